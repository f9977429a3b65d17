"""Per-node launch configuration (reference MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE
/ MADRONA_MWGPU_EXEC_CONFIG_FILE, src/mw/cuda_exec.cpp:1401-1560).

CPU: the two input formats parse as the reference reads them and malformed
input is refused.  GPU: a launch configuration changes grids only, never
results -- collisions and fantasy_vs stay byte-identical to the default
configuration with capped grid-stride grids (1 block per CU) and oversized
or minimal persistent narrowphase grids, set through the C ABI and through
the environment file."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_override_format():
    import madrona_mi355x as mw
    assert mw.parse_exec_config_override("256,2,256") == (256, 2, 256)
    assert mw.parse_exec_config_override(" 64 , 0 ,0") == (64, 0, 0)
    for bad in ("", "256", "256,2", "a,2,3", "1,2,3,4", "-1,2,3", "1,,3",
                "256,65,256", "256,4294967295,256", "256,2,70000"):
        with pytest.raises(mw.MadronaError):
            mw.parse_exec_config_override(bad)


def test_config_file_format():
    import madrona_mi355x as mw
    assert mw.parse_exec_config_file('{"0": 1, "7": 16}') == [(0, 1), (7, 16)]
    assert mw.parse_exec_config_file(json.dumps({"3": 4}, indent=2)) == [(3, 4)]
    assert mw.parse_exec_config_file(" { } ") == []
    for bad in ("", "[]", '{"a": 1}', '{"1": -2}', '{"1": 2,}', '{"1" 2}', '{"1": 2} x',
                '{"1": 2.5}', '{1: 2}',
                # out of range: keys past INT32_MAX, block counts past 64 per CU
                '{"4294967295": 1}', '{"2147483648": 1}', '{"0": 65}', '{"0": 4294967295}'):
        with pytest.raises(mw.MadronaError):
            mw.parse_exec_config_file(bad)


def _collisions(mw, W, seed):
    g = mw.default_collisions_config(128, 4, 2048, 4096)
    pos, rot = ol.gen_collisions_inits(W, 128, seed=seed)
    return mw.CollisionsSim(W, pos, rot, g)


@pytest.mark.gpu
def test_collisions_launch_config_does_not_change_results():
    import madrona_mi355x as mw
    W = 96
    base = _collisions(mw, W, 5)
    cfg = _collisions(mw, W, 5)
    names = cfg.nodes()
    assert "NarrowphaseNode" in names and "CustomParallelForNode" in names
    cfg.set_node_blocks_per_cu(-1, 1)               # every node: 1 block / CU
    narrow = names.index("NarrowphaseNode")
    cfg.set_node_blocks_per_cu(narrow, 64)          # persistent grids past residency
    assert cfg.node_blocks_per_cu(narrow) == 64 and cfg.node_blocks_per_cu(0) == 1
    base.step(20)
    cfg.step(20)
    cfg.set_node_blocks_per_cu(narrow, -1)          # back to the default (1)
    assert cfg.node_blocks_per_cu(narrow) == 1
    base.step(20)
    cfg.step(20)
    assert cfg.error_flags() == 0
    for w in range(W):
        assert base.bodies(w).tobytes() == cfg.bodies(w).tobytes(), f"world {w}"
    assert base.exported_array(2, np.float32).tobytes() == cfg.exported_array(2, np.float32).tobytes()


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import madrona_mi355x as mw, oracle_lib as ol
kind, out = sys.argv[3], sys.argv[4]
if kind == "collisions":
    g = mw.default_collisions_config(128, 4, 2048, 4096)
    pos, rot = ol.gen_collisions_inits(40, 128, seed=9)
    s = mw.CollisionsSim(40, pos, rot, g)
    names = s.nodes()
    print("CFG", s.node_blocks_per_cu(-1), s.node_blocks_per_cu(names.index("NarrowphaseNode")),
          s.node_blocks_per_cu(names.index("CustomParallelForNode")))
    s.step(15)
    assert s.error_flags() == 0
    np.save(out, np.stack([s.bodies(w) for w in range(40)]))
else:
    inits = ol.gen_fvs_inits(300, 50, 200, seed=3)
    s = mw.FvsSim(300, inits)
    s.step(700)
    np.save(out, np.concatenate([np.frombuffer(s.table(w, a).tobytes(), np.uint8)
                                 for w in range(300) for a in (0, 1)]))
"""


def _child(kind, out, env):
    r = subprocess.run([sys.executable, "-c", _CHILD,
                        os.path.join(ROOT, "gpu-ecs-madrona_amd"), os.path.join(ROOT, "tests"),
                        kind, str(out)], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


@pytest.mark.gpu
def test_one_block_grids_from_the_environment(tmp_path):
    # override "threads,blocksPerCU,numCUs" = 1 block on 1 CU: every
    # grid-stride kernel (ParallelForNode rows, PerWorldNode worlds) and
    # both persistent narrowphase kernels run as a single block
    import madrona_mi355x as mw
    env = dict(os.environ, MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE="256,1,1")
    env.pop("MADRONA_MWGPU_EXEC_CONFIG_FILE", None)
    _child("collisions", tmp_path / "c.npy", env)
    ref = _collisions(mw, 40, 9)
    ref.step(15)
    assert np.load(tmp_path / "c.npy").tobytes() == \
        np.stack([ref.bodies(w) for w in range(40)]).tobytes()
    del ref
    _child("fvs", tmp_path / "f.npy", env)
    inits = ol.gen_fvs_inits(300, 50, 200, seed=3)
    a = mw.FvsSim(300, inits)
    a.step(700)
    want = np.concatenate([np.frombuffer(a.table(w, k).tobytes(), np.uint8)
                           for w in range(300) for k in (0, 1)])
    assert np.load(tmp_path / "f.npy").tobytes() == want.tobytes()


@pytest.mark.gpu
def test_environment_config_file_is_applied(tmp_path):
    import madrona_mi355x as mw
    probe = _collisions(mw, 40, 9)
    names = probe.nodes()
    probe.step(15)
    ref = np.stack([probe.bodies(w) for w in range(40)])
    cfg_file = tmp_path / "exec.json"
    cfg_file.write_text(json.dumps({str(names.index("NarrowphaseNode")): 3}))
    env = dict(os.environ, MADRONA_MWGPU_EXEC_CONFIG_FILE=str(cfg_file),
               MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE="256,2,32")
    r = _child("collisions", tmp_path / "b.npy", env)
    assert "CFG 2 3 2" in r.stdout
    assert "Taskgraph node" in r.stderr
    assert np.load(tmp_path / "b.npy").tobytes() == ref.tobytes()
