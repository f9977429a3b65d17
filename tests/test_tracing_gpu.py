"""GPU: device tracing (reference MADRONA_TRACING,
src/mw/device/include/madrona/mw_gpu/tracing.hpp:14-128).  The records must
satisfy what scripts/parse_device_tracing.py asserts when it reads them
(madrona_mi355x.tracing.check_contract restates parse_device_logs /
block_analysis, :11-118, :146-230), and tracing must not change the
simulation.  The default library logs step and node records; block records
come from the tracing build (build_trace/, -DMW_TRACING), checked in a child
process because the library is chosen at import."""
import os
import subprocess
import sys

import pytest

from oracle_lib import gen_collisions_inits

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACE_LIB = os.path.join(ROOT, "gpu-ecs-madrona_amd", "build_trace", "libmadrona_mw.so")


def _sim(W=64, n=32, use_graph=True):
    import madrona_mi355x as mw
    cfg = mw.default_collisions_config(n, 4, 1024, 2048)
    pos, rot = gen_collisions_inits(W, n, seed=4)
    return mw.CollisionsSim(W, pos, rot, cfg, use_graph=use_graph)


@pytest.mark.parametrize("use_graph", [True, False])
def test_node_records_follow_the_parser_contract(use_graph):
    from madrona_mi355x import tracing as tr
    sim = _sim(use_graph=use_graph)
    sim.step(2)
    sim.enable_tracing(1 << 20)
    sim.step(3)
    recs, dropped = sim.trace_records()
    names = sim.trace_func_names()
    assert dropped == 0 and len(recs) > 0
    assert {"SolverNode", "NarrowphaseNode", "FindOverlappingNode", "ExportNode"} <= set(names)
    assert tr.check_contract(recs, names, 64, sim.trace_block_records()) == 3
    summ = tr.summarize(recs, names)
    assert summ["SolverNode"]["launches_per_step"] == 4
    assert summ["SolverNode"]["ns_per_step"] > 0


def test_tracing_does_not_change_the_simulation():
    a, b = _sim(), _sim()
    a.enable_tracing(1 << 18)
    a.step(6)
    b.step(6)
    for w in (0, 17, 63):
        x, y = a.bodies(w), b.bodies(w)
        assert all(x[f].tobytes() == y[f].tobytes() for f in x.dtype.names)


def test_tracing_overflow_drops_and_disable(tmp_path):
    import madrona_mi355x as mw
    sim = _sim()
    sim.enable_tracing(20)
    sim.step(2)
    recs, dropped = sim.trace_records()
    assert len(recs) == 20 and dropped > 0
    p = tmp_path / "trace.bin"
    assert sim.dump_trace(p) == 20 and p.stat().st_size == 800
    sim.enable_tracing(0)
    sim.step(1)
    assert sim.error_flags() == 0
    with pytest.raises(mw.MadronaError):
        sim.trace_records()


@pytest.mark.skipif(not os.path.exists(TRACE_LIB), reason="tracing build absent (make trace)")
def test_tracing_build_block_records(tmp_path):
    out = tmp_path / "trace.bin"
    env = dict(os.environ, MADRONA_MW_LIB=TRACE_LIB)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_check.py"), str(out)],
                       env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "trace contract ok" in r.stdout
    assert out.stat().st_size % 40 == 0 and out.stat().st_size > 0
