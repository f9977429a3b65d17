"""The CPU back end (libmadrona_cpu.so: the reference's TaskGraphExecutor /
ThreadPoolExecutor, include/madrona/mw_cpu.hpp:53-81, src/mw/cpu_exec.cpp:
31-284) steps the SAME world sources, graph and C ABI as the gfx950 library
on pinned host threads.  No GPU needed: these run in the CPU suite.

The gfx950 parity tests are re-run unchanged against the CPU back end
(mw.DEFAULT_BACKEND = "cpu"), so the CPU executor is held to the same bars:
bit-exact against the oracle, the live reference (oracle/_ref) and the
reference's golden fixtures for collisions, joints, OBJ hulls,
simple_taskgraph, fantasy_vs, both job-API examples and the out-of-tree
ecs_ops world.  Worker count never changes a bit.
"""
import importlib

import numpy as np
import pytest

import oracle_lib as ol


@pytest.fixture
def cpu(monkeypatch):
    import madrona_mi355x as mw
    monkeypatch.setattr(mw, "DEFAULT_BACKEND", "cpu")
    return mw


# (module, test function[, params]) of the gfx950 suite that also run here;
# the 8192-world sampled tests are left to the GPU (minutes of CPU time).
CASES = [
    ("test_collisions_gpu", "test_collisions_bit_exact_vs_oracle_small", {}),
    ("test_collisions_gpu", "test_collisions_bit_exact_ragged_worlds_one_substep", {}),
    ("test_collisions_gpu", "test_collisions_bvh_matches_oracle_after_first_step", {}),
    ("test_collisions_gpu", "test_collisions_bit_exact_long_horizon_contacts", {}),
    ("test_collisions_gpu", "test_episode_return_export_matches_oracle", {}),
    ("test_simple_gpu", "test_simple_taskgraph_matches_golden", {}),
    ("test_simple_gpu", "test_simple_taskgraph_matches_oracle_and_reference", {"nsub": 4, "seed": 9}),
    ("test_simple_gpu", "test_simple_taskgraph_matches_oracle_and_reference", {"nsub": 1, "seed": 0}),
    ("test_joints_gpu", "test_fixed_joints_bit_exact_vs_oracle_every_step", {}),
    ("test_joints_gpu", "test_joints_match_reference_golden", {}),
    ("test_joints_gpu", "test_hinge_joints_bit_exact_while_finite", {}),
    ("test_joints_gpu", "test_many_joints_take_the_global_record_path", {}),
    ("test_hulls_gpu", "test_hull_worlds_match_reference_golden", {}),
    ("test_fvs_gpu", "test_fvs_bit_exact_through_deaths", {}),
    ("test_fvs_gpu", "test_fvs_every_tick_around_first_deaths", {}),
    ("test_fvs_gpu", "test_fvs_golden_fixture_on_gpu", {}),
    ("test_jobs_gpu", "test_fvs_jobs_matches_oracle_through_deaths", {}),
    ("test_jobs_gpu", "test_fvs_jobs_every_tick_around_first_deaths", {}),
    ("test_jobs_gpu", "test_collisions_jobs_matches_oracle_every_tick", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_every_step_matches_reference", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_tmp_alloc_exhaustion_is_flagged_not_silent", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_tmp_alloc_chains_past_the_arena", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_reference_workload_churns", {}),
]


@pytest.mark.parametrize("module,name,params", CASES,
                         ids=[f"{m}::{n}" + ("-" + "-".join(f"{k}{v}" for k, v in p.items()) if p else "")
                              for m, n, p in CASES])
def test_gpu_parity_suite_on_cpu_backend(cpu, module, name, params):
    fn = getattr(importlib.import_module(module), name)
    fn(**params)


def test_hull_worlds_every_step_on_cpu_backend(cpu):
    import test_hulls_gpu as th
    fn = th.test_hull_worlds_bit_exact_vs_oracle_every_step
    for mark in fn.pytestmark:
        if mark.name == "parametrize":
            argnames = [a.strip() for a in mark.args[0].split(",")]
            for values in mark.args[1]:
                fn(**dict(zip(argnames, values)))


def test_cpu_backend_is_the_loaded_library(cpu):
    # the CPU executor really is libmadrona_cpu.so (not the HIP library)
    pos, rot = ol.gen_collisions_inits(2, 8, seed=1)
    sim = cpu.CollisionsSim(2, pos, rot, cpu.default_collisions_config(8, 1, 256, 256))
    assert sim.backend == "cpu" and sim._lib is cpu.cpu_library()
    sim.step(3)
    assert sim.error_flags() == 0
    with pytest.raises(cpu.MadronaError, match="gfx950"):
        sim.allgather_exported(2, 0, 4)


@pytest.mark.parametrize("workers", [1, 3])
def test_worker_count_never_changes_a_bit(cpu, workers):
    pos, rot = ol.gen_collisions_inits(6, 128, seed=4)
    g = cpu.default_collisions_config(128, 4, 4096, 4096)
    a = cpu.CollisionsSim(6, pos, rot, g, num_workers=workers)
    b = cpu.CollisionsSim(6, pos, rot, g, num_workers=0)
    a.step(40)
    b.step(40)
    for w in range(6):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
        assert a.contacts(w).tobytes() == b.contacts(w).tobytes()


def test_multi_step_world_major_equals_single_steps(cpu):
    # mw_step(n) on the CPU back end runs each world's n steps back to back on
    # one worker (every collisions node is world-local); states and the
    # exported buffers must equal n separate steps.
    pos, rot = ol.gen_collisions_inits(5, 64, seed=11)
    g = cpu.default_collisions_config(64, 4, 2048, 2048)
    a = cpu.CollisionsSim(5, pos, rot, g, num_workers=3)
    b = cpu.CollisionsSim(5, pos, rot, g, num_workers=3)
    a.step(25)
    for _ in range(25):
        b.step(1)
    for w in range(5):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
        assert a.contacts(w).tobytes() == b.contacts(w).tobytes()
    for slot in range(3):
        assert a.exported_array(slot, np.uint8).tobytes() == b.exported_array(slot, np.uint8).tobytes()


@pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_collisions_bit_exact_vs_live_reference(cpu):
    # The CPU back end against the reference itself (not the restatement),
    # every step of each world until the oracle counts the first face
    # manifold the reference leaves undefined.
    from test_collisions_gpu import _cfg_pair, _diff
    gcfg, ocfg = _cfg_pair()
    W = 3
    pos, rot = ol.gen_collisions_inits(W, 128, seed=7)
    sim = cpu.CollisionsSim(W, pos, rot, gcfg)
    ref = ol.ReferencePhys(ocfg, pos, rot)
    orc = ol.OraclePhys(ocfg, pos, rot)
    compared = 0
    for s in range(60):
        sim.step()
        ref.step()
        orc.step()
        for w in range(W):
            if orc.ub_manifolds(w):
                continue
            d = _diff(sim.bodies(w), ref.bodies(w))
            assert d is None, f"step {s} world {w}: {d}"
            compared += 1
    assert compared >= W * 30, compared
    assert np.sum(sim.counts()[1]) > 0


@pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_fvs_bit_exact_vs_live_reference(cpu):
    # fantasy_vs on the CPU back end against the reference's own ECS
    # (oracle/ref_fvs.cpp), not the restatement: every column of both tables,
    # ids, generations and the swap-remove row order, through the deaths.
    W = 3
    inits = ol.gen_fvs_inits(W, 50, 200, seed=5)
    sim = cpu.FvsSim(W, inits, backend="cpu", num_workers=2)
    ref = ol.ReferenceFvs(inits)
    for t in range(1, 13):
        sim.step(100)
        ref.step(100)
        for w in range(W):
            for arch in (0, 1):
                a, b = sim.table(w, arch), ref.table(w, arch)
                assert a.tobytes() == b.tobytes(), f"tick {100 * t} world {w} arch {arch}"
    assert sum(len(ref.table(w, 0)) for w in range(W)) < 50 * W      # dragons died



def test_node_index_timing_on_cpu_backend(cpu):
    # set_timed_node_index times one node of the graph (here the markDead
    # ParallelForNode, the fourth of five), not every node of its kind.
    inits = ol.gen_fvs_inits(4, 50, 200, seed=1)
    sim = cpu.FvsSim(4, inits, backend="cpu", num_workers=2)
    kinds = sim.nodes()
    mark = [i for i, k in enumerate(kinds) if k == "ParallelForNode"][3]
    sim.set_timed_node_index(mark)
    sim.step(3)
    ms, n = sim.timed_node()
    assert n == 3 and ms > 0
    sim.set_timed_node("ParallelForNode")
    sim.step(2)
    assert sim.timed_node()[1] == 2 * kinds.count("ParallelForNode")
    with pytest.raises(RuntimeError, match="past the graph"):
        sim.set_timed_node_index(len(kinds))
