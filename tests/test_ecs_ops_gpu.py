"""Structural ECS operations from row-parallel nodes, out-of-tree worlds and
the device graph API (reference
include/madrona/taskgraph.inl:58-104, state.inl:398-472,
src/core/state.cpp:181-202, 584-602; device taskgraph.hpp:59-182).

The "ecs_ops" world (tests/ext_env/ecs_ops_rules.hpp) is built OUT OF TREE
against include/madrona (tests/ext_env/Makefile, the recipe of
gpu-ecs-madrona_amd/world.mk), loaded with mw_load_env and created by the
name its MADRONA_BUILD_MWGPU_ENTRY registered.  Every step its lanes call
makeTemporary (one per overlapping pair, the shape of the reference's
findOverlappingEntry), makeEntityNow and destroyEntityNow (interleaved, with
double destroys) and tmpAlloc from row-parallel nodes, plus a
CustomParallelForNode (4 lanes x 2 rows per invocation), an addOneOffNode
and an addDynamicCountNode.  The reference runs the same world serially
(oracle/ref_ecs.cpp on the reference's own ECS, oracle/_ref).

Bar: agents, pair temporaries (rows AND order), spawn contents and row
order, per-world stats: bit-exact every step.  Spawn entity IDs are made by
parallel lanes, so they are checked as SURVEY.md §8c prescribes for in-step
churn: unique, alive, each mapped by the ID store to its own row.
"""
import numpy as np
import pytest

import ecs_ops_lib as el

needs_ref = pytest.mark.skipif(not el.ref_available(), reason="oracle/_ref not built")


@pytest.mark.gpu
@needs_ref
def test_ecs_ops_every_step_matches_reference():
    W, STEPS = 8, 60
    sim = el.EcsOpsSim(W)
    ref = el.RefEcsOps(W)
    for w in range(W):
        el.compare_world(sim, ref, w, "init")
    churn = 0
    for s in range(1, STEPS + 1):
        sim.step()
        ref.step()
        assert sim.error_flags() == 0, hex(sim.error_flags())
        for w in range(W):
            el.compare_world(sim, ref, w, f"step {s}")
        churn += int(sim.agents(0)["destroyed"].sum())
    st = sim.stats(0)
    assert st["tick"] == STEPS and st["dynTicks"] == STEPS
    assert st["numPairs"] > 10 and st["numSpawns"] > 20 and churn > 100
    sim.close()


@pytest.mark.gpu
@needs_ref
def test_ecs_ops_graph_without_hipgraph_matches():
    # the same step launched node by node (no graph capture)
    W, STEPS = 4, 12
    sim = el.EcsOpsSim(W, first_world=100, use_graph=False)
    ref = el.RefEcsOps(W, first_world=100)
    sim.step(STEPS)
    ref.step(STEPS)
    for w in range(W):
        el.compare_world(sim, ref, w, f"step {STEPS}")
    sim.close()


@pytest.mark.gpu
@needs_ref
def test_ecs_ops_full_size_sampled_worlds():
    W, STEPS = 8192, 40
    sim = el.EcsOpsSim(W)
    sample = [0, 1, 4097, W - 1]
    refs = {w: el.RefEcsOps(1, first_world=w) for w in sample}
    sim.step(STEPS)
    for r in refs.values():
        r.step(STEPS)
    assert sim.error_flags() == 0, hex(sim.error_flags())
    for w, r in refs.items():
        class View:                      # world w of the sim as world 0
            def __getattr__(self, name):
                f = getattr(sim, name)
                return lambda _w, *a: f(w, *a)
        el.compare_world(View(), r, 0, f"world {w}")
    sim.close()


@pytest.mark.gpu
def test_ecs_ops_tmp_alloc_exhaustion_is_flagged_not_silent():
    # 1 KiB per world and chaining off cannot hold the lanes' scratch:
    # tmpAlloc returns null (pairsMade = -1 where it did) and
    # kErrFlagTmpAllocFull is raised
    sim = el.EcsOpsSim(4, tmp_alloc_bytes=1024, tmp_pool_bytes=-1)
    sim.step(2)
    assert sim.error_flags() & (1 << 17)
    assert (sim.agents(0)["pairsMade"] == -1).any()
    sim.close()


@pytest.mark.gpu
@needs_ref
def test_ecs_ops_tmp_alloc_chains_past_the_arena():
    # 1 KiB per world, default chaining: allocations past the arena come
    # from the chained pool (host: heap blocks), as the reference chains
    # blocks (src/core/state.cpp:95-114) -- bit-exact, no flag
    W, STEPS = 4, 20
    sim = el.EcsOpsSim(W, tmp_alloc_bytes=1024)
    ref = el.RefEcsOps(W)
    for s in range(STEPS):
        sim.step()
        ref.step()
        assert sim.error_flags() == 0, hex(sim.error_flags())
        for w in range(W):
            el.compare_world(sim, ref, w, f"step {s}")
    sim.close()


@pytest.mark.gpu
def test_ecs_ops_deferred_log_overflow_is_flagged():
    # a destroy log of one entry per world per node overflows on the first
    # step with more than one destroy: kErrFlagDeferredFull, no corruption
    # of the tables (every remaining spawn still maps to its own row)
    sim = el.EcsOpsSim(2, max_deferred_destroys=1)
    sim.step(12)
    assert sim.error_flags() & (1 << 18)
    for w in range(2):
        sp = sim.spawns(w)
        assert len(set(sp["id"].tolist())) == len(sp)
        for r, (i, g) in enumerate(zip(sp["id"], sp["gen"])):
            assert sim.entity_row(w, i, g) == r
    sim.close()


def test_ecs_ops_env_loads_out_of_tree_and_registers_by_name():
    mw = el.load_env()
    assert el.ENV_NAME in mw.env_names()
    # built outside the library: not a symbol of libmadrona_mw.so
    import subprocess
    out = subprocess.run(["nm", "-DC", "--defined-only", mw.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "EcsOps" not in out
    with pytest.raises(mw.MadronaError):
        mw.load_env("/nonexistent/libnothing.so")


@needs_ref
def test_ecs_ops_reference_workload_churns():
    # the reference run of the world exercises what the GPU test checks:
    # pairs every step, spawns made and destroyed every step, children made
    # in the same node as destroys, double destroys (serial % 7 == 0)
    ref = el.RefEcsOps(3)
    made = destroyed = 0
    for _ in range(30):
        ref.step()
        a = ref.agents(1)
        made, destroyed = int(a["spawned"].sum()), int(a["destroyed"].sum())
        assert ref.stats(1)["numPairs"] > 0
    sp = ref.spawns(1)
    assert destroyed > 150 and made - destroyed == len(sp)
    assert (sp["serial"] % 7 == 0).any()
    assert len(sp) <= 4 * el.NUM_AGENTS
