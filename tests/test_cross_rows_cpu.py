"""The cross_rows world (cross-row component writes, row-to-row carried
state, entity churn whose IDs are stored in components) on the framework's
CPU back end, against the same world on the reference's ECS, every step.
The CPU back end walks every world's rows serially (reference
ParallelForNode::run, include/madrona/taskgraph.inl:63-71), so the world is
bit-exact there, entity IDs included."""
import pytest

import cross_rows_lib as cl

pytestmark = pytest.mark.skipif(not cl.ref_available(), reason="reference build absent (GPU box)")


@pytest.mark.parametrize("per_node_serial", [False, True])
def test_cross_rows_cpu_backend_matches_reference_every_step(per_node_serial):
    W, steps = 3, 60
    sim = cl.CrossSim(W, per_node_serial=per_node_serial, backend="cpu", num_workers=2)
    ref = cl.RefCross(W)
    for w in range(W):
        cl.compare_world(sim, ref, w, "init")
    grew = churned = False
    for s in range(steps):
        sim.step()
        ref.step()
        assert sim.error_flags() == 0
        for w in range(W):
            cl.compare_world(sim, ref, w, f"step {s}")
            st = ref.stats(w)
            grew |= st["cells"] > cl.NUM_CELLS
            churned |= st["sparks"] > 0
    assert grew and churned, "the workload must split cells and churn sparks"


def test_ecs_ops_cpu_backend_entity_ids_exact():
    """The CPU back end is world-serial, so even the entity IDs of spawns made
    inside a ParallelForNode are the reference's (not only up to relabelling)."""
    import ecs_ops_lib as el
    W = 4
    sim, ref = el.EcsOpsSim(W, backend="cpu", num_workers=2), el.RefEcsOps(W)
    for s in range(40):
        sim.step()
        ref.step()
        for w in range(W):
            el.compare_world(sim, ref, w, f"step {s}", exact_ids=True)
