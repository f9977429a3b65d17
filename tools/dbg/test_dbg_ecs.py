import ecs_ops_lib as el
import numpy as np

def test_dbg():
    W = 8
    for tb in (64 * 1024, 1 << 20):
        sim = el.EcsOpsSim(W, tmp_alloc_bytes=tb)
        ref = el.RefEcsOps(W)
        print("tb", tb, "created", hex(sim.error_flags()))
        sim.step(); ref.step()
        print("step1", hex(sim.error_flags()))
        for w in range(W):
            a = sim.agents(w)
            print(w, "pm", (a["pairsMade"] == -1).sum(), "destroyed", a["destroyed"].sum(), "spawned", a["spawned"].sum())
        sim.close()
