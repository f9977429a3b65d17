import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw
import ecs_ops_lib as el
mode = sys.argv[1]
W = 8
import time
sim = el.EcsOpsSim(W, use_graph=(mode != "lookup_nograph"))
ref = el.RefEcsOps(W)
for s in range(1, 61):
    sim.step(); ref.step()
    f = sim.error_flags()
    if f:
        bad = [w for w in range(W) if (sim.agents(w)["pairsMade"] == -1).any()]
        print(mode, "first flag at step", s, hex(f), "bad worlds", bad)
        break
    for w in range(W):
        if mode == "full":
            el.compare_world(sim, ref, w, f"step {s}")
        elif mode == "agents":
            sim.agents(w)
        elif mode == "spawns":
            sim.spawns(w)
        elif mode == "sleep":
            time.sleep(0.002)
        elif mode == "lookup0":
            sp = sim.spawns(w)
            if len(sp):
                for _ in range(len(sp)):
                    sim.exec.entity_loc(w, 0, 0)
        elif mode in ("lookup", "lookup_nograph"):
            sp = sim.spawns(w)
            for i, g in zip(sp["id"], sp["gen"]):
                sim.entity_row(w, i, g)
else:
    print(mode, "clean")
