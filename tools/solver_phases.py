import sys, os
sys.path.insert(0, "gpu-ecs-madrona_amd")
import madrona_mi355x as mw
cfg = mw.default_collisions_config(128, 4, max_contacts=4096, max_candidates=4096)
pos, rot = mw.gen_collisions_inits(8192, 128, seed=0)
sim = mw.CollisionsSim(8192, pos, rot, cfg)
sim.step(125)
print("DONE", sim.error_flags(), flush=True)
