import sys
sys.path.insert(0, "gpu-ecs-madrona_amd"); sys.path.insert(0, "tests")
import numpy as np
import madrona_mi355x as mw
from oracle_lib import gen_collisions_inits
from test_collisions_gpu import _cfg_pair
g, o = _cfg_pair()
pos, rot = gen_collisions_inits(2, 128, seed=0)
sim = mw.CollisionsSim(2, pos, rot, g, use_graph=False)
for a in range(mw.library().mw_num_archetypes(sim.h)):
    try:
        print(a, sim.read_column(a, 0, 0, np.uint32)[:6], sim.read_column(a, 1, 0, np.float32)[:6])
    except Exception as e:
        print(a, "err", e)
inits = mw.gen_fvs_inits(2)
f = mw.FvsSim(2, inits)
print("fvs", f.table(0, 0)[:2])
