import sys
sys.path.insert(0, "gpu-ecs-madrona_amd"); sys.path.insert(0, "tests")
import numpy as np
import madrona_mi355x as mw
from oracle_lib import OraclePhys, PhysConfig, gen_collisions_inits
from test_collisions_gpu import _cfg_pair, _diff
g, o = _cfg_pair()
pos, rot = gen_collisions_inits(2, 128, seed=0)
for backend in ("cpu", "gpu"):
    sim = mw.CollisionsSim(2, pos, rot, g, backend=backend)
    orc = OraclePhys(o, pos, rot)
    a, b = sim.bodies(0), orc.bodies(0)
    print(backend, _diff(a, b))
    for f in a.dtype.names:
        if a[f].tobytes() != b[f].tobytes():
            print(" ", f, a[f][:3], b[f][:3])
