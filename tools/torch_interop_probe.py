"""Probe: can the executor share a process with torch's GPU runtime?

  mode "madrona_first": import madrona_mi355x, then use torch.cuda.
  mode "torch_first":   torch.cuda first, then madrona_mi355x (foreign HIP
                        runtime allowed), library from $MADRONA_MW_LIB.
Runs 4 collisions worlds x 20 steps against the oracle and copies an exported
column into a torch tensor."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
mode = sys.argv[1]
if mode == "torch_first":
    import torch
    t = torch.ones(8, device="cuda")
    print("torch ok", torch.version.hip, float(t.sum()), flush=True)
    os.environ["MADRONA_MW_ALLOW_FOREIGN_HIP"] = "1"
    import madrona_mi355x as mw
else:
    import madrona_mi355x as mw
    import torch
import numpy as np
import oracle_lib as ol
from test_collisions_gpu import _cfg_pair, _diff

print("torch.cuda.is_available", torch.cuda.is_available(), flush=True)
maps = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
print("hip runtimes mapped:", maps, flush=True)
gcfg, ocfg = _cfg_pair(num_cubes=32)
pos, rot = ol.gen_collisions_inits(4, 32, seed=3)
sim = mw.CollisionsSim(4, pos, rot, gcfg)
orc = ol.OraclePhys(ocfg, pos, rot)
sim.step(20)
orc.step(20)
for w in range(4):
    d = _diff(sim.bodies(w), orc.bodies(w))
    assert d is None, d
print("parity ok", flush=True)
if torch.cuda.is_available():
    out = torch.zeros(4, device="cuda")
    sim.copy_exported(2, out.data_ptr(), 16)
    torch.cuda.synchronize()
    print("exported into torch:", out.cpu().numpy(), flush=True)
print("PROBE OK", mode)
