#!/usr/bin/env python3
"""Per-world candidate / contact count distribution of the collisions bench
workload at a few step counts (experiment tool)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402

W = 8192
cfg = mw.default_collisions_config(128, 4, 4096, 4096)
pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
sim = mw.CollisionsSim(W, pos, rot, cfg)
done = 0
for s in (20, 60, 130, 230, 330, 530):
    sim.step(s - done)
    done = s
    c, k = sim.counts()
    q = np.percentile(k, [50, 90, 99, 100])
    print(f"step {s}: cands mean {c.mean():.0f} max {c.max()}  contacts mean {k.mean():.1f} "
          f"p50/p90/p99/max {q}  worlds >128: {(k > 128).mean() * 100:.1f}%  "
          f"blocks(2w) with a world >128: {((k.reshape(-1, 2) > 128).any(1)).mean() * 100:.1f}%",
          flush=True)
