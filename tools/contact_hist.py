#!/usr/bin/env python3
"""Distribution of contacts per world in the bench's settled window
(collisions, 8192 worlds): how many worlds exceed the solver's LDS record
budget (experiment tool)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def main():
    W = 8192
    cfg = mw.default_collisions_config(128, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
    sim = mw.CollisionsSim(W, pos, rot, cfg)
    sim.step(130)
    ks = []
    for _ in range(20):
        sim.step(10)
        c, k = sim.counts()
        ks.append(k)
    k = np.concatenate(ks)
    print("contacts/world mean %.1f p50 %d p90 %d p99 %d max %d" %
          (k.mean(), np.median(k), np.percentile(k, 90), np.percentile(k, 99), k.max()))
    for t in (96, 128, 160, 192, 224, 256):
        print(f"  > {t}: {100 * (k > t).mean():5.2f} %")
    # block view: heaviest-first pairs (sorted by survivor count ~ contacts)
    for t in (128, 192, 224):
        srt = np.sort(k.reshape(20, W), axis=1)[:, ::-1]
        pairs = np.maximum(srt[:, 0::2], srt[:, 1::2])
        print(f"  blocks (sorted pairs) with a world > {t}: {100 * (pairs > t).mean():5.2f} %")


if __name__ == "__main__":
    main()
