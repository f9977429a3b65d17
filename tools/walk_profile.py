#!/usr/bin/env python3
"""World-walk profile (experiment tool): fantasy_vs with the walk, per walk
entry the mean time one world's call took and its share of the walk.

  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_wp/libmadrona_mw.so \\
      MADRONA_MW_WORLD_WALK=1 python tools/walk_profile.py [W] [preroll] [ticks]
(build: make -C gpu-ecs-madrona_amd BUILD=build_wp EXTRA=-DMW_WALK_PROFILE)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    pre = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    sim = mw.FvsSim(W, mw.gen_fvs_inits(W, 50, 200, seed=0))
    lib = mw.library()
    rd = lib.mw_debug_walk_profile_fvs
    rd.argtypes = [ctypes.c_void_p]
    out = np.zeros(128, np.uint64)
    print("walk runs per tick:", sim.world_walk_runs(), "nodes:",
          [f"{i}:{n}" for i, n in enumerate(sim.nodes())])
    sim.step(pre)
    sim.sync()
    rd(out.ctypes.data)
    t0 = time.perf_counter()
    sim.step(ticks)
    sim.sync()
    dt = time.perf_counter() - t0
    rd(out.ctypes.data)
    print(f"{ticks} ticks, {dt / ticks * 1e3:.4f} ms/tick, {W * ticks / dt / 1e6:.1f} M env-steps/s")
    tot = out[:64].astype(np.float64).sum()
    for i in range(64):
        if out[64 + i] == 0:
            continue
        per_call_us = out[i] / out[64 + i] * 0.01          # 100 MHz ticks -> us
        print(f"entry {i:2d}: sampled calls/tick {out[64 + i] / ticks:6.0f}  {per_call_us:7.3f} us per world  "
              f"{100 * out[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
