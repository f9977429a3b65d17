#!/usr/bin/env python3
"""findOverlaps phase profile (experiment tool): run with the profiling build,
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so python tools/overlap_profile.py
(build: make -C gpu-ecs-madrona_amd BUILD=build_prof EXTRA=-DMW_SOLVER_PROFILE).
Prints the mean time per findOverlaps block (thread 0's view) in each phase
over 10 settled steps."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402

PHASES = ["staging", "sweep (wave 0)", "scan (all waves)", "writes"]


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    cfg = mw.default_collisions_config(128, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
    sim = mw.CollisionsSim(W, pos, rot, cfg)
    lib = mw.library()
    out = np.zeros(8, np.uint64)
    sim.step(int(os.environ.get('SETTLE', '220')))
    lib.mw_debug_overlap_phases(out.ctypes.data_as(ctypes.c_void_p))
    sim.step(10)
    lib.mw_debug_overlap_phases(out.ctypes.data_as(ctypes.c_void_p))
    blocks = int(out[7])
    tot = out[:4].astype(np.float64).sum()
    print(f"blocks {blocks}")
    for i, n in enumerate(PHASES):
        print(f"{n:18s} {out[i] * 10 / 1e3 / blocks:8.2f} us/block  {100 * out[i] / tot:5.1f} %")
    print(f"{'total':18s} {tot * 10 / 1e3 / blocks:8.2f} us/block")


if __name__ == "__main__":
    main()
