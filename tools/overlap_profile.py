#!/usr/bin/env python3
"""findOverlaps phase profile (experiment tool): run with the profiling build,
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so python tools/overlap_profile.py
(build: make -C gpu-ecs-madrona_amd BUILD=build_prof EXTRA=-DMW_SOLVER_PROFILE).
Prints the mean time per findOverlaps block (thread 0's view) in each phase
over 10 settled steps.  [W] [n] [grid]: n cubes per world; "grid" lays them
out as tests/test_lds_fallback_gpu.py's grid worlds (MADRONA_MW_OVERLAP_DFS_LEAVES
picks the traversal)."""
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
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    if len(sys.argv) > 3 and sys.argv[3] == "grid":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_lds_fallback_gpu import _grid_world
        pos, rot = _grid_world(W, n)
        cfg = mw.default_collisions_config(n, 4, 8192, 8192)
    else:
        cfg = mw.default_collisions_config(n, 4, 4096, 4096)
        pos, rot = mw.gen_collisions_inits(W, n, seed=0)
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
    if out[5]:
        print(f"DFS queries {int(out[5])}, nodes popped per query {out[4] / out[5]:.1f}, "
              f"wide {int(out[6])}")


if __name__ == "__main__":
    main()
