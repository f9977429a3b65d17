#!/usr/bin/env python3
"""SAT stage profile (experiment tool).
  make -C gpu-ecs-madrona_amd BUILD=build_prof EXTRA=-DMW_SAT_PROFILE
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so python tools/sat_profile.py [simple|collisions]
      where the hull-hull SAT of each pair ends and the group leader's clock
      per phase over 10 settled steps (the counters' atomics slow the kernel
      several-fold: shares only);
  make -C gpu-ecs-madrona_amd BUILD=build_cut EXTRA=-DMW_SAT_CUTS
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_cut/libmadrona_mw.so python tools/sat_profile.py [simple|collisions] --cuts
      NarrowphaseNode time with the SAT cut after each phase;
  ... python tools/sat_profile.py [simple|collisions] --solver-cuts
      the solver kernel cut after each of its phases (same build)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "simple"
    W = 8192
    n = 100 if wl == "simple" else 128
    cfg = mw.default_collisions_config(n, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(W, n, seed=0)
    sim = (mw.SimpleSim if wl == "simple" else mw.CollisionsSim)(W, pos, rot, cfg)
    lib = mw.library()
    sim.step(130)
    if "--solver-cuts" in sys.argv:
        lib.mw_debug_time_solver.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        lib.mw_debug_time_solver.restype = ctypes.c_double
        sim.sync()
        names = ["load+count", "+levels", "+sort", "+positions", "+setVelocities", "+velocities",
                 "whole (no fused integration)", "+positions' loads only"]
        for cut, nm in zip((1, 2, 3, 4, 5, 6, 0, 7), names):
            ms = lib.mw_debug_time_solver(cut, 20, 3)
            print(f"solverKernel cut {cut} ({nm:30s}) {ms:.4f} ms/launch (last substep, 20 launches)")
        return
    if "--cuts" in sys.argv:
        lib.mw_debug_time_sat.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        lib.mw_debug_time_sat.restype = ctypes.c_double
        sim.sync()
        names = ["full", "staging", "+faces", "+tables", "+masks", "+edges", "full"]
        for cut, nm in zip((0, 1, 2, 3, 5, 4, 0), names):
            ms = lib.mw_debug_time_sat(cut, 20, 3)
            print(f"narrowSATKernel cut {cut} ({nm:8s}) {ms:.4f} ms/launch (last substep's list, 20 launches)")
        return
    lib.mw_debug_sat_stages.argtypes = [ctypes.c_void_p]
    out = np.zeros(16, np.uint64)
    lib.mw_debug_sat_stages(out.ctypes.data_as(ctypes.c_void_p))
    sim.step(10)
    lib.mw_debug_sat_stages(out.ctypes.data_as(ctypes.c_void_p))
    pairs = int(out[0])
    names = ["pairs", "sep face a", "sep face b", "sep edge", "face contact", "edge contact"]
    for i, nm in enumerate(names):
        print(f"{nm:14s} {int(out[i]):12d}  {100 * out[i] / max(pairs, 1):6.2f} %  per world-substep "
              f"{out[i] / (W * 40):8.2f}")
    ticks = out[8:13].astype(np.float64)
    for i, nm in enumerate(["staging", "faces a", "faces b", "edges", "job"]):
        print(f"{nm:10s} {100 * ticks[i] / ticks.sum():6.2f} % of leader clock, "
              f"{ticks[i] / max(pairs, 1) * 10:8.1f} ns/pair")


if __name__ == "__main__":
    main()
