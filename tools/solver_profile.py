#!/usr/bin/env python3
"""Solver phase profile (experiment tool): run with the profiling build,
  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_prof/libmadrona_mw.so python tools/solver_profile.py [W] [collisions|simple]
(build: make -C gpu-ecs-madrona_amd BUILD=build_prof EXTRA=-DMW_SOLVER_PROFILE).
Prints the mean time per solver block in each phase over 10 settled steps."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402

PHASES = ["load+count", "order+level", "count sort", "positions", "setVelocities",
          "velocities", "writeback"]


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    wl = sys.argv[2] if len(sys.argv) > 2 else "collisions"      # or simple (configs[1])
    n = 100 if wl == "simple" else 128
    cfg = mw.default_collisions_config(n, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(W, n, seed=0)
    sim = (mw.SimpleSim if wl == "simple" else mw.CollisionsSim)(W, pos, rot, cfg)
    lib = mw.library()
    out = np.zeros(16, np.uint64)
    sim.step(int(os.environ.get('SETTLE', '220')))
    lib.mw_debug_solver_phases(out.ctypes.data_as(ctypes.c_void_p))
    sim.step(10)
    lib.mw_debug_solver_phases(out.ctypes.data_as(ctypes.c_void_p))
    blocks = int(out[7])
    tot = out[:7].astype(np.float64).sum()
    print(f"blocks {blocks}  mean max level {out[8] / blocks:.2f}")
    for i, n in enumerate(PHASES):
        print(f"{n:14s} {out[i] * 10 / 1e3 / blocks:8.2f} us/block  {100 * out[i] / tot:5.1f} %")
    print(f"{'total':14s} {tot * 10 / 1e3 / blocks:8.2f} us/block")
    nblk = W // 2
    bt = np.zeros(2 * nblk, np.uint64)
    lib.mw_debug_solver_block_times(bt.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(nblk))
    st = bt[0::2].astype(np.int64)
    en = bt[1::2].astype(np.int64)
    t0 = st.min()
    st, en = (st - t0) * 10 / 1e3, (en - t0) * 10 / 1e3
    dur = en - st
    print(f"last launch: span {en.max():.1f} us; block duration mean {dur.mean():.1f} p50 {np.median(dur):.1f} "
          f"p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}; last start {st.max():.1f}")
    for q in (0.25, 0.5, 0.75, 0.9, 1.0):
        print(f"  blocks started by {q * en.max():6.1f} us: {(st <= q * en.max()).mean() * 100:5.1f} %  "
              f"finished: {(en <= q * en.max()).mean() * 100:5.1f} %")
    passes = max(int(out[11]), 1)
    print(f"positions: static-side items {int(out[9])}, general items {int(out[10])}; wave passes {passes}, "
          f"{100 * out[12] / passes:.1f} % mixing both kinds, {100 * out[13] / passes:.1f} % with <= 16 items, "
          f"{(out[9] + out[10]) / passes:.1f} items per pass")


if __name__ == "__main__":
    main()
