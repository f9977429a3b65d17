#!/usr/bin/env python3
"""Golden fixtures for fantasy_vs from the REFERENCE ECS (oracle/ref_fvs.cpp
compiled against /root/reference by oracle/Makefile.ref): Dragon / Knight
tables (entity gen + id, position, hp, action timer, mana / arrows) of 4
worlds at ticks 250, 1000, 1500 (seed 0) and 600, 900, 1300 (seed 7),
spanning the dragons' deaths (destroy, swap-remove, ID reuse by the
cleanup trackers).  Run in the build container:

    python tests/golden/make_golden_fvs.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

CASES = {"base": (4, 50, 200, 0, (250, 1000, 1500)),
         "seed7": (4, 50, 200, 7, (600, 900, 1300))}


def main():
    out = {}
    for name, (W, nd, nk, seed, ticks) in CASES.items():
        inits = ol.gen_fvs_inits(W, nd, nk, seed=seed)
        for k, v in inits.items():
            out[f"{name}/init/{k}"] = v
        ref = ol.ReferenceFvs(inits)
        done = 0
        for t in ticks:
            ref.step(t - done)
            done = t
            for w in range(W):
                for arch in (0, 1):
                    out[f"{name}/t{t}/w{w}/a{arch}"] = ref.table(w, arch)
    np.savez_compressed(os.path.join(HERE, "fvs_ref.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
