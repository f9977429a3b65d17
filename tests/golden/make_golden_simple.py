#!/usr/bin/env python3
"""Golden fixtures for simple_taskgraph from the REFERENCE (oracle/ref_harness
.cpp simple worlds compiled against /root/reference): per-body state of 3
worlds x (100 objects + agent + test object) after steps 1, 10, 60.

    python tests/golden/make_golden_simple.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

W, N, SEED, SNAPS = 3, 100, 0, (1, 10, 60)


def main():
    cfg = ol.default_phys_config(N, 4, max_contacts=1024)
    pos, rot = ol.gen_collisions_inits(W, N, seed=SEED)
    ref = ol.ReferenceSimple(cfg, pos, rot)
    out = {"pos": pos, "rot": rot}
    done = 0
    for s in SNAPS:
        ref.step(s - done)
        done = s
        for w in range(W):
            out[f"s{s}/w{w}"] = ref.bodies(w)
    np.savez_compressed(os.path.join(HERE, "simple_ref.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
