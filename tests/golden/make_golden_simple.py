#!/usr/bin/env python3
"""Golden fixtures for simple_taskgraph.

  * s{1,10,50}/w*: per-body state of 3 worlds x (100 objects + agent + test
    object) from the REFERENCE (oracle/ref_harness.cpp simple worlds compiled
    against /root/reference);
  * orc_s150/w*: the same worlds after 150 steps on the oracle
    (oracle/mw_oracle.cpp simple mode), past the first face manifold whose
    reference value is undefined (narrowphase.cpp:828-853 leaves a slot of an
    uninitialised Manifold unwritten; DESIGN.md "reference UB");
  * ub_first: per world, the first step with such a manifold.

The oracle is checked bit-exact against the reference on every step before
ub_first (asserted here and in tests/test_simple_oracle.py).

    python tests/golden/make_golden_simple.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

W, N, SEED, SNAPS, ORC_STEPS = 3, 100, 0, (1, 10, 50), 150


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def main():
    cfg = ol.default_phys_config(N, 4, max_contacts=1024)
    pos, rot = ol.gen_collisions_inits(W, N, seed=SEED)
    ref = ol.ReferenceSimple(cfg, pos, rot)
    orc = ol.OracleSimple(cfg, pos, rot)
    out = {"pos": pos, "rot": rot}
    ub_first = np.zeros(W, np.int32)
    for s in range(1, ORC_STEPS + 1):
        orc.step(1)
        if s <= max(SNAPS) or not ub_first.all():
            ref.step(1)
        for w in range(W):
            if ub_first[w] == 0 and orc.ub_manifolds(w):
                ub_first[w] = s
            if ub_first[w] == 0:
                assert _eq(orc.bodies(w), ref.bodies(w)), f"oracle != reference at step {s} world {w}"
            if s in SNAPS:
                assert ub_first[w] == 0, "snapshot past an undefined manifold"
                out[f"s{s}/w{w}"] = ref.bodies(w)
    for w in range(W):
        out[f"orc_s{ORC_STEPS}/w{w}"] = orc.bodies(w)
    out["ub_first"] = ub_first
    np.savez_compressed(os.path.join(HERE, "simple_ref.npz"), **out)
    print("wrote", len(out), "arrays; first undefined manifold per world:", ub_first)


if __name__ == "__main__":
    main()
