#!/usr/bin/env python3
"""Golden fixtures for the joint workload (collisions + ConstraintData rows,
reference handleJointConstraint, src/physics/physics.cpp:478-648).

  * fixed/s{1,20,50,100,150}/w*: per-body state of 4 worlds x 32 cubes + plane with
    8 fixed joints (oracle_lib.joint_inits, seed 13) from the REFERENCE
    (oracle/ref_harness.cpp compiled against /root/reference);
  * fixed/orc_s300/w*: the same worlds after 300 steps on the oracle, past the
    first undefined face manifold (DESIGN.md §4 "reference UB");
  * hinge/s{1..12}/w*: 2 worlds x 8 cubes with 2 fixed + 2 hinge joints, every
    step of the 12 the reference's hinge stays finite (it diverges: its
    positional correction has the opposite sign to the fixed joint's,
    physics.cpp:616-627 vs 597-614);
  * ub_first: per fixed-joint world, the first step with an undefined manifold.

The oracle is asserted bit-exact against the reference on every step before
ub_first.

    python tests/golden/make_golden_joints.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

FIXED = dict(W=4, N=32, J=8, H=0, SEED=13, SNAPS=(1, 20, 50, 100, 150), ORC=300)
HINGE = dict(W=2, N=8, J=4, H=2, SEED=1, STEPS=12)


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def joint_config(n, j, h):
    cfg = ol.default_phys_config(n, 4, max_contacts=1024)
    cfg.numJoints = j
    cfg.numHingeJoints = h
    return cfg


def main():
    out = {}
    F = FIXED
    cfg = joint_config(F["N"], F["J"], F["H"])
    pos, rot = ol.joint_inits(*ol.gen_collisions_inits(F["W"], F["N"], seed=F["SEED"]), F["J"])
    out["fixed/pos"], out["fixed/rot"] = pos, rot
    orc, ref = ol.OraclePhys(cfg, pos, rot), ol.ReferencePhys(cfg, pos, rot)
    ub_first = np.zeros(F["W"], np.int32)
    for s in range(1, F["ORC"] + 1):
        orc.step(1)
        if s <= max(F["SNAPS"]):
            ref.step(1)
        for w in range(F["W"]):
            if ub_first[w] == 0 and orc.ub_manifolds(w):
                ub_first[w] = s
            if s <= max(F["SNAPS"]) and ub_first[w] == 0:
                assert _eq(orc.bodies(w), ref.bodies(w)), f"oracle != reference at step {s} world {w}"
            if s in F["SNAPS"]:
                assert ub_first[w] == 0, "snapshot past an undefined manifold"
                out[f"fixed/s{s}/w{w}"] = ref.bodies(w)
    for w in range(F["W"]):
        out[f"fixed/orc_s{F['ORC']}/w{w}"] = orc.bodies(w)
    out["ub_first"] = ub_first

    H = HINGE
    cfg = joint_config(H["N"], H["J"], H["H"])
    pos, rot = ol.joint_inits(*ol.gen_collisions_inits(H["W"], H["N"], seed=H["SEED"]), H["J"],
                              H["H"])
    out["hinge/pos"], out["hinge/rot"] = pos, rot
    orc, ref = ol.OraclePhys(cfg, pos, rot), ol.ReferencePhys(cfg, pos, rot)
    for s in range(1, H["STEPS"] + 1):
        orc.step(1)
        ref.step(1)
        for w in range(H["W"]):
            b = ref.bodies(w)
            assert np.isfinite(b["pos"]).all(), f"hinge state not finite at step {s}"
            assert orc.ub_manifolds(w) == 0
            assert _eq(orc.bodies(w), b), f"hinge: oracle != reference at step {s} world {w}"
            out[f"hinge/s{s}/w{w}"] = b
    np.savez_compressed(os.path.join(HERE, "joints_ref.npz"), **out)
    print("wrote", len(out), "arrays; first undefined manifold per fixed world:", ub_first)


if __name__ == "__main__":
    main()
