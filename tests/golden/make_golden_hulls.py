#!/usr/bin/env python3
"""Golden fixtures for the physics asset path (PhysicsLoader::loadHullFromDisk,
src/physics/physics_assets.cpp:205-254; HalfEdgeMesh::construct,
src/physics/geometry.cpp:52-194) and for collisions worlds over those hulls.

  * mesh/<name>/{verts,face_counts,indices}: each asset under
    gpu-ecs-madrona_amd/data as the importer hands it over (oracle_lib.parse_obj);
  * hull/<name>/{vertices,planes,half_edges,polygons,edges,aabb}: the
    REFERENCE's half-edge hull + AABB of that mesh (oracle/ref_harness.cpp
    ref_build_hull, compiled against /root/reference);
  * <case>/pos, <case>/rot, <case>/s{k}/w{w}: per-body state from the
    REFERENCE for collisions worlds whose body i uses hull i % len(hulls)
    (the plane after them), at snapshot steps before the first undefined face
    manifold (DESIGN.md §4 "reference UB"); <case>/orc_s{k}/w{w}: the oracle
    past it.

The oracle is asserted bit-exact against the reference on every step of every
case before its first undefined manifold.

    python tests/golden/make_golden_hulls.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

DATA = os.path.join(ROOT, "gpu-ecs-madrona_amd", "data")
NAMES = ("cube", "wedge", "hex_prism", "octahedron", "disc16", "disc64")
CASES = {
    "mixed": dict(hulls=("cube", "wedge", "hex_prism"), W=3, N=24, SEED=5,
                  SNAPS=(1, 50, 150, 300), ORC=(300,)),
    "octa": dict(hulls=("octahedron",), W=3, N=64, SEED=7, SNAPS=(1, 60, 200), ORC=(200,)),
    "disc": dict(hulls=("disc16", "octahedron"), W=3, N=32, SEED=7, SNAPS=(1, 20),
                 ORC=(120,)),
    # 64-vertex caps: the GPU contact / SAT kernels' global-image variants
    "disc64": dict(hulls=("disc64", "cube"), W=3, N=32, SEED=3, SNAPS=(1, 20), ORC=(100,)),
}


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def hull_set(names):
    return ol.HullSet.from_files([os.path.join(DATA, n + ".obj") for n in names])


def main():
    out = {}
    ref_lib = ol.load_ref()
    for n in NAMES:
        mesh = ol.parse_obj(os.path.join(DATA, n + ".obj"))
        for k, a in zip(("verts", "face_counts", "indices"), mesh):
            out[f"mesh/{n}/{k}"] = a
        ref = ol.build_hull(mesh, ref_lib)
        orc = ol.build_hull(mesh)
        for k, a in ref.items():
            assert a.tobytes() == orc[k].tobytes(), f"hull {n}: oracle {k} != reference"
            out[f"hull/{n}/{k}"] = a

    for name, C in CASES.items():
        hs = hull_set(C["hulls"])
        cfg = ol.default_phys_config(C["N"], 4, max_contacts=2048)
        pos, rot = ol.gen_collisions_inits(C["W"], C["N"], seed=C["SEED"])
        out[f"{name}/pos"], out[f"{name}/rot"] = pos, rot
        orc, ref = ol.OraclePhys(cfg, pos, rot, hs), ol.ReferencePhys(cfg, pos, rot, hs)
        ub_first = np.zeros(C["W"], np.int32)
        last = max(C["SNAPS"] + C["ORC"])
        for s in range(1, last + 1):
            orc.step(1)
            if s <= max(C["SNAPS"]):
                ref.step(1)
            for w in range(C["W"]):
                if ub_first[w] == 0 and orc.ub_manifolds(w):
                    ub_first[w] = s
                if s <= max(C["SNAPS"]) and ub_first[w] == 0:
                    assert _eq(orc.bodies(w), ref.bodies(w)), \
                        f"{name}: oracle != reference at step {s} world {w}"
                    if s in C["SNAPS"]:
                        out[f"{name}/s{s}/w{w}"] = ref.bodies(w)
                if s in C["ORC"]:
                    out[f"{name}/orc_s{s}/w{w}"] = orc.bodies(w)
        out[f"{name}/ub_first"] = ub_first
        print(name, "first undefined manifold per world:", ub_first)
    np.savez_compressed(os.path.join(HERE, "hulls_ref.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
