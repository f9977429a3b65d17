"""Generate golden fixtures from the REFERENCE itself (oracle/_ref, built from
/root/reference by oracle/Makefile.ref).  Run in the build container only:

    make -C oracle && python tests/golden/make_golden.py

Writes tests/golden/collisions_ref.npz: inputs (init positions / rotations,
config) and the reference's outputs (per-body state after selected steps, the
BVH after step 1, the last substep's contacts: the reference's own count of
them (numContacts right after that narrowphase node) and exactly those rows).
These pin both the C++
restatement (oracle/) and, through it, the HIP path.

Also writes tests/golden/collisions_window_ref.npz: the bench's own window.
Worlds 0, 1, 4095 and 8191 of BASELINE.json configs[2] (8192 worlds drawn
with seed 0, serially in world order, then sliced) stepped by the reference
to steps 130, 145 (the driver's timed steps 126-145) and 330 (the end of
bench.py's default window 131-330): bodies, the step's candidate pairs (the
harness's read-only candidate log, oracle/ref_harness.cpp runLogged), the
last substep's contact count as the reference counted it (numContacts right
after that narrowphase node, runLogged) and exactly those contacts.  The GPU
test loads it at full size
(tests/test_collisions_gpu.py::test_collisions_full_size_vs_reference_window).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_lib import (ReferencePhys, default_phys_config,  # noqa: E402
                        gen_collisions_inits)

NUM_WORLDS = 3
SNAP_STEPS = (1, 2, 5, 10, 30)
CONTACT_STEPS = (1, 10, 30)


WINDOW_WORLDS = (0, 1, 4095, 8191)
WINDOW_STEPS = (130, 145, 330)


def make_window():
    cfg = default_phys_config(num_cubes=128, num_substeps=4, max_contacts=4096)
    pos, rot = gen_collisions_inits(8192, 128, seed=0)
    sel = list(WINDOW_WORLDS)
    pos, rot = np.ascontiguousarray(pos[sel]), np.ascontiguousarray(rot[sel])
    ref = ReferencePhys(cfg, pos, rot, log_candidates=True)
    out = {
        "worlds": np.array(WINDOW_WORLDS, np.int32), "num_worlds": np.int32(8192),
        "init_pos": pos, "init_rot": rot,
        "cfg": np.array([cfg.numCubes, cfg.numSubsteps, cfg.maxContacts], np.int32),
        "snap_steps": np.array(WINDOW_STEPS, np.int32),
    }
    step = 0
    for target in WINDOW_STEPS:
        ref.step(target - step)
        step = target
        for i in range(len(sel)):
            out[f"bodies_{step}_{i}"] = ref.bodies(i).view(np.uint8)
            out[f"candidates_{step}_{i}"] = ref.candidates(i)
            raw = ref.contacts_raw(i)
            n = int((raw["ref"][:, 0] != 0xFFFFFFFF).sum())
            # the last substep's own count (numContacts right after its
            # narrowphase node): the raw prefix also holds rows earlier
            # substeps wrote past it (the array is poisoned once per step)
            count = ref.last_contact_count(i)
            assert count <= n, (step, i, count, n)
            out[f"contacts_{step}_{i}"] = raw[:count].view(np.uint8).reshape(count, -1)
            out[f"contact_count_{step}_{i}"] = np.int32(count)
    path = os.path.join(HERE, "collisions_window_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    cfg = default_phys_config(num_cubes=128, num_substeps=4, max_contacts=1024)
    pos, rot = gen_collisions_inits(NUM_WORLDS, 128, seed=0)
    ref = ReferencePhys(cfg, pos, rot, log_candidates=True)
    out = {
        "init_pos": pos, "init_rot": rot,
        "cfg": np.array([cfg.numCubes, cfg.numSubsteps, cfg.maxContacts], np.int32),
        "cfg_f": np.array([cfg.deltaT, cfg.gravityZ, cfg.cubeInvMass, cfg.cubeInvInertia,
                           cfg.muS, cfg.muD], np.float32),
        "snap_steps": np.array(SNAP_STEPS, np.int32),
    }
    step = 0
    for target in SNAP_STEPS:
        ref.step(target - step)
        step = target
        bodies = np.stack([ref.bodies(w) for w in range(NUM_WORLDS)])
        out[f"bodies_{step}"] = bodies.view(np.uint8).reshape(NUM_WORLDS, -1)
        if step == 1:
            for w in range(NUM_WORLDS):
                nodes, aabbs, parents, sorted_l = ref.bvh(w)
                out[f"bvh_leaf_aabbs_{w}"] = aabbs
                out[f"bvh_leaf_parents_{w}"] = parents
                out[f"bvh_sorted_{w}"] = sorted_l
        if step in CONTACT_STEPS:
            for w in range(NUM_WORLDS):
                raw = ref.contacts_raw(w)
                n = int((raw["ref"][:, 0] != 0xFFFFFFFF).sum())
                count = ref.last_contact_count(w)
                assert count <= n, (step, w, count, n)
                out[f"contacts_{step}_{w}"] = raw[:count].view(np.uint8).reshape(count, -1)
                out[f"contact_count_{step}_{w}"] = np.int32(count)
    path = os.path.join(HERE, "collisions_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    if "--window-only" not in sys.argv:
        main()
    make_window()
