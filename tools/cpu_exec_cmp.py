#!/usr/bin/env python3
"""The framework's CPU back end (libmadrona_cpu.so) against the reference's
own ECS + physics (oracle/_ref) on the same worlds, threads and step window
(collisions, 128 cubes, S = 4): env-steps/s of each.

    python tools/cpu_exec_cmp.py [--threads 16] [--worlds 256] [--settle 130] [--steps 30]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
os.environ.setdefault("MADRONA_MW_NO_TORCH", "1")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--worlds", type=int, default=256)
    p.add_argument("--settle", type=int, default=130)
    p.add_argument("--steps", type=int, default=30)
    a = p.parse_args()
    import madrona_mi355x as mw
    import oracle_lib as ol
    pos, rot = ol.gen_collisions_inits(a.worlds, 128, seed=0)
    g = mw.default_collisions_config(128, 4, 4096, 4096)
    sim = mw.CollisionsSim(a.worlds, pos, rot, g, backend="cpu", num_workers=a.threads)
    sim.step(a.settle)
    t0 = time.perf_counter()
    sim.step(a.steps)
    fw = a.worlds * a.steps / (time.perf_counter() - t0)
    ref = ol.ReferencePhys(ol.default_phys_config(128, 4, max_contacts=4096), pos, rot)
    ref.lib.ref_phys_step_mt.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    ref.lib.ref_phys_step_mt(ref.h, a.settle, a.threads)
    t0 = time.perf_counter()
    ref.lib.ref_phys_step_mt(ref.h, a.steps, a.threads)
    rf = a.worlds * a.steps / (time.perf_counter() - t0)
    print(f"threads {a.threads} worlds {a.worlds}: framework {fw:.0f} reference {rf:.0f} env-steps/s "
          f"({fw / rf:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
