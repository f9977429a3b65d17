#!/usr/bin/env python3
"""simple_taskgraph throughput (BASELINE.json configs[1]: 8192 worlds on one
MI355X, examples/simple_taskgraph: 100 objects + test object + agent per
world, clamp + rigid-body physics, S = 4): env-steps/s over a timed window
after a settle, barrier-free single GPU, one JSON line.

    python tools/bench_simple.py [--worlds 8192] [--settle 120] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--settle", type=int, default=120)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    cfg = mw.default_collisions_config(100, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(a.worlds, 100, seed=0)
    sim = mw.SimpleSim(a.worlds, pos, rot, cfg)
    sim.step(a.settle)
    sim.sync()
    t0 = time.perf_counter()
    sim.step_async(a.steps)
    sim.sync()
    el = time.perf_counter() - t0
    cands, contacts = sim.counts()
    print(json.dumps({
        "metric": "env-steps/sec (summed worlds)", "value": round(a.worlds * a.steps / el, 1),
        "unit": "env-steps/s", "n_gpus": 1, "steps": a.steps,
        "ms_per_step": round(el / a.steps * 1e3, 4), "dtype": "f32",
        "data": "synthetic (reference example init: mt19937 seed 0 positions/rotations)",
        "config": {"workload": f"examples/simple_taskgraph: {a.worlds} worlds x 100 objects + test "
                               "object + agent, clamp + physics, S=4, dt=1/60",
                   "timed_steps": f"{a.settle + 1}-{a.settle + a.steps}"},
        "error_flags": sim.error_flags(),
        "mean_candidates_per_world": round(float(cands.mean()), 1),
        "mean_contacts_per_world": round(float(contacts.mean()), 1),
    }))
    sim.close()


if __name__ == "__main__":
    main()
