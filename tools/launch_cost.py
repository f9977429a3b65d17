#!/usr/bin/env python3
"""Host cost of enqueuing steps vs their device time (experiment tool):
    python tools/launch_cost.py [fvs|collisions] [steps]
prints, for chunks of `steps` graph replays, the wall time of the enqueue
calls alone and of enqueue + sync.  When the two are close the step rate is
bound by the host's graph launches, not by the GPU."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def main():
    env = sys.argv[1] if len(sys.argv) > 1 else "fvs"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    if env == "fvs":
        W = 16384
        sim = mw.FvsSim(W, mw.gen_fvs_inits(W, 50, 200, seed=0))
        sim.step(600)
    else:
        W = 8192
        cfg = mw.default_collisions_config(128, 4, 4096, 4096)
        pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
        sim = mw.CollisionsSim(W, pos, rot, cfg)
        sim.step(130)
    sim.sync()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            sim.step_async(1)
        t1 = time.perf_counter()
        sim.sync()
        t2 = time.perf_counter()
        print(f"{env} walk={os.environ.get('MADRONA_MW_WORLD_WALK', '0')} {n} steps: enqueue "
              f"{(t1 - t0) / n * 1e6:.1f} us/step, enqueue+sync {(t2 - t0) / n * 1e6:.1f} us/step")


if __name__ == "__main__":
    main()
