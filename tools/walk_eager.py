#!/usr/bin/env python3
"""Graph replay vs eager launches (experiment tool): ms per step of
fantasy_vs (ticks 301-400) and collisions (steps 131-230) with the step
replayed as a hipGraph and launched kernel by kernel, alternated.
    python tools/walk_eager.py [fvs|collisions|both]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gpu-ecs-madrona_amd"))
import madrona_mi355x as mw  # noqa: E402


def make(env, graph):
    if env == "fvs":
        W = 16384
        return W, mw.FvsSim(W, mw.gen_fvs_inits(W, 50, 200, seed=0), use_graph=graph), 300
    W = 8192
    cfg = mw.default_collisions_config(128, 4, 4096, 4096)
    pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
    return W, mw.CollisionsSim(W, pos, rot, cfg, use_graph=graph), 130


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    for env in (["fvs", "collisions"] if which == "both" else [which]):
        for graph in (True, False, True, False):
            W, sim, pre = make(env, graph)
            sim.step(pre)
            sim.sync()
            t0 = time.perf_counter()
            sim.step(100)
            sim.sync()
            dt = time.perf_counter() - t0
            print(env, "graph" if graph else "eager", f"{dt / 100 * 1e3:.4f} ms/step",
                  f"{W * 100 / dt / 1e6:.2f} M env-steps/s", flush=True)
            sim.close()


if __name__ == "__main__":
    main()
