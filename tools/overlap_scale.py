#!/usr/bin/env python3
"""findOverlaps scaling probe (experiment tool): grid worlds of n cubes,
W worlds, a few steps; run under rocprofv3 --kernel-trace --stats to read
findOverlapsKernel / findOverlapsGlobalKernel per launch.
  MADRONA_MW_OVERLAP_DFS_LEAVES=0 python tools/overlap_scale.py W n [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import madrona_mi355x as mw  # noqa: E402
from test_lds_fallback_gpu import _grid_world  # noqa: E402


def main():
    W, n = int(sys.argv[1]), int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    pos, rot = _grid_world(W, n)
    sim = mw.CollisionsSim(W, pos, rot, mw.default_collisions_config(n, 4, 8192, 8192))
    sim.step(2)
    sim.set_timed_node("FindOverlappingNode")
    sim.step(steps)
    ms, launches = sim.timed_node()
    c, k = sim.counts()
    print(f"W={W} n={n} dfs_leaves={os.environ.get('MADRONA_MW_OVERLAP_DFS_LEAVES')} "
          f"timed {ms / max(launches, 1):.4f} ms/launch ({launches}), cands/world {c.mean():.0f}, "
          f"variants {sim.kernel_variants()['find_overlaps']} flags {sim.error_flags():#x}")


if __name__ == "__main__":
    main()
