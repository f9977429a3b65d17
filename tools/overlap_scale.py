#!/usr/bin/env python3
"""findOverlaps scaling probe (experiment tool): grid worlds of n cubes,
W worlds, a few steps; run under rocprofv3 --kernel-trace --stats to read
findOverlapsKernel / findOverlapsGlobalKernel per launch.
  MADRONA_MW_OVERLAP_DFS_LEAVES=0 python tools/overlap_scale.py W n [steps]
  python tools/overlap_scale.py --compare      # the traversal's scaling

--compare times the traversal at 800 and 3200 cubes per world and the
sweep at 3200 (64 worlds) in child processes and prints the ratios
(round 5, one block per world: 0.28 / 2.31 ms, 8.3x for 4x the bodies;
round 6, the walk over (world, 256-row chunk) blocks: 0.082 / 0.256 ms,
3.1x, the one-block sweep 38x slower than the traversal at 3200).  A wall-clock check, so it
lives here and not in the -m gpu parity suite."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import madrona_mi355x as mw  # noqa: E402
from test_lds_fallback_gpu import _grid_world  # noqa: E402


def compare():
    import re
    import subprocess
    ms = {}
    for label, leaves, n in (("dfs800", "0", 800), ("dfs3200", "0", 3200), ("sweep3200", "-1", 3200)):
        env = dict(os.environ, MADRONA_MW_OVERLAP_DFS_LEAVES=leaves)
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "64", str(n), "6"], env=env,
                             capture_output=True, text=True, timeout=300, check=True).stdout
        print(out.strip(), flush=True)
        ms[label] = float(re.search(r"timed ([0-9.]+) ms", out).group(1))
    print(f"dfs 3200 / dfs 800 = {ms['dfs3200'] / ms['dfs800']:.2f} (bodies x4), "
          f"sweep / dfs at 3200 = {ms['sweep3200'] / ms['dfs3200']:.2f}")


def main():
    if sys.argv[1] == "--compare":
        return compare()
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
