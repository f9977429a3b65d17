"""Per-node launch-configuration autotuner: writes the JSON that
MADRONA_MWGPU_EXEC_CONFIG_FILE reads ({"<node index>": <blocks per CU>}),
the file the reference's executor consumes (src/mw/cuda_exec.cpp:1460-1517).

For every node whose kernels honour a launch configuration (grid-stride
ParallelForNode / PerWorldNode, persistent NarrowphaseNode kernels) it sweeps
blocks per CU, timing the node kind live inside the replayed step (HIP
events on the executor stream, Executor.set_timed_node), and keeps the
fastest; 0 (the node's full default grid) is always a candidate.  Nodes of
one kind are tuned together, since the live timer brackets a kind.

  python tools/autotune.py --env collisions --worlds 8192 --out gpurun_out/exec.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))

TUNABLE = ("ParallelForNode", "CustomParallelForNode", "PerWorldNode", "NarrowphaseNode")


def make_sim(mw, env, worlds):
    if env == "collisions":
        g = mw.default_collisions_config(128, 4, 2048, 4096)
        pos, rot = mw.gen_collisions_inits(worlds, 128, seed=0)
        sim = mw.CollisionsSim(worlds, pos, rot, g)
        sim.step(120)                 # the bench's settled contact regime
        return sim
    if env == "simple":
        g = mw.default_collisions_config(100, 4, 4096, 4096)
        pos, rot = mw.gen_collisions_inits(worlds, 100, seed=0)
        sim = mw.SimpleSim(worlds, pos, rot, g)
        sim.step(120)                 # bench.py --workload simple's settled window
        return sim
    if env == "fvs":
        from madrona_mi355x import gen_fvs_inits
        sim = mw.FvsSim(worlds, gen_fvs_inits(worlds, 50, 200, seed=0))
        sim.step(10)
        return sim
    raise SystemExit(f"unknown env {env}")


def time_kind(sim, kind, steps):
    sim.set_timed_node(kind)
    sim.step(2)
    sim.set_timed_node(kind)          # reset the accumulators after warmup
    for _ in range(steps):
        sim.step()
    ms, n = sim.timed_node()
    return ms / max(n, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="collisions", choices=("collisions", "simple", "fvs"))
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--candidates", default="0,1,2,4,8,16")
    ap.add_argument("--out", default="gpurun_out/exec_config.json")
    a = ap.parse_args()
    import madrona_mi355x as mw

    sim = make_sim(mw, a.env, a.worlds)
    names = sim.nodes()
    cands = [int(c) for c in a.candidates.split(",")]
    chosen, report = {}, {}
    for kind in TUNABLE:
        idx = [i for i, n in enumerate(names) if n == kind]
        if not idx:
            continue
        res = {}
        for bpc in cands:
            for i in idx:
                sim.set_node_blocks_per_cu(i, bpc)
            res[bpc] = time_kind(sim, kind, a.steps)
        best = min(res, key=res.get)
        for i in idx:
            sim.set_node_blocks_per_cu(i, best)
            if best != 0:
                chosen[str(i)] = best
        report[kind] = {"nodes": idx, "ms_per_launch": {str(k): round(v, 4) for k, v in res.items()},
                        "best_blocks_per_cu": best}
        print(f"{kind:18s} nodes {idx}: " +
              "  ".join(f"{k}:{v:.4f}" for k, v in res.items()) + f"  -> {best}", flush=True)
    sim.set_timed_node(None)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(chosen, f)
    with open(os.path.splitext(a.out)[0] + "_report.json", "w") as f:
        json.dump({"env": a.env, "worlds": a.worlds, "nodes": names, "sweep": report}, f, indent=1)
    print("wrote", a.out, chosen)


if __name__ == "__main__":
    main()
