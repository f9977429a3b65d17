#!/usr/bin/env python3
"""Summarise rocprofv3 output of a bench.py run into per-node numbers.

    python profiles/pmc_traffic.py --trace DIR_kernel_trace --fetch DIR_fetch \
        --write DIR_write --steps K --out profiles/rNN_traffic.json

* kernel time per node launch from `--kernel-trace` (run_kernel_trace.csv),
  over the last K steps' dispatches (the bench's timed window);
* HBM bytes per node launch from two separate PMC passes (FETCH_SIZE and
  WRITE_SIZE cannot share a pass on gfx950), with the MI355X_MICROARCH.md
  gfx950 correction FETCH_SIZE x 2; counters are in KB.

A node's launch may be several kernels (NarrowphaseNode = filter + order +
SAT + plane + contact); their per-launch values are summed, each weighted by
its launches per step over the node's (the first substep's integrate and
filter kernels run in one of the four substep launches).
"""
import argparse
import collections
import csv
import glob
import json
import os

# kernel -> (node, launches per step)
NODE_OF = {
    "leafUpdateKernel": ("UpdateLeafPositionsNode", 2),
    "bvhRebuildKernel": ("UpdateBVHNode", 1),
    "bvhRebuildWaveKernel": ("UpdateBVHNode", 1),
    "refitKernel": ("RefitNode", 2),
    "findOverlapsKernel": ("FindOverlappingNode", 1),
    "findOverlapsSmallKernel": ("FindOverlappingNode", 1),    # worlds of <= 256 leaves (round 5)
    "findOverlapsGlobalKernel": ("FindOverlappingNode", 1),
    "integrateKernel": ("SubstepRigidBodiesNode", 1),     # substep 0 only (later: solver tail)
    "narrowFilterKernel": ("NarrowphaseNode", 1),         # substep 0 only (later: solver tail)
    "narrowFilterWaveKernel": ("NarrowphaseNode", 1),     # the same, a wave per world
    "solverOrderKernel": ("NarrowphaseNode", 4),
    "narrowSATKernel": ("NarrowphaseNode", 4),
    "narrowSATNoGeoKernel": ("NarrowphaseNode", 4),      # hull tables read from HBM
    "narrowSATGlobalKernel": ("NarrowphaseNode", 4),
    "narrowPlaneKernel": ("NarrowphaseNode", 4),
    "narrowPlaneNoGeoKernel": ("NarrowphaseNode", 4),
    "narrowContactKernel": ("NarrowphaseNode", 4),
    "narrowContactGlobalKernel": ("NarrowphaseNode", 4),
    "solverKernel": ("SolverNode", 4),
}
PER_STEP = {"UpdateLeafPositionsNode": 2, "RefitNode": 2, "UpdateBVHNode": 1,
            "FindOverlappingNode": 1, "SubstepRigidBodiesNode": 4, "NarrowphaseNode": 4,
            "SolverNode": 4}


def kernel_key(name):
    # the kernel's own symbol name ("...phys::narrowSATKernel(...)"), so that
    # findOverlapsKernel does not match findOverlapsSmallKernel
    base = name.split("(")[0].split("::")[-1].strip()
    return base if base in NODE_OF else None


def find_csv(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def last_per_kernel(rows, steps, key_fn, val_fn):
    by = collections.defaultdict(list)
    for r in rows:
        k = key_fn(r)
        if k:
            by[k].append(val_fn(r))
    out = {}
    for k, vals in by.items():
        n = NODE_OF[k][1] * steps
        tail = vals[-n:] if n and len(vals) >= n else vals
        out[k] = sum(tail) / len(tail)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--timed-steps", default=None,
                    help="the bench's timed step range these K steps are (e.g. 131-330); "
                         "bench.py uses a profile for `traffic` only when it equals its own")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    trace = list(csv.DictReader(open(find_csv(a.trace, "kernel_trace.csv"))))
    ms = last_per_kernel(trace, a.steps, lambda r: kernel_key(r["Kernel_Name"]),
                         lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)

    def counter(d, name):
        rows = [r for r in csv.DictReader(open(find_csv(d, "counter_collection.csv")))
                if r["Counter_Name"] == name]
        return last_per_kernel(rows, a.steps, lambda r: kernel_key(r["Kernel_Name"]),
                               lambda r: float(r["Counter_Value"]) * 1024.0)

    fetch = counter(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = counter(a.write, "WRITE_SIZE") if a.write else {}

    # a node launch's share of each kernel: kernel launches per step / node
    # launches per step (the first substep's integrate / filter kernels run
    # in one of the four substep node launches)
    nodes = {}
    for k, (node, kper) in NODE_OF.items():
        if k not in ms:
            continue
        f = kper / PER_STEP[node]
        e = nodes.setdefault(node, {"kernels": [], "ms_per_launch": 0.0,
                                    "fetch_bytes": 0.0, "write_bytes": 0.0, "per_kernel": {}})
        e["kernels"].append(k)
        e["ms_per_launch"] += f * ms[k]
        e["fetch_bytes"] += f * 2.0 * fetch.get(k, 0.0)
        e["write_bytes"] += f * write.get(k, 0.0)
        # the split: each kernel per launch of its own, and its share of a
        # node launch (launches per step / node launches per step)
        e["per_kernel"][k] = {"ms_per_kernel_launch": round(ms[k], 4),
                              "bytes_per_kernel_launch": (int(2.0 * fetch.get(k, 0.0) + write.get(k, 0.0))
                                                          if (fetch or write) else None),
                              "share_of_node_launch": round(f, 4)}
    for e in nodes.values():
        e["ms_per_launch"] = round(e["ms_per_launch"], 4)
        e["bytes_per_launch"] = (int(e["fetch_bytes"] + e["write_bytes"])
                                 if (fetch or write) else None)
        e["fetch_bytes"] = int(e["fetch_bytes"])
        e["write_bytes"] = int(e["write_bytes"])
        if e["bytes_per_launch"]:
            e["hbm_gbs"] = round(e["bytes_per_launch"] / (e["ms_per_launch"] * 1e-3) / 1e9, 1)
    json.dump({"source": "rocprofv3 kernel trace + PMC FETCH_SIZE (x2, gfx950) / WRITE_SIZE",
               "steps": a.steps, "timed_steps": a.timed_steps, "nodes": nodes},
              open(a.out, "w"), indent=1)
    print(json.dumps(nodes, indent=1))


if __name__ == "__main__":
    main()
