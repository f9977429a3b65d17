#!/usr/bin/env python3
"""Per-node summary of rocprofv3 runs of tools/bench_fvs.py (fantasy_vs).

    python tools/fvs_prof_summary.py --trace T.csv [--fetch F.csv --write W.csv]
        [--ticks A B] [--out profiles/rNN_fvs_traffic.json]

A node launch of the tick graph is the run of its row kernels (one per
archetype the query matches) plus the ordered commit that follows them;
per-world nodes have no commit.  Dispatches are labelled by the system name
in the kernel symbol, commits by the node they close, and ticks are counted
by finishTickSystem launches; only ticks A+1..B (the bench's timed window,
default 601-1200) count.  For every node:
  * span_us: first kernel start to last kernel end of a launch -- what the
    bench's event pair bound to the node's kernels measures;
  * kernel_us: the sum of the launch's kernel durations;
  * bytes_per_launch: FETCH_SIZE x 2 (the gfx950 correction, calibrated in
    profiles/r03_pmc_calibration.json) + WRITE_SIZE, counters in KB, summed
    over the launch's kernels (separate PMC passes).
"""
import argparse
import collections
import csv
import json

SYSTEMS = ["casterSystem", "markDeadSystem", "actionSelectSystem", "archerSystem",
           "destroyTrackedSystem", "trackDeadSystem", "finishTickSystem"]


def label(name):
    if "structuralCommit" in name:
        return "commit"
    return next((s for s in SYSTEMS if s in name), None)


def node_launches(rows, a, b, value):
    """{system: [per-launch (start, end, kernel_sum, value_sum)]} over ticks
    a+1..b; rows: dicts with Kernel_Name, Start/End_Timestamp."""
    rows = sorted(rows, key=lambda r: (int(r["Start_Timestamp"]), int(r.get("Dispatch_Id", 0))))
    out = collections.defaultdict(list)
    tick, cur, cur_sys, closed = 0, None, None, True
    for r in rows:
        k = label(r["Kernel_Name"])
        if k is None:
            continue
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        v = value(r)
        if k == "commit":
            if cur is not None and not closed:
                cur[1] = max(cur[1], t1)
                cur[2] += t1 - t0
                cur[3] += v
                closed = True
            continue
        if k != cur_sys or closed:
            cur = [t0, t1, 0, 0.0]
            cur_sys, closed = k, False
            if a <= tick < b:
                out[k].append(cur)
        cur[1] = max(cur[1], t1)
        cur[2] += t1 - t0
        cur[3] += v
        if k == "finishTickSystem":
            tick += 1
            closed = True
    return out


def pmc(path, a, b):
    rows = list(csv.DictReader(open(path)))
    return node_launches(rows, a, b, lambda r: float(r["Counter_Value"]) * 1024.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True, help="run_kernel_trace.csv")
    ap.add_argument("--fetch", help="FETCH_SIZE run_counter_collection.csv")
    ap.add_argument("--write", help="WRITE_SIZE run_counter_collection.csv")
    ap.add_argument("--ticks", type=int, nargs=2, default=(600, 1200))
    ap.add_argument("--out")
    args = ap.parse_args()
    a, b = args.ticks
    trace = node_launches(list(csv.DictReader(open(args.trace))), a, b, lambda r: 0.0)
    fetch = pmc(args.fetch, a, b) if args.fetch else {}
    write = pmc(args.write, a, b) if args.write else {}
    nodes = {}
    for s in SYSTEMS:
        L = trace.get(s, [])
        if not L:
            continue
        e = {"launches": len(L), "launches_per_tick": round(len(L) / (b - a), 3),
             "span_us": round(sum(x[1] - x[0] for x in L) / len(L) / 1e3, 3),
             "kernel_us": round(sum(x[2] for x in L) / len(L) / 1e3, 3)}
        if s in fetch and s in write:
            f = sum(x[3] for x in fetch[s]) / len(fetch[s]) * 2.0
            w = sum(x[3] for x in write[s]) / len(write[s])
            e.update({"fetch_bytes_x2": int(f), "write_bytes": int(w),
                      "bytes_per_launch": int(f + w), "pmc_launches": len(fetch[s])})
        nodes[s] = e
    tick_us = sum(v["span_us"] * v["launches_per_tick"] for v in nodes.values())
    res = {"what": "fantasy_vs per node launch (row kernels + ordered commit) over ticks "
                   f"{a + 1}-{b}: span = first kernel start to last kernel end (what the bench's "
                   "bound event pair measures), kernel = summed kernel durations, bytes = "
                   "FETCH_SIZE x 2 + WRITE_SIZE (KB counters, separate PMC passes; "
                   "tools/fvs_prof_summary.py)",
           "node_span_us_per_tick": round(tick_us, 2), "nodes": nodes}
    txt = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
