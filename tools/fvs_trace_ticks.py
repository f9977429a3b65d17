#!/usr/bin/env python3
"""Per-tick kernel breakdown of a fantasy_vs kernel trace (rocprofv3
--kernel-trace csv of tools/bench_fvs.py): kernels are labelled by system,
commits by the node they follow; averages over ticks [A, B) of the run
(counted by finishTickSystem launches).  The runtime's copy kernels (the
bench reads sampled row counts between chunks of ticks) are left out; the
wall time per tick includes those reads.

    python tools/fvs_trace_ticks.py run_kernel_trace.csv [A B]
"""
import collections
import csv
import sys

KEYS = ["structuralCommit", "casterSystem", "markDeadSystem", "actionSelectSystem", "archerSystem",
        "destroyTrackedSystem", "trackDeadSystem", "finishTickSystem"]


def main():
    path = sys.argv[1]
    a, b = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (900, 1400)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev, tick = None, 0
    agg = collections.defaultdict(list)
    fin = []
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("__amd_rocclr"):
            continue       # the bench's row-count reads between chunks, not the tick
        k = next((x for x in KEYS if x in name), name[:40])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        if k == "structuralCommit":
            k = "commit after " + str(prev)
        else:
            prev = k
        if k == "finishTickSystem":
            tick += 1
            fin.append(int(r["Start_Timestamp"]))
        if a <= tick < b:
            agg[k].append(d)
    n = b - a
    total = 0.0
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print(f"{k:45s} launches={len(v):6d} avg={sum(v) / len(v):8.2f} us  per-tick={sum(v) / n:8.2f} us")
        total += sum(v) / n
    print(f"kernel time per tick {total:.2f} us; wall per tick {(fin[b - 1] - fin[a - 1]) / n / 1000:.2f} us")


if __name__ == "__main__":
    main()
