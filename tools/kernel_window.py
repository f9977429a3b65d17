"""Per-kernel mean duration over the last N steps of a rocprofv3 kernel trace
(the bench's timed window), instead of the whole-run average that includes
the settle phase.  A step is delimited by findOverlapsKernel (one per step).

    python tools/kernel_window.py <run_kernel_trace.csv> [N=10]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if "findOverlapsKernel" in r["Kernel_Name"]]
    t0 = marks[-n]
    agg = collections.defaultdict(list)
    for r in rows:
        s = int(r["Start_Timestamp"])
        if s >= t0:
            name = r["Kernel_Name"].split("(")[0].replace("madrona::", "")
            agg[name].append((int(r["End_Timestamp"]) - s) / 1e3)
    total = sum(sum(v) for v in agg.values())
    print(f"last {n} steps: kernel us per step {total / n:.1f}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / n:9.1f} us/step  {len(v) / n:5.1f} calls/step  {sum(v) / len(v):8.1f} us/call  {k[:90]}")


if __name__ == "__main__":
    main()
