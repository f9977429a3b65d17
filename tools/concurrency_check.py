#!/usr/bin/env python3
"""Does the hull-plane kernel overlap the hull-hull SAT + contact kernels
(physics.hip NarrowphaseNode: the plane kernel on the side stream, a
parallel branch of the step graph)?  Reads a rocprofv3 kernel trace CSV and
prints, over the last `--last` launches of `--kernel`, its mean duration and
the mean fraction of it that ran while another kernel was running (experiment
tool, GPU box).

    python3 tools/concurrency_check.py <dir>/run_kernel_trace.csv --last 80
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="narrowPlaneKernel")
    ap.add_argument("--last", type=int, default=80)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    mine = [i for i, r in enumerate(rows) if a.kernel in r[2]][-a.last:]
    if not mine:
        print("no launches of", a.kernel)
        return
    dur = ovl = 0.0
    partners = {}
    for i in mine:
        s, e, _ = rows[i]
        covered = []
        for j in range(max(0, i - 8), min(len(rows), i + 8)):
            if j == i:
                continue
            s2, e2, n2 = rows[j]
            lo, hi = max(s, s2), min(e, e2)
            if hi > lo:
                covered.append((lo, hi))
                key = n2.split("(")[0][-40:]
                partners[key] = partners.get(key, 0) + (hi - lo)
        covered.sort()
        tot, cur = 0, None
        for lo, hi in covered:
            if cur and lo <= cur[1]:
                cur[1] = max(cur[1], hi)
            else:
                if cur:
                    tot += cur[1] - cur[0]
                cur = [lo, hi]
        if cur:
            tot += cur[1] - cur[0]
        dur += e - s
        ovl += tot
    n = len(mine)
    print(f"{a.kernel}: {n} launches, mean {dur / n / 1e3:.2f} us, overlapped {ovl / max(dur, 1):.1%}")
    for k, v in sorted(partners.items(), key=lambda kv: -kv[1]):
        print(f"  with {k}: {v / n / 1e3:.2f} us per launch")


if __name__ == "__main__":
    main()
