#!/usr/bin/env python3
"""Per-tick HBM bytes and kernel time of fantasy_vs' world-walk unit (the
walk kernel + its resume kernel, one launch each per tick) over the bench's
timed window, from rocprofv3 runs of tools/bench_fvs.py:

    python tools/fvs_walk_pmc.py --trace T.csv --fetch F.csv --write W.csv \
        [--ticks 600 1200] --out profiles/rNN_fvs_traffic.json

Walk launches are numbered in dispatch order (one per tick: the pre-roll's
per-unit timing ticks included, so launch i is tick i + 1); a resume
launch belongs to the walk launch before it.  bytes_per_launch = FETCH_SIZE
x 2 (the gfx950 correction, profiles/r03_pmc_calibration.json) + WRITE_SIZE
(KB counters) summed over the tick's two kernels; kernel_us_per_launch =
their summed durations in the replayed graph (the bench's live timing reads
split ticks, which run the unit eagerly and slower)."""
import argparse
import csv
import json

WALK, RESUME = "worldWalkKernel", "worldResumeKernel"


def per_tick(rows, value, a, b):
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    ticks, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if WALK in name:
            cur = [value(r)]
            ticks.append(cur)
        elif RESUME in name and cur is not None:
            cur.append(value(r))
    return [sum(t) for t in ticks[a:b]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--ticks", type=int, nargs=2, default=(600, 1200))
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    lo, hi = a.ticks
    dur = per_tick(list(csv.DictReader(open(a.trace))),
                   lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, lo, hi)

    def counter(path):
        return per_tick(list(csv.DictReader(open(path))), lambda r: float(r["Counter_Value"]) * 1024.0, lo, hi)

    fetch, write = counter(a.fetch), counter(a.write)
    n = min(len(dur), len(fetch), len(write))
    if n == 0:
        raise SystemExit("no walk launches in the window")
    out = {"source": "rocprofv3 --kernel-trace and separate --pmc FETCH_SIZE / WRITE_SIZE passes over "
                     "tools/bench_fvs.py (tools/fvs_walk_pmc.py)",
           "ticks": f"{lo + 1}-{hi}", "launches": n,
           "nodes": {"world walk": {
               "kernels": [WALK, RESUME],
               "kernel_us_per_launch": round(sum(dur[:n]) / n, 3),
               "fetch_bytes_per_launch": round(2 * sum(fetch[:n]) / n, 1),
               "write_bytes_per_launch": round(sum(write[:n]) / n, 1),
               "bytes_per_launch": round((2 * sum(fetch[:n]) + sum(write[:n])) / n, 1)}}}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
