#!/usr/bin/env python3
"""Per-cut averages of the solver counters tools/solver_cut_pmc.sh collects:
the last 160 solverKernel dispatches of each pass are the 8 cuts x 20
relaunches (order 1,2,3,4,5,6,0,7); each row is the mean of a cut's 20."""
import collections
import csv
import glob
import os
import sys

CUTS = (1, 2, 3, 4, 5, 6, 0, 7)
NAMES = {1: "load+count", 2: "+levels", 3: "+sort", 4: "+positions", 5: "+setVelocities",
         6: "+velocities", 0: "whole (no fused tail)", 7: "positions' loads only"}


def main():
    d = sys.argv[1]
    per = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        rows = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(rows)[-160:]
        for i, cut in enumerate(CUTS):
            grp = [rows[k] for k in ids[20 * i:20 * i + 20]]
            for c in grp[0]:
                per[cut][c] = sum(g[c] for g in grp) / len(grp)
    cols = sorted({c for v in per.values() for c in v})
    print("cut " + " ".join(f"{c[:22]:>22s}" for c in cols))
    for cut in CUTS:
        print(f"{cut}   " + " ".join(f"{per[cut].get(c, 0):22.4g}" for c in cols) + f"  {NAMES[cut]}")


if __name__ == "__main__":
    main()
