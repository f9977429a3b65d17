#!/usr/bin/env python3
"""Summarise the SQ counter passes of tools/sq_counters.sh into per-kernel
averages per launch (the last --launches launches of each kernel, i.e. the
bench's settled window) plus the derived ratios used in DESIGN.md §3:

    python profiles/sq_summary.py gpurun_out/<tag> --out profiles/rNN_sq_counters.json

* valu_per_wave   = SQ_INSTS_VALU / SQ_WAVES
* valu_busy_frac  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's
                    resident cycles spent issuing VALU)
* wait_frac       = SQ_WAIT_ANY / SQ_WAVE_CYCLES, wait_inst_frac likewise
* lds_wait_frac   = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"::(\w+)\(", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                       "lds_bytes": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"]),
                       "workgroup": int(r["Workgroup_Size"])}
    return vals, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    vals, meta = load(a.dir)
    out = {}
    for k, cs in sorted(vals.items()):
        avg = {c: sum(v[-a.launches:]) / len(v[-a.launches:]) for c, v in cs.items()}
        e = {"counters_per_launch": {c: round(x, 1) for c, x in sorted(avg.items())}, **meta[k]}
        wc = avg.get("SQ_WAVE_CYCLES")
        if avg.get("SQ_WAVES"):
            e["valu_per_wave"] = round(avg.get("SQ_INSTS_VALU", 0) / avg["SQ_WAVES"], 1)
            e["lds_per_wave"] = round(avg.get("SQ_INSTS_LDS", 0) / avg["SQ_WAVES"], 1)
            e["vmem_rd_per_wave"] = round(avg.get("SQ_INSTS_VMEM_RD", 0) / avg["SQ_WAVES"], 1)
        if wc:
            for name, c in (("valu_busy_frac", "SQ_ACTIVE_INST_VALU"), ("wait_frac", "SQ_WAIT_ANY"),
                            ("wait_inst_frac", "SQ_WAIT_INST_ANY"),
                            ("lds_wait_frac", "SQ_WAIT_INST_LDS")):
                if c in avg:
                    e[name] = round(avg[c] / wc, 3)
        out[k] = e
    json.dump({"source": "rocprofv3 --pmc SQ_* (two passes, tools/sq_counters.sh), bench.py "
                         "settled window, mean of the last %d launches per kernel" % a.launches,
               "kernels": out}, open(a.out, "w"), indent=1)
    for k, e in out.items():
        print(k, {x: e.get(x) for x in ("vgpr", "scratch", "valu_per_wave", "valu_busy_frac",
                                        "wait_frac", "lds_wait_frac")})


if __name__ == "__main__":
    main()
