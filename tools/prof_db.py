#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 run database (rocpd sqlite) over the
last n steps of a bench run (the settled window), plus
the dispatch resources (VGPRs, LDS, scratch).
    python tools/prof_db.py gpurun_out/prof_xx/run_results.db [steps]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, workgroup_x, lds_size, scratch_size, vgpr_count, "
                     "accum_vgpr_count, sgpr_count, start from kernels order by start").fetchall()
    by = {}
    for r in rows:
        by.setdefault(r[0], []).append(r)
    # The window is the time span of the last `steps` steps, clocked by the
    # leaf update (2 launches per step); every dispatch that starts inside it
    # counts, so kernels outside the step (start-up fills, the bench's torch
    # reductions) only appear when they ran inside the window.
    leaf = [n for n in by if "leafUpdateKernel" in n]
    t0 = by[leaf[0]][-2 * steps][9] if leaf and len(by[leaf[0]]) >= 2 * steps else rows[0][9]
    out = []
    for n, rs in by.items():
        last = [r for r in rs if r[9] >= t0]
        if not last:
            continue
        calls = len(last) / steps
        mean = sum(r[1] for r in last) / len(last) / 1e3
        r0 = last[-1]
        out.append((mean * calls, n, calls, mean, r0))
    out.sort(reverse=True)
    tot = sum(o[0] for o in out)
    print(f"{'us/step':>8} {'%':>5} {'calls':>5} {'us/call':>8} {'grid':>7} {'wg':>4} {'lds':>6} "
          f"{'scr':>4} {'vgpr':>4} kernel")
    for ms, n, k, mean, r in out[:16]:
        short = n.split("(")[0].replace("madrona::phys::", "").replace("madrona::", "")[:60]
        print(f"{ms:8.1f} {100 * ms / tot:5.1f} {k:5.2g} {mean:8.2f} {r[2]:7d} {r[3]:4d} {r[4]:6d} "
              f"{r[5]:4d} {r[6]:4d} {short}")
    print(f"{tot:8.1f} us/step of kernel time over the last {steps} steps")


if __name__ == "__main__":
    main()
