#!/usr/bin/env python3
"""Benchmark of the fantasy_vs workload (BASELINE.json configs[4]: 16 384
worlds x 50 dragons + 200 knights, deaths destroy entities) on one MI355X.
Same JSON contract as bench.py; a step = one tick of every world (action
select, casters, archers, cleanup with device-side destroy / ID release).
Timed window: the CHURN window, ticks preroll+1 .. preroll+K (default
601-1200): the dragons of the reference init start dying at tick ~550 and
most of them die before tick 1200 (oracle run of the same init: 3197 of the
sampled 3200 alive at 600, ~490 at 1200), so every timed tick destroys
entities, releases IDs and compacts rows (the ordered commit's wave-parallel
swap-removes) up to the window's end.  The sampled worlds' dragons alive
after every chunk of ticks are reported (read between chunks, outside the
timed steps).  The CPU
baseline is the reference's own ECS (oracle/_ref) on the same tick window,
one pinned worker per usable core, batches of 2048 worlds (the reference
reserves 48 GiB of address space per world) until ~4 s is timed.

    python tools/bench_fvs.py [--worlds 16384 --preroll 750 --steps 750]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))

HBM_PEAK_GBS = 8000.0
# Algorithmic bytes per launch and world (Entity 8,
# Position 12, Health 64 (cache-line aligned), Action 4, Mana / Quiver 4).
# The three ParallelForNodes are timed together, so their bytes are averaged:
# actionSelect reads Entity + Position + Action and writes Position + Action
# on every row, the caster reads Entity + Action + Mana and writes Mana on
# dragon rows, the archer reads Entity + Action + Quiver on knight rows.
def world_bytes(node, nd, nk):
    if node == "ParallelForNode":
        return ((nd + nk) * (8 + 2 * 12 + 2 * 4) + nd * (8 + 4 + 2 * 4) + nk * (8 + 4 + 4)) / 3
    return (nd + nk) * (8 + 64)                     # cleanup scan: Entity + Health


def pmc_traffic(node):
    """HBM bytes per launch of the node kind from the committed rocprofv3 PMC
    passes (profiles/r03_fvs_traffic.json, tools/gpu_fvs_pmc.sh); None if
    absent."""
    try:
        with open(os.path.join(ROOT, "profiles", "r03_fvs_traffic.json")) as f:
            return json.load(f)["nodes"][node]["bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--worlds", type=int, default=16384)
    p.add_argument("--steps", type=int, default=600)
    p.add_argument("--preroll", type=int, default=600,
                   help="untimed ticks before the window (the warmup)")
    p.add_argument("--dragons", type=int, default=50)
    p.add_argument("--knights", type=int, default=200)
    p.add_argument("--cpu-worlds", type=int, default=2048,
                   help="worlds per CPU batch (the reference reserves address space per world)")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable core")
    p.add_argument("--cpu-target-s", type=float, default=4.0)
    p.add_argument("--cpu-max-batches", type=int, default=48)
    p.add_argument("--cpu-first-world", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--chunk", type=int, default=50,
                   help="ticks launched back-to-back per host sync (the reference "
                        "benchmark runs all ticks in one go)")
    p.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


def cpu_child(args):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol                      # no torch import in the child
    first = args.cpu_first_world
    inits = {k: v[first:] for k, v in
             ol.gen_fvs_inits(first + args.cpu_worlds, args.dragons, args.knights, seed=0).items()}
    threads = max(1, args.cpu_threads)
    ref = ol.ReferenceFvs(inits, first_world_index=args.cpu_first_world)
    ref.lib.ref_fvs_step_mt.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    ref.lib.ref_fvs_step_mt(ref.h, args.preroll, threads)
    t0 = time.perf_counter()
    ref.lib.ref_fvs_step_mt(ref.h, args.steps, threads)
    dt = time.perf_counter() - t0
    alive = sum(len(ref.table(w, 0)) for w in range(0, args.cpu_worlds, max(1, args.cpu_worlds // 64)))
    print(json.dumps({"kind": "reference", "seconds": dt, "threads": threads, "alive": alive}))


def cpu_baseline(args):
    sys.path.insert(0, ROOT)
    from bench import cpu_model, usable_cores
    threads = args.cpu_threads if args.cpu_threads > 0 else usable_cores()
    total_s, batches, t_wall = 0.0, 0, time.perf_counter()
    while batches < args.cpu_max_batches and total_s < args.cpu_target_s:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child",
                            "--cpu-worlds", str(args.cpu_worlds), "--cpu-threads", str(threads),
                            "--cpu-first-world", str(batches * args.cpu_worlds),
                            "--steps", str(args.steps), "--preroll", str(args.preroll),
                            "--dragons", str(args.dragons), "--knights", str(args.knights)],
                           capture_output=True, text=True, timeout=1200)
        if r.returncode != 0:
            raise RuntimeError(f"cpu baseline child failed: {r.stderr[-2000:]}")
        res = json.loads(r.stdout.strip().splitlines()[-1])
        total_s += res["seconds"]
        batches += 1
    worlds = batches * args.cpu_worlds
    return {"value": round(worlds * args.steps / total_s, 1), "unit": "env-steps/s",
            "cores": threads, "cpu_model": cpu_model(), "kind": "reference",
            "sample": f"fantasy_vs {batches} batches x {args.cpu_worlds} worlds (worlds 0-{worlds - 1}) "
                      f"x ({args.dragons} dragons + {args.knights} knights), ticks "
                      f"{args.preroll + 1}-{args.preroll + args.steps} (the GPU's timed window), "
                      f"{threads} host threads pinned one per usable core, {total_s:.2f} s timed / "
                      f"{time.perf_counter() - t_wall:.1f} s wall"}


def main():
    args = parse()
    if args.cpu_child:
        return cpu_child(args)
    import madrona_mi355x as mw
    W = args.worlds
    inits = mw.gen_fvs_inits(W, args.dragons, args.knights, seed=0)
    sim = mw.FvsSim(W, inits)

    node_ms = {}
    for name in ("ParallelForNode", "PerWorldNode"):
        node_ms[name] = sim.time_node(name, 1)     # untimed pre-roll (2 ticks)
    # restart from the init so the timed window is ticks warmup+1..warmup+K
    sim.close()
    sim = mw.FvsSim(W, inits)
    dom = max(node_ms, key=lambda n: node_ms[n] * (4 if n == "ParallelForNode" else 1))
    left = args.preroll
    while left > 0:
        n = min(args.chunk, left)
        sim.step(n)
        left -= n
    sim.sync()
    sampled = range(0, W, max(1, W // 64))
    alive0 = sum(sim.num_rows(w, 0) for w in sampled)
    # throughput: the plain step graph, chunks of ticks per host sync; only
    # the stepping is timed (the sampled alive counts are read between chunks)
    elapsed = 0.0
    left, tick = args.steps, args.preroll
    alive_by_tick = [[tick, int(alive0)]]
    while left > 0:
        n = min(args.chunk, left)
        t0 = time.perf_counter()
        sim.step(n)              # n graph replays back-to-back, one sync
        sim.sync()
        elapsed += time.perf_counter() - t0
        left -= n
        tick += n
        alive_by_tick.append([tick, int(sum(sim.num_rows(w, 0) for w in sampled))])
    alive = alive_by_tick[-1][1]
    # per-launch kernel time: HIP events around every launch of the dominant
    # node kind (graph split at that node), one tick per sync, 100 ticks
    sim.set_timed_node(dom)
    for _ in range(100):
        sim.step(1)
    ms1, n1 = sim.timed_node()
    ms0, n0 = 0.0, 0
    sim.set_timed_node(None)
    flags = sim.error_flags()

    launch_ms = (ms1 - ms0) / max(1, n1 - n0)
    nbytes = W * world_bytes(dom, args.dragons, args.knights)
    achieved = nbytes / (launch_ms * 1e-3) / 1e9
    cpu = None if args.no_cpu_baseline else cpu_baseline(args)
    out = {
        "metric": "env-steps/sec (summed worlds)", "value": round(W * args.steps / elapsed, 1),
        "unit": "env-steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.preroll,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "warmup_note": "warmup = the untimed preroll ticks",
        "scaling": "weak", "vs_baseline": None, "dtype": "f32+i32",
        "data": "synthetic (reference example init, mt19937 seed 0; counter-based in-tick draws)",
        "config": {"workload": f"examples/fantasy_vs restated: {W} worlds x ({args.dragons} "
                               f"dragons + {args.knights} knights), Game::tick with cleanup",
                   "timed_ticks": f"{args.preroll + 1}-{args.preroll + args.steps}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": pmc_traffic(dom), "ms_per_launch": round(launch_ms, 4),
                     "timing": "HIP events around every launch of the node kind over 100 "
                               "ticks right after the timed region (executor stream)",
                     "bytes_per_launch": int(nbytes)},
        "cpu_baseline": cpu, "error_flags": flags,
        "nodes_ms_per_launch_preroll": {k: round(v, 4) for k, v in node_ms.items()},
        "dragons_alive_sampled_worlds": {"window_start": int(alive0), "window_end": int(alive),
                                          "sampled_worlds": len(sampled),
                                          "at_init": args.dragons * len(sampled),
                                          "by_tick": alive_by_tick},
    }
    print(json.dumps(out))
    sim.close()


if __name__ == "__main__":
    main()
