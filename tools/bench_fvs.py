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
swap-removes) up to the window's end.  The live dragons and knights of 256
sampled worlds are read after every chunk of ticks (outside the timed
steps); their window mean sizes the dominant node's algorithmic bytes.  The CPU
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
# The tick graph's nodes in sorted order (fvs.hip): the ParallelForNodes and
# the PerWorldNodes, by system.
ROW_SYSTEMS = ["actionSelectSystem", "casterSystem", "archerSystem", "markDeadSystem",
               "destroyTrackedSystem"]
WORLD_SYSTEMS = ["trackDeadSystem", "finishTickSystem"]
# Algorithmic bytes per launch and world of a node (SURVEY.md §8(d) C5:
# Entity 8, Position 12, Health 64 -- alignas(MADRONA_CACHE_LINE) --,
# Action 4, Mana / Quiver 4), nd / nk = live dragons / knights of the world:
# every column of the node's query read once per row, every column it
# modifies written once.  The caster's blasts re-read Position / Health of the
# world (L2-resident after the first) and are not counted; the cleanup nodes
# touch a few tracker rows.
SYS_BYTES = {
    "actionSelectSystem": lambda nd, nk: (nd + nk) * (8 + 2 * 12 + 2 * 4),
    "casterSystem": lambda nd, nk: nd * (8 + 4 + 2 * 4),
    "archerSystem": lambda nd, nk: nk * (8 + 4 + 2 * 4),
    "markDeadSystem": lambda nd, nk: (nd + nk) * (8 + 64),
}


def node_systems(kinds):
    """{node index: system} from the executor's node kinds."""
    rows, worlds = iter(ROW_SYSTEMS), iter(WORLD_SYSTEMS)
    return {i: next(rows) if k == "ParallelForNode" else next(worlds)
            for i, k in enumerate(kinds)}


# committed PMC / kernel-trace summaries of the timed window (ticks 601-1200):
# the world-walk unit (tools/gpu_fvs_walk_pmc.sh -> profiles/r06_fvs_traffic.json),
# per-node launches of the per-node graph (tools/gpu_fvs_pmc.sh ->
# profiles/r03_fvs_traffic.json)
FVS_TRAFFIC = ("r06_fvs_traffic.json", "r03_fvs_traffic.json")


def committed_unit(system):
    """The committed summary entry of the launch unit (None if absent) and its
    file: HBM bytes per launch (PMC) and, for the walk, its kernel time per
    replayed tick."""
    key = "world walk" if system.startswith("world walk") else system
    for name in FVS_TRAFFIC:
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
            if d.get("ticks", "601-1200") == "601-1200" and key in d["nodes"]:
                return d["nodes"][key], "profiles/" + name
        except (OSError, ValueError, KeyError):
            continue
    return None, None


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
    p.add_argument("--no-node-timing", action="store_true",
                   help="no live node timing in the window (every tick replays the whole graph)")
    p.add_argument("--chunk", type=int, default=50,
                   help="ticks launched back-to-back per host sync (the reference "
                        "benchmark runs all ticks in one go)")
    p.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cpu-executor", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--no-cpu-executor", action="store_true",
                   help="skip the framework's CPU back end leg")
    return p.parse_args()


def cpu_child(args):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol                      # no torch import in the child
    first = args.cpu_first_world
    inits = {k: v[first:] for k, v in
             ol.gen_fvs_inits(first + args.cpu_worlds, args.dragons, args.knights, seed=0).items()}
    threads = max(1, args.cpu_threads)
    if args.cpu_executor:
        # the framework's CPU back end (libmadrona_cpu.so) on the same worlds
        os.environ["MADRONA_MW_NO_TORCH"] = "1"
        import madrona_mi355x as mw
        sim = mw.FvsSim(args.cpu_worlds, inits, first_world=first, backend="cpu", num_workers=threads)
        sim.step(args.preroll)
        t0 = time.perf_counter()
        sim.step(args.steps)
        dt = time.perf_counter() - t0
        print(json.dumps({"kind": "port", "seconds": dt, "threads": threads}))
        return
    ref = ol.ReferenceFvs(inits, first_world_index=args.cpu_first_world)
    ref.lib.ref_fvs_step_mt.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    ref.lib.ref_fvs_step_mt(ref.h, args.preroll, threads)
    t0 = time.perf_counter()
    ref.lib.ref_fvs_step_mt(ref.h, args.steps, threads)
    dt = time.perf_counter() - t0
    alive = sum(len(ref.table(w, 0)) for w in range(0, args.cpu_worlds, max(1, args.cpu_worlds // 64)))
    print(json.dumps({"kind": "reference", "seconds": dt, "threads": threads, "alive": alive}))


def cpu_baselines(args, legs):
    """CPU legs on the same tick window: "reference" = the reference's own ECS
    (oracle/_ref), "executor" = the framework's CPU back end; with both, their
    batches alternate over the same worlds (one stretch of host load)."""
    sys.path.insert(0, ROOT)
    from bench import cpu_model, usable_cores
    threads = args.cpu_threads if args.cpu_threads > 0 else usable_cores()
    acc = {leg: 0.0 for leg in legs}
    batches, t_wall = 0, time.perf_counter()
    while batches < args.cpu_max_batches and min(acc.values()) < args.cpu_target_s:
        for leg in legs:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child",
                                "--cpu-worlds", str(args.cpu_worlds), "--cpu-threads", str(threads),
                                "--cpu-first-world", str(batches * args.cpu_worlds),
                                "--steps", str(args.steps), "--preroll", str(args.preroll),
                                "--dragons", str(args.dragons), "--knights", str(args.knights)] +
                               (["--cpu-executor"] if leg == "executor" else []),
                               capture_output=True, text=True, timeout=1200)
            if r.returncode != 0:
                raise RuntimeError(f"cpu {leg} child failed: {r.stderr[-2000:]}")
            acc[leg] += json.loads(r.stdout.strip().splitlines()[-1])["seconds"]
        batches += 1
    worlds = batches * args.cpu_worlds
    wall = time.perf_counter() - t_wall
    out = {}
    for leg in legs:
        out[leg] = {"value": round(worlds * args.steps / acc[leg], 1), "unit": "env-steps/s",
                    "cores": threads, "cpu_model": cpu_model(),
                    "kind": "reference" if leg == "reference" else "port",
                    "sample": ("libmadrona_cpu.so: " if leg == "executor" else "")
                              + f"fantasy_vs {batches} batches x {args.cpu_worlds} worlds (worlds 0-"
                              f"{worlds - 1}) x ({args.dragons} dragons + {args.knights} knights), ticks "
                              f"{args.preroll + 1}-{args.preroll + args.steps} (the GPU's timed window), "
                              f"{threads} host threads pinned one per usable core, {acc[leg]:.2f} s timed"
                              + (f"; batches alternated with the other leg over the same worlds, "
                                 f"{wall:.1f} s wall for both" if len(legs) > 1 else f" / {wall:.1f} s wall")}
    return out


def main():
    args = parse()
    if args.cpu_child:
        return cpu_child(args)
    import madrona_mi355x as mw
    W = args.worlds
    inits = mw.gen_fvs_inits(W, args.dragons, args.knights, seed=0)
    sim = mw.FvsSim(W, inits)

    systems = node_systems(sim.nodes())
    # launch units: a world-walk run (the nodes one walk launch covers,
    # mw_walk_run_end) or a single node
    units, i = {}, 0
    while i < len(systems):
        units[i] = sim.walk_run_end(i)
        i = units[i]

    def unit_name(i):
        names = [systems[k] for k in range(i, units[i])]
        return names[0] if len(names) == 1 else "world walk: " + " + ".join(names)

    def unit_bytes(i, nd, nk):
        return sum(SYS_BYTES[systems[k]](nd, nk) for k in range(i, units[i]) if systems[k] in SYS_BYTES)

    # untimed pre-roll: the first ticks time each modelled unit in turn (its
    # kernels bound to an event pair) to pick the dominant one
    node_ms = {}
    for i in units:
        if not any(systems[k] in SYS_BYTES for k in range(i, units[i])):
            continue
        sim.set_timed_node_index(i)
        sim.step(5)
        ms, n = sim.timed_node()
        node_ms[i] = ms / max(1, n)
    sim.set_timed_node(None)
    dom = max(node_ms, key=node_ms.get)
    dom_sys = unit_name(dom)
    left = args.preroll - 5 * len(node_ms)
    if left < 0:
        raise SystemExit("--preroll too short for the node timing")
    while left > 0:
        n = min(args.chunk, left)
        sim.step(n)
        left -= n
    sim.sync()
    sampled = range(0, W, max(1, W // 256))

    def live():
        return (sum(sim.num_rows(w, 0) for w in sampled) / len(sampled),
                sum(sim.num_rows(w, 1) for w in sampled) / len(sampled))

    # throughput: the step graph, chunks of ticks per host sync; only the
    # stepping is timed (the sampled row counts are read between chunks).
    # The dominant node is timed live in the window: every 10th tick runs the
    # graph split at that node with an event pair bound to its kernels.
    if not args.no_node_timing:
        sim.set_timed_node_index(dom, every=10)
    elapsed = 0.0
    left, tick = args.steps, args.preroll
    rows_by_tick = [[tick, *live()]]
    while left > 0:
        n = min(args.chunk, left)
        t0 = time.perf_counter()
        sim.step(n)              # n graph replays back-to-back, one sync
        sim.sync()
        elapsed += time.perf_counter() - t0
        left -= n
        tick += n
        rows_by_tick.append([tick, *live()])
    ms1, n1 = sim.timed_node()
    ms0, n0 = 0.0, 0
    sim.set_timed_node(None)
    flags = sim.error_flags()
    # mean live rows over the window (trapezoid over the chunk boundaries)
    span = rows_by_tick[-1][0] - rows_by_tick[0][0]
    nd_mean = sum((b[0] - a[0]) * (a[1] + b[1]) / 2 for a, b in zip(rows_by_tick, rows_by_tick[1:])) / span
    nk_mean = sum((b[0] - a[0]) * (a[2] + b[2]) / 2 for a, b in zip(rows_by_tick, rows_by_tick[1:])) / span

    launch_ms = (ms1 - ms0) / max(1, n1 - n0)
    nbytes = W * unit_bytes(dom, nd_mean, nk_mean)
    achieved = nbytes / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    unit, unit_src = committed_unit(dom_sys)
    # the same bytes over the unit's kernel time in the replayed graph (the
    # committed trace of this window): the split ticks the live timing reads
    # run the unit eagerly, slower than a replayed tick
    replayed = None
    if unit and unit.get("kernel_us_per_launch"):
        r_ms = unit["kernel_us_per_launch"] / 1e3
        replayed = {"ms_per_launch": round(r_ms, 4), "achieved": round(nbytes / (r_ms * 1e-3) / 1e9, 2),
                    "frac": round(nbytes / (r_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                    "frac_pmc": round(unit["bytes_per_launch"] / (r_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                    "source": unit_src}
    cpu = cpu_exec = None
    if not args.no_cpu_baseline:
        legs = ["reference"] + ([] if args.no_cpu_executor else ["executor"])
        res = cpu_baselines(args, legs)
        cpu, cpu_exec = res["reference"], res.get("executor")
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
        "roofline": {"bound": "hbm",
                     "kernel": (f"{dom_sys} (nodes {dom}-{units[dom] - 1}: the walk kernel + its resume "
                                "kernel)" if units[dom] > dom + 1 else
                                f"{dom_sys} (node {dom}: row kernels + ordered commit)"),
                     "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": (unit or {}).get("bytes_per_launch"),
                     "traffic_source": unit_src,
                     "ms_per_launch": round(launch_ms, 4),
                     "timed_launches": int(n1 - n0),
                     "timing": "a HIP event pair bound to each of the unit's kernels (start to end, "
                               "summed over its kernels) on every 10th tick of the timed window (the "
                               "step graph is split at that unit on those ticks only)",
                     "bytes_per_launch": int(nbytes),
                     "replayed_tick": replayed,
                     "bytes_model": f"{W} worlds x SYS_BYTES of {dom_sys} at the window's mean live "
                                    f"rows per world: {nd_mean:.1f} dragons, {nk_mean:.1f} knights"},
        "cpu_baseline": cpu, "cpu_executor": cpu_exec, "error_flags": flags,
        "world_walk_runs": sim.world_walk_runs(),
        "nodes_ms_per_launch_preroll": {unit_name(i): round(v, 4) for i, v in node_ms.items()},
        "live_rows_sampled_worlds": {"sampled_worlds": len(sampled),
                                     "at_init": [args.dragons, args.knights],
                                     "by_tick_dragons_knights_per_world":
                                         [[t, round(d, 2), round(k, 2)] for t, d, k in rows_by_tick]},
    }
    print(json.dumps(out))
    sim.close()


if __name__ == "__main__":
    main()
