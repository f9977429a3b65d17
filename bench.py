#!/usr/bin/env python3
"""Benchmark: env-steps/s of the `collisions` rigid-body workload
(BASELINE.json configs[2]: 8192 worlds x 128 cube hulls + ground plane, S=4,
dt=1/60) on MI355X.

    python bench.py [--gpus N --steps K --warmup W] [--workload simple]

--workload simple measures BASELINE.json configs[1] instead
(examples/simple_taskgraph, 8192 worlds x 100 objects + test object + agent,
clamp + physics, S=4) with the same roofline / CPU-baseline legs; its
hand-off is the exported agent positions (getExported slot 0).

A "step" = one taskgraph step of every world (broadphase, 4 XPBD substeps of
integrate / narrowphase / solve, cleanup, episode-return node) replayed as one
hipGraph, followed by the training hand-off: the per-world episode returns are
copied into a torch tensor on the device and, for N > 1, all-gathered over
RCCL (xGMI) into it, by the framework on its step stream.  Steps and
hand-offs are enqueued back to back (no host round trip per step); the timed
region is closed by a device sync.
Worlds are sharded contiguously across ranks (weak scaling: 8192 per GPU;
N = 8 is BASELINE.json configs[3], 65 536 worlds).

Prints ONE JSON line on rank 0 (metric / value / roofline / cpu_baseline; see
DESIGN.md §6 for the byte model behind `roofline`).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, HBM3E 8.0 TB/s spec

# Algorithmic bytes each node moves per unit, per launch (SURVEY.md §8(d),
# DESIGN.md §3 "Roofline in bench.py"): body = one physics body row, cand =
# one candidate pair, surv = one narrowphase survivor pair, contact = one
# contact manifold; "fused" = the work a launch does only when it also runs
# the next substep's integration + filter (SolverNode, substeps 0..S-2) or
# the first substep's filter (NarrowphaseNode, substep 0), weighted by the
# timed launches that did.  The overlap query's 116 B per visited BVH node
# is not counted (lower bound).
BYTES = {
    "UpdateLeafPositionsNode": {"body": 96 + 68},
    # whole BVH nodes read and written back (0.69 nodes of 116 B per body: the
    # oracle's trees hold 81-97 nodes per 129-body world in the timed window)
    # + the leaf AABB, parent and LeafID per body; PMC (calibrated): 1.0x
    "RefitNode": {"body": 32 + 160},
    "UpdateBVHNode": {"body": 0},
    # per body: its leaf's node slot (the node's lines, 80 B per body), leaf
    # parent / order / entity, the entity's IDNode, ResponseType, LeafID and
    # leaf AABB; per candidate: the pair (16 B) and its packed slots (8 B)
    "FindOverlappingNode": {"body": 80 + 4 + 4 + 8 + 12 + 4 + 4 + 24, "cand": 16 + 8},
    "SubstepRigidBodiesNode": {"body": 84 + 108},
    # filter (substep 0 only): the candidate and both bodies' poses per
    # candidate; SAT / plane: the packed work entry (16 B) and both bodies'
    # poses (Position 12 + Rotation 16 + Scale 12 + ObjectID 4) per survivor
    # pair; the manifold written per contact
    "NarrowphaseNode": {"surv": 16 + 2 * 44, "contact": 112,
                        "fused": {"cand": 16 + 2 * 44}},
    # solverKernel (one wave per world): each body's image in once (Position
    # 12, Rotation 16, Velocity 24, ObjectID 4, ResponseType 4) and out once
    # (Position, Rotation, Velocity); per contact and per pass (positions,
    # velocities) the 112-byte manifold and both bodies' read-only substep
    # columns (positions: PreSolvePositional + SubstepPrevState, 2 x 56;
    # velocities: PreSolvePositional + PreSolveVelocity, 2 x 52), lambdaN
    # written (16), survivor info read and contact order written (4 + 4);
    # fused tail: the next substep's integration (192 / body, as
    # SubstepRigidBodiesNode) and narrowphase filter (104 / cand)
    "SolverNode": {"body": 60 + 52,
                   "contact": (112 + 2 * 56 + 16) + (112 + 2 * 52) + 4 + 4,
                   "fused": {"body": 84 + 108, "cand": 16 + 2 * 44}},
}


def launch_bytes(node, units):
    """Algorithmic bytes of one launch of `node` for `units` (per-launch
    means; units["fused"] = fraction of launches that ran the fused work)."""
    m = BYTES[node]
    b = sum(v * units.get(u, 0.0) for u, v in m.items() if u != "fused")
    b += units.get("fused", 0.0) * sum(v * units.get(u, 0.0) for u, v in m.get("fused", {}).items())
    return b


NODE_KINDS = list(BYTES.keys()) + ["CustomParallelForNode", "ParallelForNode"]


def pmc_traffic(kernel_node, workload="collisions", timed_steps=None):
    """HBM bytes per launch of the node's kernel from the committed rocprofv3
    PMC passes of the same workload (profiles/rNN_traffic*.json for
    collisions, profiles/rNN_<workload>_traffic*.json otherwise, written by
    profiles/pmc_traffic.py via profiles/collect.sh: FETCH_SIZE x 2 (gfx950
    correction) + WRITE_SIZE), from the latest file whose step window is
    exactly `timed_steps` (the window this run timed).  (None, note) when no
    committed profile covers that window."""
    import glob
    import re
    tag = "" if workload == "collisions" else workload + "_"
    pat = re.compile(r"r\d+_" + tag + r"traffic(_w\d+-\d+)?\.json$")
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_traffic*.json"))
                   if pat.search(os.path.basename(f)))
    seen = []
    for path in reversed(files):
        try:
            with open(path) as f:
                data = json.load(f)
        except (OSError, ValueError):
            continue
        seen.append(f"{os.path.basename(path)}: {data.get('timed_steps')}")
        if data.get("timed_steps") != timed_steps:
            continue
        entry = data.get("nodes", {}).get(kernel_node)
        if entry is None or entry.get("bytes_per_launch") is None:
            continue
        return entry["bytes_per_launch"], f"profiles/{os.path.basename(path)}, steps {timed_steps}"
    return None, (f"no committed PMC profile for steps {timed_steps} "
                  f"(have: {'; '.join(seen) or 'none'})")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--worlds", type=int, default=8192, help="worlds per GPU")
    p.add_argument("--settle", type=int, default=120,
                   help="untimed pre-roll steps so the timed window is the settled, "
                        "contact-heavy regime (cubes fall from z<=10 for ~85 steps)")
    p.add_argument("--workload", choices=("collisions", "simple"), default="collisions")
    p.add_argument("--cubes", type=int, default=0,
                   help="bodies per world besides the fixed ones (0: 128 collisions, 100 simple)")
    p.add_argument("--substeps", type=int, default=4)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-worlds", type=int, default=0,
                   help="worlds per CPU batch (0 = 16 per CPU thread, at least 256)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = every core this process may use (affinity, capped by the cgroup CPU quota)")
    p.add_argument("--cpu-steps", type=int, default=0,
                   help="timed steps per CPU batch (0 = --steps: the GPU's timed window)")
    p.add_argument("--cpu-target-s", type=float, default=10.0)
    p.add_argument("--cpu-max-batches", type=int, default=12)
    p.add_argument("--cpu-port", action="store_true", help="time oracle/ instead of oracle/_ref")
    p.add_argument("--cpu-executor", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--no-cpu-executor", action="store_true",
                   help="skip timing the framework's own CPU back end (libmadrona_cpu.so)")
    p.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cpu-first-world", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--timed-every", type=int, default=10,
                   help="time the dominant kernel's launches in every N-th timed step (the "
                        "graph is split at that node only in those steps)")
    p.add_argument("--no-handoff", action="store_true")
    p.add_argument("--backend", choices=("gpu", "cpu"), default="gpu",
                   help="cpu: the framework's CPU back end with a gloo hand-off -- a rehearsal of "
                        "the multi-rank path without a GPU (tests/test_bench_launch.py), never "
                        "the headline")
    p.add_argument("--dry-launch", action="store_true",
                   help="spawn the ranks as for a real run; each prints its launch environment "
                        "and exits without touching a GPU")
    p.add_argument("--ref-ticks", type=int, default=1000,
                   help="the reference's own timing definition (examples/collisions/gpu.cpp:32-43): "
                        "a fresh executor, this many synchronous steps from init, wall time; "
                        "reported beside the headline (0 = skip)")
    args = p.parse_args()
    if args.cubes <= 0:
        args.cubes = 128 if args.workload == "collisions" else 100
    # at least one timed launch of the dominant kernel however short the run
    args.timed_every = max(1, min(args.timed_every, args.steps))
    return args


def _cpu_child(args):
    """One bounded CPU sample in a fresh process: the reference executor
    reserves virtual address space per world that it never releases, so each
    batch of worlds lives in its own short-lived child."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol
    threads = max(1, args.cpu_threads)
    W, first = args.cpu_worlds, args.cpu_first_world
    pos, rot = ol.gen_collisions_inits(first + W, args.cubes, seed=0)
    pos, rot = pos[first:], rot[first:]
    ocfg = ol.default_phys_config(args.cubes, args.substeps, max_contacts=4096)
    simple = args.workload == "simple"
    if args.cpu_executor:
        # the framework's CPU back end: same world sources, pinned workers
        import madrona_mi355x as mw
        g = mw.default_collisions_config(args.cubes, args.substeps, 4096, 4096)
        Sim = mw.SimpleSim if simple else mw.CollisionsSim
        sim = Sim(W, pos, rot, g, backend="cpu", num_workers=threads)
        kind = "port"
        sim.step(args.settle + args.warmup)
        t0 = time.perf_counter()
        sim.step(args.cpu_steps)
        dt = time.perf_counter() - t0
        assert sim.error_flags() == 0
    elif ol.ref_available() and not args.cpu_port:
        sim = ol.ReferenceSimple(ocfg, pos, rot) if simple else ol.ReferencePhys(ocfg, pos, rot)
        lib = sim.lib
        lib.ref_phys_step_mt.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        kind = "reference"
        lib.ref_phys_step_mt(sim.h, args.settle + args.warmup, threads)
        t0 = time.perf_counter()
        lib.ref_phys_step_mt(sim.h, args.cpu_steps, threads)
        dt = time.perf_counter() - t0
    else:
        sim = ol.OracleSimple(ocfg, pos, rot) if simple else ol.OraclePhys(ocfg, pos, rot)
        kind = "port"
        sim.step(args.settle + args.warmup, threads)
        t0 = time.perf_counter()
        sim.step(args.cpu_steps, threads)
        dt = time.perf_counter() - t0
    print(json.dumps({"kind": kind, "seconds": dt, "env_steps": W * args.cpu_steps}))


def usable_cores():
    """Cores this process may run on: the affinity mask, capped by the cgroup
    v2 CPU quota when one is set (a GPU box's share of a larger host)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baselines(args, legs):
    """CPU legs on a bounded sample of the same workload and the same step
    window as the timed GPU region (steps warmup+1 .. warmup+K of consecutive
    world batches): "reference" = the reference's own executor (oracle/_ref,
    built from its src/core + src/physics; the parity-pinned restatement in
    oracle/ when that build is absent), "executor" = the framework's CPU back
    end (libmadrona_cpu.so).  With both legs their batches alternate over the
    same worlds (reference batch i, then executor batch i), so the two rates
    come from the same worlds in the same stretch of host load; batches are
    added until every leg has cpu_target_s of timed work."""
    import subprocess
    threads = args.cpu_threads if args.cpu_threads > 0 else usable_cores()
    if args.cpu_worlds <= 0:
        args.cpu_worlds = max(256, 16 * threads)
    if args.cpu_steps <= 0:
        args.cpu_steps = args.steps
    acc = {leg: {"s": 0.0, "steps": 0, "kind": None} for leg in legs}
    batches = 0
    t_wall = time.perf_counter()
    while batches < args.cpu_max_batches and min(a["s"] for a in acc.values()) < args.cpu_target_s:
        for leg in legs:
            cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child",
                   "--cpu-worlds", str(args.cpu_worlds),
                   "--cpu-first-world", str(batches * args.cpu_worlds),
                   "--cpu-threads", str(threads), "--cubes", str(args.cubes),
                   "--workload", args.workload,
                   "--substeps", str(args.substeps), "--cpu-steps", str(args.cpu_steps),
                   "--settle", str(args.settle), "--warmup", str(args.warmup)] + \
                  (["--cpu-port"] if args.cpu_port else []) + \
                  (["--cpu-executor"] if leg == "executor" else [])
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                raise RuntimeError(f"cpu {leg} child failed: {r.stderr[-2000:]}")
            res = json.loads(r.stdout.strip().splitlines()[-1])
            acc[leg]["kind"] = res["kind"]
            acc[leg]["s"] += res["seconds"]
            acc[leg]["steps"] += res["env_steps"]
        batches += 1
    wall = time.perf_counter() - t_wall
    out = {}
    for leg in legs:
        a = acc[leg]
        out[leg] = {
            "value": round(a["steps"] / a["s"], 1),
            "unit": "env-steps/s",
            "cores": threads,
            "cpu_model": cpu_model(),
            "host_cpus_visible": os.cpu_count(),
            "kind": a["kind"],
            "sample": ("libmadrona_cpu.so: " if leg == "executor" else "")
                      + f"{args.workload} {batches} batches x {args.cpu_worlds} worlds (worlds 0-"
                      f"{batches * args.cpu_worlds - 1}) x {args.cubes} cubes, S={args.substeps}; "
                      f"timed steps {args.settle + args.warmup + 1}-"
                      f"{args.settle + args.warmup + args.cpu_steps} ("
                      + ("the GPU's timed window" if args.cpu_steps == args.steps
                         else "starts where the GPU's timed window starts")
                      + f"), {threads} host threads pinned one per usable core, "
                      f"{a['s']:.2f} s timed"
                      + (f"; batches alternated with the {' / '.join(l for l in legs if l != leg)} "
                         f"leg over the same worlds, {wall:.1f} s wall for all legs"
                         if len(legs) > 1 else f" / {wall:.1f} s wall"),
        }
    return out


LAUNCH_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` without a launcher: start N rank processes of this script
    (one per GPU, LOCAL_RANK = GPU ordinal; the environment
    torch.distributed.run would give them, rendezvous on 127.0.0.1) and exit
    with the first non-zero status among them.  Called before this process
    imports the framework or torch, so the parent never touches a GPU.  A
    rank that fails takes the others down (they would wait at a barrier)."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench: rank {procs.index(p)} exited with status {code}; stopping the "
                      "other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


def main():
    args = parse()
    if args.cpu_child:
        return _cpu_child(args)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher "
                             f"disagrees with --gpus {args.gpus}")
    elif args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_launch:
        print(json.dumps({"dry_launch": {k: os.environ.get(k) for k in LAUNCH_VARS},
                          "pid": os.getpid(), "gpus": args.gpus}), flush=True)
        return None
    cpu_backend = args.backend == "cpu"
    if cpu_backend:
        # rehearsal of the rank / hand-off plumbing: no per-node GPU timing,
        # no CPU-baseline legs, no reference-definition leg
        args.no_roofline = args.no_cpu_baseline = True
        args.ref_ticks = 0
    breakdown_steps = 0 if args.no_roofline else 2 * len(NODE_KINDS)
    startup_steps = 0 if args.no_roofline else 20
    if args.settle < breakdown_steps + startup_steps:
        raise SystemExit(f"--settle must be >= {breakdown_steps + startup_steps} "
                         "(the start-up and per-node breakdown steps)")

    # The framework owns the step stream and the hand-off collective (RCCL
    # over xGMI from the C ABI, enqueued right behind the step); the hand-off
    # lands in a learner-owned torch tensor on the same device.  torch and the
    # framework share one HIP runtime (madrona_mi355x imports torch first);
    # the timing barrier / max-reduce run over gloo on the CPU.
    import madrona_mi355x as mw
    import torch
    from madrona_mi355x.sharding import bootstrap_rccl, gather_world_returns, world_shard
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
    if not cpu_backend:
        torch.cuda.set_device(local_rank)

    cfg = mw.default_collisions_config(args.cubes, args.substeps, max_contacts=4096,
                                       max_candidates=4096)
    first_world, W = world_shard(rank, args.worlds)
    simple = args.workload == "simple"
    Sim = mw.SimpleSim if simple else mw.CollisionsSim

    def make_sim():
        pos, rot = mw.gen_collisions_inits(W, args.cubes, seed=0, first_world=first_world)
        if cpu_backend:
            return Sim(W, pos, rot, cfg, backend="cpu", num_workers=max(1, args.cpu_threads))
        return Sim(W, pos, rot, cfg, gpu_id=local_rank)

    sim = make_sim()
    # the training hand-off: collisions -- the per-world episode return
    # (export slot 2, 1 float); simple -- the agent's position (slot 0, 3)
    ho_slot, ho_floats = (0, 3) if simple else (2, 1)

    if dist is not None and not cpu_backend:
        bootstrap_rccl(sim, rank, world_size)
    # per-world returns of every rank, in world order: a torch tensor
    returns = torch.empty(W * world_size * ho_floats, dtype=torch.float32,
                          device="cpu" if cpu_backend else f"cuda:{local_rank}")
    handoff = returns.data_ptr()

    # Every step is enqueued without a host round trip: the step graph, then
    # the hand-off (D2D copy / RCCL all-gather of the returns into the torch
    # tensor) on the same stream; the timed region ends with a device sync.
    # The CPU back end steps synchronously and gathers over gloo.
    def step():
        sim.step_async(1)
        if args.no_handoff:
            return
        if cpu_backend:
            local = torch.from_numpy(sim.exported_array(ho_slot, np.float32).copy())
            if dist is not None:
                gather_world_returns(local, out=returns)
            else:
                returns.copy_(local)
        elif dist is not None:
            sim.allgather_exported(ho_slot, handoff, 4 * ho_floats * W)
        else:
            sim.copy_exported_async(ho_slot, handoff, 4 * ho_floats * W)

    def barrier():
        if dist is not None:
            dist.barrier()

    # Per-node breakdown (eager, untimed, part of the settle pre-roll: each
    # kind's 2 timed steps advance the simulation, so they count towards
    # --settle and the timed window starts exactly at step settle+warmup+1):
    # picks the dominant kernel, whose launches are then timed live inside
    # the replayed graph.
    launches = {"SubstepRigidBodiesNode": args.substeps, "NarrowphaseNode": args.substeps,
                "SolverNode": args.substeps, "FindOverlappingNode": 1,
                "UpdateLeafPositionsNode": 2, "RefitNode": 2, "UpdateBVHNode": 1,
                "CustomParallelForNode": 1, "ParallelForNode": 1}
    node_table = {}
    dom = None
    # Start-up cost (untimed, part of the settle pre-roll): step 1 carries the
    # forced BVH rebuild (its kernel timed with HIP events), then the wall
    # time of steps 2-20, each synchronised, while the cubes fall and land.
    startup = None
    if startup_steps:
        rebuild_ms = sim.time_node("UpdateBVHNode", 1)
        wall = []
        for _ in range(startup_steps - 1):
            sim.sync()
            t0 = time.perf_counter()
            sim.step(1)
            sim.sync()
            wall.append((time.perf_counter() - t0) * 1e3)
        startup = {"step1_bvh_rebuild_ms": round(rebuild_ms, 4),
                   "steps_2_20_ms": [round(x, 3) for x in wall],
                   "steps_2_20_total_ms": round(sum(wall), 3)}
    sim.step(args.settle - breakdown_steps - startup_steps)
    if not args.no_roofline:
        for name in NODE_KINDS:
            ms = sim.time_node(name, 2)
            if ms > 0:
                node_table[name] = {"ms_per_launch": round(ms, 4),
                                    "ms_per_step": round(ms * launches[name], 4)}
        dom = max((n for n in node_table if n in BYTES),
                  key=lambda n: node_table[n]["ms_per_step"])
        sim.set_timed_node(dom, every=args.timed_every)

    for _ in range(args.warmup):
        step()
    ev_ms0, ev_n0 = sim.timed_node() if dom else (0.0, 0)
    if dom:
        sim.take_units()       # (syncs) units of the timed launches only

    # timed region: barrier + device sync on both sides (the framework's
    # stream is the only GPU work in this process), max over ranks
    barrier()
    sim.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sim.sync()
    own_elapsed = time.perf_counter() - t0      # this rank's own steps (before the barrier)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    flags = sim.error_flags()
    total_worlds = W * world_size
    value = total_worlds * args.steps / elapsed

    roofline = None
    if dom:
        ev_ms1, ev_n1 = sim.timed_node()
        if ev_n1 - ev_n0 <= 0:
            raise RuntimeError(f"bench: no timed launch of {dom} in {args.steps} steps")
        ms = (ev_ms1 - ev_ms0) / (ev_n1 - ev_n0)
        # the work units of exactly the timed launches (their candidates,
        # survivors and manifolds, summed on the device right after each
        # timed launch; mw_phys_take_units)
        n_l, u_cand, u_cont, n_fused, u_surv = sim.take_units()
        if n_l != ev_n1 - ev_n0:
            raise RuntimeError(f"bench: {n_l} unit probes for {ev_n1 - ev_n0} timed launches")
        units = {"body": W * (args.cubes + (2 if simple else 1)), "cand": u_cand / n_l,
                 "surv": u_surv / n_l, "contact": u_cont / n_l, "fused": n_fused / n_l}
        nbytes = launch_bytes(dom, units)
        achieved = nbytes / (ms * 1e-3) / 1e9
        # whole step: every modelled node at the timed launches' mean units
        # (NarrowphaseNode's survivors only when it was the timed node)
        step_units = dict(units, fused=(args.substeps - 1) / args.substeps)
        step_bytes = sum(launches[n] * launch_bytes(n, step_units) for n in BYTES
                         if n not in ("SolverNode", "NarrowphaseNode"))
        step_bytes += args.substeps * launch_bytes("SolverNode", step_units)
        if dom == "NarrowphaseNode":
            step_bytes += args.substeps * launch_bytes(
                "NarrowphaseNode", dict(units, fused=1.0 / args.substeps))
        timed_steps = f"{args.settle + args.warmup + 1}-{args.settle + args.warmup + args.steps}"
        traffic, traffic_src = pmc_traffic(dom, args.workload, timed_steps)
        roofline = {
            "bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_launch": int(nbytes), "ms_per_launch": round(ms, 4),
            "timed_launches": int(ev_n1 - ev_n0),
            "timing": ("a HIP event pair bound to each of the node's kernels (hipExtLaunchKernelGGL: "
                       "kernel start to kernel end, summed over the node's kernels, no dispatch gap) "
                       "on every launch of the node in "
                       + ("every timed step" if args.timed_every <= 1 else
                          f"every {args.timed_every}th timed step (the first of each run of "
                          f"{args.timed_every}; the step graph is split at that node in those "
                          "steps only, the others replay the unsplit graph)")),
            "units_per_launch": {k: round(v, 3) for k, v in units.items()},
            "units_source": (f"summed on the device after each of the {n_l} timed launches "
                             "(mw_phys_take_units)"),
            "step_algorithmic_bytes": int(step_bytes),
            "step_achieved_gbs": round(step_bytes / (elapsed / args.steps) / 1e9, 2),
            "mean_candidates_per_world": round(units["cand"] / W, 1),
            "mean_contacts_per_world": round(units["contact"] / W, 1),
        }
        if traffic:
            # the counters' HBM bytes over the same launches: the model counts
            # reads that LDS / L2 serve, so this rate is the HBM-true one
            roofline["frac_pmc"] = round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
            roofline["model_over_pmc"] = round(nbytes / traffic, 3)

    # N > 1: every rank's own step time, error flags and dominant-kernel time
    # (a shard imbalance or a failing shard shows here, not only in the max)
    ranks = None
    if dist is not None:
        mine = torch.tensor([own_elapsed, float(flags), roofline["ms_per_launch"] if roofline else -1.0],
                            dtype=torch.float64)
        got = [torch.zeros_like(mine) for _ in range(world_size)]
        dist.all_gather(got, mine)
        per = []
        for r, (el, fl, dms) in enumerate(x.tolist() for x in got):
            e = {"rank": r, "worlds": W, "ms_per_step": round(el / args.steps * 1e3, 4),
                 "value": round(W * args.steps / el, 1), "error_flags": int(fl)}
            if dms >= 0:
                e["dominant_ms_per_launch"] = round(dms, 4)
            per.append(e)
        mss = [e["ms_per_step"] for e in per]
        ranks = {"per_rank": per,
                 "ms_per_step": {"min": min(mss), "max": max(mss), "mean": round(sum(mss) / len(mss), 4)},
                 "imbalance": round(max(mss) / min(mss), 4) if min(mss) > 0 else None}
        for e in per:
            flags |= e["error_flags"]

    assert bool(torch.isfinite(returns).all()), "non-finite returns in the hand-off tensor"
    sim.close()

    # The reference's own definition (examples/collisions/gpu.cpp:32-43): a
    # fresh executor, ref_ticks synchronous run() calls from init (start-up
    # transient included), wall time; beside the settled-window headline.
    ref_def = None
    if rank == 0 and world_size == 1 and args.ref_ticks > 0:
        sim = make_sim()
        sim.sync()
        t0 = time.perf_counter()
        for _ in range(args.ref_ticks):
            sim.step(1)
        dt = time.perf_counter() - t0
        ref_def = {"value": round(W * args.ref_ticks / dt, 1), "unit": "env-steps/s",
                   "ticks": f"1-{args.ref_ticks}", "seconds": round(dt, 4),
                   "ms_per_step": round(dt / args.ref_ticks * 1e3, 4),
                   "definition": "examples/collisions/gpu.cpp:32-43: a fresh executor, "
                                 f"{args.ref_ticks} synchronous steps from init timed by wall clock "
                                 "(each mw_step waits for its step, as run() syncs its stream; "
                                 "no hand-off)",
                   "error_flags": sim.error_flags()}
        sim.close()

    cpu = cpu_exec = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        # the framework's own CPU back end (the reference's
        # TaskGraphExecutor restated, libmadrona_cpu.so) on the same cores,
        # worlds and step window, reported beside the reference
        legs = ["reference"] + ([] if args.no_cpu_executor else ["executor"])
        res = cpu_baselines(args, legs)
        cpu, cpu_exec = res["reference"], res.get("executor")

    if rank == 0:
        out = {
            "metric": "env-steps/sec (summed worlds)",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference example init: mt19937 seed 0 positions/rotations)",
            "config": {
                "workload": (f"examples/simple_taskgraph: {W} worlds/GPU x {args.cubes} objects + "
                             f"test object + agent, clamp + physics, S={args.substeps}, dt=1/60"
                             if simple else
                             f"examples/collisions physics: {W} worlds/GPU x {args.cubes} cube hulls "
                             f"+ ground plane, S={args.substeps}, dt=1/60"),
                "worlds_per_gpu": W, "total_worlds": total_worlds,
                "timed_steps": f"{args.settle + args.warmup + 1}-{args.settle + args.warmup + args.steps}",
                "parallelism": f"world-sharded x{world_size}" +
                               ("" if args.no_handoff else ", per-step return hand-off"
                                + ((" (gloo all-gather)" if cpu_backend else " (RCCL all-gather over xGMI)")
                                   if world_size > 1 else "")),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_executor": cpu_exec,
            "reference_definition": ref_def,
            "error_flags": flags,
            "nodes": node_table,
            **({"ranks": ranks} if ranks else {}),
            "startup": startup,
        }
        if cpu_backend:
            out["backend"] = "cpu (rehearsal of the rank plumbing, not a GPU measurement)"
        print(json.dumps(out), flush=True)
    del returns
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
