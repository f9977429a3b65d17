#!/usr/bin/env python3
"""A/B of bench.py over library builds / environment switches (experiment
tool, GPU box).  Each variant is LABEL or LABEL:VAR=VAL[,VAR=VAL...]; a
variable LIB=<build dir> selects gpu-ecs-madrona_amd/<dir>/libmadrona_mw.so.

    python tools/ab_bench.py --workload simple new old:LIB=build_ab notab:MADRONA_MW_SAT_TABLES=0

Runs each variant once (a child process under its own time limit), prints
value and the per-node ms per launch, and stops at the first child that
ends by a signal or a time limit (no retries)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="simple")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--timeout", type=int, default=200)
    ap.add_argument("--out", default="gpurun_out/ab")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, os.path.dirname(a.out)), exist_ok=True)
    for var in a.variants:
        label, _, spec = var.partition(":")
        env = dict(os.environ)
        for kv in filter(None, spec.split(",")):
            k, _, v = kv.partition("=")
            if k == "LIB":
                env["MADRONA_MW_LIB"] = os.path.join(ROOT, "gpu-ecs-madrona_amd", v, "libmadrona_mw.so")
            else:
                env[k] = v
        cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", os.path.join(ROOT, "bench.py"),
               "--workload", a.workload, "--steps", str(a.steps), "--no-cpu-baseline", "--no-cpu-executor"]
        out = f"{a.out}_{a.workload}_{label}.json"
        with open(os.path.join(ROOT, out), "w") as f, open(os.path.join(ROOT, out + ".err"), "w") as e:
            rc = subprocess.run(cmd, env=env, stdout=f, stderr=e, cwd=ROOT).returncode
        if rc != 0:
            print(f"{label}: rc={rc}, see {out}.err", flush=True)
            if rc < 0 or rc in (124, 134, 137, 139):
                sys.exit(rc if rc > 0 else 128 - rc)
            continue
        d = json.loads(open(os.path.join(ROOT, out)).read().strip().splitlines()[-1])
        nodes = {k: v["ms_per_launch"] for k, v in d.get("nodes", {}).items()}
        print(f"{label}: {d['value']:.0f} env-steps/s flags={d.get('error_flags')} {nodes}", flush=True)


if __name__ == "__main__":
    main()
