#!/usr/bin/env python3
"""Device-trace contract check on the tracing build (run by
tests/test_tracing_gpu.py in a child process, since the library is chosen at
import):  MADRONA_MW_LIB=gpu-ecs-madrona_amd/build_trace/libmadrona_mw.so \
python tools/trace_check.py [out.bin]

Steps a small collisions batch with tracing on, checks the records against
the parser contract (madrona_mi355x.tracing.check_contract, block records
included), prints a per-node-kind summary, optionally dumps the records in
the scripts/parse_device_tracing.py input format."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))

import madrona_mi355x as mw  # noqa: E402
from madrona_mi355x import tracing as tr  # noqa: E402


def main():
    assert mw.Executor.trace_block_records(), "not the tracing build (MADRONA_MW_LIB)"
    W, n = 64, 32
    cfg = mw.default_collisions_config(n, 4, 1024, 2048)
    pos, rot = mw.gen_collisions_inits(W, n, seed=4)
    sim = mw.CollisionsSim(W, pos, rot, cfg)
    sim.step(2)
    sim.enable_tracing(1 << 20)
    sim.step(3)
    recs, dropped = sim.trace_records()
    names = sim.trace_func_names()
    assert dropped == 0
    assert tr.check_contract(recs, names, W, block_records=True) == 3
    for k, v in sorted(tr.summarize(recs, names).items(), key=lambda kv: -kv[1]["ns_per_step"]):
        print(f"{k:28s} {v['launches_per_step']:4.0f} launches/step {v['ns_per_step'] / 1e3:9.1f} us/step")
    if len(sys.argv) > 1:
        sim.dump_trace(sys.argv[1])
    print("trace contract ok:", len(recs), "records")


if __name__ == "__main__":
    main()
