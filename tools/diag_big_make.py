"""Diagnose tests/test_big_make_gpu.py: step the big_make world with
progress output; dump Python stacks if a call hangs."""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
faulthandler.dump_traceback_later(50, exit=True)
import test_big_make_gpu as T  # noqa: E402

backend = sys.argv[1] if len(sys.argv) > 1 else "gpu"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 64
t0 = time.time()
print("create", backend, W, flush=True)
ex = T._sim(W, backend)
print("created", time.time() - t0, flush=True)
for t in range(6):
    ex.step()
    print("tick", t, "flags", hex(ex.error_flags()), time.time() - t0, flush=True)
    m = T._rows(ex, T.ARCH_MARK, 1, 0, T.MARK_DTYPE)
    print("  marks w0", len(m), flush=True)
print("done", flush=True)
