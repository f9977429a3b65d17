"""Prints, for each reset method x size x host-copy setting, how many of the
graph replays left a counter wrong (tests/diag/memset_node.hip).  TEST
INFRASTRUCTURE: a diagnosis run, results recorded in DESIGN.md.
host_copies: 0 none, 1 synchronous H2D / D2H copies between replays, 2 the
same after scribbling the host stack with the fault log's counter value
(the graph is captured in a helper whose frame is gone by then), 3 also a
D2H read-back and a hipMalloc / hipFree between replays, 4 also 4096 host
heap blocks filled with that value and freed between replays."""
import ctypes
import json
import os

import torch  # noqa: F401  (the same HIP runtime the framework's library uses)

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    lib = ctypes.CDLL(os.path.join(HERE, "build", "libmemset_node.so"))
    lib.memset_node_run.argtypes = [ctypes.c_int32] * 4 + [ctypes.POINTER(ctypes.c_int64)]
    lib.memset_node_run.restype = ctypes.c_int
    return lib


def run(lib, reset, n, replays, host_copies):
    out = (ctypes.c_int64 * 3)()
    rc = lib.memset_node_run(reset, n, replays, host_copies, out)
    assert rc == 0, rc
    return {"bad_replays": out[0], "first_bad": out[1], "bad_counters": out[2]}


if __name__ == "__main__":
    torch.cuda.init()
    lib = load()
    rows = []
    for reset in (0, 1, 2):
        for n in (1, 2, 64, 8192, 8193):
            for hc in (0, 1, 2, 3, 4):
                r = run(lib, reset, n, 200, hc)
                r.update(reset=["kernel", "hipMemsetAsync", "hipMemsetD32Async"][reset], n=n, host_copies=hc)
                rows.append(r)
                print(json.dumps(r), flush=True)
