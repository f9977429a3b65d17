"""GPU: row-parallel makeEntityNow from a node that walks more rows per world
than the row-ordered make path covers (tests/ext_env/big_make.hip: 6000
cells = 94 waves per world; waves 0..63 take IDs in row order, the rest
through the per-world ID-store lock).  Every ID handed out must be unique,
and the rows must match the same world on the CPU back end (world-serial,
the reference's walk) byte for byte outside the ID columns.  ADVICE r3
(high): the ordered path used to skip the lock, so an ordered and an
unordered wave could run the ID store's acquire at the same time."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV_SO = os.path.join(ROOT, "tests", "ext_env", "build", "libbig_make.so")
ENV_SO_CPU = os.path.join(ROOT, "tests", "ext_env", "build", "libbig_make_cpu.so")
ENV_NAME = "BigMake::World"
NUM_CELLS = 6000
ARCH_CELL, ARCH_MARK = 0, 1

CELL_DTYPE = np.dtype([("k", np.int32), ("made", np.int32), ("mark_gen", np.uint32),
                       ("mark_id", np.int32)])
MARK_DTYPE = np.dtype([("src_gen", np.uint32), ("src_id", np.int32), ("born", np.int32),
                       ("k", np.int32)])
ENTITY_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32)])


class Cfg(ctypes.Structure):
    _fields_ = [("numCells", ctypes.c_int32)]


class Init(ctypes.Structure):
    _fields_ = [("worldIndex", ctypes.c_int32)]


def _sim(W, backend):
    import madrona_mi355x as mw
    so = ENV_SO_CPU if backend == "cpu" else ENV_SO
    if ENV_NAME not in mw.env_names(backend):
        assert mw.load_env(so, backend) == 1
    inits = (Init * W)(*[Init(w) for w in range(W)])
    # up to 261 destroys per world per tick (the drop node)
    kw = {"num_workers": 4} if backend == "cpu" else {"max_deferred_destroys": 1024}
    return mw.Executor(ENV_NAME, W, Cfg(NUM_CELLS), inits, ctypes.sizeof(Init), backend=backend,
                       **kw)


def cpu_rows(W, ticks, worlds):
    """The same worlds on the CPU back end (world-serial: the reference's
    walk): per tick and world, the Cell and Mark component rows."""
    ex = _sim(W, "cpu")
    out = {}
    for t in range(ticks):
        ex.step()
        assert ex.error_flags() == 0, t
        for w in worlds:
            out[f"cells_{t}_{w}"] = _rows(ex, ARCH_CELL, 1, w, CELL_DTYPE)
            out[f"marks_{t}_{w}"] = _rows(ex, ARCH_MARK, 1, w, MARK_DTYPE)
    ex.close()
    return out


def _makes(k, tick):
    return (k * 7 + tick * 13) % 23 == 0


def _rows(ex, arch, col, w, dtype):
    return ex.read_column(arch, col, w, np.uint8, max_rows=8192).view(dtype)


def test_big_make_cpu_backend_invariants():
    # the CPU reference side of the GPU test below: every tick makes the
    # expected marks, two ticks of marks stay alive, no flag
    rows = cpu_rows(8, 4, range(0, 8, 7))
    for t in range(4):
        cells, marks = rows[f"cells_{t}_0"], rows[f"marks_{t}_0"]
        assert len(cells) == NUM_CELLS
        made_now = int(sum(_makes(k, t) for k in cells["k"]))
        assert made_now == int((marks["born"] == t).sum()) > 4 * 64
        assert set(np.unique(marks["born"]).tolist()) == set(range(max(0, t - 1), t + 1))


@pytest.mark.gpu
def test_big_table_row_parallel_makes_unique_ids_and_serial_rows(tmp_path):
    import subprocess
    import sys
    W, ticks = 64, 6
    ref = str(tmp_path / "cpu.npz")
    subprocess.run([sys.executable, os.path.abspath(__file__), str(W), str(ticks), ref],
                   check=True, timeout=120)
    ref = np.load(ref)
    gpu = _sim(W, "gpu")
    for t in range(ticks):
        gpu.step()
        assert gpu.error_flags() == 0, (t, hex(gpu.error_flags()))
        for w in range(0, W, 7):
            cells = _rows(gpu, ARCH_CELL, 1, w, CELL_DTYPE)
            cells_c = ref[f"cells_{t}_{w}"]
            assert len(cells) == NUM_CELLS
            # (plain bools: pytest's diff of two long byte strings takes minutes)
            same = (np.array_equal(cells["k"], cells_c["k"]) and
                    np.array_equal(cells["made"], cells_c["made"]))
            assert same, (t, w)
            marks = _rows(gpu, ARCH_MARK, 1, w, MARK_DTYPE)
            marks_c = ref[f"marks_{t}_{w}"]
            # the ordered commit lands the marks in the serial walk's order
            same = marks.tobytes() == marks_c.tobytes()
            assert same, (t, w, len(marks), len(marks_c))
            made_now = int(sum(_makes(k, t) for k in cells["k"]))
            assert made_now > 4 * 64          # rows made by waves past the 64th too
            assert made_now == int((marks["born"] == t).sum())
            ids = np.concatenate([_rows(gpu, ARCH_CELL, 0, w, ENTITY_DTYPE)["id"],
                                  _rows(gpu, ARCH_MARK, 0, w, ENTITY_DTYPE)["id"]])
            assert (ids >= 0).all() and len(np.unique(ids)) == len(ids), (t, w)
            # every cell that made a mark this tick points at a live mark row
            ent = _rows(gpu, ARCH_MARK, 0, w, ENTITY_DTYPE)
            live = set(zip(ent["gen"].tolist(), ent["id"].tolist()))
            fresh = cells[np.array([_makes(k, t) for k in cells["k"]])]
            assert all((int(g), int(i)) in live for g, i in zip(fresh["mark_gen"], fresh["mark_id"]))
    gpu.close()


if __name__ == "__main__":           # child of the GPU test: no GPU in this process
    import sys
    sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))
    W, ticks, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    np.savez(path, **cpu_rows(W, ticks, range(0, W, 7)))
