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
    return mw.Executor(ENV_NAME, W, Cfg(NUM_CELLS), inits, ctypes.sizeof(Init), backend=backend)


def _makes(k, tick):
    return (k * 7 + tick * 13) % 23 == 0


def _rows(ex, arch, col, w, dtype):
    return ex.read_column(arch, col, w, np.uint8, max_rows=8192).view(dtype)


@pytest.mark.gpu
def test_big_table_row_parallel_makes_unique_ids_and_serial_rows():
    W, ticks = 64, 6
    gpu = _sim(W, "gpu")
    cpu = _sim(W, "cpu")
    for t in range(ticks):
        gpu.step()
        cpu.step()
        assert gpu.error_flags() == 0 and cpu.error_flags() == 0, t
        for w in range(0, W, 7):
            cells = _rows(gpu, ARCH_CELL, 1, w, CELL_DTYPE)
            cells_c = _rows(cpu, ARCH_CELL, 1, w, CELL_DTYPE)
            assert len(cells) == NUM_CELLS
            assert cells[["k", "made"]].tobytes() == cells_c[["k", "made"]].tobytes(), (t, w)
            marks = _rows(gpu, ARCH_MARK, 1, w, MARK_DTYPE)
            marks_c = _rows(cpu, ARCH_MARK, 1, w, MARK_DTYPE)
            # the ordered commit lands the marks in the serial walk's order
            assert marks.tobytes() == marks_c.tobytes(), (t, w)
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
    cpu.close()
