"""Table growth (reference src/common/table.cpp:44-61:
Table::addRow doubles a full per-world table, state.inl registerArchetype).
The ecs_ops world with grow_spawns registers Spawn with registerArchetype
(no fixed size): it starts at mw_config.default_capacity rows per world and
the executor grows it between steps, at half full, doubling.  Its spawn
count climbs to ~120 per world within 40 steps, so a table declared at 16
rows ends 8x larger, and every step stays bit-exact with the same world on
the reference's own ECS (oracle/ref_ecs.cpp, whose tables grow by
themselves) -- with no table-full flag.  The ID store and the ordered
commit's shape grow with it."""
import ctypes

import pytest

import ecs_ops_lib as el

needs_ref = pytest.mark.skipif(not el.ref_available(), reason="oracle/_ref not built")

DECLARED = 16


def _capacity(sim, arch, col=1):
    b, c = ctypes.c_int32(), ctypes.c_int32()
    assert sim.exec._lib.mw_column_info(sim.exec.h, arch, col, ctypes.byref(b), ctypes.byref(c)) == 0
    return c.value


def _run(sim, ref, steps, exact_ids):
    W = sim.num_worlds
    caps = []
    for s in range(steps):
        sim.step()
        ref.step()
        assert sim.error_flags() == 0, (s, sim.error_flags())
        for w in range(W):
            el.compare_world(sim, ref, w, f"step {s}", exact_ids=exact_ids)
        caps.append(_capacity(sim, el.ARCH_SPAWN))
    live = max(len(sim.spawns(w)) for w in range(W))
    return caps, live


@needs_ref
def test_growth_cpu_backend_bit_exact_with_reference_ecs():
    W = 8
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED, backend="cpu", num_workers=2)
    ref = el.RefEcsOps(W)
    assert _capacity(sim, el.ARCH_SPAWN) == DECLARED
    caps, live = _run(sim, ref, 40, exact_ids=True)
    assert live > 4 * DECLARED, live                 # 4x past the declared capacity
    assert caps[-1] >= 2 * live and caps == sorted(caps), caps
    # fixed-size tables never grow
    assert _capacity(sim, el.ARCH_AGENT) == el.NUM_AGENTS


@needs_ref
def test_fixed_size_table_is_not_grown_cpu():
    W = 4
    sim = el.EcsOpsSim(W, grow_spawns=False, default_capacity=DECLARED, backend="cpu", num_workers=1)
    sim.step(5)
    assert _capacity(sim, el.ARCH_SPAWN) == 512      # registerFixedSizeArchetype(kMaxSpawns)


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("serial", [False, True])
def test_growth_gpu_bit_exact_with_reference_ecs(serial):
    """Row-parallel makes append into the grown slabs (their keys re-strided
    with them); world-serially the IDs are the reference's exactly."""
    W = 64
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED, serial_nodes=serial)
    ref = el.RefEcsOps(W)
    assert _capacity(sim, el.ARCH_SPAWN) == DECLARED
    caps, live = _run(sim, ref, 40, exact_ids=serial)
    assert live > 4 * DECLARED, live
    assert caps[-1] >= 2 * live and caps == sorted(caps), caps


@pytest.mark.gpu
@needs_ref
def test_growth_gpu_with_world_walk_and_exports(monkeypatch):
    """The walk plan and the step graph are rebuilt after a growth (a row
    node over the grown table moves from the walk to its own launches once
    its lanes exceed a wave's); results stay exact through it."""
    monkeypatch.setenv("MADRONA_MW_WORLD_WALK", "1")
    W = 32
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED)
    ref = el.RefEcsOps(W)
    runs0 = sim.exec.world_walk_runs()
    caps, live = _run(sim, ref, 40, exact_ids=False)
    assert caps[-1] > DECLARED and runs0 >= 1


SPAWN_EXPORT = 1            # exportColumn<Spawn, SpawnInfo>(1)


def _check_export(sim, where):
    """The packed SpawnInfo export equals the worlds' Spawn rows, world-major
    (reference getExported: every world's rows of the column, in order)."""
    import numpy as np
    ptr, rows = sim.exec.exported(SPAWN_EXPORT)
    want = [sim._cols(el.ARCH_SPAWN, w, (1,))[0] for w in range(sim.num_worlds)]
    want = np.concatenate(want) if want else np.zeros(0, np.uint8)
    assert rows * 24 == len(want), (where, rows, len(want))
    got = sim.exec.exported_array(SPAWN_EXPORT, np.uint8)
    assert got.tobytes() == want.tobytes(), f"{where}: packed export differs from the Spawn rows"
    return ptr


def _compare_all(sim, ref, where, exact_ids=False):
    assert sim.error_flags() == 0, (where, sim.error_flags())
    for w in range(sim.num_worlds):
        el.compare_world(sim, ref, w, where, exact_ids=exact_ids)


@needs_ref
def test_growth_cpu_backend_multi_step_call():
    """mw_step(40) in one call: the CPU back end steps one step at a time
    when a table can grow (its world-major multi-step run would overflow)."""
    W = 8
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED, backend="cpu", num_workers=2)
    ref = el.RefEcsOps(W)
    sim.step(40)
    ref.step(40)
    _compare_all(sim, ref, "after step(40)", exact_ids=True)
    assert _capacity(sim, el.ARCH_SPAWN) >= 8 * DECLARED
    _check_export(sim, "cpu step(40)")


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("mode", ["one_call", "async_burst"])
def test_growth_gpu_without_host_sync_per_step(mode):
    """SURVEY §8 a2 (reference Table::addRow grows inside the step loop):
    the table grows 8x inside one mw_step(40) call, and inside a burst of 40
    mw_step_async calls closed by one sync -- no table-full flag, every
    world bit-exact with the reference ECS afterwards."""
    W = 64
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED)
    ref = el.RefEcsOps(W)
    if mode == "one_call":
        sim.step(40)
    else:
        for _ in range(40):
            sim.exec.step_async(1)
        sim.exec.sync()
    ref.step(40)
    _compare_all(sim, ref, f"{mode} after 40 steps")
    assert _capacity(sim, el.ARCH_SPAWN) >= 8 * DECLARED
    _check_export(sim, mode)


@pytest.mark.gpu
@needs_ref
def test_growth_gpu_export_pointer_stable_and_filled():
    """the export buffer of a growing table keeps its address
    (a reserved range extended in place) and, on the step a growth follows,
    holds that step's packed rows -- never uninitialised memory."""
    W = 32
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED)
    ref = el.RefEcsOps(W)
    ptr0 = _check_export(sim, "initial")
    caps = []
    for s in range(30):
        sim.step()
        ref.step()
        _compare_all(sim, ref, f"step {s}")
        assert _check_export(sim, f"step {s}") == ptr0, f"step {s}: export moved"
        caps.append(_capacity(sim, el.ARCH_SPAWN))
    assert caps[-1] >= 8 * DECLARED and len(set(caps)) >= 2, caps


@pytest.mark.gpu
@needs_ref
def test_growth_gpu_export_relocated_without_vmm(monkeypatch):
    """MADRONA_MW_EXPORT_VMM=0: a growth moves the export to a new buffer with
    the rows copied over; the pointer fetched again reads the right rows."""
    monkeypatch.setenv("MADRONA_MW_EXPORT_VMM", "0")
    W = 16
    sim = el.EcsOpsSim(W, grow_spawns=True, default_capacity=DECLARED)
    ref = el.RefEcsOps(W)
    for s in range(12):
        sim.step()
        ref.step()
        _compare_all(sim, ref, f"step {s}")
        _check_export(sim, f"step {s}")
