"""AddressSanitizer + UBSan over the host code (SURVEY.md §5 race / failure
detection): the CPU back end (gpu-ecs-madrona_amd/build_cpu_asan/
libmadrona_cpu.so, `make cpu_asan`) and the oracle restatement
(oracle/_build_asan/liborc.so, `make -C oracle asan`) run a slice of the
parity suite in a child process with the sanitizer runtimes preloaded; any
report (heap overflow, use after free, undefined behaviour) fails the child.
GPU sanitizers are not available on this pool, so device code is covered by
the kernels' index guards and the launch checks instead."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CPU_ASAN = os.path.join(ROOT, "gpu-ecs-madrona_amd", "build_cpu_asan", "libmadrona_cpu.so")
ORC_ASAN = os.path.join(ROOT, "oracle", "_build_asan", "liborc.so")

CHILD = r"""
import importlib, sys
import madrona_mi355x as mw
mw.DEFAULT_BACKEND = "cpu"
cases = [
    ("test_collisions_gpu", "test_collisions_bit_exact_vs_oracle_small", {}),
    ("test_collisions_gpu", "test_collisions_bit_exact_ragged_worlds_one_substep", {}),
    ("test_joints_gpu", "test_many_joints_take_the_global_record_path", {}),
    ("test_fvs_gpu", "test_fvs_every_tick_around_first_deaths", {}),
    ("test_jobs_gpu", "test_collisions_jobs_matches_oracle_every_tick", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_every_step_matches_reference", {}),
    ("test_ecs_ops_gpu", "test_ecs_ops_tmp_alloc_chains_past_the_arena", {}),
    ("test_cross_rows_cpu", "test_cross_rows_cpu_backend_matches_reference_every_step",
     {"per_node_serial": True}),
]
for mod, name, kw in cases:
    getattr(importlib.import_module(mod), name)(**kw)
    print("ok", mod, name, flush=True)
"""


def _runtime(name):
    r = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(not (os.path.exists(CPU_ASAN) and os.path.exists(ORC_ASAN)),
                    reason="sanitizer builds absent (make -C gpu-ecs-madrona_amd cpu_asan; "
                           "make -C oracle asan)")
def test_cpu_backend_and_oracle_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not found")
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": f"{asan}:{ubsan}",
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=23",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "MADRONA_MW_NO_TORCH": "1",
        "MADRONA_MW_LIB": CPU_ASAN,          # no HIP library in this process
        "MADRONA_MW_CPU_LIB": CPU_ASAN,
        "MADRONA_MW_BACKEND": "cpu",
        "MADRONA_ORC_LIB": ORC_ASAN,
        "PYTHONPATH": os.pathsep.join([HERE, os.path.join(ROOT, "gpu-ecs-madrona_amd")]),
    })
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=900, cwd=HERE)
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, report
    assert r.stdout.count("ok ") == 8, report
