"""CPU checks of the drop-in boundary (no GPU work): the C-ABI library loads,
exports every function include/madrona_mw.h declares, its structs have the
layout the header gives a C compiler, the host-side init generator matches
the oracle bit for bit, and the Python surface refuses to run without the
native library (no silent CPU fallback)."""
import ctypes
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "madrona_mw.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mw_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    names = _declared_functions()
    assert "mw_create" in names and "mw_step" in names and "mw_get_exported" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    import madrona_mi355x as mw
    lib = ctypes.CDLL(mw.LIB_PATH)
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python wrapper binds exactly the header's functions
    assert sorted(mw.C_ABI_SYMBOLS) == _declared_functions()


def test_exported_symbols_are_unmangled_c():
    import madrona_mi355x as mw
    for path in (mw.LIB_PATH, mw.CPU_LIB_PATH):
        out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True,
                             text=True, check=True).stdout
        exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
        for n in _declared_functions():
            assert n in exported, (path, n)


def test_cpu_library_exports_every_declared_symbol_without_hip():
    # the CPU back end is the same ABI with no HIP / RCCL dependency
    import madrona_mi355x as mw
    lib = mw.cpu_library()
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    deps = subprocess.run(["readelf", "-d", mw.CPU_LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    assert "amdhip" not in deps and "rccl" not in deps, deps


def test_struct_layout_matches_header(tmp_path):
    import madrona_mi355x as mw
    prog = tmp_path / "layout.c"
    prog.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <stddef.h>
        #include "madrona_mw.h"
        int main(void) {
            printf("%zu %zu %zu\\n", sizeof(mw_config), sizeof(mw_collisions_config),
                   sizeof(mw_collisions_init));
            printf("%zu %zu %zu %zu\\n", offsetof(mw_collisions_config, max_contacts),
                   offsetof(mw_collisions_config, mu_d), offsetof(mw_config, use_graph),
                   offsetof(mw_collisions_config, hull_paths));
            return 0;
        }
    """))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(prog), "-o",
                    str(exe)], check=True)
    sizes, offs = subprocess.run([str(exe)], capture_output=True, text=True,
                                 check=True).stdout.split("\n")[:2]
    assert [int(x) for x in sizes.split()] == [ctypes.sizeof(mw.MwConfig),
                                                ctypes.sizeof(mw.CollisionsConfig),
                                                ctypes.sizeof(mw.CollisionsInit)]
    assert [int(x) for x in offs.split()] == [mw.CollisionsConfig.max_contacts.offset,
                                              mw.CollisionsConfig.mu_d.offset,
                                              mw.MwConfig.use_graph.offset,
                                              mw.CollisionsConfig.hull_paths.offset]


def test_init_generator_matches_oracle_including_shard_offsets():
    # mw_gen_collisions_inits is host code in the product library; the
    # oracle restates examples/collisions/collisions.cpp:20-80.
    import madrona_mi355x as mw
    from oracle_lib import gen_collisions_inits
    pos, rot = gen_collisions_inits(7, 16, seed=0)
    p2, r2 = mw.gen_collisions_inits(3, 16, seed=0, first_world=4)
    assert p2.tobytes() == pos[4:7].tobytes()
    assert r2.tobytes() == rot[4:7].tobytes()


def test_missing_native_library_fails_loudly():
    code = "import madrona_mi355x"
    env = dict(os.environ, MADRONA_MW_LIB="/nonexistent/libmadrona_mw.so")
    env["PYTHONPATH"] = os.path.join(ROOT, "gpu-ecs-madrona_amd")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    assert r.returncode != 0
    assert "libmadrona_mw.so" in r.stderr
