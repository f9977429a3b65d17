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


def test_mw_config_size_and_version_are_checked():
    # a caller compiled against another mw_config layout is
    # refused with a message instead of being misread (CPU library: no GPU)
    import madrona_mi355x as mw
    lib = mw.cpu_library()
    ccfg = mw.default_collisions_config(4, 1, 64, 64)
    pos, rot = mw.gen_collisions_inits(1, 4, seed=0)
    inits = (mw.CollisionsInit * 1)(mw.CollisionsInit(pos[0].ctypes.data, rot[0].ctypes.data))

    def create(size, version):
        cfg = mw.MwConfig(size, version, 1, 0, 0, 1, 0, 0, 1, 0, 0)
        return lib.mw_create(b"collisions", ctypes.byref(cfg), ctypes.byref(ccfg),
                             ctypes.sizeof(ccfg), ctypes.cast(inits, ctypes.c_void_p),
                             ctypes.sizeof(mw.CollisionsInit))

    for size, version in ((ctypes.sizeof(mw.MwConfig) - 8, mw.MW_ABI_VERSION),
                          (ctypes.sizeof(mw.MwConfig), mw.MW_ABI_VERSION + 1),
                          (1, 0)):   # a pre-round-5 struct: num_worlds where struct_size is
        assert not create(size, version)
        assert b"struct_size" in lib.mw_last_error()
    h = create(ctypes.sizeof(mw.MwConfig), mw.MW_ABI_VERSION)
    assert h, lib.mw_last_error()
    assert lib.mw_step(h, 1) == 0
    lib.mw_destroy(h)
    # the environment's own config is checked through user_cfg_bytes
    cfg = mw.MwConfig(ctypes.sizeof(mw.MwConfig), mw.MW_ABI_VERSION, 1, 0, 0, 1, 0, 0, 1, 0, 0)
    assert not lib.mw_create(b"collisions", ctypes.byref(cfg), ctypes.byref(ccfg),
                             ctypes.sizeof(ccfg) - 4, ctypes.cast(inits, ctypes.c_void_p),
                             ctypes.sizeof(mw.CollisionsInit))
    assert b"user config" in lib.mw_last_error()


def test_c_caller_with_mw_config_init(tmp_path):
    # the header's initialiser from C, against the CPU library
    import madrona_mi355x as mw
    prog = tmp_path / "cfg.c"
    prog.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include "madrona_mw.h"
        int main(void) {
            mw_config c = MW_CONFIG_INIT;
            c.num_worlds = 2; c.use_graph = 1; c.num_workers = 1;
            mw_collisions_config cc = { .num_cubes = 8, .num_substeps = 1, .delta_t = 1.f / 60.f,
                .gravity_z = -9.8f, .max_contacts = 256, .max_candidates = 256,
                .cube_inv_mass = 1.f, .cube_inv_inertia = 0.375f, .mu_s = 0.5f, .mu_d = 0.5f };
            static float pos[2 * 8 * 3], rot[2 * 8 * 4];
            mw_gen_collisions_inits(0, 2, 8, 0, pos, rot);
            mw_collisions_init in[2] = { { pos, rot }, { pos + 24, rot + 32 } };
            mw_exec *e = mw_create("collisions", &c, &cc, sizeof(cc), in, sizeof(in[0]));
            if (!e) { printf("ERR %s\\n", mw_last_error()); return 1; }
            if (mw_step(e, 3)) { printf("ERR %s\\n", mw_last_error()); return 1; }
            printf("OK %d\\n", mw_num_worlds(e));
            return mw_destroy(e);
        }
    """))
    exe = tmp_path / "cfg"
    libdir = os.path.dirname(mw.CPU_LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(prog), "-o",
                    str(exe), "-L", libdir, "-lmadrona_cpu", "-Wl,-rpath," + libdir], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "OK 2", (out.stdout, out.stderr)
