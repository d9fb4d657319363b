"""The C-ABI library loads and exports every symbol include/el_gpu.h declares (no compute:
there is no GPU here); without a device every entry point fails loudly (EL_EHIP)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "el_gpu.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void\*?|const char\*)\s*(el_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build_lib()
    from distel_amd import engine
    return engine.load_library()


def test_header_declares_expected(lib):
    from distel_amd import engine
    assert _declared() == sorted(engine.EXPORTED_SYMBOLS)


def test_exports_every_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "distel_amd", "lib", "libel_gpu.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (el_\w+)$", out, re.M))
    for sym in _declared():
        assert sym in exported, sym
        assert getattr(lib, sym) is not None


def test_abi_version(lib):
    from distel_amd import engine
    assert lib.el_abi_version() == engine.ABI_VERSION == 8


def test_config_struct_layout():
    """The ctypes mirror of el_config matches the C layout (offset of every field)."""
    import ctypes as C
    from distel_amd import engine
    src = '#include <stddef.h>\n#include <stdio.h>\n#include "el_gpu.h"\nint main(void){printf("%zu %zu %zu %zu\\n",' \
          'offsetof(el_config, exchange), offsetof(el_config, group), offsetof(el_config, rccl_id), sizeof(el_config));}'
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "t.c"), "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(d, "t"), os.path.join(d, "t.c")],
                       check=True)
        got = list(map(int, subprocess.run([os.path.join(d, "t")], capture_output=True, text=True).stdout.split()))
    T = engine._ElConfig
    assert got == [T.exchange.offset, T.group.offset, T.rccl_id.offset, C.sizeof(T)]


def test_partition_config_validation(lib):
    """Bad partition configs are refused before any device work."""
    import ctypes as C
    from distel_amd import engine
    cfg = engine._ElConfig(0, 0, 0)
    cfg.exchange, cfg.part_rank, cfg.part_count = engine.XCHG_LOCAL, 0, 2  # LOCAL without a group
    ctx = C.c_void_p()
    assert lib.el_create(C.byref(ctx), C.byref(cfg)) == engine.EL_EINVAL
    cfg.exchange, cfg.part_rank, cfg.part_count = 7, 0, 1
    assert lib.el_create(C.byref(ctx), C.byref(cfg)) == engine.EL_EINVAL
    g = engine.LocalGroup(2)
    cfg.exchange, cfg.part_rank, cfg.part_count, cfg.group = engine.XCHG_LOCAL, 2, 2, g.ptr  # rank out of range
    assert lib.el_create(C.byref(ctx), C.byref(cfg)) == engine.EL_EINVAL
    g.close()


def test_no_device_fails_loudly(lib):
    from distel_amd import engine
    if engine.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(engine.ElError) as e:
        engine.Engine(device=0)
    assert e.value.code == engine.EL_EHIP


def test_null_arguments(lib):
    assert lib.el_create(None, None) == -1
    assert lib.el_init(None) == -1
    assert lib.el_saturate(None, None) == -1
    lib.el_destroy(None)


def test_no_oracle_in_product():
    """The product package never imports or links the CPU oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "distel_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dirpath, f), encoding="utf-8").read()
                for bad in ('#include "el_oracle', "libel_oracle", "import oracle", "from oracle"):
                    assert bad not in src, (f, bad)


def test_stream_run_decode():
    """The streamed result's row-run encoding (el_stream: values + (x, end) runs) decodes to the
    per-entry rows; a run table that does not end at the entry count is refused."""
    import numpy as np
    from distel_amd import engine
    s = engine.Stream()
    s.s_b = np.array([5, 7, 9, 1, 2, 3, 4], np.uint32)
    s.s_run = np.array([[10, 2], [11, 3], [10, 7]], np.uint32)  # x = 10, 10, 11, 10, 10, 10, 10
    s.n_facts, s.n_s_runs = 7, 3
    x, b = s.fact_rows()
    assert x.tolist() == [10, 10, 11, 10, 10, 10, 10] and b.tolist() == [5, 7, 9, 1, 2, 3, 4]
    fx, fb = s.facts()
    assert fx.tolist() == [10] * 6 + [11] and fb.tolist() == [1, 2, 3, 4, 5, 7, 9]
    s.s_run = np.array([[10, 2], [11, 6]], np.uint32)
    s.n_s_runs = 2
    with pytest.raises(ValueError):
        s.fact_rows()
    empty = engine.Stream()
    empty.s_b, empty.s_run = np.zeros(0, np.uint32), np.zeros((0, 2), np.uint32)
    x, b = empty.fact_rows()
    assert len(x) == 0 and len(b) == 0
