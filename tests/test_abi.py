"""The drop-in boundary: libkolm_hip.so loads and exports exactly what include/kolm.h
declares; the ctypes layer binds every symbol; no compute call is made here (CPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from kolm import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "kolm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kolm_[a-z0-9_]+)\s*\(", src)))


def test_header_parses():
    fns = declared_functions()
    assert "kolm_encode_blocks" in fns and "kolm_bbwt_forward" in fns and len(fns) >= 15


def test_library_exports_header_symbols():
    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (kolm_[a-z0-9_]+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert hasattr(lib, f)


def test_ctypes_signatures_cover_header():
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared_functions()) == bound


def test_stats_struct_size_matches_header(tmp_path):
    # kolm_stats: 2 u32 + 4 u64 + 5 double + KOLM_NKT(12) x {double, u64, u64} + double + 5 u64
    nkt = int(re.search(r"#define KOLM_NKT (\d+)", open(HEADER).read()).group(1))
    assert nkt == len(_lib.KT_NAMES) == 12
    assert ctypes.sizeof(_lib.Stats) == 8 + 4 * 8 + 5 * 8 + nkt * 24 + 8 + 5 * 8
    # the C compiler's layout of the header struct: size and every field offset
    src = tmp_path / "sz.c"
    fields = [f for f, _ in _lib.Stats._fields_]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "kolm.h"\nint main(void){printf("%zu'
                   + "".join(" %zu" for _ in fields) + '\\n", sizeof(kolm_stats)'
                   + "".join(f", offsetof(kolm_stats, {f})" for f in fields) + ");return 0;}\n")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got[0] == ctypes.sizeof(_lib.Stats)
    assert got[1:] == [getattr(_lib.Stats, f).offset for f in fields]


def test_candidate_constants_match_header():
    src = open(HEADER).read()
    val = lambda name: int(re.search(rf"#define {name} (0x[0-9A-Fa-f]+|\d+)", src).group(1), 0)  # noqa: E731
    assert val("KOLM_NCAND") == _lib.KOLM_NCAND == 11
    assert val("KOLM_FULL_MASK") == _lib.KOLM_FULL_MASK == 0x7FF
    assert val("KOLM_DEFAULT_MASK") == _lib.KOLM_DEFAULT_MASK
    assert val("KOLM_HOTPATH_MASK") == _lib.KOLM_HOTPATH_MASK


def test_gpu_entry_fails_loudly_without_device():
    if _lib.device_count() > 0:
        pytest.skip("a HIP device is visible")
    import kolm
    with pytest.raises(_lib.KolmUnavailable):
        kolm.bbwt_forward(b"banana")
    with pytest.raises(_lib.KolmUnavailable):
        kolm.compress_blocks_fixed(b"abc", 2)


def test_error_codes_without_init():
    lib = _lib.load()
    if _lib._inited_device is not None:
        pytest.skip("default context already initialised")
    assert lib.kolm_bbwt_forward(b"ab", 2, ctypes.create_string_buffer(2)) == -5  # KOLM_ENOINIT
    assert lib.kolm_ctx_destroy(None) == -1
