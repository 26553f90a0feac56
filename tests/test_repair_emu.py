"""The device Re-Pair's batch logic (kolmogorovlike-datacompressor_amd/csrc/repair_core.h)
checked on the CPU: tools/repair_emu.cpp runs the kernel's phases with 1024 virtual
threads (one barrier = one loop over the threads, optionally in a shuffled order per
phase) and must reproduce the oracle's exact Re-Pair (PY:1817-1911) byte for byte.
This is test infrastructure only; the product runs the same header as a HIP kernel."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import oracle as O
from kolm import datagen as D

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "repair_emu.cpp")


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("emu") / "repair_emu.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", SRC, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.repair_emu.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_void_p, ctypes.c_uint64]
    lib.repair_emu.restype = ctypes.c_int64

    def run(data: bytes, seed: int = 0):
        cap = 4 * len(data) + 64
        buf = ctypes.create_string_buffer(cap)
        res = (ctypes.c_uint32 * 8)()
        r = lib.repair_emu(data, len(data), buf, cap, res, seed)
        assert r >= 0, f"emulated kernel error {-r}"
        return buf.raw[:r], list(res)
    return run


def test_emu_small_random(emu):
    rng = random.Random(7)
    cases = [b"a", b"aa", b"aaa", b"aaaa", b"abab", b"aaaaa" * 3, b"abcabcabc", bytes(100), b"ab" * 50]
    for _ in range(250):
        n = rng.randint(1, 400)
        alpha = rng.choice([1, 2, 3, 4, 16, 256])
        cases.append(bytes(rng.randrange(alpha) for _ in range(n)))
    for i, c in enumerate(cases):
        want = O.repair_fast(c)
        assert emu(c)[0] == want, c[:40]
        if i % 5 == 0:  # thread order inside a phase must not matter
            assert emu(c, seed=1000 + i)[0] == want, c[:40]


def test_emu_golden(emu, golden_kernels, manifest):
    for name in manifest["kernels"]:
        inp = golden_kernels[f"{name}/input"].tobytes()
        if inp:
            assert emu(inp)[0] == golden_kernels[f"{name}/repair"].tobytes(), name


@pytest.mark.parametrize("kind", ["enwik", "gradient", "random", "zeros", "pattern"])
def test_emu_256k(emu, kind):
    n = 1 << 18
    data = {"enwik": lambda: D.enwik_like(n), "gradient": lambda: D.gradient_bmp()[:n],
            "random": lambda: D.splitmix64_bytes(n), "zeros": lambda: bytes(n),
            "pattern": lambda: D.pattern_blocks()[6 * 65536:6 * 65536 + n]}[kind]()
    got, res = emu(data, seed=3)
    assert got == O.repair_fast(data)
    assert res[3] <= res[1]  # batches <= rounds (rules)


@pytest.mark.parametrize("kind", ["random", "gradient", "enwik"])
def test_emu_1m_level_cache(emu, kind):
    """1 MiB blocks: far more than QLIM pairs occur twice (random: ~65536 pairs sharing a few
    top counts), so the level cache rescans with falling thresholds many times."""
    n = 1 << 20
    data = {"enwik": lambda: D.enwik_like(n, seed=5), "gradient": lambda: D.gradient_bmp()[-n:],
            "random": lambda: D.splitmix64_bytes(n, seed=11)}[kind]()
    got, res = emu(data)
    assert got == O.repair_fast(data)
