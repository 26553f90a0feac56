"""Content-defined blocks: FastCDC chunking (PY:140-309) and compress_blocks_cdc
(PY:2213-2326).

CPU: the oracle (oracle/cdc_oracle.cpp + oracle.compress_blocks_cdc) against PY's own
outputs (tests/golden/cdc.npz, made by tests/golden/make_golden_cdc.py).
GPU: the device chunker (k_cdc.hip) and the variable-geometry batch encode against the
same goldens and against the oracle on seeded inputs, bit-exact.
"""
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

import oracle as O
from kolm import datagen as D

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import make_golden_cdc as G  # noqa: E402  (inputs only; the reference is imported by its main())

with open(os.path.join(GOLDEN, "cdc.json")) as _f:
    MAN = json.load(_f)
BNAMES = sorted(MAN["boundaries"])
CNAMES = sorted(MAN["containers"])
_INPUTS = {}


@pytest.fixture(scope="module")
def cdc_npz():
    return np.load(os.path.join(GOLDEN, "cdc.npz"))


def case(name):
    """(data, params, merge) of a boundary case, rebuilt and checked against its hash."""
    if not _INPUTS:
        _INPUTS.update(G.boundary_cases())
    data, params, merge = _INPUTS[name]
    ent = MAN["boundaries"][name]
    assert hashlib.sha256(data).hexdigest() == ent["input"]["sha256"]
    assert list(params) == ent["params"] and merge == ent["merge"]
    return data, params, merge


def golden_bounds(z, name):
    return [(int(a), int(b)) for a, b in z[f"{name}/bounds"].reshape(-1, 2)]


def container_case(z, name):
    ent = MAN["containers"][name]
    return z[f"c_{name}/input"].tobytes(), ent["params"]


# ---------------------------------------------------------------------------- CPU

@pytest.mark.parametrize("name", BNAMES)
def test_oracle_cdc_golden(cdc_npz, name):
    data, (mn, av, mx), merge = case(name)
    assert O.cdc_boundaries(data, mn, av, mx, merge) == golden_bounds(cdc_npz, name)


def test_oracle_cdc_errors():
    with pytest.raises(ValueError, match="Require"):
        O.cdc_boundaries(b"abc", 0, 64, 128)
    with pytest.raises(ValueError, match="Require"):
        O.cdc_boundaries(b"abc", 128, 64, 256)
    with pytest.raises(ValueError, match="too small"):
        O.cdc_boundaries(b"abc", 1, 32, 256)
    assert O.cdc_boundaries(b"", 0, 0, 0) == []  # PY returns before validating


@pytest.mark.parametrize("name", CNAMES)
def test_oracle_cdc_container_golden(cdc_npz, name):
    data, (mn, av, mx) = container_case(cdc_npz, name)
    assert O.compress_blocks_cdc(data, mn, av, mx, ids=range(9)) == cdc_npz[f"c_{name}/ids0_8"].tobytes()
    assert O.compress_blocks_cdc(data, mn, av, mx, ids=range(10)) == cdc_npz[f"c_{name}/full"].tobytes()


def test_cdc_host_decode_golden(cdc_npz):
    import kolm
    for name in CNAMES:
        data, _ = container_case(cdc_npz, name)
        assert kolm.decompress(cdc_npz[f"c_{name}/full"].tobytes(), device=False) == data


# ---------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("name", BNAMES)
def test_gpu_cdc_golden(kolm_gpu, cdc_npz, name):
    data, (mn, av, mx), merge = case(name)
    assert kolm_gpu.cdc_fast_boundaries_strict(data, mn, av, mx, merge) == golden_bounds(cdc_npz, name)


@pytest.mark.gpu
def test_gpu_cdc_errors(kolm_gpu):
    with pytest.raises(ValueError, match="Require"):
        kolm_gpu.cdc_fast_boundaries_strict(b"abc", 0, 64, 128)
    with pytest.raises(ValueError, match="too small"):
        kolm_gpu.cdc_fast_boundaries_strict(b"abc", 1, 32, 256)
    assert kolm_gpu.cdc_fast_boundaries_strict(b"") == []
    from kolm import _lib
    with pytest.raises(_lib.KolmError):  # the C ABI rejects them too
        _lib.cdc_boundaries(b"abcdef", 0, 64, 128)


CDC_PARAMS = [(4096, 8192, 16384), (64, 128, 256), (1, 64, 1024), (3000, 5000, 20000), (1000, 1000, 1000),
              (100, 4096, 100003), (2048, 65536, 1 << 20), (7, 64, 65)]


@pytest.mark.gpu
@pytest.mark.parametrize("params", CDC_PARAMS)
@pytest.mark.parametrize("kind", ["enwik", "random", "zeros", "mixed"])
def test_gpu_cdc_vs_oracle(kolm_gpu, params, kind):
    n = {"enwik": 3_000_017, "random": 1 << 20, "zeros": 777_777, "mixed": 2_500_000}[kind]
    data = {"enwik": lambda: D.enwik_like(n), "random": lambda: D.splitmix64_bytes(n), "zeros": lambda: bytes(n),
            "mixed": lambda: D.mixed_corpus()[:n]}[kind]()
    mn, av, mx = params
    for merge in (True, False):
        assert kolm_gpu.cdc_fast_boundaries_strict(data, mn, av, mx, merge) == O.cdc_boundaries(data, mn, av, mx, merge)


@pytest.mark.gpu
def test_gpu_cdc_large(kolm_gpu):
    """64 MiB: thousands of segments through the speculative chain + stitch."""
    data = D.enwik_like(64 << 20)
    for mn, av, mx in ((4096, 8192, 16384), (5000, 9000, 33333)):
        got = kolm_gpu.cdc_fast_boundaries_strict(data, mn, av, mx)
        assert got == O.cdc_boundaries(data, mn, av, mx)
        assert got[0][0] == 0 and got[-1][1] == len(data)
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CNAMES)
def test_gpu_cdc_container_golden(kolm_gpu, cdc_npz, name):
    data, (mn, av, mx) = container_case(cdc_npz, name)
    got = kolm_gpu.compress_blocks_cdc(data, mn, av, mx)
    assert got == cdc_npz[f"c_{name}/full"].tobytes()  # PY's container, byte for byte
    assert kolm_gpu.decompress(got) == data
    assert kolm_gpu.compress_blocks_cdc(data, mn, av, mx, hot_path=True) == cdc_npz[f"c_{name}/ids0_8"].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_variable_blocks_vs_oracle(kolm_gpu, seed):
    """Arbitrary content-defined partitions (1-byte blocks, odd lengths, one long block)
    through the variable geometry: every candidate size and the winner's payload."""
    from kolm import _lib
    rng = random.Random(seed)
    data = D.enwik_like(30000, seed=seed) + D.splitmix64_bytes(9000, seed=seed) + bytes(7000) + \
        bytes(i & 0xFF for i in range(5000))
    edges = [0]
    while edges[-1] < len(data):
        edges.append(min(len(data), edges[-1] + rng.choice([1, 2, 3, 17, 64, 333, 1000, 2047, 4096, 9000])))
    sizes, method, payloads, _ = _lib.encode_blocks_var(data, edges)
    for i in range(len(edges) - 1):
        blk = data[edges[i]:edges[i + 1]]
        want = [len(O.candidate(m, blk)) for m in range(10)]
        assert list(map(int, sizes[i][:10])) == want, (i, len(blk))
        assert int(method[i]) == int(np.argmin(want))
        assert payloads[i] == O.candidate(int(method[i]), blk)


@pytest.mark.gpu
def test_gpu_compress_cdc_vs_oracle(kolm_gpu):
    data = D.enwik_like(300_000) + D.splitmix64_bytes(100_000) + D.gradient_bmp()[:120_000]
    got = kolm_gpu.compress_blocks_cdc(data, hot_path=True)
    assert got == O.compress_blocks_cdc(data, ids=range(9))
    assert kolm_gpu.decompress(got) == data
