"""Both forms of the cyclic sort's round 0 against the oracle (PY:351-423 BBWT order):
KOLM_R0_MSD=1 — MSD radix partitions of (key, position) by key byte + LDS bucket sorts
(csrc/k_r0m.hip) — and KOLM_R0_MSD=0 — eight stable LSD passes (csrc/k_lsd.hip).  The inputs
cover every path of the MSD form: text whose buckets finish after one, two or more key
bytes (LDS sorts of all four size classes), random bytes (8-bit codes: the first level's
buckets must be <= 256 to fit the index bits), tie groups longer than the LDS classes
(zeros, short periods: key bits exhausted), singletons, ragged and one-byte blocks, and
bit-plane-like binary data (1-bit codes, 32 characters)."""
import numpy as np
import pytest

import oracle as O
from kolm import _lib
from kolm import datagen as D

pytestmark = pytest.mark.gpu


def _inputs():
    text = D.enwik_like(3 * 65536 + 777, seed=41)
    rnd = D.splitmix64_bytes(2 * 65536, seed=5)
    per = (b"abcab" * 30000)[:100000]
    bits = bytes(np.random.default_rng(3).integers(0, 2, 70000, dtype=np.uint8))
    return [
        ("text_64k", text, 65536),
        ("random_64k", rnd, 65536),
        ("zeros_period", bytes(40000) + per, 65536),
        ("mixed_small_blocks", text[:20000] + rnd[:5000] + bytes(3000), 4096),
        ("bits", bits, 32768),
        ("two_symbols", bytes(np.random.default_rng(4).choice([97, 98], 50000).astype(np.uint8)), 50000),
        ("tiny", b"b" + b"a" * 9 + b"xyz", 5),
        ("one_byte_blocks", b"hello world", 1),
    ]


@pytest.mark.parametrize("mode", ["1", "0"])
@pytest.mark.parametrize("case", range(8))
def test_round0_forms_match_oracle(kolm_gpu, monkeypatch, mode, case):
    name, data, bs = _inputs()[case]
    monkeypatch.setenv("KOLM_R0_MSD", mode)
    sizes, method, pays, _ = _lib.encode_blocks(data, bs, _lib.KOLM_HOTPATH_MASK)
    for i in range(len(method)):
        blk = data[i * bs:(i + 1) * bs]
        for m in (2, 3, 4, 5, 6):  # the BBWT family: BBWT -> MTF -> map -> Rice
            assert int(sizes[i][m]) == len(O.candidate(m, blk)), (name, i, m)
        assert pays[i] == O.candidate(int(method[i]), blk), (name, i)
    assert kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True) == O.compress_blocks_fixed(data, bs, range(9))


@pytest.mark.parametrize("mode", ["1", "0"])
def test_round0_forms_bbwt_1mib(kolm_gpu, monkeypatch, mode):
    """1 MiB blocks (the bench's block size): LDS classes up to 8192 elements, three or more
    MSD levels for the long common prefixes of the text's frequent words."""
    monkeypatch.setenv("KOLM_R0_MSD", mode)
    data = D.enwik_like(1 << 20, seed=77)
    assert _lib.bbwt_forward(data) == O.bbwt_forward(data)
    grad = D.gradient_bmp()[: 1 << 20]
    assert _lib.bbwt_forward(grad) == O.bbwt_forward(grad)
