"""The cyclic sort's round 0 (stable LSD passes over the packed codes of the first C rotation
characters, csrc/k_lsd.hip) against the oracle (PY:351-423 BBWT order) on inputs that reach
each of its forms: text (6-bit codes, C = 10: record passes, the packed first-half pass, the
partial next character), random bytes (8-bit codes, C = 8), tie groups longer than a tile
(zeros, short periods), singletons, ragged and one-byte blocks, bit-plane-like binary data
(1-bit codes, 32 characters: four passes, no second half) and two symbols.  (Round 5's MSD
form of round 0 measured slower and was removed in round 6.)"""
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


@pytest.mark.parametrize("case", range(8))
def test_round0_matches_oracle(kolm_gpu, case):
    name, data, bs = _inputs()[case]
    sizes, method, pays, _ = _lib.encode_blocks(data, bs, _lib.KOLM_HOTPATH_MASK)
    for i in range(len(method)):
        blk = data[i * bs:(i + 1) * bs]
        for m in (2, 3, 4, 5, 6):  # the BBWT family: BBWT -> MTF -> map -> Rice
            assert int(sizes[i][m]) == len(O.candidate(m, blk)), (name, i, m)
        assert pays[i] == O.candidate(int(method[i]), blk), (name, i)
    assert kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True) == O.compress_blocks_fixed(data, bs, range(9))


def test_round0_bbwt_1mib(kolm_gpu):
    """1 MiB blocks (the bench's block size): 256 LSD tiles per block, position windows for RK."""
    data = D.enwik_like(1 << 20, seed=77)
    assert _lib.bbwt_forward(data) == O.bbwt_forward(data)
    grad = D.gradient_bmp()[: 1 << 20]
    assert _lib.bbwt_forward(grad) == O.bbwt_forward(grad)
