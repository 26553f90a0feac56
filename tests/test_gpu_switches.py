"""Product forms chosen by batch shape, forced onto inputs they would not otherwise see (DESIGN.md
§9; the switches that selected measured-slower forms were removed in round 6).  Each case runs
the hot-path candidates with the switch set and compares every block's sizes and winner payload
with the oracle (PY:351-423 BBWT order, PY:460 MTF, PY:1413 Rice, PY:2350-2369 MDL).

  KOLM_MTF_WAVE=0   the per-thread MTF replay (and its SWAR Rice sums) on batches of few blocks,
                    with chunks of 128..512 bytes and ragged block ends
  KOLM_MTF_WAVE=1   the position-parallel MTF replay on a batch of 64 blocks or more
  KOLM_PREVC_IDX=1  k_prevc on the index stream below 16 blocks (with 16+ blocks: the early BBWT
                    gather from doubling round 3 on the third stream)
  KOLM_LZ_BIGWIN=0/1  the LZ77 stitch's 5 KiB / 62 KiB brute-force window
  KOLM_LZ_IDX=0     the LZ77 parse's in-LDS window sort (the full-batch form) on batches under 64 blocks
"""
import pytest

import oracle as O
from kolm import _lib
from kolm import datagen as D

pytestmark = pytest.mark.gpu

SWITCHES = [
    {"KOLM_MTF_WAVE": "0"},
    {"KOLM_MTF_WAVE": "1"},
    {"KOLM_PREVC_IDX": "1"},
    {"KOLM_LZ_BIGWIN": "0"},
    {"KOLM_LZ_BIGWIN": "1"},
    {"KOLM_LZ_IDX": "0"},
]


def _inputs():
    text = D.enwik_like(5 * 65536 + 333, seed=57)
    rnd = D.splitmix64_bytes(65536, seed=9)
    per = (b"abcab" * 20000)[:60000]
    return [
        ("text_64k", text, 65536),
        ("mixed_16k", text[:30000] + rnd[:9000] + bytes(5000) + per[:7000], 16384),
        ("gradient_128k", D.gradient_bmp()[: 1 << 17], 1 << 17),
        # 20 blocks of 16 KiB: prevc on the index stream and the early BBWT gather (from 16 blocks)
        ("text_20x16k", D.enwik_like(20 * 16384, seed=58), 16384),
    ]


@pytest.mark.parametrize("sw", range(len(SWITCHES)), ids=lambda i: "+".join(f"{k}={v}" for k, v in SWITCHES[i].items()))
def test_switch_off_matches_oracle(kolm_gpu, monkeypatch, sw):
    for k, v in SWITCHES[sw].items():
        monkeypatch.setenv(k, v)
    for name, data, bs in _inputs():
        sizes, method, pays, _ = _lib.encode_blocks(data, bs, _lib.KOLM_HOTPATH_MASK)
        for i in range(len(method)):
            blk = data[i * bs:(i + 1) * bs]
            for m in (2, 3, 4, 5, 6):  # the BBWT family: BBWT -> MTF -> map -> Rice
                assert int(sizes[i][m]) == len(O.candidate(m, blk)), (name, i, m)
            assert pays[i] == O.candidate(int(method[i]), blk), (name, i)
