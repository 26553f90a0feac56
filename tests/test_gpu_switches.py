"""The measured-and-kept round-5 forms of the cyclic sort and the MTF stage have A/B switches that
restore the previous form.  Both sides of every switch must stay exact: each case
runs the hot-path candidates with the switch off and compares every block's sizes and winner
payload with the oracle (PY:351-423 BBWT order, PY:460 MTF, PY:1413 Rice, PY:2350-2369 MDL).

  KOLM_LSD_REC=0    LSD passes exchange (key, position) in two u32 arrays instead of u64 records
  KOLM_R0_PART=0    round 0's padding bits stay zero (no partial next character)
  KOLM_R0_PART=2    only the top 2 bits of the next character
  KOLM_LSD_PACK=0   no packed first-half pass;  KOLM_LSD_SCAN2=0: per-block LSD scans
  KOLM_MTF_CP=0     one-workgroup-per-block MTF compose
  KOLM_DUVAL_GRP=0  Duval span merges a thread per merge (a wave from level 4096)
  KOLM_MTF_WAVE=0   the per-thread MTF replay (and its SWAR Rice sums) on batches of few blocks,
                    with chunks of 128..512 bytes and ragged block ends
  KOLM_EARLY_GATHER=0/1/2  one BBWT gather after the rounds / the early gather on the third stream
                    from doubling round 1 / 2 on, the slots of that round's segments again after them
"""
import pytest

import oracle as O
from kolm import _lib
from kolm import datagen as D

pytestmark = pytest.mark.gpu

SWITCHES = [
    {"KOLM_LSD_REC": "0"},
    {"KOLM_R0_PART": "0"},
    {"KOLM_R0_PART": "2"},
    {"KOLM_LSD_PACK": "0", "KOLM_LSD_SCAN2": "0"},
    {"KOLM_MTF_CP": "0"},
    {"KOLM_DUVAL_GRP": "0"},
    {"KOLM_MTF_WAVE": "0"},
    {"KOLM_EARLY_GATHER": "0"},
    {"KOLM_EARLY_GATHER": "1"},
    {"KOLM_EARLY_GATHER": "2"},
]


def _inputs():
    text = D.enwik_like(5 * 65536 + 333, seed=57)
    rnd = D.splitmix64_bytes(65536, seed=9)
    per = (b"abcab" * 20000)[:60000]
    return [
        ("text_64k", text, 65536),
        ("mixed_16k", text[:30000] + rnd[:9000] + bytes(5000) + per[:7000], 16384),
        ("gradient_128k", D.gradient_bmp()[: 1 << 17], 1 << 17),
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
