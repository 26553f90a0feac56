"""Exactness at benchmark scale.

* The benchmarked stream itself — bench.py's rank-0 input, 256 x 1 MiB blocks of
  enwik-style text — encoded in ONE batched call, every field of every block against the
  oracle's per-block answers (tests/golden/bench_stream.json, make_golden_bench.py): the
  sizes of candidates 0..9, the MDL winner over ids 0..8 (the hot path) and over 0..9
  (PY's full list, PY:2350-2369), the winners' sha256, and the LZ77 stream's sha256
  (PY:1711-1763) of every block — so a different-but-valid LZ77 parse or a size that
  flips the argmin is caught on every block, not only block 0.
* BASELINE config 5 at its stated shape: the whole mixed corpus in 1 MiB fixed blocks
  (3 blocks, a short tail), per-block selection, the containers for ids 0..8 and 0..9,
  decoded back; and config 2 (the gradient 1 MiB block).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from kolm import datagen as D

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _bench_golden():
    with open(os.path.join(GOLDEN, "bench_stream.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def bench_rank0():
    g = _bench_golden()["ranks"]["0"]
    data = D.enwik_like(g["bytes"], seed=g["seed"])
    assert sha(data) == g["input_sha256"]
    return g, data


def _mismatches(g, sizes, method, payloads, ncand, wkey, shakey):
    bad = []
    for i, rec in enumerate(g["blocks"]):
        want_sz = rec["sizes"][:ncand]
        if list(map(int, sizes[i][:ncand])) != want_sz:
            bad.append((i, "sizes", list(map(int, sizes[i][:ncand])), want_sz))
            continue
        if int(method[i]) != rec[wkey]:
            bad.append((i, "winner", int(method[i]), rec[wkey]))
            continue
        want_sha = rec.get(shakey, rec["sha9"])
        if sha(payloads[i]) != want_sha:
            bad.append((i, "payload sha256"))
    return bad


def test_bench_stream_hot_path(kolm_gpu, bench_rank0):
    """The bench's own workload (ids 0..8 + MDL, 256 x 1 MiB) block by block."""
    from kolm import _lib
    g, data = bench_rank0
    bs = g["block_size"]
    sizes, method, payloads, st = _lib.encode_blocks(data, bs, cand_mask=_lib.KOLM_HOTPATH_MASK)
    assert len(payloads) == len(g["blocks"]) == 256
    bad = _mismatches(g, sizes, method, payloads, 9, "w9", "sha9")
    assert not bad, bad[:8]


def test_bench_stream_lz77_every_block(kolm_gpu, bench_rank0):
    """The LZ77 stream of every block of the bench stream (forced id 7), whatever wins."""
    from kolm import _lib
    g, data = bench_rank0
    nb = len(g["blocks"])
    _, method, payloads, st = _lib.encode_blocks(data, g["block_size"], cand_mask=1 << 7, force=[7] * nb)
    bad = [i for i in range(nb) if sha(payloads[i]) != g["blocks"][i]["lz"]]
    assert not bad, bad[:16]


def test_bench_stream_full_candidates(kolm_gpu, bench_rank0):
    """PY's full candidate list (ids 0..9, Re-Pair on the device) on the bench stream."""
    from kolm import _lib
    g, data = bench_rank0
    sizes, method, payloads, st = _lib.encode_blocks(data, g["block_size"], cand_mask=_lib.KOLM_DEFAULT_MASK)
    bad = _mismatches(g, sizes, method, payloads, 10, "w10", "sha10")
    assert not bad, bad[:8]


def _mixed_golden():
    with open(os.path.join(GOLDEN, "mixed_corpus.json")) as f:
        return json.load(f)


CASES = {"mixed_corpus": D.mixed_corpus, "gradient_1m": lambda: D.gradient_bmp()[: 1 << 20]}


@pytest.mark.parametrize("case", sorted(CASES))
def test_config_shapes(kolm_gpu, case):
    """config 5 (mixed corpus, 1 MiB blocks, short tail) and config 2 (gradient 1 MiB):
    per-block sizes / winners / payloads and both containers, then decompress."""
    from kolm import _lib
    g = _mixed_golden()[case]
    data = CASES[case]()
    assert sha(data) == g["input"]["sha256"]
    bs = g["block_size"]
    for mask, wkey, shakey, ncand in ((_lib.KOLM_HOTPATH_MASK, "w9", "sha9", 9),
                                      (_lib.KOLM_DEFAULT_MASK, "w10", "sha10", 10)):
        sizes, method, payloads, _ = _lib.encode_blocks(data, bs, cand_mask=mask)
        bad = _mismatches(g, sizes, method, payloads, ncand, wkey, shakey)
        assert not bad, (mask, bad)
    c9 = kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True)
    assert (len(c9), sha(c9)) == (g["container_ids0_8"]["len"], g["container_ids0_8"]["sha256"])
    c10 = kolm_gpu.compress_blocks_fixed(data, bs)
    assert (len(c10), sha(c10)) == (g["container_full"]["len"], g["container_full"]["sha256"])
    assert kolm_gpu.decompress(c9) == data
    assert kolm_gpu.decompress(c10) == data
    if case == "mixed_corpus":  # per-block model selection is exercised: winners differ
        assert len({r["w9"] for r in g["blocks"]}) > 1
