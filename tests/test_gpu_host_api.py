"""The host-buffer API (kolm_compress_fixed behind kolm.compress_blocks_fixed): the
multi-batch path (inputs split into several device batches, forced small with
KOLM_BATCH_BYTES), statistics summed over the batches, and concurrent callers on several
threads (the context's result buffer is read under the binding's lock).  Containers are
compared with the oracle's (PY:2332-2445)."""
import os
import threading

import pytest

import oracle as O
from kolm import datagen as D

pytestmark = pytest.mark.gpu


def test_multibatch_container_and_stats(kolm_gpu, monkeypatch):
    bs = 65536
    data = D.enwik_like(5 * bs + 4321, seed=3) + bytes(bs) + D.splitmix64_bytes(bs)
    want = O.compress_blocks_fixed(data, bs, range(9))
    one = kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True)
    st1 = kolm_gpu.last_stats()
    assert one == want
    monkeypatch.setenv("KOLM_BATCH_BYTES", str(2 * bs + 100))  # 2 blocks per batch: 4 batches
    many = kolm_gpu.compress_blocks_fixed(data, bs, hot_path=True)
    st4 = kolm_gpu.last_stats()
    assert many == want
    # statistics of the batches add up: the LZ77 token count is a function of each block
    # alone (the doubling-round sum is not: it counts the rounds of each batch)
    assert st4["lz_tokens"] == st1["lz_tokens"]
    assert kolm_gpu.decompress(many) == data


def test_concurrent_callers(kolm_gpu):
    cases = [(D.enwik_like(200000, seed=s), 32768) for s in range(4)]
    want = [O.compress_blocks_fixed(d, bs, range(9)) for d, bs in cases]
    got = [None] * len(cases)
    errs = []

    def run(i):
        try:
            for _ in range(3):
                got[i] = kolm_gpu.compress_blocks_fixed(cases[i][0], cases[i][1], hot_path=True)
                assert got[i] == want[i]
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    assert got == want
