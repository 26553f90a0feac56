"""N>1 path on CPU: world_size-2 gloo process group.  Each rank encodes its contiguous
block shard (here with the oracle standing in for the GPU encoder, which needs a
device), the payload arenas and method ids are gathered with the same
kolm.parallel.gather_payloads used on MI355X (RCCL there), and rank 0's reassembled
container must equal the single-process container."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, data, bs, q, use_async=False, partition="contiguous"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "kolmogorovlike-datacompressor_amd"), os.path.join(repo, "oracle")]
    import oracle as O
    from kolm.parallel import assemble_container, gather_payloads, rank_blocks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nb = (len(data) + bs - 1) // bs
        mids, pays = [], []
        for i in rank_blocks(nb, rank, world, partition):
            blk = data[i * bs:(i + 1) * bs]
            cands = [O.candidate(m, blk) for m in range(10)]
            m = int(np.argmin([len(c) for c in cands]))
            mids.append(m)
            pays.append(cands[m])
        blob = b"".join(pays)
        offs = np.concatenate([[0], np.cumsum([len(p) for p in pays])]).astype(np.int64).tolist()
        mx = torch.tensor([len(blob)], dtype=torch.int64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        arena = torch.zeros(max(int(mx[0]), 1), dtype=torch.uint8)
        if blob:
            arena[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        ids = torch.tensor(mids, dtype=torch.int32)
        if use_async:  # bench.py's double-buffered form: the gather completes at wait()/result()
            got_p, got_i = gather_payloads(arena, len(blob), ids, dst=0, async_op=True).result()
        else:
            got_p, got_i = gather_payloads(arena, len(blob), ids, dst=0)
        all_offs = [None] * world
        dist.all_gather_object(all_offs, offs)
        if rank == 0:
            c = assemble_container(bs, len(data), [i.tolist() for i in got_i],
                                   [p.numpy().tobytes() for p in got_p], all_offs, partition)
            q.put(c)
        else:
            assert got_p is None and got_i is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bs,n,use_async,partition", [
    (2, 4096, 4096 * 5 + 123, False, "contiguous"), (2, 1000, 999, False, "contiguous"),
    (3, 2048, 2048 * 4, False, "contiguous"), (2, 4096, 4096 * 3 + 7, True, "contiguous"),
    (2, 4096, 4096 * 5 + 123, False, "round_robin"), (3, 2048, 2048 * 7 + 5, True, "round_robin")])
def test_gloo_sharded_reassembly(world, bs, n, use_async, partition):
    import oracle as O
    from kolm import datagen as D
    data = (D.enwik_like(n // 2, seed=5) + bytes(n // 4) + D.splitmix64_bytes(n, seed=9))[:n]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, bs, q, use_async, partition))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == O.compress_blocks_fixed(data, bs, range(10))
