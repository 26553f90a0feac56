"""Distributed compress with real GPU encoding: 2 ranks share the box's one GPU (RCCL
needs one GPU per rank, so the shards travel through the gloo test transport here), each
encodes its block shard through the C ABI into a device arena, rank 0 reassembles with
the product's kolm.parallel.compress_blocks_fixed_distributed; the container must equal
the oracle's."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, data, bs, q, partition):
    import sys
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "kolmogorovlike-datacompressor_amd"), os.path.join(repo, "tests")]
    from gloo_transport import GlooTransport
    from kolm import _lib
    from kolm.parallel import compress_blocks_fixed_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = GlooTransport(0, _lib.device_ctx(0))
        out = compress_blocks_fixed_distributed(data, bs, comm=comm, partition=partition)
        if rank == 0:
            q.put(out)
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("partition", ["contiguous", "round_robin"])
def test_distributed_gpu_encode_matches_single(partition):
    import oracle as O
    from kolm import datagen as D
    bs = 65536
    data = (D.enwik_like(5 * bs) + bytes(bs) + D.splitmix64_bytes(bs + 777))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, data, bs, q, partition)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == O.compress_blocks_fixed(data, bs, range(10))
