"""The RCCL reassembly path on the box's one GPU: a world-1 ``nccl`` process group (RCCL),
the payload arenas, method ids and offsets gathered straight from HBM — both through the
library entry compress_blocks_fixed_distributed and through bench.py's double-buffered
async form (gather_payloads(async_op=True) while the next batch encodes).  The containers
must equal the oracle's (PY:2350-2369 per-block MDL, PY:2375-2445 container).  RCCL does
not allow two ranks on one device, so world 1 is what one GPU can run; world > 1 is
covered by the gloo tests (same code, host tensors)."""
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


def _worker(port, cases, q):
    import sys
    import numpy as np
    import torch
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "kolmogorovlike-datacompressor_amd")]
    from kolm import _lib
    from kolm.parallel import assemble_container, compress_blocks_fixed_distributed, gather_payloads
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out = {"backend": dist.get_backend()}
    try:
        for name, data, bs, partition in cases:
            out[name] = compress_blocks_fixed_distributed(data, bs, partition=partition)
        # bench.py's form: two device arenas, the gather of batch k in flight (async, on
        # RCCL's stream) while batch k + 1 encodes into the other arena
        name, data, bs, _ = cases[0]
        n = len(data)
        d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        d_in[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        torch.cuda.synchronize()
        ctx = _lib.device_ctx(0)
        cap = _lib.arena_capacity(n, (n + bs - 1) // bs, _lib.KOLM_DEFAULT_MASK)
        arenas = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(2)]
        pend, got = [None, None], []
        for k in range(4):
            j = k % 2
            if pend[j] is not None:
                got.append(pend[j].result())
                pend[j] = None
            _, method, off, _ = _lib.encode_blocks_device(ctx, d_in.data_ptr(), n, bs, arenas[j].data_ptr(), cap)
            ids = torch.from_numpy(method.astype(np.int32)).cuda()
            offs = torch.from_numpy(off.astype(np.int64)).cuda()
            pend[j] = gather_payloads(arenas[j], int(off[-1]), ids, dst=0, async_op=True, offsets=offs)
        got += [p.result() for p in pend if p is not None]
        out["async"] = [assemble_container(bs, n, [i.cpu().tolist() for i in ids_l],
                                           [p.cpu().numpy().tobytes() for p in pays_l],
                                           [o.cpu().tolist() for o in offs_l])
                        for pays_l, ids_l, offs_l in got]
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_rccl_world1_reassembly_matches_oracle():
    import oracle as O
    from kolm import datagen as D
    bs = 65536
    mixed = D.enwik_like(5 * bs) + bytes(bs) + D.splitmix64_bytes(bs + 777)
    cases = [("mixed_rr", mixed, bs, "round_robin"), ("mixed_contig", mixed, bs, "contiguous"),
             ("text_rr", D.enwik_like(300000, seed=11), 65536, "round_robin"),
             ("one_short", b"abracadabra" * 3, 4096, "round_robin")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), cases, q))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert got["backend"] == "nccl"
    for name, data, bs, _ in cases:
        assert got[name] == O.compress_blocks_fixed(data, bs, range(10)), name
    want = O.compress_blocks_fixed(cases[0][1], cases[0][2], range(10))
    assert len(got["async"]) == 4 and all(c == want for c in got["async"])
