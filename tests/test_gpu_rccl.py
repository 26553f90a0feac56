"""RCCL behind the C ABI on the box's one GPU, with no PyTorch in the process: a world-1
communicator (kolm_comm_init) — both block partitions through
kolm.parallel.compress_blocks_fixed_distributed, the double-buffered asynchronous form
bench.py uses (the gather of batch k on RCCL's stream while batch k + 1 encodes), the
all-reduce / barrier, KOLM_ERCCL on an RCCL error, and kolm_encode_blocks_multi's
ncclCommInitAll reassembly.  Every container must equal the oracle's (PY:2350-2369 per-block
MDL, PY:2375-2445 container).  One device cannot hold two RCCL ranks, so world > 1 is
covered by the gloo tests (same reassembly code) and by the driver's multi-GPU bench."""
import multiprocessing as mpc
import os

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(cases, q):
    import ctypes
    import sys
    sys.path[:0] = [os.path.join(REPO, "kolmogorovlike-datacompressor_amd")]
    import numpy as np
    from kolm import _lib
    from kolm.parallel import Comm, compress_blocks_fixed_distributed, container_from_gathered
    out = {}
    try:
        comm = Comm(1, 0, Comm.unique_id(), 0)
        out["rank"] = (comm.rank, comm.nranks)
        for name, data, bs, partition in cases:
            out[name] = compress_blocks_fixed_distributed(data, bs, comm=comm, partition=partition)
        # bench.py's form: two device arenas, the gather of batch k in flight while batch
        # k + 1 encodes into the other arena; each gather lands in its own destination buffer
        name, data, bs, _ = cases[0]
        n = len(data)
        nb = (n + bs - 1) // bs
        ctx = _lib.device_ctx(0)
        d_in = _lib.input_buffer(ctx, data)
        cap = _lib.arena_capacity(n, nb, _lib.KOLM_DEFAULT_MASK)
        arenas = [_lib.DeviceBuffer(ctx, cap) for _ in range(2)]
        dsts = [_lib.DeviceBuffer(ctx, cap) for _ in range(2)]
        pend, got = [None, None], []
        for k in range(4):
            j = k % 2
            if pend[j] is not None:
                got.append(container_from_gathered(pend[j].result(), bs, n))
                pend[j] = None
            _, method, off, _ = _lib.encode_blocks_device(ctx, d_in.ptr, n, bs, arenas[j].ptr, cap)
            pend[j] = comm.gather_payloads(arenas[j].ptr, int(off[-1]), method, off, dst=0, dst_buf=dsts[j],
                                           async_op=True, dst_cap_blocks=nb)
        for j in range(2):
            if pend[j] is not None:
                got.append(container_from_gathered(pend[j].result(), bs, n))
        out["async"] = got
        out["sum"] = comm.allreduce([5, 7]).tolist()
        out["max"] = comm.allreduce([2.5], op="max").tolist()
        comm.barrier()
        # an RCCL error comes back as KOLM_ERCCL (rank 1 of a 1-rank communicator:
        # ncclInvalidArgument, raised by RCCL before any bootstrap traffic)
        h = ctypes.c_void_p()
        rc = _lib.load().kolm_comm_init(ctx, 1, 1, Comm.unique_id(), ctypes.byref(h))
        out["erccl"] = (rc, _lib.load().kolm_last_error().decode())
        comm.close()
        # kolm_encode_blocks_multi: ncclCommInitAll over this process's devices (one here),
        # payloads received into device 0, one copy to the host
        _, method, pays, _ = _lib.encode_blocks_multi(data, bs, 1)
        out["multi"] = (method.tolist(), pays)
        out["torch_loaded"] = "torch" in sys.modules
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    q.put(out)


def test_rccl_c_abi_world1_matches_oracle():
    import oracle as O
    from kolm import datagen as D
    bs = 65536
    mixed = D.enwik_like(5 * bs) + bytes(bs) + D.splitmix64_bytes(bs + 777)
    cases = [("mixed_rr", mixed, bs, "round_robin"), ("mixed_contig", mixed, bs, "contiguous"),
             ("text_rr", D.enwik_like(300000, seed=11), 65536, "round_robin"),
             ("one_short", b"abracadabra" * 3, 4096, "round_robin")]
    ctx = mpc.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(cases, q))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert "error" not in got, got.get("error")
    assert got["rank"] == (0, 1)
    assert not got["torch_loaded"]
    for name, data, bs, _ in cases:
        assert got[name] == O.compress_blocks_fixed(data, bs, range(10)), name
    want = O.compress_blocks_fixed(cases[0][1], cases[0][2], range(10))
    assert len(got["async"]) == 4 and all(c == want for c in got["async"])
    assert got["sum"] == [5, 7] and got["max"] == [2.5]
    rc, msg = got["erccl"]
    assert rc == -4 and "RCCL" in msg, (rc, msg)
    ids, pays = got["multi"]
    data, bs0 = cases[0][1], cases[0][2]
    wids = []
    for i in range(0, len(data), bs0):
        blk = data[i:i + bs0]
        c = [O.candidate(m, blk) for m in range(10)]
        m = min(range(10), key=lambda k: len(c[k]))
        wids.append(m)
        assert pays[len(wids) - 1] == c[m]
    assert ids == wids
