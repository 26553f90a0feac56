"""CPU stand-in for kolm.parallel.Comm in the tests: the same rank / nranks / device /
gather_payloads interface over a torch ``gloo`` process group on host memory (test
transport only — the product gathers with RCCL behind the C ABI, kolm_gather_payloads).
Returns kolm.parallel.Gathered records, so the reassembly code under test is the
product's own (container_from_gathered)."""
import numpy as np
import torch
import torch.distributed as dist

from kolm.parallel import Gathered


class GlooTransport:
    def __init__(self, device: int = 0, ctx=None):
        self.rank = dist.get_rank()
        self.nranks = dist.get_world_size()
        self.device = device
        self.ctx = ctx  # set: d_arena is a device pointer of this context (GPU encode)

    def gather_host(self, blob: bytes, method, off, dst: int = 0):
        """The gather of host payload bytes (the oracle-encoded CPU tests)."""
        meth = np.asarray(method, np.int64)
        offs = np.asarray(off, np.int64)
        meta = torch.tensor([len(blob), meth.size], dtype=torch.int64)
        metas = [torch.empty_like(meta) for _ in range(self.nranks)]
        dist.all_gather(metas, meta)
        sizes = [int(m[0]) for m in metas]
        counts = [int(m[1]) for m in metas]
        maxb, maxc = max(max(sizes), 1), max(counts)
        pay = torch.zeros(maxb, dtype=torch.uint8)
        if blob:
            pay[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        ids = torch.zeros(maxc, dtype=torch.int64)
        ids[:meth.size] = torch.from_numpy(meth)
        ot = torch.zeros(maxc + 1, dtype=torch.int64)
        ot[:offs.size] = torch.from_numpy(offs)
        is_dst = self.rank == dst
        pl = [torch.empty(maxb, dtype=torch.uint8) for _ in range(self.nranks)] if is_dst else None
        il = [torch.empty(maxc, dtype=torch.int64) for _ in range(self.nranks)] if is_dst else None
        ol = [torch.empty(maxc + 1, dtype=torch.int64) for _ in range(self.nranks)] if is_dst else None
        dist.gather(pay, pl, dst=dst)
        dist.gather(ids, il, dst=dst)
        dist.gather(ot, ol, dst=dst)
        if not is_dst:
            return None
        parts, m_all, o_all, base = [], [], [0], 0
        for r in range(self.nranks):
            parts.append(pl[r][:sizes[r]].numpy().tobytes())
            m_all += il[r][:counts[r]].tolist()
            o_all += [base + int(x) for x in ol[r][1:counts[r] + 1].tolist()]
            base += sizes[r]
        return Gathered(b"".join(parts), np.array(sizes, np.uint64), np.array(counts, np.uint32),
                        np.array(m_all, np.uint32), np.array(o_all, np.uint64))

    def gather_payloads(self, d_arena, nbytes, method, off, dst=0, dst_cap_blocks=0, async_op=False):
        """kolm.parallel.Comm's interface: the device arena comes to the host first."""
        from kolm import _lib
        blob = b""
        if nbytes:
            buf = np.zeros(int(nbytes), np.uint8)
            _lib.check(_lib.load().kolm_memcpy_d2h(self.ctx, buf.ctypes.data, d_arena, int(nbytes)))
            blob = buf.tobytes()
        return self.gather_host(blob, method, off, dst)
