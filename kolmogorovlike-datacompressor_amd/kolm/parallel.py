"""Multi-GPU block sharding + container reassembly (one process per GPU), over the C ABI.

Blocks are independent (PY:2350-2369: no state crosses blocks), so a batch shards with
no data-path collective: rank r encodes the blocks ``rank_blocks(nblocks, r, world,
partition)`` — by default the contiguous range ``shard_blocks(nblocks, r, world)`` (a
rank's blocks are one contiguous slice of the input: one upload, and rank order is
container order), or ``partition="round_robin"`` (block i on rank i mod world, BASELINE
config 4's assignment; for equal blocks both give every rank the same work).  The only
exchange step is reassembling the output stream on the destination rank
(``kolm_gather_payloads``, csrc/kolm_comm.cpp: RCCL over xGMI, straight from HBM — each
rank's payload arena exactly as long as it is, plus its method ids and payload offsets),
after which the destination writes the container (PY:2375-2445).

No PyTorch: device memory, the communicator (``Comm``: ncclCommInitRank behind
``kolm_comm_init``), barriers and reductions all go through libkolm_hip.so with ctypes
and numpy.  The communicator id is moved between the processes by ``exchange_unique_id``
(a TCP socket at MASTER_ADDR, as torch.distributed.run sets it).  Anything with the same
``rank`` / ``nranks`` / ``device`` / ``gather_payloads`` interface can stand in for
``Comm`` (the CPU tests use a gloo transport of their own).
"""
from __future__ import annotations

import ctypes
import os
import socket
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_blocks(nblocks: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced block range [first, first+count) of `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(nblocks, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


PARTITIONS = ("contiguous", "round_robin")


def rank_blocks(nblocks: int, rank: int, world: int, partition: str = "contiguous") -> range:
    """Global block indices encoded by `rank`, in container order."""
    if partition == "contiguous":
        first, count = shard_blocks(nblocks, rank, world)
        return range(first, first + count)
    if partition == "round_robin":
        if world <= 0 or not 0 <= rank < world:
            raise ValueError("bad rank/world")
        return range(rank, nblocks, world)
    raise ValueError(f"partition must be one of {PARTITIONS}")


# ---------------------------------------------------------------------------------------
# bootstrap: the communicator id from rank 0 to every rank
# ---------------------------------------------------------------------------------------
_ID_BYTES = 128


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("kolm comm bootstrap: peer closed the connection")
        buf += chunk
    return bytes(buf)


def exchange_unique_id(rank: int, world: int, addr: str, port: int, uid: Optional[bytes] = None,
                       timeout: float = 300.0) -> bytes:
    """Rank 0 (which passes `uid`) serves the id's bytes to the other world - 1 ranks at
    addr:port; every other rank connects (retrying until rank 0 listens) and receives
    them.  Returns the id on every rank.  Each client first sends its rank (4 bytes), so a
    stray or repeated connection is refused instead of being counted."""
    if world <= 1:
        if uid is None:
            raise ValueError("rank 0 must supply the id")
        return uid
    deadline = time.monotonic() + timeout
    if rank == 0:
        if uid is None or len(uid) != _ID_BYTES:
            raise ValueError("rank 0 must supply a 128-byte id")
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        try:
            srv.bind((addr, port))
            srv.listen(max(world, 8))
            seen = set()
            while len(seen) < world - 1:
                srv.settimeout(max(deadline - time.monotonic(), 0.1))
                conn, _ = srv.accept()
                with conn:
                    conn.settimeout(30.0)
                    r = int.from_bytes(_recv_exact(conn, 4), "little")
                    if not 0 < r < world or r in seen:
                        continue
                    conn.sendall(uid)
                    seen.add(r)
        finally:
            srv.close()
        return uid
    while True:
        try:
            with socket.create_connection((addr, port), timeout=5.0) as s:
                s.sendall(int(rank).to_bytes(4, "little"))
                return _recv_exact(s, _ID_BYTES)
        except (ConnectionError, OSError):
            if time.monotonic() > deadline:
                raise TimeoutError(f"kolm comm bootstrap: rank {rank} could not reach {addr}:{port}")
            time.sleep(0.05)


def env_rendezvous() -> Tuple[int, int, int, str, int]:
    """(rank, world, local_rank, addr, port) from torch.distributed.run's environment
    (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  The id is served on
    KOLM_COMM_PORT, default MASTER_PORT + 1 (the launcher's own store holds MASTER_PORT)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("KOLM_COMM_PORT", str(int(os.environ.get("MASTER_PORT", "29500")) + 1)))
    return rank, world, local, addr, port


# ---------------------------------------------------------------------------------------
# the communicator (RCCL, csrc/kolm_comm.cpp)
# ---------------------------------------------------------------------------------------
@dataclass
class Gathered:
    """What the destination rank holds after a gather: the ranks' payloads back to back in
    rank order (``payloads``: a DeviceBuffer for RCCL, or host bytes), each rank's
    (bytes, blocks), and the concatenated method ids and offsets into the payloads."""
    payloads: object
    rank_bytes: np.ndarray
    rank_blocks: np.ndarray
    method_all: np.ndarray
    off_all: np.ndarray

    def payload_bytes(self) -> bytes:
        """The gathered payloads as host bytes (one device-to-host copy for RCCL)."""
        total = int(self.off_all[-1]) if len(self.off_all) else 0
        if isinstance(self.payloads, (bytes, bytearray, memoryview)):
            return bytes(self.payloads[:total])
        return self.payloads.download(total)


class PendingGather:
    """An in-flight gather (async_op=True): wait() blocks until every transfer of it is
    done (the arena may be reused after that); result() waits, then returns what the
    synchronous call would (the Gathered record on the destination, None elsewhere)."""

    def __init__(self, comm, result):
        self._comm = comm
        self._result = result
        self._done = False

    def wait(self):
        if not self._done:
            self._comm.wait()
            self._done = True

    def result(self):
        self.wait()
        return self._result


class Comm:
    """One rank of an RCCL communicator on this process's device (kolm_comm_init).

    Comm(nranks, rank, uid, device): explicit id (``Comm.unique_id()`` on one rank, the same
    bytes everywhere); ``Comm.from_env()``: the launcher's environment + the TCP bootstrap."""

    def __init__(self, nranks: int, rank: int, uid: bytes, device: int = 0):
        from . import _lib
        self._lib = _lib
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)
        self.ctx = _lib.device_ctx(self.device)
        p = ctypes.c_void_p()
        _lib.check(_lib.load().kolm_comm_init(self.ctx, self.nranks, self.rank, bytes(uid), ctypes.byref(p)))
        self._h = p
        self._dst_buf = None  # grow-only destination arena of the gathers (device memory)

    @staticmethod
    def unique_id() -> bytes:
        from . import _lib
        buf = ctypes.create_string_buffer(_lib.KOLM_COMM_ID_BYTES)
        _lib.check(_lib.load().kolm_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def from_env(cls, device: Optional[int] = None, timeout: float = 300.0) -> "Comm":
        rank, world, local, addr, port = env_rendezvous()
        uid = exchange_unique_id(rank, world, addr, port, cls.unique_id() if rank == 0 else None, timeout)
        return cls(world, rank, uid, local if device is None else device)

    def close(self):
        if self._h is not None and self._h.value:
            self._dst_buf = None
            self._lib.check(self._lib.load().kolm_comm_destroy(self._h))
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def barrier(self):
        self._lib.check(self._lib.load().kolm_comm_barrier(self._h))

    def allreduce(self, values, op: str = "sum") -> np.ndarray:
        """Host values (int -> uint64, float -> float64) reduced over the ranks ("sum"/"max")."""
        arr = np.asarray(values)
        dt = 1 if arr.dtype.kind == "f" else 0
        buf = np.ascontiguousarray(arr, dtype=np.float64 if dt else np.uint64).reshape(-1).copy()
        self._lib.check(self._lib.load().kolm_comm_allreduce(self._h, buf.ctypes.data, buf.size, dt,
                                                             {"sum": 0, "max": 1}[op]))
        return buf

    def wait(self):
        self._lib.check(self._lib.load().kolm_comm_wait(self._h))

    def _dst_arena(self, nbytes: int):
        if self._dst_buf is None or self._dst_buf.nbytes < nbytes:
            self._dst_buf = None
            self._dst_buf = self._lib.DeviceBuffer(self.ctx, max(nbytes, 1))
        return self._dst_buf

    def gather_payloads(self, d_arena: int, nbytes: int, method, off, dst: int = 0, dst_buf=None,
                        async_op: bool = False, dst_cap_blocks: int = 1 << 20):
        """kolm_gather_payloads: this rank's device arena prefix d_arena[0, nbytes), its
        method ids and payload offsets (host arrays, as the encoder returned them) onto
        `dst`.  dst_buf: the destination's DeviceBuffer (default: a grow-only buffer of the
        communicator, sized after a first call that reports the ranks' sizes).  Returns a
        Gathered record on dst, None elsewhere (a PendingGather of either with async_op).

        Without dst_buf the payloads of every gather land in that one communicator buffer:
        a Gathered record (and PendingGather.result()) stays valid only until the next
        gather_payloads call of this communicator overwrites it.  A caller that keeps
        several gathers alive (double-buffered steps) passes its own dst_buf per gather."""
        L = self._lib.load()
        R = self.nranks
        meth = np.ascontiguousarray(np.asarray(method, dtype=np.uint32))
        offs = np.ascontiguousarray(np.asarray(off, dtype=np.uint64))
        nb = int(meth.size)
        if offs.size != nb + 1:
            raise ValueError("off must hold len(method) + 1 entries")
        rbytes = np.zeros(R, np.uint64)
        rblocks = np.zeros(R, np.uint32)
        is_dst = self.rank == dst
        cap_b = int(dst_cap_blocks) if is_dst else 0
        m_all = np.zeros(max(cap_b, 1), np.uint32)
        o_all = np.zeros(max(cap_b, 1) + 1, np.uint64)
        buf = dst_buf if dst_buf is not None else (self._dst_buf if is_dst else None)
        for attempt in range(2):
            cap = buf.nbytes if (is_dst and buf is not None) else 0
            rc = L.kolm_gather_payloads(self._h, d_arena, int(nbytes), meth.ctypes.data if nb else None,
                                        offs.ctypes.data, nb, int(dst), buf.ptr if (is_dst and buf) else None,
                                        cap, cap_b, rbytes.ctypes.data, rblocks.ctypes.data,
                                        m_all.ctypes.data if is_dst else None,
                                        o_all.ctypes.data if is_dst else None, 1 if async_op else 0)
            if rc == self._lib.KOLM_ECAP and attempt == 0:
                # every rank saw the sizes and returned KOLM_ECAP: the destination takes a
                # large enough buffer of its own (a caller's dst_buf that is too small is
                # replaced), and every rank calls again
                if is_dst:
                    buf = self._dst_arena(int(rbytes.sum()))
                    if int(rblocks.sum()) > cap_b:
                        cap_b = int(rblocks.sum())
                        m_all = np.zeros(cap_b, np.uint32)
                        o_all = np.zeros(cap_b + 1, np.uint64)
                continue
            self._lib.check(rc)
            break
        res = None
        if is_dst:
            tb = int(rblocks.sum())
            res = Gathered(buf, rbytes, rblocks, m_all[:tb], o_all[:tb + 1])
        return PendingGather(self, res) if async_op else res


_default_comm = None


def default_comm() -> Comm:
    """The process's communicator from the launcher's environment (created once)."""
    global _default_comm
    if _default_comm is None:
        _default_comm = Comm.from_env()
    return _default_comm


# ---------------------------------------------------------------------------------------
# reassembly (host logic, shared by every transport)
# ---------------------------------------------------------------------------------------
def container_from_gathered(g: Gathered, block_size: int, total_len: int, partition: str = "contiguous") -> bytes:
    """The container (PY:2332-2445) from a gather's record: blocks of rank r are
    rank_blocks(.., r, ..) in order; the ranks' payloads lie back to back in rank order."""
    from .container import MODE_FIXED, write_container
    world = len(g.rank_blocks)
    nb = int(np.sum(g.rank_blocks))
    if nb != (total_len + block_size - 1) // block_size:
        raise ValueError("gathered block count does not match the input")
    blob = g.payload_bytes()
    mids: List[int] = [0] * nb
    pays: List[bytes] = [b""] * nb
    k = 0
    for r in range(world):
        blocks = rank_blocks(nb, r, world, partition)
        if len(blocks) != int(g.rank_blocks[r]):
            raise ValueError("per-rank block counts do not match the partition")
        for gi in blocks:
            mids[gi] = int(g.method_all[k])
            pays[gi] = blob[int(g.off_all[k]):int(g.off_all[k + 1])]
            k += 1
    orig = [min(block_size, total_len - i * block_size) for i in range(nb)]
    return write_container(MODE_FIXED, block_size, total_len, mids, orig, pays)


def assemble_container(block_size: int, total_len: int, per_rank_ids: Sequence[Sequence[int]],
                       per_rank_payloads: Sequence[bytes], per_rank_offsets: Sequence[Sequence[int]],
                       partition: str = "contiguous") -> bytes:
    """Host TOC + payloads in global block order from per-rank lists (each rank's blocks:
    rank_blocks); the same as container_from_gathered on separate per-rank pieces."""
    blob = b"".join(bytes(p[:int(o[-1])]) if len(o) else b"" for p, o in zip(per_rank_payloads, per_rank_offsets))
    m_all, o_all, base = [], [0], 0
    for ids, off in zip(per_rank_ids, per_rank_offsets):
        m_all += [int(x) for x in ids]
        o_all += [base + int(x) for x in list(off)[1:]]
        base += int(off[-1]) if len(off) else 0
    g = Gathered(blob, np.array([int(o[-1]) if len(o) else 0 for o in per_rank_offsets], np.uint64),
                 np.array([len(i) for i in per_rank_ids], np.uint32), np.array(m_all, np.uint32),
                 np.array(o_all, np.uint64))
    return container_from_gathered(g, block_size, total_len, partition)


def compress_blocks_fixed_distributed(data: bytes, block_size: int, comm=None, dst: int = 0,
                                      cand_mask: Optional[int] = None,
                                      partition: str = "contiguous") -> Optional[bytes]:
    """Every rank calls this with the same `data`; rank r encodes its blocks
    (rank_blocks(.., partition)) on its GPU into a device arena (kolm_encode_blocks_device),
    the arenas, method ids and offsets are gathered onto `dst` (comm.gather_payloads; RCCL
    over xGMI by default), and `dst` returns the container (others return None) —
    bit-identical to compress_blocks_fixed(data) for either partition.  Only `dst` copies
    payloads to the host, once, to write the container."""
    from . import _lib, candidate_mask
    if block_size <= 0:
        raise ValueError("block_size must be positive")
    comm = default_comm() if comm is None else comm
    rank, world = comm.rank, comm.nranks
    mask = candidate_mask() if cand_mask is None else cand_mask
    n = len(data)
    nb = (n + block_size - 1) // block_size
    mine = rank_blocks(nb, rank, world, partition)
    # the rank's blocks back to back: equal blocks, the input's short tail (if it is this
    # rank's) last, so they form one fixed-size batch
    if partition == "contiguous" and len(mine):
        part = memoryview(data)[mine.start * block_size:min(n, mine.stop * block_size)]
    else:
        part = b"".join(data[i * block_size:(i + 1) * block_size] for i in mine)
    m = len(part)
    ctx = _lib.device_ctx(comm.device)
    arena = _lib.DeviceBuffer(ctx, _lib.arena_capacity(m, len(mine), mask))
    if m:
        d_in = _lib.input_buffer(ctx, part)
        _, method, off, _ = _lib.encode_blocks_device(ctx, d_in.ptr, m, block_size, arena.ptr, arena.nbytes, mask)
        d_in.free()
    else:
        method, off = np.zeros(0, np.uint32), np.zeros(1, np.uint64)
    g = comm.gather_payloads(arena.ptr, int(off[-1]), method, off, dst=dst, dst_cap_blocks=max(nb, 1))
    if rank != dst:
        return None
    return container_from_gathered(g, block_size, n, partition)
