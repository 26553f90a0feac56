"""Multi-GPU block sharding + container reassembly (one process per GPU).

Blocks are independent (PY:2350-2369: no state crosses blocks), so a batch shards with
no data-path collective: rank r encodes the blocks ``rank_blocks(nblocks, r, world,
partition)`` — by default the contiguous range ``shard_blocks(nblocks, r, world)`` (a
rank's blocks are one contiguous slice of the input: one upload, and rank order is
container order), or ``partition="round_robin"`` (block i on rank i mod world, BASELINE
config 4's assignment; for equal blocks both give every rank the same work).  The only exchange step is reassembling the output
stream on the destination rank: a tiny all-gather of per-rank (nblocks, payload bytes),
then a gather of the per-rank payload arenas (padded to the largest) and of the method
ids.  With the ``nccl`` backend (RCCL over xGMI on MI355X) the tensors live in HBM; with
``gloo`` (CPU tests) they are host tensors — the logic is identical.

torch is imported lazily (plumbing only); a process that also loads libkolm_hip.so must
import torch first so both share one HIP runtime (see kolm._lib).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple


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


class PendingGather:
    """An in-flight gather_payloads(async_op=True): wait() blocks the host until the
    collectives are done (the arena may be reused after that); result() waits, then
    returns what the synchronous call would."""

    def __init__(self, works, result):
        self._works = works
        self._result = result

    def wait(self):
        import torch
        for w in self._works:
            w.wait()
        self._works = []
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()

    def result(self):
        self.wait()
        return self._result


def gather_payloads(arena, nbytes: int, method_ids, dst: int = 0, group=None, async_op: bool = False,
                    offsets=None):
    """Gather every rank's payload arena prefix, method ids (and payload offsets) onto `dst`.

    arena: 1-D uint8 tensor (device for nccl, host for gloo) holding this rank's payloads
    back to back; nbytes: its used length; method_ids: 1-D int32 tensor of this rank's
    per-block winners (same device); offsets (optional): 1-D int64 tensor of its
    len(method_ids) + 1 payload offsets.  An arena shorter than the largest rank's payload
    bytes is padded into a temporary first.
    Returns on dst: (list of per-rank uint8 tensors trimmed to their nbytes, list of
    per-rank int32 method-id tensors[, list of per-rank int64 offset tensors when offsets
    were given]); on other ranks Nones.
    async_op: the small size exchange completes here, the payload / id / offset gathers are
    left in flight and a PendingGather is returned (the caller must not overwrite `arena`
    before its wait()) — bench.py double-buffers the arena so the gather of step k runs
    over xGMI while step k+1 computes.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = arena.device
    meta = torch.tensor([nbytes, method_ids.numel()], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    sizes_counts = torch.stack(metas).cpu().tolist()  # one device -> host read
    sizes = [int(s) for s, _ in sizes_counts]
    counts = [int(c) for _, c in sizes_counts]
    maxb, maxc = max(max(sizes), 1), max(counts)
    src = arena[:maxb]
    if arena.numel() < maxb:
        src = torch.zeros(maxb, dtype=torch.uint8, device=dev)
        src[:nbytes] = arena[:nbytes]
    ids = torch.zeros(maxc, dtype=torch.int32, device=dev)
    ids[: method_ids.numel()] = method_ids
    if offsets is not None:
        offs = torch.zeros(maxc + 1, dtype=torch.int64, device=dev)
        offs[: offsets.numel()] = offsets
    if rank == dst:
        pay_list = [torch.empty(maxb, dtype=torch.uint8, device=dev) for _ in range(world)]
        id_list = [torch.empty(maxc, dtype=torch.int32, device=dev) for _ in range(world)]
        off_list = [torch.empty(maxc + 1, dtype=torch.int64, device=dev) for _ in range(world)]
    else:
        pay_list = id_list = off_list = None
    works = [dist.gather(src.contiguous(), pay_list, dst=dst, group=group, async_op=async_op),
             dist.gather(ids, id_list, dst=dst, group=group, async_op=async_op)]
    if offsets is not None:
        works.append(dist.gather(offs, off_list, dst=dst, group=group, async_op=async_op))
    if rank != dst:
        res = (None, None) if offsets is None else (None, None, None)
    else:
        res = ([p[: sizes[r]] for r, p in enumerate(pay_list)], [i[: counts[r]] for r, i in enumerate(id_list)])
        if offsets is not None:
            res = res + ([o[: counts[r] + 1] for r, o in enumerate(off_list)],)
    if async_op:
        return PendingGather([w for w in works if w is not None], res)
    return res


def assemble_container(block_size: int, total_len: int, per_rank_ids: Sequence[Sequence[int]],
                       per_rank_payloads: Sequence[bytes], per_rank_offsets: Sequence[Sequence[int]],
                       partition: str = "contiguous") -> bytes:
    """Host TOC + payloads in global block order (each rank's blocks: rank_blocks)."""
    from .container import MODE_FIXED, write_container
    world = len(per_rank_ids)
    nb = sum(len(ids) for ids in per_rank_ids)
    mids: List[int] = [0] * nb
    pays: List[bytes] = [b""] * nb
    for r, (ids, buf, off) in enumerate(zip(per_rank_ids, per_rank_payloads, per_rank_offsets)):
        blocks = rank_blocks(nb, r, world, partition)
        if len(blocks) != len(ids):
            raise ValueError("per-rank block counts do not match the partition")
        for i, g in enumerate(blocks):
            mids[g] = int(ids[i])
            pays[g] = bytes(buf[int(off[i]):int(off[i + 1])])
    orig = [min(block_size, total_len - i * block_size) for i in range(nb)]
    return write_container(MODE_FIXED, block_size, total_len, mids, orig, pays)


def compress_blocks_fixed_distributed(data: bytes, block_size: int, dst: int = 0, group=None,
                                      cand_mask: Optional[int] = None, partition: str = "contiguous") -> Optional[bytes]:
    """Every rank calls this with the same `data`; rank r encodes its blocks
    (rank_blocks(.., partition)) on its GPU, payloads + ids + offsets are gathered to `dst`
    over the process group, `dst` returns the container (others return None).
    Bit-identical to compress_blocks_fixed(data) for either partition.

    The rank's blocks go up once and are encoded into a device arena
    (kolm_encode_blocks_device); with ``nccl`` (RCCL over xGMI) the arena, the method ids
    and the payload offsets are gathered straight from HBM, and only `dst` copies the
    gathered payloads to the host, once, to write the container.  With ``gloo`` (CPU
    process groups) the arena is copied to the host before the gather."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from . import _lib, candidate_mask
    if block_size <= 0:
        raise ValueError("block_size must be positive")
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mask = candidate_mask() if cand_mask is None else cand_mask
    n = len(data)
    nb = (n + block_size - 1) // block_size
    mine = rank_blocks(nb, rank, world, partition)
    device = torch.cuda.current_device()
    gpu = torch.device("cuda", device)
    coll = gpu if dist.get_backend(group) == "nccl" else torch.device("cpu")
    # the rank's blocks back to back: equal blocks, the input's short tail (if it is this
    # rank's) last, so they form one fixed-size batch
    if partition == "contiguous" and len(mine):
        part = memoryview(data)[mine.start * block_size:min(n, mine.stop * block_size)]
    else:
        part = b"".join(data[i * block_size:(i + 1) * block_size] for i in mine)
    m = len(part)
    cap = _lib.arena_capacity(m, len(mine), mask)
    arena = torch.empty(cap, dtype=torch.uint8, device=gpu)
    if m:
        d_in = torch.empty(m + 64, dtype=torch.uint8, device=gpu)
        d_in[:m].copy_(torch.frombuffer(bytearray(part), dtype=torch.uint8))
        torch.cuda.synchronize()
        _, method, off, _ = _lib.encode_blocks_device(_lib.device_ctx(device), d_in.data_ptr(), m, block_size,
                                                      arena.data_ptr(), cap, mask)
        del d_in
    else:
        method, off = np.zeros(0, np.uint32), np.zeros(1, np.uint64)
    nbytes = int(off[-1])
    ids = torch.from_numpy(method.astype(np.int32)).to(coll)
    offs = torch.from_numpy(off.astype(np.int64)).to(coll)
    src = arena if coll.type == "cuda" else arena[:max(nbytes, 1)].cpu()
    pays, idl, offl = gather_payloads(src, nbytes, ids, dst=dst, group=group, offsets=offs)
    if rank != dst:
        return None
    # one device -> host copy of all gathered payloads
    lens = [int(p.numel()) for p in pays]
    blob = torch.cat(pays).cpu().numpy().tobytes() if sum(lens) else b""
    starts = np.concatenate([[0], np.cumsum(lens)]).tolist()
    per_rank = [blob[starts[r]:starts[r + 1]] for r in range(world)]
    return assemble_container(block_size, n, [i.cpu().tolist() for i in idl], per_rank,
                              [o.cpu().tolist() for o in offl], partition)
