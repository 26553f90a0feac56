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


def gather_payloads(arena, nbytes: int, method_ids, dst: int = 0, group=None, async_op: bool = False):
    """Gather every rank's payload arena prefix and method ids onto `dst`.

    arena: 1-D uint8 tensor (device for nccl, host for gloo) holding this rank's payloads
    back to back (at least max-over-ranks bytes long); nbytes: its used length;
    method_ids: 1-D int32 tensor of this rank's per-block winners (same device).
    Returns on dst: (list of per-rank uint8 tensors trimmed to their nbytes,
    list of per-rank int32 method-id tensors); on other ranks (None, None).
    async_op: the small size exchange completes here, the payload and id gathers are left
    in flight and a PendingGather is returned (the caller must not overwrite `arena`
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
    sizes = [int(m[0]) for m in metas]
    counts = [int(m[1]) for m in metas]
    maxb, maxc = max(sizes), max(counts)
    if arena.numel() < maxb:
        raise ValueError("arena shorter than the largest rank payload")
    ids = torch.zeros(maxc, dtype=torch.int32, device=dev)
    ids[: method_ids.numel()] = method_ids
    if rank == dst:
        pay_list = [torch.empty(maxb, dtype=torch.uint8, device=dev) for _ in range(world)]
        id_list = [torch.empty(maxc, dtype=torch.int32, device=dev) for _ in range(world)]
    else:
        pay_list = id_list = None
    w1 = dist.gather(arena[:maxb].contiguous(), pay_list, dst=dst, group=group, async_op=async_op)
    w2 = dist.gather(ids, id_list, dst=dst, group=group, async_op=async_op)
    res = (None, None) if rank != dst else ([p[: sizes[r]] for r, p in enumerate(pay_list)],
                                            [i[: counts[r]] for r, i in enumerate(id_list)])
    if async_op:
        return PendingGather([w for w in (w1, w2) if w is not None], res)
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
    (rank_blocks(.., partition)) on its GPU, payloads + ids are gathered to `dst` over the
    process group, `dst` returns the container (others return None).  Bit-identical to
    compress_blocks_fixed(data) for either partition."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from . import encode_blocks
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = len(data)
    nb = (n + block_size - 1) // block_size
    mine = rank_blocks(nb, rank, world, partition)
    # the rank's blocks back to back: equal blocks, the input's short tail (if it is this
    # rank's) last, so they form one fixed-size batch
    part = b"".join(data[i * block_size:(i + 1) * block_size] for i in mine)
    mids, orig, payloads, _ = encode_blocks(part, block_size, cand_mask) if len(mine) else ([], [], [], None)
    blob = b"".join(payloads)
    offs = np.concatenate([[0], np.cumsum([len(p) for p in payloads])]).astype(np.int64)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    meta = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    dist.all_reduce(meta, op=dist.ReduceOp.MAX, group=group)
    arena = torch.zeros(max(int(meta[0]), 1), dtype=torch.uint8, device=dev)
    if blob:
        arena[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    ids = torch.tensor(mids, dtype=torch.int32, device=dev)
    pays, idl = gather_payloads(arena, len(blob), ids, dst=dst, group=group)
    # offsets are tiny: gather them through an object collective on the host
    all_offs = [None] * world
    dist.all_gather_object(all_offs, offs.tolist(), group=group)
    if rank != dst:
        return None
    return assemble_container(block_size, n, [i.cpu().tolist() for i in idl],
                              [p.cpu().numpy().tobytes() for p in pays], all_offs, partition)
