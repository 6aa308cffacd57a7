"""Data-parallel sharding of a word array across ranks (one process per GPU).

Word i of every Amphora array depends only on word i of the other arrays
(SURVEY.md 8e), so a W-word job splits into contiguous shards with no
data-path exchange.  The one cross-shard value is the verify verdict: the
smallest failing word index over all shards (min-reduce of global indices).

For a root-held array (BASELINE config C4: the word array lives on one GPU
and is split over 8) the shards travel by torch.distributed scatter/gather,
which is RCCL over xGMI with the "nccl" backend (and gloo on CPU in tests).
Shards are padded to equal size (ceil(W / world) words) for the collective.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

NO_FAILURE = 0x7F7F7F7F7F7F7F7F


def shard_range(words: int, rank: int, world: int) -> Tuple[int, int]:
    """(start, count) of rank's contiguous shard; shard size ceil(W/world)."""
    per = -(-words // world) if world else 0
    start = min(words, rank * per)
    return start, max(0, min(per, words - start))


def padded_shard_words(words: int, world: int) -> int:
    return -(-words // world)


def scatter_words(full, words: int, width: int, root: int = 0, group=None, like=None):
    """Scatter a (words, width) uint8 tensor held by `root` into equal padded
    shards; every rank returns its (count, width) shard view.
    `like` gives device/dtype on non-root ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = padded_shard_words(words, world)
    ref = full if full is not None else like
    out = torch.empty((per, width), dtype=torch.uint8, device=ref.device)
    chunks = None
    if rank == root:
        pad = per * world - words
        src = full if pad == 0 else torch.cat(
            [full, torch.zeros((pad, width), dtype=torch.uint8, device=full.device)])
        chunks = list(src.view(world, per, width).unbind(0))
    dist.scatter(out, chunks, src=root, group=group)
    _, count = shard_range(words, rank, world)
    return out[:count]


def gather_words(local, words: int, width: int, root: int = 0, group=None):
    """Inverse of scatter_words: root returns the (words, width) tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = padded_shard_words(words, world)
    buf = torch.zeros((per, width), dtype=torch.uint8, device=local.device)
    buf[: local.shape[0]] = local
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, bufs, dst=root, group=group)
    if rank != root:
        return None
    return torch.cat(bufs)[:words]


def global_first_fail(local_ff: int, start: int) -> int:
    """Local verdict (-1 / index / device sentinel) -> global index or NO_FAILURE."""
    if local_ff < 0 or local_ff == NO_FAILURE:
        return NO_FAILURE
    return start + local_ff


def combine_first_fail(local_ff: int, start: int, group=None, device="cpu") -> int:
    """min over ranks of the global failing index; -1 if every word verified."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([global_first_fail(local_ff, start)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    v = int(t.item())
    return -1 if v == NO_FAILURE else v
