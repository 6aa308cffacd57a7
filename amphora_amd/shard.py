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
    full = None
    bufs = None
    if rank == root:  # every rank's padded shard lands in its slice of one buffer
        full = torch.empty((per * world, width), dtype=torch.uint8, device=local.device)
        bufs = list(full.view(world, per, width).unbind(0))
    dist.gather(buf, bufs, dst=root, group=group)
    if rank != root:
        return None
    return full[:words]


def _p2p(ops, timeout=None):
    """Run a list of (op, tensor, peer) as ONE batch_isend_irecv group (RCCL:
    one ncclGroupStart/End, every send and receive in flight at once).  gloo
    moves host memory only, so for a gloo rehearsal with device tensors the
    sends are staged through host copies and the receives land in host
    buffers copied back afterwards.

    `timeout` (seconds): the host blocks until every operation of the batch
    has completed or the time is up, and then raises (torch's
    `Work.wait(timeout)`, which for RCCL also blocks the CPU) -- a peer that
    never posts its half turns into an exception here instead of a stream
    that never drains."""
    import datetime
    import torch.distributed as dist
    if not ops:
        return
    host = dist.get_backend() == "gloo" and any(t.is_cuda for _, t, _ in ops)
    staged, back = [], []
    for op, t, peer in ops:
        if host:
            h = t.cpu() if op is dist.isend else t.new_empty(t.shape, device="cpu")
            if op is dist.irecv:
                back.append((t, h))
            t = h
        staged.append(dist.P2POp(op, t, peer))
    td = datetime.timedelta(seconds=timeout) if timeout else None
    for req in dist.batch_isend_irecv(staged):
        if td is None:
            req.wait()
        elif not req.wait(timeout=td):
            raise TimeoutError("point-to-point batch not complete after %.0f s" % timeout)
    for dev, h in back:
        dev.copy_(h)


class RootScatterGather:
    """BASELINE C4 with the word arrays held by one GPU: the
    root scatters `n_in` input arrays of `words` words to the ranks in
    contiguous shards and gathers `n_out` output arrays back.

    Each direction is ONE grouped point-to-point batch (root: a send per
    (peer, array) slice; peer: a receive per array into its preallocated
    `[n_in, per, width]` buffer), so on the GPU node all of the root's xGMI
    links carry their peers' shards at once.  Nothing is allocated per step:
    the root's own shard is a view of its full arrays (its kernels read and
    write them in place), peers receive into and send from buffers made
    once, and the gathered outputs land directly in their slices of the
    root's `[n_out, words, width]` array (no concatenation)."""

    def __init__(self, words: int, n_in: int, n_out: int, width: int = 16, root: int = 0,
                 device="cpu", group=None):
        import torch
        import torch.distributed as dist
        self.words, self.n_in, self.n_out, self.width, self.root = words, n_in, n_out, width, root
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.spans = [shard_range(words, r, self.world) for r in range(self.world)]
        self.start, self.count = self.spans[self.rank]
        per = padded_shard_words(words, self.world)
        self.inbuf = self.outbuf = None
        if self.rank != root:
            self.inbuf = torch.empty((n_in, per, width), dtype=torch.uint8, device=device)
            self.outbuf = torch.empty((n_out, per, width), dtype=torch.uint8, device=device)

    def _peer(self, r):
        import torch.distributed as dist
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def scatter(self, full_in=None, timeout=None):
        """Root passes its `[n_in, words, width]` arrays; every rank gets the
        `[n_in, count, width]` view of its own shard."""
        import torch.distributed as dist
        s, c = self.start, self.count
        ops = []
        if self.rank == self.root:
            assert full_in is not None and tuple(full_in.shape) == (self.n_in, self.words, self.width)
            for r, (rs, rc) in enumerate(self.spans):
                if r != self.root and rc:
                    ops += [(dist.isend, full_in[a, rs:rs + rc], self._peer(r)) for a in range(self.n_in)]
            _p2p(ops, timeout)
            return full_in[:, s:s + c]
        if c:
            ops = [(dist.irecv, self.inbuf[a, :c], self._peer(self.root)) for a in range(self.n_in)]
        _p2p(ops, timeout)
        return self.inbuf[:, :c]

    def out_view(self, full_out=None):
        """Where this rank's kernels write their outputs: the root's own
        slice of `full_out`, a peer's send buffer."""
        s, c = self.start, self.count
        if self.rank == self.root:
            return full_out[:, s:s + c]
        return self.outbuf[:, :c]

    def gather(self, full_out=None, timeout=None):
        """Peers send their `out_view()`; the root receives every peer's
        shard straight into its slice of `full_out` `[n_out, words, width]`."""
        import torch.distributed as dist
        ops = []
        if self.rank == self.root:
            assert full_out is not None and tuple(full_out.shape) == (self.n_out, self.words, self.width)
            for r, (rs, rc) in enumerate(self.spans):
                if r != self.root and rc:
                    ops += [(dist.irecv, full_out[a, rs:rs + rc], self._peer(r)) for a in range(self.n_out)]
        elif self.count:
            ops = [(dist.isend, self.outbuf[a, :self.count], self._peer(self.root))
                   for a in range(self.n_out)]
        _p2p(ops, timeout)
        return full_out if self.rank == self.root else None

    def moved_bytes(self) -> int:
        """Bytes that cross the root's links per step (scatter + gather)."""
        peers = sum(c for r, (_, c) in enumerate(self.spans) if r != self.root)
        return peers * (self.n_in + self.n_out) * self.width


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
