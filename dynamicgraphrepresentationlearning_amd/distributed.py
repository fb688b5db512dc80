"""Multi-GPU walk sharding and corpus reassembly (one process per GPU).

The graph snapshot is replicated on every rank; rank g owns the walks of a
contiguous start-vertex range [lo_g, hi_g) (walk ids {r*n + v : r < wpv, v in
[lo_g, hi_g)}), chosen so every rank holds the same number of non-isolated
start vertices.  Generation and re-walks need no exchange: the deterministic
RNG depends only on (wid / n, step) and the MH Philox stream on (seed, wid,
pos, epoch), so a walk is identical whichever rank computes it.

The only collective is the corpus all-gatherv used to hand the whole walk
corpus to a downstream consumer (yskip in the reference,
vertex-classification.cpp:142-158): a full-mesh exchange of batched
point-to-point sends/receives (torch.distributed.batch_isend_irecv, RCCL over
xGMI with backend "nccl", gloo on CPU) — every peer pair uses its own link at
once instead of a ring, and shards of different sizes need no padding.

Two forms:
  * allgatherv_corpus: the whole [n*wpv, L] corpus on every rank (fits while
    the corpus is small next to the graph: configs[1]-[3]);
  * gather_corpus_chunked: bounded memory, for corpora larger than a device
    (configs[4]: 656 M walks x 80 x 4 B = 210 GB against 288 GB of HBM, 253 GB
    of which the rank's graph and shard already hold).  Chunk c is local rows
    [c*K, (c+1)*K) of EVERY rank, so each chunk is a full-mesh exchange; the
    chunk lands in one buffer of K * world rows (or K rows on a rank that only
    sends, gatherv to a root), is handed to a sink with the global walk ids of
    its row runs, and the buffer is reused.  Local rows come from a callback
    (WharfMH.export_walk_rows: one device gather per chunk), so neither the
    corpus nor the rank's own walk-major copy is ever whole in memory.

Collective safety: a rank that fails between collectives must not leave its
peers waiting inside one.  `agree` is the one rule every multi-rank phase
follows (bench.py's jobs, the chunked gather): each rank runs its local,
fallible work, then all ranks meet in ONE small all-reduce that says whether
any rank failed; if one did, every rank raises RankFailure (carrying the
failing rank's error) at the same point, so the job is abandoned together.
Sizes that shape a collective (the gather's rows per chunk) are agreed the
same way (all-reduce MIN) instead of trusted to be equal.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


class RankFailure(RuntimeError):
    """Raised on EVERY rank when any rank failed a phase (see `agree`)."""

    def __init__(self, rank: int, phase: str, message: str):
        super().__init__(f"rank {rank} failed in {phase}: {message}")
        self.rank = rank
        self.phase = phase
        self.message = message


def _dist_active(group=None) -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def agree(err, phase: str, group=None, device="cpu"):
    """Collective: every rank reports whether its part of `phase` failed (err =
    the exception or None).  Returns only if no rank failed; otherwise raises
    RankFailure(first failing rank, phase, its error text) on every rank.
    Without an initialised process group it re-raises err."""
    if not _dist_active(group):
        if err is not None:
            raise err
        return
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = torch.tensor([rank if err is not None else world], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    src = int(t.item())
    if src == world:
        return
    msg = [f"{type(err).__name__}: {str(err)[:400]}" if err is not None else None]
    dist.broadcast_object_list(msg, src=src if group is None else dist.get_global_rank(group, src), group=group,
                               device=torch.device(device) if device != "cpu" else None)
    raise RankFailure(src, phase, msg[0]) from err


def agree_min(value: int, group=None, device="cpu") -> int:
    """Collective: the minimum of `value` over the ranks (a size every rank must share)."""
    if not _dist_active(group):
        return int(value)
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def injected_fault(phase: str, rank: int):
    """Test hook: WHARF_TEST_FAIL="<rank>:<phase>[,...]" makes that rank raise at
    that phase (tests/test_collective_safety.py drives a one-rank failure
    through bench.py's jobs and the chunked gather).  A phase ending in "_oom"
    raises torch.OutOfMemoryError, once per process."""
    spec = os.environ.get("WHARF_TEST_FAIL")
    key = f"{rank}:{phase}"
    if spec and key in spec.split(",") and key not in _FIRED:
        if phase.endswith("_oom"):
            import torch
            _FIRED.add(key)
            raise torch.OutOfMemoryError(f"injected out of memory (WHARF_TEST_FAIL) at {phase} on rank {rank}")
        raise RuntimeError(f"injected fault (WHARF_TEST_FAIL) at {phase} on rank {rank}")


_FIRED: set = set()


def _is_oom(ex) -> bool:
    import torch
    return isinstance(ex, torch.OutOfMemoryError) or "out of memory" in str(ex).lower()


def alloc_or_reclaim(alloc, on_oom, rank: int = 0):
    """alloc(); if it runs out of device memory and on_oom is given (e.g.
    WharfMH.release_caches: the library's reverse-slot index), free that and
    try once more.  Local to the rank: the caller agrees the outcome."""
    try:
        injected_fault("alloc_oom", rank)
        return alloc()
    except Exception as ex:   # noqa: BLE001
        if on_oom is None or not _is_oom(ex):
            raise
        on_oom()
        return alloc()


def balanced_shards(deg: np.ndarray, parts: int):
    """Contiguous start-vertex ranges with equal numbers of non-isolated vertices."""
    deg = np.asarray(deg)
    act = np.cumsum(deg > 0)
    total = int(act[-1]) if len(act) else 0
    bounds = [0]
    for k in range(1, parts):
        bounds.append(int(np.searchsorted(act, (total * k) // parts, side="right")))
    bounds.append(len(deg))
    return [(bounds[i], bounds[i + 1]) for i in range(parts)]


def shard_walk_ids(n: int, wpv: int, lo: int, hi: int) -> np.ndarray:
    """Global walk ids of a shard, in its local (export) order: r-major, then v."""
    v = np.arange(lo, hi, dtype=np.int64)
    return (np.arange(wpv, dtype=np.int64)[:, None] * n + v[None, :]).ravel()


@dataclass(frozen=True)
class BlockShard:
    """The start vertices of blocks part, part + parts, ... of 2^bits
    consecutive vertices (WharfMH.set_shard_blocks, include/wharf_gpu.h).
    Contiguous ranges of an RMAT graph re-walk at rates 10-12 % apart (hub
    regions vs the rest); dealing 64 Ki-vertex blocks round-robin
    gives every rank the same mix."""
    part: int
    parts: int
    bits: int
    n: int

    def blocks(self):
        B = 1 << self.bits
        nb = -(-self.n // B)
        return [(q * B, min(self.n, (q + 1) * B)) for q in range(self.part, nb, self.parts)]

    def size(self) -> int:
        return sum(b - a for a, b in self.blocks())

    def vertices(self) -> np.ndarray:
        return np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in self.blocks()] or
                              [np.zeros(0, dtype=np.int64)])


def block_shards(n: int, parts: int, bits: int = 16):
    return [BlockShard(g, parts, bits, n) for g in range(parts)]


def shard_size(shard) -> int:
    """Start vertices of a shard: a (lo, hi) range or a BlockShard."""
    return shard.size() if isinstance(shard, BlockShard) else shard[1] - shard[0]


def shard_walk_ids_of(shard, n: int, wpv: int) -> np.ndarray:
    """shard_walk_ids for either kind of shard (local order: r-major, then ascending v)."""
    if not isinstance(shard, BlockShard):
        return shard_walk_ids(n, wpv, *shard)
    v = shard.vertices()
    return (np.arange(wpv, dtype=np.int64)[:, None] * n + v[None, :]).ravel()


def allgatherv_corpus(local_walks, shards, n: int, wpv: int, group=None):
    """Reassemble the global corpus [n*wpv, L] (row = walk id) on every rank.

    local_walks: torch tensor [W_local, L] (walk-major, this rank's export
    order: round-major, rows r*(hi-lo) + (v-lo)).  Returns a tensor on
    local_walks.device.  Row r*n + v of the output holds walk r*n + v.

    Each round of a peer's shard is a contiguous row block of the output
    (rows r*n + lo .. r*n + hi), so receives land in place: the only buffer
    is the output itself (a staging copy of every part would double the
    footprint — at 8 ranks of weak scaling the whole corpus is 107 GB).  One
    batch of point-to-point operations per round keeps every peer link busy
    at once; a round's blocks are hi-lo rows per peer.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    L = local_walks.shape[1]
    lo_r, hi_r = shards[rank]
    own = hi_r - lo_r
    if local_walks.shape[0] != own * wpv:
        raise ValueError(f"rank {rank}: {local_walks.shape[0]} local walks, expected {own} x {wpv} rounds")
    local_walks = local_walks.contiguous()
    out = torch.empty((n * wpv, L), dtype=local_walks.dtype, device=local_walks.device)
    ov = out.view(wpv, n, L)
    ov[:, lo_r:hi_r, :] = local_walks.view(wpv, own, L)
    for r in range(wpv):
        ops = []
        for peer in range(world):
            if peer == rank:
                continue
            lo, hi = shards[peer]
            if own:
                ops.append(dist.P2POp(dist.isend, local_walks[r * own:(r + 1) * own], peer, group))
            if hi > lo:
                ops.append(dist.P2POp(dist.irecv, ov[r, lo:hi], peer, group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
    return out


def local_rows_to_global(lo: int, hi: int, n: int, first: int, count: int):
    """Global walk-id runs of local rows [first, first + count) of shard [lo, hi)
    (local row i = round i // (hi-lo), vertex lo + i % (hi-lo)):
    [(local_first, count, global_first)], each run inside one round."""
    own = hi - lo
    runs, i, end = [], first, first + count
    while i < end:
        r, j = divmod(i, own)
        c = min(end - i, own - j)
        runs.append((i, c, r * n + lo + j))
        i += c
    return runs


def shard_rows_to_global(shard, n: int, first: int, count: int):
    """local_rows_to_global for either kind of shard: runs of consecutive walk
    ids (a BlockShard's run also ends at each of its blocks)."""
    if not isinstance(shard, BlockShard):
        return local_rows_to_global(shard[0], shard[1], n, first, count)
    B = 1 << shard.bits
    own = shard.size()
    runs, i, end = [], first, first + count
    while i < end:
        r, j = divmod(i, own)
        q, o = divmod(j, B)                      # the part's q-th block, offset o
        v = (q * shard.parts + shard.part) * B + o
        c = min(end - i, own - j, B - o)
        runs.append((i, c, r * n + v))
        i += c
    return runs


def gather_corpus_chunked(read_local, shards, n: int, wpv: int, L: int, rows_per_rank: int, sink=None,
                          root: int | None = None, group=None, device="cpu", dtype=None, on_oom=None):
    """Bounded-memory corpus gather: all-gatherv (root None) or gatherv to `root`.

    shards: per rank, a (lo, hi) start-vertex range or a BlockShard;
    read_local(first, count, out): writes this rank's walk-major local rows
        [first, first + count) into the contiguous 2-D tensor `out` ([count, L]);
    sink(chunk, segments): called on every receiving rank once per chunk, with
        chunk = [R, L] tensor (valid until sink returns) and segments =
        [(chunk_row, count, global_walk_id_first)] covering its R rows.
    At most rows_per_rank * world rows (rows_per_rank on a sending-only rank)
    are resident.  rows_per_rank may differ between ranks (each derives it from
    its own free memory): the chunk size used is the minimum over the ranks,
    agreed before the first exchange, because chunk boundaries and receive
    sizes must be the same on every rank.  A failure on one rank (buffer,
    read_local, sink) is agreed before the next exchange and raises
    RankFailure on every rank.  on_oom (e.g. WharfMH.release_caches): called
    once when the chunk buffer does not fit, before one more try (the
    library's droppable caches make room for it).  Returns {"chunks",
    "rows_per_rank", "bytes_received", "bytes_sent"} of this rank.
    """
    import torch
    import torch.distributed as dist

    dtype = dtype or torch.int32
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    owns = [shard_size(sh) * wpv for sh in shards]
    if len(owns) != world:
        raise ValueError(f"{len(owns)} shards for a world of {world}")
    K = max(1, agree_min(max(1, int(rows_per_rank)), group, device))
    nchunks = -(-max(owns) // K) if max(owns) else 0
    receives = root is None or rank == root
    buf, err = None, None
    try:
        buf = alloc_or_reclaim(lambda: torch.empty((K * (world if receives else 1), L), dtype=dtype, device=device),
                               on_oom, rank)
    except Exception as ex:   # noqa: BLE001 (agreed below: every rank abandons the gather together)
        err = ex
    agree(err, "corpus gather buffer", group, device)
    cuda = buf.is_cuda
    stats = {"chunks": nchunks, "rows_per_rank": K, "bytes_received": 0, "bytes_sent": 0}
    for c in range(nchunks):
        parts = [(min(c * K, own), min((c + 1) * K, own)) for own in owns]
        cnt = [b - a for a, b in parts]
        base, acc = [], 0
        for g in range(world):
            base.append(acc if receives else 0)
            if receives:
                acc += cnt[g]
        my0 = base[rank] if receives else 0
        mine = buf[my0:my0 + cnt[rank]]
        if cnt[rank] and err is None:
            try:
                read_local(parts[rank][0], cnt[rank], mine)
            except Exception as ex:   # noqa: BLE001
                err = ex
        agree(err, f"corpus gather chunk {c}", group, device)
        ops = []
        for peer in range(world):
            if peer == rank:
                continue
            peer_receives = root is None or peer == root
            if cnt[rank] and peer_receives:
                ops.append(dist.P2POp(dist.isend, mine, peer, group))
                stats["bytes_sent"] += mine.numel() * mine.element_size()
            if receives and cnt[peer]:
                dst = buf[base[peer]:base[peer] + cnt[peer]]
                ops.append(dist.P2POp(dist.irecv, dst, peer, group))
                stats["bytes_received"] += dst.numel() * dst.element_size()
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if cuda:   # the library's export of the next chunk runs on its own stream: the buffer must be free
            torch.cuda.current_stream(buf.device).synchronize()
        if receives and sink is not None:
            segs = []
            for g, sh in enumerate(shards):
                if cnt[g]:
                    for lf, k, gf in shard_rows_to_global(sh, n, parts[g][0], cnt[g]):
                        segs.append((base[g] + lf - parts[g][0], k, gf))
            try:
                sink(buf[:sum(cnt)], segs)
                if cuda:
                    torch.cuda.current_stream(buf.device).synchronize()
            except Exception as ex:   # noqa: BLE001 (agreed before the next exchange or at the end)
                err = ex
    agree(err, "corpus gather sink", group, device)
    return stats


_K1 = 0x9E3779B97F4A7C15 - (1 << 64)   # as signed int64 (torch has no uint64 arithmetic)
_K2 = 0xBF58476D1CE4E5B9 - (1 << 64)


def corpus_checksum(rows, global_first: int, L: int, block_rows: int = 1 << 16):
    """Order-independent checksum of walk-major rows whose first row is walk id
    `global_first` (consecutive ids): sum over entries of (value + 1) * mix(id*L + pos),
    int64 wrapping (mod 2^64).  The checksum of a whole corpus is the sum of its
    pieces', so the sum of every rank's local checksum must equal the checksum
    of what a gather delivered (the full-size property of bench.py's gather)."""
    import torch

    total = torch.zeros((), dtype=torch.int64, device=rows.device)
    pos = torch.arange(L, dtype=torch.int64, device=rows.device)
    for r0 in range(0, rows.shape[0], block_rows):
        blk = rows[r0:r0 + block_rows]
        ids = torch.arange(global_first + r0, global_first + r0 + blk.shape[0], dtype=torch.int64, device=rows.device)
        h = (ids[:, None] * L + pos[None, :]) * _K1
        h = (h ^ (h >> 31)) * _K2
        total += (((blk.to(torch.int64) & 0xFFFFFFFF) + 1) * h).sum()
    return total


def local_corpus_checksum(read_local, shard, n: int, wpv: int, L: int, rows_per_call: int, device="cpu"):
    """corpus_checksum of this rank's own walks (shard: a (lo, hi) range or a
    BlockShard), read chunk by chunk."""
    import torch

    own = shard_size(shard) * wpv
    buf = torch.empty((max(1, min(rows_per_call, own)), L), dtype=torch.int32, device=device)
    total = torch.zeros((), dtype=torch.int64, device=device)
    for f in range(0, own, buf.shape[0]):
        k = min(buf.shape[0], own - f)
        read_local(f, k, buf[:k])
        for lf, c, gf in shard_rows_to_global(shard, n, f, k):
            total += corpus_checksum(buf[lf - f:lf - f + c], gf, L)
    return total
