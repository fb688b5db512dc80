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
"""
from __future__ import annotations

import numpy as np


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
