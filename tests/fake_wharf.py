"""A host-only stand-in for the library and for torch.cuda, so that bench.py's
multi-rank job logic (phases, agreed failures, the bounded corpus gather) runs
under gloo on a machine without a GPU (tests/test_collective_safety.py).

The fake handle's walks are a pure function of (global walk id, position), so
what a gather delivers is checkable; it does no walking.  Nothing here is used
by the product or by any GPU test."""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch


def walk_value(gid, pos):
    """The fake corpus: entry (walk gid, position pos)."""
    return (np.asarray(gid, dtype=np.int64) * 131 + np.asarray(pos, dtype=np.int64) * 7) % (1 << 31)


class FakeHandle:
    def __init__(self, n: int, cfg):
        self.n, self.cfg = n, cfg
        self.shard = (0, n)
        self.number_of_walks = n * cfg.walks_per_vertex
        self._steps = 0

    def offsets(self):
        return (np.arange(self.n + 1, dtype=np.uint64) * 2)

    def _set(self, shard):
        from dynamicgraphrepresentationlearning_amd.distributed import shard_size
        self.shard = shard
        self.number_of_walks = shard_size(shard) * self.cfg.walks_per_vertex

    def apply_shard(self, shard):
        self._set(shard)

    def set_shard(self, lo, hi):
        self._set((lo, hi))

    def generate_initial_random_walks(self):
        self._steps = self.number_of_walks * (self.cfg.walk_length - 1)

    def stats(self):
        return {"last_walk_kernel_ms": 1.0, "steps": self._steps, "last_anchor_inits": 0,
                "last_graph_update_ms": 0.1, "last_walk_update_ms": 0.5, "last_csr_move_ms": 0.01,
                "affected": self.number_of_walks // 2, "accepts": self._steps}

    def number_of_edges(self):
        return 2 * self.n

    def memory_footprint(self, verbose=False):
        return {"total_bytes": 1}

    def export_walk_rows(self, first, count, out):
        from dynamicgraphrepresentationlearning_amd.distributed import shard_rows_to_global
        L = self.cfg.walk_length
        for lf, c, gf in shard_rows_to_global(self.shard, self.n, first, count):
            vals = walk_value(np.arange(gf, gf + c)[:, None], np.arange(L)[None, :])
            out[lf - first:lf - first + c].copy_(torch.from_numpy(vals.astype(np.int32)))

    def insert_edges_batch(self, batch, remove_dups=True, out=None, apply_walk_updates=True):
        self._steps = self.number_of_walks
        return np.zeros(0, dtype=np.uint32)

    delete_edges_batch = insert_edges_batch

    released = 0   # release_caches calls (class-wide: the tests read it after a job)

    def release_caches(self):
        FakeHandle.released += 1
        return 0

    def destroy(self):
        pass


class _WharfMH:
    @staticmethod
    def from_rmat(n, samples, nn, seed=0, config=None, device=None):
        return FakeHandle(n, config)


FakeW = SimpleNamespace(
    WharfConfig=lambda **kw: SimpleNamespace(**kw), DEEPWALK=0, NODE2VEC=1, WharfMH=_WharfMH,
    generate_batch_of_edges=lambda m, n, seed, self_loops, directed, device=None: np.zeros((8, 2), dtype=np.uint32))


class _Cuda:
    free = 8 << 30

    @staticmethod
    def synchronize(*a, **k):
        pass

    @classmethod
    def mem_get_info(cls, *a):
        return (cls.free, cls.free)

    @staticmethod
    def empty_cache():
        pass


class TorchProxy:
    """torch, with device tensors made on the host and torch.cuda's calls no-ops."""
    cuda = _Cuda

    def __getattr__(self, k):
        return getattr(torch, k)

    @staticmethod
    def empty(*a, device=None, **k):
        if device is not None and str(device).startswith("cuda"):
            device = "cpu"
        return torch.empty(*a, device=device, **k)
