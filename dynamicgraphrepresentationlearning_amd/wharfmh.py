"""Python host mirror of dygrl::WharfMH (graph/wharfmh.h) over the HIP C ABI.

Method names, argument order and meaning follow the reference class so driver
code ports line by line:

    reference (C++)                                     here
    ------------------------------------------------    -----------------------------------------
    WharfMH(n, m, offsets, edges)        wharfmh.h:58   WharfMH(n, m, offsets, edges, config=...)
    WharfMH(n, m)                        wharfmh.h:26   WharfMH(n, 0)
    number_of_vertices / number_of_edges :117 / :130    same
    generate_initial_random_walks        :250           same
    insert_edges_batch(m, edges, sorted, remove_dups,   insert_edges_batch(edges, sorted, remove_dups,
        nn, apply_walk_updates, run_seq) :439               nn, apply_walk_updates, run_seq)
    delete_edges_batch                   :588           same
    walk(wid) -> "v0 v1 ... "            :365           same
    vertex_at_walk(wid, pos)             :404           same
    flatten_graph                        :175           flatten_graph() -> (offsets[n+1], targets[m])
    destroy / destroy_index              :228 / :237    same
    config::* globals                    globals.h      WharfConfig (per instance)

Errors raise RuntimeError (the reference calls std::exit(1) / asserts).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import weakref
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

DEEPWALK, NODE2VEC = L.WHARF_DEEPWALK, L.WHARF_NODE2VEC
RANDOM, BURNIN, WEIGHT = L.WHARF_INIT_RANDOM, L.WHARF_INIT_BURNIN, L.WHARF_INIT_WEIGHT
SENTINEL = L.SENTINEL


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


@dataclass
class WharfConfig:
    """config::* (config/globals.h:7-29) plus the MH seed and the walk shard."""

    walks_per_vertex: int = 10
    walk_length: int = 80
    model: int = NODE2VEC          # globals.h:13 (in deterministic mode both models give the same walks)
    paramP: float = 4.0
    paramQ: float = 1.0
    sampler_init: int = WEIGHT
    deterministic: bool = True
    seed: int = 0x5EED
    shard_lo: int = 0
    shard_hi: int = 0

    def to_c(self) -> L.wharf_config:
        c = L.wharf_config()
        c.walks_per_vertex = self.walks_per_vertex
        c.walk_length = self.walk_length
        c.model = self.model
        c.paramP = self.paramP
        c.paramQ = self.paramQ
        c.sampler_init = self.sampler_init
        c.deterministic = int(bool(self.deterministic))
        c.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        c.shard_lo = self.shard_lo
        c.shard_hi = self.shard_hi
        return c


class WharfMH:
    """Streaming random-walk engine: CSR snapshot + position-major walk matrix in HBM."""

    # every live handle (weakly): destroy_all() frees the device memory of handles a caller lost
    # track of, e.g. a test that failed with its handle still referenced by the traceback
    _live: "weakref.WeakSet[WharfMH]" = weakref.WeakSet()

    @classmethod
    def destroy_all(cls) -> int:
        n = 0
        for g in list(cls._live):
            if getattr(g, "_h", None):
                g.destroy()
                n += 1
        return n

    def __init__(self, n: int, m: int = 0, offsets=None, edges=None, config: WharfConfig | None = None,
                 device: int = 0, _handle=None):
        WharfMH._live.add(self)
        # a copy: set_shard records the shard here, not in the caller's object
        self.config = dataclasses.replace(config) if config is not None else WharfConfig()
        self._cfg = self.config.to_c()
        self.device = device
        if _handle is not None:
            self._h = _handle
            return
        h = C.c_void_p()
        if m == 0 and offsets is None:
            rc = L.lib.wharf_create_empty(C.byref(self._cfg), n, device, C.byref(h))
        else:
            off = np.ascontiguousarray(offsets, dtype=np.uint64)[:n]
            tgt = np.ascontiguousarray(edges, dtype=np.uint32)
            if len(off) != n or len(tgt) < m:
                raise ValueError("offsets must have n entries and edges m entries")
            rc = L.lib.wharf_create(C.byref(self._cfg), n, m, _ptr(off), _ptr(tgt), device, C.byref(h))
        L.check(rc, None, "wharf_create")
        self._h = h

    @classmethod
    def from_csr(cls, offsets_np1, targets, config: WharfConfig | None = None, device: int = 0) -> "WharfMH":
        off = np.asarray(offsets_np1, dtype=np.uint64)
        return cls(len(off) - 1, int(off[-1]), off[:-1], targets, config=config, device=device)

    @classmethod
    def from_rmat(cls, n: int, edges_number: int, vertices_number: int | None = None, seed: int = 0,
                  a: float = 0.5, b: float = 0.2, c: float = 0.1, config: WharfConfig | None = None,
                  device: int = 0) -> "WharfMH":
        """Undirected RMAT base graph built on the device:
        generate_batch_of_edges(edges_number, vertices_number, seed, false, false) (utility.h:55)."""
        config = config or WharfConfig()
        cfg = config.to_c()
        h = C.c_void_p()
        vn = vertices_number if vertices_number is not None else 2 * n
        rc = L.lib.wharf_create_rmat(C.byref(cfg), n, edges_number, vn, seed, a, b, c, device, C.byref(h))
        L.check(rc, None, "wharf_create_rmat")
        return cls(n, config=config, device=device, _handle=h)

    # -- lifetime ---------------------------------------------------------------------------
    def destroy(self) -> None:
        if getattr(self, "_h", None):
            L.lib.wharf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def destroy_index(self) -> None:
        L.check(L.lib.wharf_destroy_index(self._h), self._h, "destroy_index")

    def release_caches(self) -> int:
        """Free the droppable device caches (the reverse-slot index) for an allocation of the
        caller's that ran out of device memory; results are unchanged.  Returns the bytes freed."""
        freed = C.c_uint64(0)
        L.check(L.lib.wharf_release_caches(self._h, C.byref(freed)), self._h, "release_caches")
        return int(freed.value)

    # -- queries ----------------------------------------------------------------------------
    def number_of_vertices(self) -> int:
        v = C.c_uint64()
        L.check(L.lib.wharf_number_of_vertices(self._h, C.byref(v)), self._h, "number_of_vertices")
        return v.value

    def number_of_edges(self) -> int:
        v = C.c_uint64()
        L.check(L.lib.wharf_number_of_edges(self._h, C.byref(v)), self._h, "number_of_edges")
        return v.value

    def shard(self):
        lo, hi, w = C.c_uint64(), C.c_uint64(), C.c_uint64()
        L.check(L.lib.wharf_shard(self._h, C.byref(lo), C.byref(hi), C.byref(w)), self._h, "shard")
        return lo.value, hi.value, w.value

    def set_shard(self, lo: int, hi: int) -> None:
        """Own the walks of start vertices [lo, hi) (drops current walks)."""
        L.check(L.lib.wharf_set_shard(self._h, lo, hi), self._h, "set_shard")
        self.config.shard_lo, self.config.shard_hi = lo, hi

    def set_shard_blocks(self, part: int, parts: int, block_bits: int = 16) -> None:
        """Own the walks of the start vertices in blocks part, part + parts, ...
        of 2^block_bits consecutive vertices (drops current walks): every part
        gets the same mix of the graph's regions (distributed.BlockShard)."""
        L.check(L.lib.wharf_set_shard_blocks(self._h, part, parts, block_bits), self._h, "set_shard_blocks")
        self.config.shard_lo, self.config.shard_hi = 0, 0

    def shard_blocks(self):
        """(part, parts, block_bits); (0, 1, 0) for a contiguous shard."""
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        L.check(L.lib.wharf_shard_blocks(self._h, C.byref(a), C.byref(b), C.byref(c)), self._h, "shard_blocks")
        return a.value, b.value, c.value

    def apply_shard(self, shard) -> None:
        """A shard of distributed.py: a (lo, hi) start-vertex range or a BlockShard."""
        if isinstance(shard, tuple):
            self.set_shard(*shard)
        else:
            self.set_shard_blocks(shard.part, shard.parts, shard.bits)

    @property
    def number_of_walks(self) -> int:
        return self.shard()[2]

    def stats(self) -> dict:
        s = L.wharf_stats()
        L.check(L.lib.wharf_get_stats(self._h, C.byref(s)), self._h, "stats")
        return {k: getattr(s, k) for k, _ in L.wharf_stats._fields_}

    def memory_footprint(self, verbose: bool = True) -> dict:
        """WharfMH::memory_footprint (wharfmh.h:928-998): device bytes by role
        (printed like the reference when verbose)."""
        r = L.wharf_memory()
        L.check(L.lib.wharf_memory_footprint(self._h, C.byref(r)), self._h, "memory_footprint")
        d = {f: getattr(r, f) for f, _ in r._fields_}
        if verbose:
            gb = lambda b: f"{b / 2**20:.2f} MB = {b / 2**30:.3f} GB"
            print(f"\nGraph: \n\tVertices: {d['n']}, Edges: {d['m']}")
            for k, name in (("csr_bytes", "CSR"), ("records_bytes", "Row records"), ("walks_bytes", "Walks"),
                            ("samplers_bytes", "Samplers"), ("edge_hash_bytes", "Edge hash"),
                            ("update_buffers_bytes", "Update buffers"), ("scratch_bytes", "Scratch")):
                print(f"{name}: \n\tMemory usage: {gb(d[k])}")
            print(f"Total memory used: \n\t{gb(d['total_bytes'])}\n")
        return d

    def flatten_graph(self):
        n, m = self.number_of_vertices(), self.number_of_edges()
        off = np.zeros(n + 1, dtype=np.uint64)
        adj = np.zeros(max(m, 1), dtype=np.uint32)
        L.check(L.lib.wharf_get_graph(self._h, _ptr(off), _ptr(adj)), self._h, "flatten_graph")
        return off, adj[:m]

    def offsets(self) -> np.ndarray:
        """CSR row offsets only (n + 1 u64; the targets stay on the device)."""
        off = np.zeros(self.number_of_vertices() + 1, dtype=np.uint64)
        L.check(L.lib.wharf_get_graph(self._h, _ptr(off), None), self._h, "offsets")
        return off

    # -- the walk path ------------------------------------------------------------------------
    def generate_initial_random_walks(self) -> None:
        L.check(L.lib.wharf_generate(self._h), self._h, "generate_initial_random_walks")

    def _update(self, fn, edges, sorted, remove_dups, apply_walk_updates, out) -> np.ndarray:
        e = np.ascontiguousarray(np.asarray(edges, dtype=np.uint32).reshape(-1, 2))
        flags = (L.WHARF_SORTED if sorted else 0) | (L.WHARF_REMOVE_DUPS if remove_dups else 0) | \
                (L.WHARF_APPLY_WALK_UPDATES if apply_walk_updates else 0)
        W = max(self.number_of_walks, 1)
        if out is not None and getattr(out, "is_cuda", False):
            # device output (torch int32/uint32 tensor on this handle's GPU): ids stay in HBM
            import torch
            if out.dtype not in (torch.int32, torch.uint32) or out.numel() < W or not out.is_contiguous():
                raise ValueError("device out must be a contiguous 32-bit tensor with >= number_of_walks entries")
            cnt = C.c_uint64()
            L.check(fn(self._h, len(e), _ptr(e), flags | L.WHARF_AFFECTED_DEVICE, C.c_void_p(out.data_ptr()),
                       C.byref(cnt)), self._h, fn.__name__)
            return out[: cnt.value]
        buf = out if out is not None else np.empty(W, dtype=np.uint32)
        if buf.dtype != np.uint32 or len(buf) < W or not buf.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint32 array with >= number_of_walks entries")
        cnt = C.c_uint64()
        L.check(fn(self._h, len(e), _ptr(e), flags, _ptr(buf), C.byref(cnt)), self._h, fn.__name__)
        return buf[: cnt.value]

    def insert_edges_batch(self, edges, sorted: bool = False, remove_dups: bool = False, nn: int | None = None,
                           apply_walk_updates: bool = True, run_seq: bool = False, out=None) -> np.ndarray:
        """wharfmh.h:439.  `edges`: (m, 2) (src, dst).  Returns the affected walk ids
        (ascending; a view of `out` when given — a torch tensor on the GPU keeps
        them in HBM, WHARF_AFFECTED_DEVICE).  `nn` and `run_seq` are CPU
        sort/scheduling hints of the reference and have no effect here; the
        caller's buffer is not modified."""
        return self._update(L.lib.wharf_insert_edges, edges, sorted, remove_dups, apply_walk_updates, out)

    def delete_edges_batch(self, edges, sorted: bool = False, remove_dups: bool = False, nn: int | None = None,
                           apply_walk_updates: bool = True, run_seq: bool = False, out=None) -> np.ndarray:
        """wharfmh.h:588."""
        return self._update(L.lib.wharf_delete_edges, edges, sorted, remove_dups, apply_walk_updates, out)

    def batch_walk_update(self, sources, out=None) -> np.ndarray:
        """wharfmh.h:733: re-walk every walk from its first position holding a
        vertex of `sources` (the vertex set of the reference's MapOfChanges) on
        the current graph; returns the affected walk ids (ascending).  After an
        update with apply_walk_updates=False, passing that batch's sources gives
        exactly the walks the update would have produced."""
        src = np.ascontiguousarray(np.asarray(sources, dtype=np.uint32).reshape(-1))
        buf = out if out is not None else np.empty(max(self.number_of_walks, 1), dtype=np.uint32)
        if buf.dtype != np.uint32 or len(buf) < self.number_of_walks or not buf.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint32 array with >= number_of_walks entries")
        cnt = C.c_uint64()
        L.check(L.lib.wharf_batch_walk_update(self._h, _ptr(src), len(src), 0, _ptr(buf), C.byref(cnt)), self._h,
                "batch_walk_update")
        return buf[: cnt.value]

    def walk(self, walk_id: int) -> str:
        """WharfMH::walk (wharfmh.h:365): "v0 v1 ... " with a trailing space."""
        n = C.c_size_t()
        L.check(L.lib.wharf_walk_string(self._h, walk_id, None, 0, C.byref(n)), self._h, "walk")
        buf = C.create_string_buffer(n.value + 1)
        L.check(L.lib.wharf_walk_string(self._h, walk_id, buf, n.value + 1, C.byref(n)), self._h, "walk")
        return buf.value.decode()

    def walk_vertices(self, walk_id: int) -> np.ndarray:
        out = np.zeros(self.config.walk_length, dtype=np.uint32)
        ln = C.c_uint32()
        L.check(L.lib.wharf_walk(self._h, walk_id, _ptr(out), C.byref(ln)), self._h, "walk")
        return out[: ln.value]

    def vertex_at_walk(self, walk_id: int, position: int) -> int:
        v = C.c_uint32()
        L.check(L.lib.wharf_vertex_at_walk(self._h, walk_id, position, C.byref(v)), self._h, "vertex_at_walk")
        return v.value

    def walks(self, layout: str = "walk") -> np.ndarray:
        """The owned corpus, SENTINEL-padded: 'walk' -> [walks][L], 'position' -> [L][walks]."""
        W, Lw = self.number_of_walks, self.config.walk_length
        if layout == "walk":
            out = np.zeros((W, Lw), dtype=np.uint32)
            L.check(L.lib.wharf_export_walks(self._h, _ptr(out), 0), self._h, "export_walks")
        else:
            out = np.zeros((Lw, W), dtype=np.uint32)
            L.check(L.lib.wharf_export_walks(self._h, _ptr(out), 1), self._h, "export_walks")
        return out

    def walk_ids(self) -> np.ndarray:
        out = np.zeros(max(self.number_of_walks, 1), dtype=np.uint32)
        L.check(L.lib.wharf_walk_ids(self._h, _ptr(out)), self._h, "walk_ids")
        return out[: self.number_of_walks]

    def export_walks_device(self, device_ptr: int, layout: str = "walk") -> None:
        L.check(L.lib.wharf_export_walks_device(self._h, C.c_void_p(device_ptr), 0 if layout == "walk" else 1),
                self._h, "export_walks_device")

    def export_walk_rows(self, first: int, count: int, out=None) -> np.ndarray:
        """Walk-major rows [first, first + count) of walks() (the handle's owned
        walks in ascending id), one bounded chunk of the corpus.  `out`: a host
        uint32 array of >= count * L entries, or a contiguous 32-bit torch tensor
        on this handle's GPU (the rows stay in HBM: the chunked corpus gather)."""
        Lw = self.config.walk_length
        if out is not None and getattr(out, "is_cuda", False):
            import torch
            if out.dtype not in (torch.int32, torch.uint32) or out.numel() < count * Lw or not out.is_contiguous():
                raise ValueError("device out must be a contiguous 32-bit tensor with >= count * walk_length entries")
            L.check(L.lib.wharf_export_walk_rows_device(self._h, first, count, C.c_void_p(out.data_ptr())), self._h,
                    "export_walk_rows_device")
            return out
        buf = out if out is not None else np.empty((count, Lw), dtype=np.uint32)
        if buf.dtype != np.uint32 or buf.size < count * Lw or not buf.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint32 array with >= count * walk_length entries")
        L.check(L.lib.wharf_export_walk_rows(self._h, first, count, _ptr(buf)), self._h, "export_walk_rows")
        return buf

    def write_corpus(self, path: str, walk_ids=None, append: bool = False) -> None:
        """Text corpus for yskip (vertex-classification.cpp:142-150): one
        WharfMH::walk line per walk; all owned walks, or `walk_ids` in order."""
        if walk_ids is None:
            rc = L.lib.wharf_write_corpus(self._h, path.encode(), None, 0, int(append))
        else:
            ids = np.ascontiguousarray(walk_ids, dtype=np.uint32)
            rc = L.lib.wharf_write_corpus(self._h, path.encode(), _ptr(ids), len(ids), int(append))
        L.check(rc, self._h, "write_corpus")

    def inverted_index(self, v0: int | None = None, v1: int | None = None):
        """Per-vertex ascending (key = wid*L + pos, next) lists (walks/inverted_index.h):
        returns (counts, keys, nexts) for every vertex, or for the vertex window
        [v0, v1) only (counts[v1 - v0]).  Keys are 64-bit."""
        sz = C.c_uint64()
        if v0 is None and v1 is None:
            L.check(L.lib.wharf_index_size(self._h, C.byref(sz)), self._h, "index_size")
            counts = np.zeros(self.number_of_vertices(), dtype=np.uint64)
        else:
            v0 = 0 if v0 is None else v0
            v1 = self.number_of_vertices() if v1 is None else v1
            L.check(L.lib.wharf_index_size_range(self._h, v0, v1, C.byref(sz)), self._h, "index_size_range")
            counts = np.zeros(max(v1 - v0, 1), dtype=np.uint64)
        keys = np.zeros(max(sz.value, 1), dtype=np.uint64)
        nexts = np.zeros(max(sz.value, 1), dtype=np.uint32)
        if v0 is None and v1 is None:
            L.check(L.lib.wharf_export_index(self._h, _ptr(counts), _ptr(keys), _ptr(nexts)), self._h, "export_index")
        else:
            L.check(L.lib.wharf_export_index_range(self._h, v0, v1, _ptr(counts), _ptr(keys), _ptr(nexts)), self._h,
                    "export_index_range")
            counts = counts[: v1 - v0]
        return counts, keys[: sz.value], nexts[: sz.value]

    def compressed_walks(self):
        """The pairing-encoded CompressedWalks form (walks/compressed_walks.h:49-66):
        per vertex, Szudzik(wid*L + pos, next) of its stored positions, ascending,
        as 64-bit values.  Returns (counts[n], paired)."""
        sz = C.c_uint64()
        L.check(L.lib.wharf_index_size(self._h, C.byref(sz)), self._h, "index_size")
        counts = np.zeros(self.number_of_vertices(), dtype=np.uint64)
        paired = np.zeros(max(sz.value, 1), dtype=np.uint64)
        L.check(L.lib.wharf_export_index_paired(self._h, _ptr(counts), _ptr(paired)), self._h, "export_index_paired")
        return counts, paired[: sz.value]


def generate_batch_of_edges(edges_number: int, vertices_number: int, batch_seed: int, self_loops: bool = False,
                            directed: bool = True, a: float = 0.5, b: float = 0.2, c: float = 0.1,
                            device: int = 0) -> np.ndarray:
    """utility::generate_batch_of_edges (utils/utility.h:55-146) on the device -> (k, 2) uint32."""
    cap = edges_number * (1 if directed else 2)
    out = np.zeros((max(cap, 1), 2), dtype=np.uint32)
    cnt = C.c_uint64()
    L.check(L.lib.wharf_generate_batch_of_edges(device, edges_number, vertices_number, batch_seed, int(self_loops),
                                                int(directed), a, b, c, _ptr(out), C.byref(cnt)),
            None, "generate_batch_of_edges")
    return out[: cnt.value].copy()


def read_adjacency_graph(path: str):
    """read_unweighted_graph (common/IO.h:67-106) -> (offsets[n+1] u64, targets[m] u32)."""
    n, m = C.c_uint64(), C.c_uint64()
    L.check(L.lib.wharf_read_adjacency_graph(path.encode(), C.byref(n), C.byref(m), None, None), None,
            "read_adjacency_graph")
    off = np.zeros(n.value + 1, dtype=np.uint64)
    adj = np.zeros(max(m.value, 1), dtype=np.uint32)
    L.check(L.lib.wharf_read_adjacency_graph(path.encode(), C.byref(n), C.byref(m), _ptr(off), _ptr(adj)), None,
            "read_adjacency_graph")
    off[n.value] = m.value
    return off, adj[: m.value]


def snap_to_adj(snap_path: str, adj_path: str, symmetric: bool = True) -> None:
    """experiments/bin/SNAPtoAdj [-s]: SNAP edge list -> AdjacencyGraph text."""
    L.check(L.lib.wharf_snap_to_adj(snap_path.encode(), adj_path.encode(), int(symmetric)), None, "snap_to_adj")


def szudzik64_pair(x, y, device: int = 0) -> np.ndarray:
    """pairings::Szudzik<uint64_t>::pair (walks/pairings.h:124-176), elementwise on the device."""
    x = np.ascontiguousarray(x, dtype=np.uint64).copy()
    y = np.ascontiguousarray(y, dtype=np.uint64).copy()
    z = np.zeros_like(x)
    L.check(L.lib.wharf_szudzik64(device, 0, len(x), _ptr(x), _ptr(y), _ptr(z)), None, "szudzik64")
    return z


def szudzik64_unpair(z, device: int = 0):
    """pairings::Szudzik<uint64_t>::unpair (walks/pairings.h:197-210) with an exact integer sqrt."""
    z = np.ascontiguousarray(z, dtype=np.uint64).copy()
    x = np.zeros_like(z)
    y = np.zeros_like(z)
    L.check(L.lib.wharf_szudzik64(device, 1, len(z), _ptr(x), _ptr(y), _ptr(z)), None, "szudzik64")
    return x, y
