"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the C oracle (wharf_oracle.c).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker.  The product package
(``dynamicgraphrepresentationlearning_amd``) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
SENT = 0xFFFFFFFE

DEEPWALK, NODE2VEC = 0, 1
INIT_RANDOM, INIT_BURNIN, INIT_WEIGHT = 0, 1, 2
SORTED, REMOVE_DUPS, APPLY_WALK_UPDATES = 1, 2, 4

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u64, u32, p = C.c_uint64, C.c_uint32, C.c_void_p
        L.wo_random_init.argtypes = [u64, p]
        L.wo_lrand.argtypes = [p]
        L.wo_lrand.restype = u64
        L.wo_drand.argtypes = [p]
        L.wo_drand.restype = C.c_double
        L.wo_hash32.argtypes = [u32]
        L.wo_hash32.restype = u32
        L.wo_hash64.argtypes = [u64]
        L.wo_hash64.restype = u64
        L.wo_philox4x32_10.argtypes = [p, p, p]
        L.wo_generate_batch_of_edges.argtypes = [u64, u64, u64, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, p]
        L.wo_generate_batch_of_edges.restype = u64
        L.wo_szudzik32_pair.argtypes = [u32, u32]
        L.wo_szudzik32_pair.restype = u32
        L.wo_szudzik32_unpair.argtypes = [u32, p, p]
        L.wo_szudzik64_pair.argtypes = [u64, u64]
        L.wo_szudzik64_pair.restype = u64
        L.wo_szudzik64_unpair.argtypes = [u64, p, p]
        L.wo_create.argtypes = [u64, u64, p, p, u32, u32, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, u64]
        L.wo_create.restype = p
        L.wo_free.argtypes = [p]
        L.wo_generate.argtypes = [p]
        L.wo_update.argtypes = [p, C.c_int, u64, p, u32, p]
        L.wo_update.restype = u64
        for f in ("wo_num_edges", "wo_num_walks", "wo_get_accepts", "wo_get_steps", "wo_index_size"):
            getattr(L, f).argtypes = [p]
            getattr(L, f).restype = u64
        L.wo_get_csr.argtypes = [p, p, p]
        L.wo_get_walks.argtypes = [p, p]
        L.wo_get_walks_range.argtypes = [p, u64, u64, p]
        L.wo_export_index.argtypes = [p, p, p, p]
        L.wo_time_generate_range.argtypes = [p, u64, u64, C.c_int]
        L.wo_time_generate_range.restype = C.c_double
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Random:
    """utility::Random (utils/utility.h:152-223)."""

    def __init__(self, seed: int):
        self.s = np.zeros(2, dtype=np.uint64)
        lib().wo_random_init(seed & 0xFFFFFFFFFFFFFFFF, _ptr(self.s))

    def lrand(self) -> int:
        return int(lib().wo_lrand(_ptr(self.s)))

    def drand(self) -> float:
        return float(lib().wo_drand(_ptr(self.s)))

    def irand(self, mx: int) -> int:
        return self.lrand() % mx


def hash32(x: int) -> int:
    return int(lib().wo_hash32(x))


def hash64(x: int) -> int:
    return int(lib().wo_hash64(x))


def philox4x32_10(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().wo_philox4x32_10(_ptr(c), _ptr(k), _ptr(o))
    return [int(x) for x in o]


def generate_batch_of_edges(edges_number, vertices_number, batch_seed, self_loops=False, directed=True,
                            a=0.5, b=0.2, c=0.1) -> np.ndarray:
    """utility::generate_batch_of_edges (utils/utility.h:55-146) -> (k, 2) uint32."""
    cap = edges_number * (1 if directed else 2)
    out = np.zeros((max(cap, 1), 2), dtype=np.uint32)
    k = lib().wo_generate_batch_of_edges(edges_number, vertices_number, batch_seed, int(self_loops),
                                         int(directed), a, b, c, _ptr(out))
    return out[:k].copy()


def szudzik32_pair(x, y):
    return int(lib().wo_szudzik32_pair(x, y))


def szudzik32_unpair(z):
    x = np.zeros(1, np.uint32)
    y = np.zeros(1, np.uint32)
    lib().wo_szudzik32_unpair(z, _ptr(x), _ptr(y))
    return int(x[0]), int(y[0])


def szudzik64_pair(x, y):
    return int(lib().wo_szudzik64_pair(x, y))


def szudzik64_unpair(z):
    x = np.zeros(1, np.uint64)
    y = np.zeros(1, np.uint64)
    lib().wo_szudzik64_unpair(z, _ptr(x), _ptr(y))
    return int(x[0]), int(y[0])


def csr_from_edges(n: int, pairs: np.ndarray):
    """CSR (off u64[n+1], adj u32[m]) from sorted, deduplicated (src, dst) pairs."""
    pairs = np.asarray(pairs, dtype=np.uint32).reshape(-1, 2)
    counts = np.bincount(pairs[:, 0].astype(np.int64), minlength=n)[:n]
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(counts, out=off[1:])
    return off, np.ascontiguousarray(pairs[:, 1])


class Engine:
    """CPU restatement of dygrl::WharfMH's walk path (graph/wharfmh.h)."""

    def __init__(self, off, adj, wpv=10, L=80, model=DEEPWALK, p=4.0, q=1.0, init=INIT_WEIGHT,
                 deterministic=True, seed=0x5EED):
        off = np.ascontiguousarray(off, dtype=np.uint64)
        adj = np.ascontiguousarray(adj, dtype=np.uint32)
        self.n = len(off) - 1
        self.wpv, self.L = wpv, L
        self._h = lib().wo_create(self.n, len(adj), _ptr(off), _ptr(adj), wpv, L, model, p, q, init,
                                  int(deterministic), seed)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().wo_free(self._h)
            self._h = None

    def generate(self):
        lib().wo_generate(self._h)

    def update(self, insert: bool, pairs, flags=REMOVE_DUPS | APPLY_WALK_UPDATES) -> np.ndarray:
        pairs = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1, 2)
        aff = np.zeros(max(self.num_walks, 1), dtype=np.uint32)
        k = lib().wo_update(self._h, int(insert), len(pairs), _ptr(pairs), flags, _ptr(aff))
        return aff[:k].copy()

    def insert_edges_batch(self, pairs, flags=REMOVE_DUPS | APPLY_WALK_UPDATES):
        return self.update(True, pairs, flags)

    def delete_edges_batch(self, pairs, flags=REMOVE_DUPS | APPLY_WALK_UPDATES):
        return self.update(False, pairs, flags)

    @property
    def num_walks(self) -> int:
        return int(lib().wo_num_walks(self._h))

    @property
    def num_edges(self) -> int:
        return int(lib().wo_num_edges(self._h))

    @property
    def accepts(self) -> int:
        return int(lib().wo_get_accepts(self._h))

    @property
    def steps(self) -> int:
        return int(lib().wo_get_steps(self._h))

    def csr(self):
        off = np.zeros(self.n + 1, dtype=np.uint64)
        adj = np.zeros(max(self.num_edges, 1), dtype=np.uint32)
        lib().wo_get_csr(self._h, _ptr(off), _ptr(adj))
        return off, adj[: self.num_edges]

    def walks(self) -> np.ndarray:
        """[W][L] walk-major, SENT-padded."""
        out = np.zeros((self.num_walks, self.L), dtype=np.uint32)
        lib().wo_get_walks(self._h, _ptr(out))
        return out

    def walks_range(self, w0: int, w1: int) -> np.ndarray:
        """walks [w0, w1) of the [W][L] corpus (no copy of the rest)."""
        out = np.zeros((w1 - w0, self.L), dtype=np.uint32)
        lib().wo_get_walks_range(self._h, w0, w1, _ptr(out))
        return out

    def index(self):
        tot = int(lib().wo_index_size(self._h))
        counts = np.zeros(self.n, dtype=np.uint64)
        keys = np.zeros(max(tot, 1), dtype=np.uint64)
        nexts = np.zeros(max(tot, 1), dtype=np.uint32)
        lib().wo_export_index(self._h, _ptr(counts), _ptr(keys), _ptr(nexts))
        return counts, keys[:tot], nexts[:tot]

    def time_generate_range(self, w0: int, w1: int, threads: int = 0) -> float:
        return float(lib().wo_time_generate_range(self._h, w0, w1, threads))


def walk_string(walk_row: np.ndarray) -> str:
    """WharfMH::walk text (wharfmh.h:365-394): ids separated by and ending with a space."""
    return "".join(f"{int(v)} " for v in walk_row if v != SENT)
