"""ctypes binding of libwharf_gpu.so (include/wharf_gpu.h).

The HIP library is the only implementation: if it is missing this module
raises on import — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

# One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 and its
# libraries ask for it as "libamdhip64.so"; libwharf_gpu.so asks for the soname
# "libamdhip64.so.7".  Loaded torch-first, our request resolves to torch's
# runtime; loaded the other way round the process would map two HIP/HSA
# runtimes and torch's would find no GPU ("No HIP GPUs are available").
try:
    import torch  # noqa: F401
except ImportError:   # torch is plumbing (device buffers, streams, torch.distributed), not required
    pass

_HERE = os.path.dirname(os.path.abspath(__file__))
# WHARF_LIB_PATH: an alternative build of the same library (A/B experiments in tools/)
LIB_PATH = os.environ.get("WHARF_LIB_PATH") or os.path.join(_HERE, "libwharf_gpu.so")

ABI_VERSION = 8   # WHARF_ABI_VERSION of include/wharf_gpu.h
WHARF_OK = 0
WHARF_DEEPWALK, WHARF_NODE2VEC = 0, 1
WHARF_INIT_RANDOM, WHARF_INIT_BURNIN, WHARF_INIT_WEIGHT = 0, 1, 2
WHARF_SORTED, WHARF_REMOVE_DUPS, WHARF_APPLY_WALK_UPDATES, WHARF_AFFECTED_DEVICE = 1, 2, 4, 8
SENTINEL = 0xFFFFFFFE


class wharf_config(C.Structure):
    _fields_ = [
        ("walks_per_vertex", C.c_uint32),
        ("walk_length", C.c_uint32),
        ("model", C.c_int32),
        ("paramP", C.c_float),
        ("paramQ", C.c_float),
        ("sampler_init", C.c_int32),
        ("deterministic", C.c_int32),
        ("seed", C.c_uint64),
        ("shard_lo", C.c_uint64),
        ("shard_hi", C.c_uint64),
    ]


class wharf_stats(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("m", C.c_uint64),
        ("walks", C.c_uint64),
        ("steps", C.c_uint64),
        ("accepts", C.c_uint64),
        ("affected", C.c_uint64),
        ("batch_edges", C.c_uint64),
        ("last_walk_kernel_ms", C.c_double),
        ("last_graph_update_ms", C.c_double),
        ("last_walk_update_ms", C.c_double),
        ("last_total_ms", C.c_double),
        ("hbm_bytes_walks", C.c_uint64),
        ("hbm_bytes_graph", C.c_uint64),
        ("last_csr_move_ms", C.c_double),
        ("last_moved_slots", C.c_uint64),
        ("pool_slots", C.c_uint64),
        ("pool_capacity", C.c_uint64),
        ("last_moved_row_slots", C.c_uint64),
        ("repacks", C.c_uint64),
        ("dead_slots", C.c_uint64),
        ("last_anchor_inits", C.c_uint64),
        ("last_rewalk_passes", C.c_uint64),
        ("last_in_edge_mode", C.c_uint64),
        ("rev_fallbacks", C.c_uint64),
    ]


class wharf_memory(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("n", "m", "csr_bytes", "records_bytes", "walks_bytes", "samplers_bytes",
                                          "edge_hash_bytes", "update_buffers_bytes", "scratch_bytes", "total_bytes")]


# every symbol declared in include/wharf_gpu.h, with its ctypes signature
_P, _U64, _U32, _I = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
SIGNATURES = {
    "wharf_config_default": (None, [_P]),
    "wharf_last_error": (C.c_char_p, [_P]),
    "wharf_abi_version": (_I, []),
    "wharf_device_count": (_I, [_P]),
    "wharf_create": (_I, [_P, _U64, _U64, _P, _P, _I, _P]),
    "wharf_create_empty": (_I, [_P, _U64, _I, _P]),
    "wharf_create_rmat": (_I, [_P, _U64, _U64, _U64, _U64, C.c_double, C.c_double, C.c_double, _I, _P]),
    "wharf_destroy": (_I, [_P]),
    "wharf_destroy_index": (_I, [_P]),
    "wharf_release_caches": (_I, [_P, _P]),
    "wharf_generate": (_I, [_P]),
    "wharf_insert_edges": (_I, [_P, _U64, _P, _U32, _P, _P]),
    "wharf_delete_edges": (_I, [_P, _U64, _P, _U32, _P, _P]),
    "wharf_batch_walk_update": (_I, [_P, _P, _U64, _U32, _P, _P]),
    "wharf_number_of_vertices": (_I, [_P, _P]),
    "wharf_number_of_edges": (_I, [_P, _P]),
    "wharf_shard": (_I, [_P, _P, _P, _P]),
    "wharf_set_shard": (_I, [_P, _U64, _U64]),
    "wharf_set_shard_blocks": (_I, [_P, _U32, _U32, _U32]),
    "wharf_shard_blocks": (_I, [_P, _P, _P, _P]),
    "wharf_get_graph": (_I, [_P, _P, _P]),
    "wharf_walk": (_I, [_P, _U64, _P, _P]),
    "wharf_walk_string": (_I, [_P, _U64, _P, C.c_size_t, _P]),
    "wharf_vertex_at_walk": (_I, [_P, _U64, _U32, _P]),
    "wharf_export_walks": (_I, [_P, _P, _I]),
    "wharf_export_walks_device": (_I, [_P, _P, _I]),
    "wharf_export_walk_rows": (_I, [_P, _U64, _U64, _P]),
    "wharf_export_walk_rows_device": (_I, [_P, _U64, _U64, _P]),
    "wharf_walk_ids": (_I, [_P, _P]),
    "wharf_index_size": (_I, [_P, _P]),
    "wharf_export_index": (_I, [_P, _P, _P, _P]),
    "wharf_index_size_range": (_I, [_P, C.c_uint64, C.c_uint64, _P]),
    "wharf_export_index_range": (_I, [_P, C.c_uint64, C.c_uint64, _P, _P, _P]),
    "wharf_get_stats": (_I, [_P, _P]),
    "wharf_export_index_paired": (_I, [_P, _P, _P]),
    "wharf_memory_footprint": (_I, [_P, _P]),
    "wharf_generate_batch_of_edges": (_I, [_I, _U64, _U64, _U64, _I, _I, C.c_double, C.c_double, C.c_double, _P, _P]),
    "wharf_szudzik64": (_I, [_I, _I, _U64, _P, _P, _P]),
    "wharf_read_adjacency_graph": (_I, [C.c_char_p, _P, _P, _P, _P]),
    "wharf_snap_to_adj": (_I, [C.c_char_p, C.c_char_p, _I]),
    "wharf_write_corpus": (_I, [_P, C.c_char_p, _P, _U64, _I]),
    "wharf_format_corpus": (_I, [_P, _U64, _U32, C.c_char_p, _I]),
}


def load(path: str = LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(f"{path} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(make -C dynamicgraphrepresentationlearning_amd/csrc)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    # the structs above mirror include/wharf_gpu.h of this ABI version: a library
    # of another version (an A/B build through WHARF_LIB_PATH) would write a
    # wharf_stats of another size into the ctypes buffer
    ver = lib.wharf_abi_version()
    if ver != ABI_VERSION:
        raise ImportError(f"{path}: WHARF_ABI_VERSION {ver}, this binding expects {ABI_VERSION}; rebuild the library")
    return lib


lib = load()


def last_error(handle=None) -> str:
    msg = lib.wharf_last_error(handle)
    return msg.decode() if msg else ""


def check(rc: int, handle=None, what: str = "") -> None:
    if rc != WHARF_OK:
        raise RuntimeError(f"{what} failed ({rc}): {last_error(handle)}")
