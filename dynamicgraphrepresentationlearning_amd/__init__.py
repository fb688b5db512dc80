"""MI355X-native streaming random-walk engine (WharfMH walk path).

The compute path is libwharf_gpu.so (hand-written HIP for gfx950) behind the
C ABI in include/wharf_gpu.h; this package is the Python host mirror of the
reference's dygrl::WharfMH interface.  Importing it fails loudly when the HIP
library has not been built.
"""
from .wharfmh import (  # noqa: F401
    BURNIN,
    DEEPWALK,
    NODE2VEC,
    RANDOM,
    SENTINEL,
    WEIGHT,
    WharfConfig,
    WharfMH,
    generate_batch_of_edges,
    read_adjacency_graph,
    snap_to_adj,
    szudzik64_pair,
    szudzik64_unpair,
)
from ._lib import LIB_PATH  # noqa: F401

__all__ = ["WharfMH", "WharfConfig", "generate_batch_of_edges", "read_adjacency_graph", "snap_to_adj",
           "szudzik64_pair", "szudzik64_unpair", "DEEPWALK", "NODE2VEC", "RANDOM", "BURNIN", "WEIGHT", "SENTINEL"]
