/*
 * wharf_gpu.h — C ABI of the MI355X-native WharfMH walk engine.
 *
 * This is the drop-in boundary for the reference's walk-generation and
 * incremental re-walk path (djordjijeK/DynamicGraphRepresentationLearning,
 * graph/wharfmh.h).  Every entry point names the reference interface it
 * replaces.  Plain pointers and sizes only; no C++ or torch types.
 *
 * Conventions
 *   - every call returns 0 (WHARF_OK) or a negative WHARF_E* code; the message
 *     is available from wharf_last_error(handle) (handle may be NULL for errors
 *     raised before a handle exists).  The reference exits or asserts instead
 *     (wharfmh.h:270,758; utility.h:220 divides by zero).
 *   - input buffers are host memory owned by the caller and copied on entry
 *     (the reference takes ownership of the CSR, wharfmh.h:99-103, and sorts the
 *     caller's edge batch in place, wharfmh.h:450-453; this ABI does neither).
 *   - output buffers are caller-allocated host memory; sizes are queried first.
 *   - one host thread per handle; a handle owns one HIP device and one stream.
 *     Calls are synchronous (they return after the device work completed).
 *   - the graph, the walk matrix and all scratch stay resident in HBM between
 *     calls.
 */
#ifndef WHARF_GPU_H
#define WHARF_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WHARF_ABI_VERSION 8

enum {
    WHARF_OK = 0,
    WHARF_E_INVALID = -1,   /* bad argument (sizes, ids >= n, null pointers) */
    WHARF_E_HIP = -2,       /* HIP runtime error */
    WHARF_E_NOMEM = -3,     /* device allocation failed */
    WHARF_E_STATE = -4,     /* call not valid in the current state */
    WHARF_E_RANGE = -5      /* walk id / position out of range or not owned by this shard */
};

/* types::RandomWalkModelType (config/types.h:28) */
enum { WHARF_DEEPWALK = 0, WHARF_NODE2VEC = 1 };
/* types::SamplerInitStartegy (config/types.h:31) */
enum { WHARF_INIT_RANDOM = 0, WHARF_INIT_BURNIN = 1, WHARF_INIT_WEIGHT = 2 };
/* insert_edges_batch / delete_edges_batch boolean arguments (wharfmh.h:439,588) */
enum { WHARF_SORTED = 1, WHARF_REMOVE_DUPS = 2, WHARF_APPLY_WALK_UPDATES = 4,
       WHARF_AFFECTED_DEVICE = 8 /* affected_out is device memory of the handle's GPU (no PCIe copy) */ };

#define WHARF_SENTINEL 0xFFFFFFFEu  /* std::numeric_limits<uint32_t>::max() - 1 (wharfmh.h:282) */

/* The reference's mutable globals (config/globals.h:7-29) as a POD. */
typedef struct wharf_config {
    uint32_t walks_per_vertex;  /* config::walks_per_vertex (u8 in the reference), default 10 */
    uint32_t walk_length;       /* config::walk_length (u8), default 80, 2..255 */
    int32_t  model;             /* config::random_walk_model, default WHARF_NODE2VEC (globals.h:13) */
    float    paramP;            /* config::paramP, default 4.0 */
    float    paramQ;            /* config::paramQ, default 1.0 */
    int32_t  sampler_init;      /* config::sampler_init_strategy, default WHARF_INIT_WEIGHT */
    int32_t  deterministic;     /* config::deterministic_mode, default 1 */
    uint64_t seed;              /* MH-mode Philox key (replaces config::random(time(nullptr))), default 0x5EED */
    uint64_t shard_lo;          /* walks of start vertices [shard_lo, shard_hi) live on this handle; */
    uint64_t shard_hi;          /*   shard_hi == 0 means all vertices */
} wharf_config;

typedef struct wharf_stats {
    uint64_t n, m;                 /* number_of_vertices(), number_of_edges() (wharfmh.h:117,130) */
    uint64_t walks;                /* walks owned by this handle */
    uint64_t steps;                /* transitions appended by the last generate/update */
    uint64_t accepts;              /* MH acceptances in the last generate/update */
    uint64_t affected;             /* walks re-walked by the last update */
    uint64_t batch_edges;          /* edges in the last batch after sort/dedup */
    double   last_walk_kernel_ms;  /* device time of the last walk / re-walk kernel (HIP events) */
    double   last_graph_update_ms; /* device time of the last CSR update (graph_update_time_on_*, config.h:10-14) */
    double   last_walk_update_ms;  /* device time of the last scan + re-walk (walk_update_time_on_*) */
    double   last_total_ms;        /* host wall time of the last call */
    uint64_t hbm_bytes_walks;      /* resident bytes: walk matrix */
    uint64_t hbm_bytes_graph;      /* resident bytes: CSR + vertex records (+ anchors) */
    double   last_csr_move_ms;     /* device time of the last update's in-edge record pass (the records of the
                                      batch sources' in-edges): k_patch_in_edges, a streaming pass over the slot
                                      pool, or k_patch_rev through the reverse-slot index (last_in_edge_mode) */
    uint64_t last_moved_slots;     /* slots that pass read: the whole pool (scan: live, slack and dead slots
                                      alike), or the sources' new rows, sum of their degrees (reverse index) */
    /* slack-row CSR: row v = slots [off, off + deg) of a pool with cap >= deg reserved */
    uint64_t pool_slots;           /* slots handed out to rows (live edges + slack + rows' old places) */
    uint64_t pool_capacity;        /* slots allocated */
    uint64_t last_moved_row_slots; /* slots given to rows that outgrew their place in the last batch */
    uint64_t repacks;              /* pool repacks (fresh slack for every row, or dead slots squeezed out) so far */
    uint64_t dead_slots;           /* slots of rows' old places (moved rows leave them kGap): read by every
                                      in-edge pass until a repack reclaims them (one is started past 1/4 of the pool) */
    uint64_t last_anchor_inits;    /* node2vec MH: anchors (MH sampler inits) computed by the last generate/update */
    uint64_t last_rewalk_passes;   /* node2vec MH re-walk by passes (k_rewalk_park): passes of the last update,
                                      0 when the lock-step kernel ran */
    uint64_t last_in_edge_mode;    /* 0: the last update scanned the pool for in-edges, 1: reverse-slot index */
    uint64_t rev_fallbacks;        /* updates so far whose reverse-slot pass found an edge without its reverse or
                                      a stale entry: the index was dropped and the pool scan rewrote the records
                                      (0 on a healthy undirected stream; tests assert it) */
} wharf_stats;

typedef struct wharf_handle wharf_handle;

void        wharf_config_default(wharf_config* cfg);
const char* wharf_last_error(const wharf_handle* h);
int         wharf_abi_version(void);
int         wharf_device_count(int* count);

/* WharfMH(long n, long m, uintE* offsets, uintV* edges, bool free_memory) (wharfmh.h:58-110).
 * offsets: n entries (row v = [offsets[v], offsets[v+1]) with offsets[n] := m), targets: m.
 * Rows are canonicalised (sorted ascending, duplicates removed), the form
 * CompressedEdges::get_edges returns (tree_plus.h:233-243). */
int wharf_create(const wharf_config* cfg, uint64_t n, uint64_t m, const uint64_t* offsets,
                 const uint32_t* targets, int device, wharf_handle** out);

/* WharfMH(long n, long m) (wharfmh.h:26-47): n isolated vertices. */
int wharf_create_empty(const wharf_config* cfg, uint64_t n, int device, wharf_handle** out);

/* A synthetic base graph built on the device without a host round trip:
 * the undirected RMAT graph utility::generate_batch_of_edges(edges_number,
 * vertices_number, seed, self_loops=false, directed=false, a, b, c)
 * (utils/utility.h:55-146) on n vertices (n >= the RMAT size). */
int wharf_create_rmat(const wharf_config* cfg, uint64_t n, uint64_t edges_number, uint64_t vertices_number,
                      uint64_t seed, double a, double b, double c, int device, wharf_handle** out);

/* ~WharfMH / WharfMH::destroy (wharfmh.h:228). */
int wharf_destroy(wharf_handle* h);
/* WharfMH::destroy_index (wharfmh.h:237): drops every walk. */
int wharf_destroy_index(wharf_handle* h);
/* Frees the handle's droppable device caches -- the reverse-slot index (up to 4 B per pool slot,
 * 16 GB at configs[4]) -- for a caller whose own allocation (e.g. a corpus gather buffer) ran out of
 * device memory; the library does the same for its own failed allocations.  Results are unchanged
 * (updates then scan the pool for in-edges); the index is not rebuilt lazily.  *freed_bytes (may be
 * null) = bytes released, 0 when there was nothing to drop.  No reference counterpart. */
int wharf_release_caches(wharf_handle* h, uint64_t* freed_bytes);

/* WharfMH::generate_initial_random_walks (wharfmh.h:250-356). */
int wharf_generate(wharf_handle* h);

/* WharfMH::insert_edges_batch / delete_edges_batch (wharfmh.h:439-726) followed,
 * when WHARF_APPLY_WALK_UPDATES is set, by batch_walk_update (733-923).
 * pairs: m (src, dst) u32 pairs.  affected_out (may be NULL) receives the
 * affected walk ids in ascending order (the reference returns them in hash
 * order); capacity >= the owned walk count.  *n_affected receives the count.
 * With WHARF_AFFECTED_DEVICE, affected_out is a device pointer and the ids
 * stay in HBM (the call still returns after the update completed). */
int wharf_insert_edges(wharf_handle* h, uint64_t m, const uint32_t* pairs, uint32_t flags,
                       uint32_t* affected_out, uint64_t* n_affected);
int wharf_delete_edges(wharf_handle* h, uint64_t m, const uint32_t* pairs, uint32_t flags,
                       uint32_t* affected_out, uint64_t* n_affected);

/* WharfMH::batch_walk_update (wharfmh.h:733-923) on its own: re-walk every owned
 * walk from its first position holding one of the k `sources` (the vertex set
 * of the reference's MapOfChanges, wharfmh.h:519-537), on the current graph.
 * Samplers are not reset (the reference resets them in insert/delete,
 * wharfmh.h:504,539,652,689), and MH draws are keyed by the epoch of the last
 * applied batch, so insert_edges(flags without WHARF_APPLY_WALK_UPDATES)
 * followed by batch_walk_update(that batch's sources) gives exactly the walks
 * of insert_edges(WHARF_APPLY_WALK_UPDATES).  flags: WHARF_AFFECTED_DEVICE
 * only; affected_out / n_affected as for wharf_insert_edges. */
int wharf_batch_walk_update(wharf_handle* h, const uint32_t* sources, uint64_t k, uint32_t flags,
                            uint32_t* affected_out, uint64_t* n_affected);

/* number_of_vertices / number_of_edges (wharfmh.h:117-133). */
int wharf_number_of_vertices(const wharf_handle* h, uint64_t* n);
int wharf_number_of_edges(const wharf_handle* h, uint64_t* m);
/* walks owned by this handle and the [lo, hi) start-vertex shard. */
int wharf_shard(const wharf_handle* h, uint64_t* lo, uint64_t* hi, uint64_t* walks);

/* Re-partition the walks: this handle owns the walks of start vertices
 * [lo, hi) (hi == 0: all).  Drops the current walks (like destroy_index). */
int wharf_set_shard(wharf_handle* h, uint64_t lo, uint64_t hi);

/* Re-partition the walks by vertex blocks: this handle owns the walks of the
 * start vertices in blocks part, part + parts, part + 2 parts, ... of
 * 2^block_bits consecutive vertices (6 <= block_bits <= 31).  Every part gets
 * the same mix of the graph's regions, so the parts' walks re-walk at the same
 * rate (contiguous ranges of an RMAT graph do not: DESIGN.md §8).  Local walk
 * order stays ascending in walk id.  Drops the current walks; wharf_set_shard
 * returns to a contiguous range.  wharf_shard reports lo = 0, hi = n. */
int wharf_set_shard_blocks(wharf_handle* h, uint32_t part, uint32_t parts, uint32_t block_bits);
int wharf_shard_blocks(const wharf_handle* h, uint32_t* part, uint32_t* parts, uint32_t* block_bits);

/* flatten_graph (wharfmh.h:175-208): offsets_out n+1 entries, targets_out m
 * (targets_out NULL: offsets only). */
int wharf_get_graph(wharf_handle* h, uint64_t* offsets_out, uint32_t* targets_out);

/* WharfMH::walk / vertex_at_walk (wharfmh.h:365-427).
 * wharf_walk: vertices of walk `wid` into out (capacity walk_length), *len = count. */
int wharf_walk(wharf_handle* h, uint64_t wid, uint32_t* out, uint32_t* len);
/* text form "v0 v1 ... " (trailing space), *len excludes the terminating NUL. */
int wharf_walk_string(wharf_handle* h, uint64_t wid, char* buf, size_t cap, size_t* len);
int wharf_vertex_at_walk(wharf_handle* h, uint64_t wid, uint32_t position, uint32_t* vertex);

/* Whole corpus of this handle's walks, SENT-padded.
 *   layout 0: walk-major [walks][walk_length], rows in ascending walk id
 *   layout 1: position-major [walk_length][walks] (the resident HBM layout)
 * dst: host buffer of walks*walk_length u32; or, with wharf_export_walks_device,
 * a device pointer on the handle's device (used for the RCCL corpus gather). */
int wharf_export_walks(wharf_handle* h, uint32_t* dst, int layout);
int wharf_export_walks_device(wharf_handle* h, uint32_t* dst_device, int layout);
/* Walk-major rows [first, first + count) of the layout-0 export (row i = the
 * handle's i-th owned walk in ascending walk id), so a corpus can leave the
 * device one bounded chunk at a time (the chunked corpus gather of
 * distributed.py; vertex-classification.cpp:142-158 consumes the corpus). */
int wharf_export_walk_rows(wharf_handle* h, uint64_t first, uint64_t count, uint32_t* dst);
int wharf_export_walk_rows_device(wharf_handle* h, uint64_t first, uint64_t count, uint32_t* dst_device);
/* global walk id of each owned walk, in export row order (walks entries). */
int wharf_walk_ids(wharf_handle* h, uint32_t* ids_out);

/* The inverted index (walks/inverted_index.h:12-93): for each vertex v the
 * ascending (key = wid*walk_length + pos, next) entries of the walks owned by
 * this handle; next = SENT at the last position.
 * First call wharf_index_size, then wharf_export_index with counts[n],
 * keys[size], nexts[size]. */
int wharf_index_size(wharf_handle* h, uint64_t* size);
int wharf_export_index(wharf_handle* h, uint64_t* counts, uint64_t* keys, uint32_t* nexts);

/* The same for the vertex window [v0, v1) only: counts[v1 - v0], keys/nexts of
 * wharf_index_size_range() entries.  Keys stay 64-bit: past n*wpv*L > 2^32
 * (configs[3]/[4]) the reference's u32 keys (inverted_index.h:14) would wrap.
 * Lets a caller export a corpus whose whole index does not fit the host. */
int wharf_index_size_range(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* size);
int wharf_export_index_range(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* counts, uint64_t* keys,
                             uint32_t* nexts);

/* The walks in the reference's pairing-encoded CompressedWalks form
 * (walks/compressed_walks.h:49-66, pairings.h): per vertex, the values
 * Szudzik(wid*L + pos, next) of its stored positions, ascending (the C-tree's
 * iteration order), in 64 bits (the reference's 32-bit Szudzik<Vertex> would
 * overflow past 2^16 keys).  counts[n] as for wharf_export_index; paired
 * receives wharf_index_size() values. */
int wharf_export_index_paired(wharf_handle* h, uint64_t* counts, uint64_t* paired);

int wharf_get_stats(const wharf_handle* h, wharf_stats* out);

/* WharfMH::memory_footprint (wharfmh.h:928-998), which prints the bytes of the
 * vertex tree, edge C-trees, walk trees and samplers: here the device bytes
 * held by the handle, by role. */
typedef struct wharf_memory {
    uint64_t n, m;
    uint64_t csr_bytes;             /* offsets + targets (the edge trees' content) + reverse-slot index */
    uint64_t records_bytes;         /* vertex + edge row records */
    uint64_t walks_bytes;           /* walk matrix + per-walk rewalk positions (the walk trees) */
    uint64_t samplers_bytes;        /* MH anchors + per-row sampler epochs (the samplers) */
    uint64_t edge_hash_bytes;       /* node2vec has_edge set + per-row neighbour filters */
    uint64_t update_buffers_bytes;  /* second CSR / record buffers of the batch merge */
    uint64_t scratch_bytes;         /* sort / select temporaries, batch and draw tables */
    uint64_t total_bytes;
} wharf_memory;
int wharf_memory_footprint(const wharf_handle* h, wharf_memory* out);

/* utility::generate_batch_of_edges (utils/utility.h:55-146) on the device:
 * sorted, deduplicated (src,dst) pairs.  out_pairs capacity: 2*edges_number
 * pairs when undirected, edges_number otherwise. */
int wharf_generate_batch_of_edges(int device, uint64_t edges_number, uint64_t vertices_number, uint64_t batch_seed,
                                  int self_loops, int directed, double a, double b, double c,
                                  uint32_t* out_pairs, uint64_t* count);

/* ---- IO (host side) ------------------------------------------------------ */

/* read_unweighted_graph (libs/compressed_trees/common/IO.h:67-106): Ligra
 * "AdjacencyGraph" text.  Call with offsets == NULL for n and m, then with
 * offsets[n] and targets[m]. */
int wharf_read_adjacency_graph(const char* path, uint64_t* n, uint64_t* m, uint64_t* offsets, uint32_t* targets);

/* The prebuilt experiments/bin/SNAPtoAdj (-s): SNAP edge list ('#' comments)
 * -> AdjacencyGraph text, symmetrised when `symmetric`, sorted, duplicates and
 * self loops removed, n = largest id + 1. */
int wharf_snap_to_adj(const char* snap_path, const char* adj_path, int symmetric);

/* Text corpus for yskip (vertex-classification.cpp:142-150): one line per walk,
 * WharfMH::walk format "v0 v1 ... " + '\n'.  wids == NULL writes every owned
 * walk in ascending id order; otherwise the listed (owned) walks in list order
 * (e.g. the affected ids of an update).  append != 0 appends to the file. */
int wharf_write_corpus(wharf_handle* h, const char* path, const uint32_t* wids, uint64_t count, int append);

/* Formatting half of wharf_write_corpus for walk-major rows already on the host. */
int wharf_format_corpus(const uint32_t* rows, uint64_t count, uint32_t walk_length, const char* path, int append);

/* pairings::Szudzik (walks/pairings.h:113-226) on the device, elementwise.
 * op 0: pair(x[i], y[i]) -> z[i]; op 1: unpair(z[i]) -> x[i], y[i].  64-bit
 * unpair uses an exact integer square root (the reference's floor(sqrt(double))
 * is only exact below 2^52). */
int wharf_szudzik64(int device, int op, uint64_t count, uint64_t* x, uint64_t* y, uint64_t* z);

#ifdef __cplusplus
}
#endif
#endif /* WHARF_GPU_H */
