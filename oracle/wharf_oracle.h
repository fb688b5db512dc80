/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle for the WharfMH walk path.
 *
 * A clean-room C restatement of the reference's walk-generation / re-walk
 * algorithm (djordjijeK/DynamicGraphRepresentationLearning @ 2024-10-08).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker.  The product (libwharf_gpu.so) never
 * links or calls it.
 *
 * Pinned: every deterministic-mode function is checked bit-for-bit against
 * golden vectors produced by the reference itself (oracle/_ref/ref_harness,
 * tests/golden/make_golden.py).  The MH-mode functions restate the build's
 * own counter-based (Philox) MH semantics, which the reference
 * cannot reproduce (it uses a shared, time-seeded RNG); they are pinned by the
 * Random123 Philox known-answer vectors and checked statistically against the
 * reference's transition-class frequencies.
 */
#ifndef WHARF_ORACLE_H
#define WHARF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WO_SENT 0xFFFFFFFEu

/* utils/utility.h:157-222 */
void     wo_random_init(uint64_t seed, uint64_t state[2]);
uint64_t wo_lrand(uint64_t state[2]);
double   wo_drand(uint64_t state[2]);

/* pbbslib/utilities.h:108-146, 286-291 */
uint32_t wo_hash32(uint32_t a);
uint64_t wo_hash64(uint64_t u);
uint32_t wo_log2_up(uint64_t i);

/* Philox4x32-10 (Salmon et al., SC'11; Random123 reference algorithm) */
void wo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* utils/utility.h:55-146 + rmat_util.h:7-43.  Writes sorted, deduplicated
 * (src,dst) pairs into out (capacity 2*edges_number pairs when undirected) and
 * returns the count. */
uint64_t wo_generate_batch_of_edges(uint64_t edges_number, uint64_t vertices_number, uint64_t batch_seed,
                                    int self_loops, int directed, double a, double b, double c,
                                    uint32_t* out_pairs);

/* walks/pairings.h:113-226 (reference arithmetic, including floor(sqrt)). */
uint32_t wo_szudzik32_pair(uint32_t x, uint32_t y);
void     wo_szudzik32_unpair(uint32_t z, uint32_t* x, uint32_t* y);
uint64_t wo_szudzik64_pair(uint64_t x, uint64_t y);
void     wo_szudzik64_unpair(uint64_t z, uint64_t* x, uint64_t* y);

/* ---- engine (graph/wharfmh.h) ------------------------------------------- */
typedef struct wo_engine wo_engine;

enum { WO_DEEPWALK = 0, WO_NODE2VEC = 1 };
enum { WO_INIT_RANDOM = 0, WO_INIT_BURNIN = 1, WO_INIT_WEIGHT = 2 };
enum { WO_SORTED = 1, WO_REMOVE_DUPS = 2, WO_APPLY_WALK_UPDATES = 4 };

/* CSR: off[n+1] (u64), adj[m] (u32, ascending & unique per row) */
wo_engine* wo_create(uint64_t n, uint64_t m, const uint64_t* off, const uint32_t* adj,
                     uint32_t wpv, uint32_t L, int model, float p, float q, int init,
                     int deterministic, uint64_t seed);
void     wo_free(wo_engine* e);
void     wo_generate(wo_engine* e);                       /* wharfmh.h:250-356 */
/* wharfmh.h:439-576 / 588-726 + batch_walk_update 733-923.  Returns number of
 * affected walks; affected_out (capacity n*wpv) receives them ascending. */
uint64_t wo_update(wo_engine* e, int insert, uint64_t m, const uint32_t* pairs, uint32_t flags,
                   uint32_t* affected_out);
uint64_t wo_num_edges(const wo_engine* e);
uint64_t wo_num_walks(const wo_engine* e);
void     wo_get_csr(const wo_engine* e, uint64_t* off_out, uint32_t* adj_out);
void     wo_get_walks(const wo_engine* e, uint32_t* out);   /* [W][L] walk-major */
void     wo_get_walks_range(const wo_engine* e, uint64_t w0, uint64_t w1, uint32_t* out);   /* walks [w0, w1) */
uint64_t wo_get_accepts(const wo_engine* e);               /* MH acceptances since last reset */
uint64_t wo_get_steps(const wo_engine* e);
/* Inverted index (walks/inverted_index.h:12-93): counts[n], then per vertex
 * ascending (key, next) pairs.  key = wid*L + pos (64-bit). */
uint64_t wo_index_size(const wo_engine* e);
void     wo_export_index(const wo_engine* e, uint64_t* counts, uint64_t* keys, uint32_t* nexts);

/* Time deterministic generation over walk ids [w0, w1) only (cpu_baseline). */
double   wo_time_generate_range(wo_engine* e, uint64_t w0, uint64_t w1, int threads);

#ifdef __cplusplus
}
#endif
#endif
