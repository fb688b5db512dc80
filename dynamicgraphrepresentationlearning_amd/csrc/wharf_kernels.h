// Kernel-side interface of the WharfMH walk engine (shared by the kernels and
// the C-ABI implementation).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "wharf_device.h"

namespace wharf {

enum { kDeepWalk = 0, kNode2Vec = 1 };
enum { kInitRandom = 0, kInitBurnin = 1, kInitWeight = 2 };
constexpr uint64_t kMemoPad = 64;   // >= the chunk of k_rewalk_chunked

struct RunInfo {
    uint64_t off, end;   // old row [off, end)
    uint32_t src, rs, re, pad;
};

struct WalkArgs {
    const ERec* vrec;            // [n]: the row of each vertex
    const ERec* erec;            // [m]: per CSR slot, the target's row (16 B, 32 B with the anchor, or 8 B: rf)
    RecFmt rf;                   // edge-record layout (compact 8-B records: DeepWalk / deterministic)
    const uint32_t* deg;         // [n]: row degrees (a compact record's degree escape)
    const uint32_t* adj;         // [m]: CSR targets (binary searches, anchor proposals)
    uint64_t* anchor;            // node2vec MH: anchor entry of CSR slot e at anchor[e * kAnchorStride]
                                 //   (bytes 16-23 of the slot's 32-B edge record)
    const uint64_t* ehash;       // node2vec: edge hash set (u << 32 | v), or null -> binary search
    uint64_t ehash_mask;         // capacity - 1 (power of two)
    const uint64_t* fdir;        // node2vec MH: per-row neighbour filter {word offset | log2 words << 48}, or null
    const uint32_t* fpool;       //   and its 32-bit words (in front of has_edge in anchor inits)
    uint32_t* walks;             // [L][W]
    const uint64_t* rtab;        // deterministic draws [wpv][L]
    const uint32_t* bitmap;      // batch sources (re-walk)
    const uint32_t* bloom;       // Bloom filter of the batch sources, kBloomWords
    uint8_t* aff;                // per owned walk: re-walk position or kNoRewalk
    unsigned long long* counters;  // [0] steps, [1] accepts, [2] re-walk list, [3..6] WHARF_INIT_STATS, [7] anchor inits
    uint64_t n, n_loc, lo, W;
    uint32_t sh_part, sh_parts, sh_bits;   // the shard's blocks (ShardMap; contiguous: 0, 1, 0)
    uint32_t L, epoch;
    uint32_t key0, key1;
    float inv_p, inv_q;
    int model, init, det;
    int scan_only;               // re-walk: only find rewalk points (apply_walk_updates=false)
    uint64_t* defer;             // node2vec re-walk list {li | p << 56}, tickets << 40 | count in counters[2]
    uint64_t* bdesc;             //   per 256-walk block: its run of the list {offset | count << 40}, or null
    uint64_t* stab;              // node2vec MH re-walk: start-state table, buckets of 4 {key, anchor entry}, or null
    uint64_t stab_mask;          //   buckets - 1
    // deterministic re-walk by suffix table (k_det_suffix + k_rewalk_chunked<true>), or memo == null
    uint32_t* memo;              // [wpv][k][memo_stride]: walk from batch source i in round r, new graph
    const uint32_t* src_idx;     // [n]: index of a batch source in the run table (kNoSource elsewhere when src_exact)
    const RunInfo* runs;         // the batch's source runs
    uint64_t memo_k;             // sources (runs) in the batch
    uint32_t memo_stride;        // L rounded up to 4 (16-B aligned rows)
                                 // (the table has kMemoPad readable words on either side)
    uint32_t wpv;
    int nt_rows;                 // chunked scans: non-temporal walk-matrix row loads (most walks re-walk)
    int park;                    // node2vec MH re-walk by passes (k_rewalk_park / k_park_init), run by the host
    int no_sure;                 // A/B: initialise every uncached anchor a step meets (no sure-accept skip)
    int lane_sort;               // node2vec sorted re-walk: a wave's 64 list entries in column order
    int src_exact;               // src_idx holds kNoSource for every non-source (the copy settles positives by it)
    int ret_first;               // node2vec MH, WEIGHT, 1/p the unique heaviest weight: return-first inits (walk_step)
    unsigned long long* err;     // re-walk list consumers: bit 0 an entry out of range, bit 1 an entry outside its block
    int stage;                   // node2vec re-walk launch: 0 plan + consumer, 1 plan only, 2 consumer only
    int plan_group;              // k_rewalk_plan_lean: bin the 4 blocks of a workgroup together (A/B, no bdesc)
};

__host__ __device__ __forceinline__ ShardMap shard_map(const WalkArgs& a)
{
    return ShardMap{a.n, a.n_loc, a.lo, a.sh_part, a.sh_parts, a.sh_bits};
}

constexpr uint64_t kListMask = (1ull << 40) - 1;   // counters[2]: tickets << 40 | re-walk list entries
constexpr uint64_t kParkRecBytes = 32;   // one parked walker of the node2vec re-walk passes


// per batch source: the new row (slack-row CSR update, k_plan_rows .. k_commit_rows)
constexpr uint64_t kRelocate = ~0ull;   // RowPlan.noff before the merge: the row moves to the pool's end
struct RowPlan {
    uint64_t noff;         // new row start
    uint32_t ndeg, ncap;   // new degree and capacity
    uint32_t ocap, pad;    // old capacity
};

unsigned grid_for(uint64_t work, unsigned block);
unsigned cu_count();

void launch_walk(const WalkArgs& a, bool rewalk, hipStream_t s);
// node2vec MH re-walk passes: fresh = the input is k_rewalk_plan's list, park = walkers that need
// an uncached anchor are appended to `out` instead of initialising it in the wave
void launch_rewalk_park(const WalkArgs& a, int fresh, int park, const void* in, const unsigned long long* in_cnt,
                        void* out, unsigned long long* out_cnt, hipStream_t s);
void launch_park_init(const WalkArgs& a, const void* in, const unsigned long long* in_cnt, hipStream_t s);
void launch_src_index(const RunInfo* runs, uint64_t k, uint32_t* src_idx, hipStream_t s);
void launch_source_degrees(const RunInfo* runs, uint64_t k, const ERec* vrec, uint64_t* out, hipStream_t s);
void launch_anchor_preinit(const WalkArgs& a, const uint64_t* preoff, uint64_t k, hipStream_t s);
void launch_slot_owner_fill(const uint64_t* off, const uint32_t* deg, uint64_t n, uint32_t* owner, hipStream_t s);
// Which order computes a state's anchor up front (round 6, undirected graphs with the reverse-slot
// index): state (cur y, prev x) goes in cur order iff cur's row spans at least t[lg(x)] 128-B lines,
// lg(x) = filt_log2_words(deg x) (the size of prev's neighbour filter).  The host fills t from a
// line-count model (wharf_api.hip, init_order_table); integers, so both kernels decide alike.
constexpr uint32_t kWeightProposals = 21;   // WEIGHT inits: the best of 21 proposals (metropolis_hastings_sampler.h:87-107)
constexpr uint32_t kInitOrderLg = 40;
struct InitOrder {
    uint32_t t[kInitOrderLg];
};
// by_cur_y != 0 (undirected graphs): the states of hub curs (deg > by_cur_y) with small prevs
// (deg <= by_cur_x) computed in cur order by a second kernel (k_anchor_init_by_cur, round 5).
// ridx != null (undirected, reverse-slot index): every state in the cheaper of the two orders by
// `ord` (k_anchor_init_all + k_anchor_init_cur); verify: check each reverse slot before writing.
void launch_anchor_init_all(const WalkArgs& a, const uint32_t* owner, uint64_t slots, uint32_t by_cur_y,
                            uint32_t by_cur_x, const uint32_t* ridx, const InitOrder& ord, bool verify,
                            hipStream_t s);
void launch_vrec(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* row_epoch, ERec* vrec,
                 hipStream_t s);
void launch_erec(const uint32_t* adj, uint64_t slots, const ERec* vrec, ERec* erec, uint32_t rs, int keep_anchors,
                 RecFmt rf, hipStream_t s);
void launch_rmat_keys(const RmatParams& p, uint64_t M, int directed, uint64_t* keys, hipStream_t s);
void launch_pairs_to_keys(const uint32_t* pairs, uint64_t m, uint64_t n, uint64_t* keys, unsigned long long* err, hipStream_t s);
void launch_csr_to_keys(const uint64_t* off, uint64_t n, const uint32_t* tgt, uint64_t* keys, unsigned long long* err, hipStream_t s);
void launch_unique_flags(const uint64_t* keys, uint64_t m, int drop_loops, uint8_t* keep, hipStream_t s);
void launch_offsets_from_keys(const uint64_t* keys, uint64_t m, uint64_t n, uint64_t* off, hipStream_t s);
void launch_low32(const uint64_t* keys, uint64_t m, uint32_t* out, hipStream_t s);
void launch_batch_change(const uint64_t* bkeys, uint64_t mb, const uint64_t* off, const uint32_t* deg, const uint32_t* adj,
                         int insert, uint32_t* chg, hipStream_t s);
void launch_run_flags(const uint64_t* bkeys, uint64_t mb, uint8_t* f, hipStream_t s);
void launch_run_info(const uint64_t* bkeys, const uint32_t* run_start, uint64_t k, uint64_t mb, const uint64_t* off,
                     const uint32_t* deg, RunInfo* runs, uint32_t* bitmap, uint32_t* bloom, hipStream_t s);
void launch_mark_sources(const uint32_t* src, uint64_t k, RunInfo* runs, uint32_t* bitmap, uint32_t* bloom,
                         hipStream_t s);
void launch_row_degrees(const uint64_t* coff, uint64_t n, uint32_t* deg, uint32_t* cap, uint64_t* capw, int slack,
                        hipStream_t s);
void launch_row_recap(const uint32_t* deg, uint64_t n, uint32_t* cap, uint64_t* capw, int slack, hipStream_t s);
void launch_deg_u64(const uint32_t* deg, uint64_t n, uint64_t* out, hipStream_t s);
void launch_copy_rows(const uint64_t* soff, const uint32_t* deg, const uint32_t* src, const uint64_t* doff, uint64_t n,
                      uint32_t* dst, const uint64_t* sanc, uint64_t* danc, hipStream_t s);
void launch_plan_rows(const RunInfo* runs, uint64_t k, const uint32_t* cap, const uint32_t* cf, int insert, int slack,
                      uint64_t* need, uint64_t* save, RowPlan* plan, unsigned long long* dead, hipStream_t s);
// in-place pool compaction (wharf_handle::compact)
void launch_slot_order_keys(const uint64_t* off, const uint32_t* cap, uint64_t n, uint64_t* keys, uint32_t* vals,
                            hipStream_t s);
void launch_ordered_caps(const uint32_t* order, const uint32_t* cap, uint64_t n, uint64_t* capw, hipStream_t s);
void launch_compact_gather(const uint32_t* order, const uint64_t* snoff, uint64_t r0, uint64_t r1, const uint64_t* off,
                           const uint32_t* deg, const uint32_t* adj, const uint64_t* anc, uint64_t D, uint64_t C,
                           uint32_t* sadj, uint64_t* sanc, hipStream_t s);
void launch_compact_put(const uint32_t* sadj, const uint64_t* sanc, uint64_t cnt, uint64_t D, uint32_t* adj,
                        uint64_t* anc, hipStream_t s);
void launch_scatter_offsets(const uint32_t* order, const uint64_t* snoff, uint64_t n, uint64_t* off, hipStream_t s);
// source rows in chunks (`pre`: exclusive prefix of launch_run_chunks' counts; null: a workgroup per row)
void launch_run_chunks(const RunInfo* runs, const RowPlan* plan, uint64_t k, uint32_t* cnt, hipStream_t s);
void launch_save_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint32_t* adj, const uint64_t* sofs,
                      uint32_t* scratch, const uint64_t* anc, uint64_t* sanc, const uint32_t* rev, uint32_t* srev,
                      hipStream_t s);
void launch_merge_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* bkeys, const uint32_t* chg,
                       const uint32_t* cf, const uint32_t* scratch, const uint64_t* sofs, const uint64_t* relofs,
                       uint64_t pool_end, int insert, RowPlan* plan, uint32_t* adj, const uint64_t* sanc, uint64_t* anc,
                       const uint32_t* srev, uint32_t* rev, hipStream_t s);
void launch_anchor_invalidate(const uint64_t* bkeys, uint64_t mb, const uint32_t* chg, const uint64_t* off,
                              const uint32_t* deg, const uint32_t* adj, uint64_t* anc, const uint64_t* fdir,
                              const uint32_t* fpool, hipStream_t s);
void launch_keys_symmetric(const uint64_t* keys, uint64_t m, unsigned long long* asym, hipStream_t s);
void launch_commit_rows(const RunInfo* runs, uint64_t k, const RowPlan* plan, uint32_t epoch, uint64_t* off,
                        uint32_t* deg, uint32_t* cap, ERec* vrec, uint32_t* row_epoch, hipStream_t s);
void launch_erec_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* off, const uint32_t* deg,
                      const uint32_t* adj, const ERec* vrec, ERec* erec, uint32_t rs, int keep_anc, RecFmt rf,
                      hipStream_t s);
void launch_patch_in_edges(const uint32_t* adj, uint64_t slots, const uint32_t* bitmap, const uint32_t* bloom,
                           const ERec* vrec, ERec* erec, uint32_t rs, RecFmt rf, hipStream_t s);
// reverse-slot index (undirected graphs): ridx[e] = the index of x in y's row for slot e = (x -> y)
constexpr uint32_t kNoRidx = 0xFFFFFFFFu;
void launch_rev_build(const uint64_t* off, const uint32_t* deg, const uint32_t* adj, uint64_t n, uint64_t slots,
                      uint32_t* ridx, unsigned long long* miss, hipStream_t s);
void launch_patch_rev(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* off, const uint32_t* deg,
                      const uint32_t* adj, const uint32_t* bitmap, const ERec* vrec, ERec* erec, uint32_t rs,
                      RecFmt rf, uint32_t* ridx, unsigned long long* miss, hipStream_t s);
void launch_transpose(const uint32_t* in, uint64_t W, uint32_t L, uint32_t* out, hipStream_t s);
void launch_gather_rows(const uint32_t* walks, uint64_t W, uint32_t L, const uint64_t* list, uint64_t base,
                        uint64_t count, uint32_t* out, hipStream_t s);
void launch_walk_lengths(const uint32_t* walks, uint64_t W, uint32_t L, uint32_t v0, uint32_t v1, uint64_t* len,
                         hipStream_t s);
void launch_index_entries(const uint32_t* walks, uint64_t W, uint32_t L, const ShardMap& sm, int kb,
                          uint32_t v0, uint32_t v1, const uint64_t* col_base, uint64_t* skeys, uint32_t* vals,
                          hipStream_t s);
void launch_index_split(const uint64_t* skeys, uint64_t E, int kb, unsigned long long* counts, uint64_t* keys,
                        hipStream_t s);
unsigned aff_blocks(uint64_t W);
void launch_aff_count(const uint8_t* aff, uint64_t W, uint32_t* counts, hipStream_t s);
void launch_aff_write(const uint8_t* aff, uint64_t W, const uint32_t* offs, const ShardMap& sm,
                      uint32_t* out, hipStream_t s);
void launch_index_pair(const uint64_t* keys, const uint32_t* nexts, uint64_t E, uint64_t* out, hipStream_t s);
void launch_rel_offsets(const uint64_t* off, uint64_t v0, uint64_t cnt, uint32_t* rel, hipStream_t s);
void launch_fill_u32(uint32_t* p, uint64_t cnt, uint32_t v, hipStream_t s);
void launch_fill_u64(uint64_t* p, uint64_t cnt, uint64_t v, hipStream_t s);
void launch_edge_hash_update(const uint64_t* bkeys, uint64_t mb, const uint32_t* chg, int insert, uint64_t* table,
                             uint64_t mask, hipStream_t s);
void launch_edge_hash_build(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* adj, uint64_t* table,
                            uint64_t mask, hipStream_t s);
void launch_filter_sizes(const uint32_t* deg, uint64_t n, uint64_t* words, hipStream_t s);
void launch_filter_pack(const uint32_t* deg, uint64_t n, uint64_t* fdir, hipStream_t s);
void launch_filter_fill(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* adj, const uint64_t* fdir,
                        uint32_t* pool, hipStream_t s);
void launch_filter_plan(const RunInfo* runs, uint64_t k, const uint32_t* deg, const uint64_t* fdir, uint64_t* need,
                        hipStream_t s);
void launch_filter_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* noff, const uint32_t* deg,
                        const uint32_t* adj, const uint64_t* need, const uint64_t* gofs, uint64_t base, uint64_t* fdir,
                        uint32_t* pool, hipStream_t s);
void launch_szudzik64(int op, uint64_t cnt, uint64_t* x, uint64_t* y, uint64_t* z, hipStream_t s);

}  // namespace wharf
