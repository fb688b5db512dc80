// HIP kernels of the WharfMH walk engine, written for gfx950 (CDNA4).
//
// Layout in HBM:
//   vrec[n]        16-B row record {v, deg, row offset:40 | row epoch:24}
//   erec[m]        per CSR slot, its target's row record (one 16-B gather per
//                  walk step); node2vec MH: 32-B records, bytes 16-23 = the
//                  slot's frozen-anchor cache entry
//   adj[m]         u32 targets, rows ascending (the order CompressedEdges::get_edges yields)
//   walks[L][W]    position-major walk matrix: lane i of a wave owns walk i, so every
//                  store/load of one position by a wave is one contiguous 256-B segment
//   ehash          node2vec: edge set for has_edge (32-B buckets)
//   bitmap[n/32]   batch-source set for the rewalk-point scan, + its Bloom filter
#include <cstdlib>
#include <string>
#include <type_traits>

#include "wharf_kernels.h"

namespace wharf {

// ---------------------------------------------------------------------------
// wave-level sum + one atomic per wave for the step / acceptance counters
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_add(unsigned long long* dst, uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

// std::binary_search over the ascending row (node2vec.h:112-119)
__device__ __forceinline__ int64_t row_find(const uint32_t* __restrict__ adj, const Row& r, uint32_t x)
{
    uint64_t lo = r.off, hi = r.off + r.deg;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (adj[mid] < x) lo = mid + 1; else hi = mid;
    }
    return (lo < r.off + r.deg && adj[lo] == x) ? (int64_t)lo : -1;
}

// Edge set of the snapshot: open addressing over 64-bit keys (u << 32 | v),
// 4-key (32-B) buckets, load <= 1/2.  One bucket read answers has_edge in
// almost every case, instead of the log2(deg) dependent probes of
// std::binary_search (node2vec.h:112-119).
__device__ __forceinline__ uint64_t edge_hash(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ bool has_edge(const WalkArgs& a, const Row& rprev, uint32_t c)
{
    if (!a.ehash) return row_find(a.adj, rprev, c) >= 0;
    const uint64_t key = ((uint64_t)rprev.v << 32) | c;
    uint64_t b = (edge_hash(key) & a.ehash_mask) & ~3ull;
    for (;;) {
        const ulonglong2 q0 = *reinterpret_cast<const ulonglong2*>(a.ehash + b);
        const ulonglong2 q1 = *reinterpret_cast<const ulonglong2*>(a.ehash + b + 2);
        if (q0.x == key || q0.y == key || q1.x == key || q1.y == key) return true;
        if (q0.x == kEmptyKey || q0.y == kEmptyKey || q1.x == kEmptyKey || q1.y == kEmptyKey) return false;
        b = (b + 4) & a.ehash_mask;
    }
}

// Per-row neighbour filter (a Bloom filter of each row's targets) in front of
// has_edge in anchor inits.  Row u owns 2^k 32-bit words of `fpool` at
// fdir[u] = word offset | k << 48, 8-16 bits per neighbour; target c sets 3
// bits of one word.  No false negatives, so has_edge's answer is unchanged; a
// negative (most proposals: triangles are rare) saves the random 32-B bucket
// read of the edge hash, and the ~18 probes of one init all land in prev's
// deg-byte filter (2.8 distinct lines on average, visit-weighted, for the
// RMAT graphs of configs[1]) instead of ~18 random buckets.
__device__ __forceinline__ uint64_t filt_hash(uint32_t c)
{
    uint64_t h = (uint64_t)c * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31;
    h *= 0xD6E8FEB86659FD93ull;
    h ^= h >> 32;
    return h;
}
__device__ __forceinline__ uint32_t filt_bits(uint64_t h)
{
    return (1u << (h & 31)) | (1u << ((h >> 5) & 31)) | (1u << ((h >> 10) & 31));
}
__device__ __forceinline__ uint64_t filt_word(uint64_t fd, uint64_t h)
{
    return (fd & kFiltOffMask) + ((h >> 32) & ((1ull << (fd >> kFiltOffBits)) - 1));
}

// has_edge(prev, c) with prev's filter descriptor fd (fdir[prev.v]) loaded once per init
__device__ __forceinline__ bool has_edge_filtered(const WalkArgs& a, const Row& rprev, uint64_t fd, uint32_t c)
{
    if (a.fpool) {
        const uint64_t h = filt_hash(c);
        const uint32_t b = filt_bits(h);
        if ((a.fpool[filt_word(fd, h)] & b) != b) return false;
    }
    return has_edge(a, rprev, c);
}

// node2vec.h:74-88 (DeepWalk: deepwalk.h:67-70 returns 1); rprev = row of prev.
// Weight class: 0 -> 1/p (return), 1 -> 1 (triangle), 2 -> 1/q (outward).
template <int MODEL>
__device__ __forceinline__ uint32_t weight_class(const WalkArgs& a, const Row& rprev, uint32_t c)
{
    if constexpr (MODEL == kDeepWalk) return 1;
    if (c == rprev.v) return 0;
    return has_edge(a, rprev, c) ? 1 : 2;
}

__device__ __forceinline__ float class_weight(const WalkArgs& a, uint32_t cls)
{
    return cls == 0 ? a.inv_p : (cls == 1 ? 1.0f : a.inv_q);
}

template <int MODEL>
__device__ __forceinline__ float weight(const WalkArgs& a, const Row& rprev, uint32_t c)
{
    return class_weight(a, weight_class<MODEL>(a, rprev, c));
}

// MetropolisHastingsSampler::init (metropolis_hastings_sampler.h:69-108) with
// proposals from the (cur, prev, epoch of cur's row) Philox stream: RANDOM
// and BURNIN, one lane at a time.  Returns the anchor as a slot of cur's row,
// and its weight class.  WEIGHT (best of 1 + 20 proposals) is evaluated by
// the whole wave: anchor_init_wave below.

__device__ uint32_t anchor_init(const WalkArgs& a, const Row& rc, const Row& rp, uint32_t& cls)
{
    const uint32_t ep = rc.epoch << 4;
    P4 r = philox4x32_10(rc.v, rp.v, 0, ep | kStreamAnchor, a.key0, a.key1);
    uint32_t last = (uint32_t)pick32(r.x0, rc.deg);
    uint32_t lcls = weight_class<kNode2Vec>(a, rp, a.adj[rc.off + last]);
    if (a.init == kInitBurnin) {
        const uint64_t fd = a.fpool ? a.fdir[rp.v] : 0;
        // 100 MH moves (metropolis_hastings_sampler.h:96-104); the current
        // anchor's class is carried instead of re-probed, and a candidate's
        // has_edge is skipped when it is rejected whatever its class
        for (uint32_t i = 0; i < 100; i++) {
            r = philox4x32_10(rc.v, rp.v, i, ep | kStreamBurnin, a.key0, a.key1);
            const uint32_t cand = (uint32_t)pick32(r.x0, rc.deg);
            const uint32_t cv = a.adj[rc.off + cand];
            const float wl = class_weight(a, lcls);
            const double u = u01(r.x1, r.x2);
            auto move = [&](float wn) { return (wl < wn) || (u <= (double)wn / (double)wl); };
            if (cv == rp.v) {
                if (move(a.inv_p)) { last = cand; lcls = 0; }
                continue;
            }
            const bool m_tri = move(1.0f), m_out = move(a.inv_q);
            if (!m_tri && !m_out) continue;   // rejected whatever the class
            const uint32_t c = has_edge_filtered(a, rp, fd, cv) ? 1u : 2u;
            if (c == 1 ? m_tri : m_out) { last = cand; lcls = c; }
        }
    }
    cls = lcls;
    return last;
}

// SamplerManager::find (a copy, so the anchor stays frozen: libcuckoo find()
// returns by value, cuckoohash_map.hh:596-609).  The anchor of state
// (cur, prev) is cached on the edge prev->cur the walker just crossed (`ac`,
// that slot's entry, or null), tagged with the epoch it was written in.  The
// reference keeps the sampler in cur's SamplerManager (wharfmh.h:296-301),
// which is reset only when cur is a batch source (wharfmh.h:504,539): the
// anchor stays valid while cur's row is unchanged since the tag (checked here)
// AND while prev's row is unchanged — the entry sits in prev's row, which a
// batch with prev as a source rebuilds.  On a directed graph (or with
// WHARF_ANCHOR_CARRY=0) the rebuilt row's entries start empty (k_erec_rows);
// on an undirected graph the anchor carry keeps them through the merge
// (k_save_rows / k_merge_rows) and k_anchor_invalidate resets only the entries
// (y, prev) with y in N(prev) and in a changed edge's other end's filter — the
// only states whose re-initialisation could pick differently — so a kept entry
// equals what re-initialising would compute.  That prev-row
// reset is a deliberate divergence: the reference's surviving
// sampler was initialised against prev's row as it was at the first visit, a
// function of which walks visited the state when, which differs per GPU shard;
// re-initialising keeps every entry a pure function of the current snapshot
// (same Philox proposals, since cur's row epoch is unchanged; only the weight
// classes prev's new row gives them can change the pick), so lazy races are
// benign and the corpus does not depend on which walks (or which GPU) touched
// it first.  The entry also keeps the anchor's weight class (node2vec.h:74-88,
// has_edge(prev, anchor)), valid with the entry since prev's row is unchanged,
// so an accepted step needs one has_edge, not two.
// Entry = slot | tag << 32 | class << 62.
//
// node2vec MH keeps the entry of slot e inside e's 32-B edge record (bytes
// 16-23), so the gather that crosses an edge also brings the anchor of the
// state it enters: `anc` is that entry, carried by the walker.
//
// WEIGHT inits are evaluated by the whole wave at once (anchor_init_wave):
// the lanes that need one publish their (cur, prev) rows, and the proposals
// of all of them (21 each) are dealt over the lanes active at the call,
// whichever they are.  Targets, then prev's filter words, then has_edge for
// filter positives: each one round of independent loads for up to
// kInitRounds proposals per active lane.  Before, each lane walked its 21
// proposals in dependent groups of 4 while the rest of its lock-step wave
// waited (configs[2] node2vec re-walk 88.6 ms, first generation 224 ms; now
// 76.7 / 178 ms).  A per-init LDS minimum over (weight rank, proposal index)
// keeps the reference's choice: the first proposal of maximal weight (strict
// '>', metropolis_hastings_sampler.h:87-107).  Proposals need no has_edge
// when q == 1 (triangle and outward weigh the same) or when prev's neighbour
// filter says no (exact).
#ifndef WHARF_INIT_ROUNDS
#define WHARF_INIT_ROUNDS 2
#endif
constexpr uint32_t kInitRounds = WHARF_INIT_ROUNDS;   // proposals per active lane in flight
#ifndef WHARF_RET_PRUNE
#define WHARF_RET_PRUNE 0   // A/B (round 6): 1 = return pruning below; measured neutral, off by default
#endif
constexpr uint32_t kWavesPerBlock = 4;                // every walk kernel runs 256-thread blocks

struct InitReq {     // a lane's init, published for the wave
    uint32_t cv, cdeg, cep, pv, pdeg, tonly;
    uint64_t coff, poff, fd;
};

// LDS traffic of one wave is processed in order; the barrier keeps the
// compiler from moving the per-init table accesses across the phases
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_wave_barrier(); }

// TONLY (return-first inits, WalkArgs::ret_first): a lane whose step is settled
// whenever the anchor is not a return asks for its proposals' targets only; no
// filter word or edge-hash bucket is read for them.  `resolved` comes back
// false when none of the 21 proposals is the return (the anchor is then not
// known, only that it weighs at most max(1, 1/q)); with a return among them the
// anchor is the first return (the heaviest class when ret_first is set).
template <uint32_t ROUNDS = kInitRounds>
__device__ void anchor_init_wave(const WalkArgs& a, bool need, const Row& rc, const Row& rp, uint32_t& slot,
                                 uint32_t& cls, bool tonly = false, bool* resolved = nullptr)
{
    constexpr uint32_t kInitRounds = ROUNDS;
    __shared__ InitReq s_req[kWavesPerBlock][64];
    __shared__ uint32_t s_key[kWavesPerBlock][64];
    const uint64_t mask = __ballot(need);
    if (!mask) return;
    if (blockDim.x > 64 * kWavesPerBlock) __builtin_trap();   // the per-wave LDS tables assume <= 4 waves
    // proposals are dealt over the lanes active here (the caller's walking lanes), not all 64
    const uint64_t act = __ballot(1), below = (1ull << __lane_id()) - 1;
    const uint32_t wv = threadIdx.x >> 6, nact = (uint32_t)__popcll(act), lane = (uint32_t)__popcll(act & below);
    const uint32_t cnt = (uint32_t)__popcll(mask), me = (uint32_t)__popcll(mask & below);
    const bool use_f = a.fpool && a.inv_q != 1.0f;
    if (need) {
        s_req[wv][me] = InitReq{rc.v, rc.deg, rc.epoch, rp.v, rp.deg, (uint32_t)tonly, rc.off, rp.off,
                                use_f && !tonly ? a.fdir[rp.v] : 0ull};
        s_key[wv][me] = ~0u;
    }
    wave_lds_sync();
    // rank of each class by weight (ties share a rank, so the first proposal wins among them)
    const float w0 = a.inv_p, w1 = 1.0f, w2 = a.inv_q;
    const uint32_t rk0 = (w1 > w0) + (w2 > w0), rk1 = (w0 > w1) + (w2 > w1), rk2 = (w0 > w2) + (w1 > w2);
    // Return pruning: when the return (1/p) is strictly the heaviest class, an init with a return
    // among its proposals is settled by its first return whatever the others' classes, so once the
    // targets are known the returns are published (key < 128: rank 0) and the other proposals of
    // those inits read no filter word and probe no edge-hash bucket (exact; configs[4]'s p = .5,
    // q = 2: ~24 % of the inits hold a return).  Measured neutral (round 6, profiles/r06/ret_prune:
    // configs[4] first generation 1088-1098 vs 1094-1105 ms; the skipped filter words are lines of
    // prev's own filter, mostly cache hits, and the 21 target loads bound the init), so it stays an
    // A/B build (-DWHARF_RET_PRUNE=1, the GPU suite passed with it on).
    const bool prune = WHARF_RET_PRUNE && rk0 == 0 && rk1 > 0 && rk2 > 0;
    const uint32_t total = cnt * kWeightProposals;
    for (uint32_t base = 0; base < total; base += nact * kInitRounds) {
        uint32_t t[kInitRounds], j[kInitRounds], cv[kInitRounds], fw[kInitRounds], fb[kInitRounds];
#pragma unroll
        for (uint32_t b = 0; b < kInitRounds; b++) {
            const uint32_t it = base + b * nact + lane;
            t[b] = it < total ? it / kWeightProposals : cnt;
            j[b] = it - t[b] * kWeightProposals;
            cv[b] = 0;
            if (t[b] < cnt) {
                const InitReq q = s_req[wv][t[b]];
                const P4 r = philox4x32_10(q.cv, q.pv, j[b], (q.cep << 4) | kStreamAnchor, a.key0, a.key1);
                cv[b] = a.adj[q.coff + pick32(r.x0, q.cdeg)];
            }
        }
        bool settled[kInitRounds];   // this proposal's init has a return (prune): its class cannot win
        if (prune) {
#pragma unroll
            for (uint32_t b = 0; b < kInitRounds; b++)
                if (t[b] < cnt && cv[b] == s_req[wv][t[b]].pv) atomicMin(&s_key[wv][t[b]], j[b] << 2);
            wave_lds_sync();
#pragma unroll
            for (uint32_t b = 0; b < kInitRounds; b++) settled[b] = t[b] < cnt && s_key[wv][t[b]] < 128u;
        } else {
#pragma unroll
            for (uint32_t b = 0; b < kInitRounds; b++) settled[b] = false;
        }
#pragma unroll
        for (uint32_t b = 0; b < kInitRounds; b++) {
            fw[b] = 0, fb[b] = 0;
            if (t[b] < cnt && use_f && cv[b] != s_req[wv][t[b]].pv && !s_req[wv][t[b]].tonly && !settled[b]) {
                const uint64_t h = filt_hash(cv[b]);
                fb[b] = filt_bits(h);
                fw[b] = a.fpool[filt_word(s_req[wv][t[b]].fd, h)];
            }
        }
#pragma unroll
        for (uint32_t b = 0; b < kInitRounds; b++) {
            if (t[b] >= cnt) continue;
            const InitReq q = s_req[wv][t[b]];
            uint32_t c;
            if (cv[b] == q.pv) c = 0;
            else if (q.tonly || settled[b]) continue;   // only a return can settle a targets-only init;
                                                        // a return already settles this one
            else if (a.inv_q == 1.0f) c = 1;   // triangle and outward weigh the same
            else if (use_f && (fw[b] & fb[b]) != fb[b]) c = 2;   // filter negative: exact
            else c = has_edge(a, Row{q.pv, q.pdeg, 0u, q.poff}, cv[b]) ? 1 : 2;
            const uint32_t rk = c == 0 ? rk0 : (c == 1 ? rk1 : rk2);
            atomicMin(&s_key[wv][t[b]], (rk << 7) | (j[b] << 2) | c);
        }
    }
    wave_lds_sync();
    if (need) {
        const uint32_t key = s_key[wv][me];
        if (resolved) *resolved = key != ~0u;
        if (key == ~0u) return;   // targets-only, no return among the proposals
        const P4 r = philox4x32_10(rc.v, rp.v, (key >> 2) & 31, (rc.epoch << 4) | kStreamAnchor, a.key0, a.key1);
        slot = (uint32_t)pick32(r.x0, rc.deg);
        cls = key & 3;
    }
}

// The cached anchor of the walker's state, or need = true (no valid entry).
// Class 3 is the return-first marker (walk_step): the state's 21 proposals hold
// no return, the anchor itself is not known yet (need stays true, noret is set).
constexpr uint32_t kClassNoReturn = 3;
__device__ __forceinline__ uint64_t noreturn_entry(uint32_t epoch)
{
    return ((uint64_t)kClassNoReturn << 62) | ((uint64_t)epoch << 32) | 0xFFFFFFFEull;
}
__device__ __forceinline__ void anchor_lookup(const WalkArgs& a, const Row& rc, const Row& rp, const uint64_t* ac,
                                              uint64_t anc, uint32_t& an, uint32_t& cls, bool& need, bool& noret)
{
    need = true;
    noret = false;
    if (ac) {
        const uint32_t tag = (uint32_t)(anc >> 32) & 0x3FFFFFFFu;
        if (anc != kAnchorNone64 && tag >= rc.epoch) {
            if ((uint32_t)(anc >> 62) == kClassNoReturn) {
                noret = true;
            } else {
                need = false;
                an = (uint32_t)anc;
                cls = (uint32_t)(anc >> 62);
            }
        }
    }
}

// The anchor of a state whose cache entry is empty (need), computed and
// cached.  Called by every active lane of the wave together (WEIGHT inits are
// wave-cooperative); lanes with need = false pass an / cls through.
__device__ __forceinline__ uint32_t anchor_fill(const WalkArgs& a, bool need, const Row& rc, const Row& rp,
                                                uint64_t* ac, uint64_t anc, uint32_t an, uint32_t& cls, uint32_t& inits,
                                                bool tonly, bool& resolved)
{
    inits += need;   // per lane; the kernel adds them up once (counters[7])
    resolved = true;
    if (a.init == kInitWeight) {
        anchor_init_wave(a, need, rc, rp, an, cls, tonly, &resolved);
        if (!resolved) {   // the anchor is not known; cache what is: no proposal returns
            if (need && ac) *ac = noreturn_entry(a.epoch);
            return an;
        }
    } else if (need) {
        an = anchor_init(a, rc, rp, cls);
    }
#ifdef WHARF_INIT_STATS
    // A/B probe: inits vs distinct states initialised (the first writer's CAS
    // from the stale entry succeeds; a duplicate finds the value already there)
    if (need && ac) {
        const uint64_t nv = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(ac);
        const bool won = atomicCAS(slot, (unsigned long long)anc, (unsigned long long)nv) == (unsigned long long)anc;
        atomicAdd(a.counters + 3, 1ull);
        if (won) atomicAdd(a.counters + 4, 1ull);
    }
    return an;
#endif
    if (need && ac) *ac = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
    return an;
}

// Heaviest weight class (node2vec.h:74-88: 1/p, 1, 1/q) and the lightest a
// non-return candidate can have (triangle 1 or outward 1/q).
__device__ __forceinline__ float w_heaviest(const WalkArgs& a) { return fmaxf(fmaxf(a.inv_p, 1.0f), a.inv_q); }
__device__ __forceinline__ float w_lightest_nonreturn(const WalkArgs& a) { return fminf(1.0f, a.inv_q); }

// ---------------------------------------------------------------------------
// The walk kernels.  One lane per walk; lane li owns walk matrix column li.
// The walker carries the record of its current vertex, so a step is ONE
// dependent gather: erec[cur.off + pick] = {next vertex, its degree, row
// offset, row epoch} (+ for node2vec MH the anchor entry of the edge).
// ---------------------------------------------------------------------------

// edge records per slot: 16 B, or 32 B with the anchor entry (node2vec MH)
template <int MODEL, bool DET>
constexpr uint64_t kRecStride = (MODEL == kNode2Vec && !DET) ? 2 : 1;

struct Walker {
    Row rc, rp;      // rows of the current and previous vertex
    uint64_t* ac;    // node2vec MH: the anchor cache entry of the state (cur, prev) — the entry of the
                     // edge prev -> cur, or of the re-walk start table — or null
    uint64_t anc;    // node2vec MH: anchor entry of that slot
};

// RL: the edge-record layout fixed at compile time -- 0 the 16-B records, 1 the compact 8-B ones
// (a.rf) -- or -1, read from a.rf per load.  The hot kernels (k_walk, k_rewalk_sweep) are
// instantiated per layout: a per-step branch on a.rf changed the lock-step sweep's code layout
// and cost the 16-B path ~30 % (configs[3] re-walk 18 -> 24.5 ms, profiles/r06/compact_rec).
template <int MODEL, bool DET, int RL = -1>
__device__ __forceinline__ Row load_edge(const WalkArgs& a, uint64_t e, uint64_t& anc)
{
    if constexpr (kRecStride<MODEL, DET> == 2) {
        const Row r = load_rec(a.erec, e * 2);
        anc = a.anchor[e * kAnchorStride];   // same 32-B record
        return r;
    } else if constexpr (RL == 0) {
        return load_rec(a.erec, e);
    } else if constexpr (RL == 1) {
        return unpack_rec8(reinterpret_cast<const uint64_t*>(a.erec)[e], a.rf, a.deg);
    } else {
        return load_erec(a.erec, e, 1, a.rf, a.deg);   // 16 B, or 8 B (compact)
    }
}

// One transition cur -> next from position `pos` (deepwalk.h:64-87 /
// node2vec.h:52-72 through MetropolisHastingsSampler::sample, or the
// deterministic adj(cur)[Random(wid/n).lrand() % deg] of wharfmh.h:296-304).
// Advances the walker; returns the new vertex.
// PARK (node2vec MH re-walk by passes, k_rewalk_park): a state whose anchor is
// not cached and is needed for the decision is not initialised here; the step
// returns with `parked` set and the walker unchanged, and k_park_init computes
// the anchor with full waves before the walker resumes.
template <int MODEL, bool DET, bool PARK = false, bool RF = false, int RL = -1>
__device__ __forceinline__ uint32_t walk_step(const WalkArgs& a, Walker& w, const uint64_t* __restrict__ rt,
                                              uint32_t pos, uint32_t wlo, uint32_t whi, uint32_t ep, uint32_t& accepts,
                                              uint32_t& inits, bool* parked = nullptr)
{
    Row nx;
    if constexpr (DET) {
        // rt = Random(wid / n) restarted at the walk's first re-walked position
        uint64_t unused_anc;
        nx = load_edge<MODEL, DET, RL>(a, w.rc.off + umod64_32(rt[pos], w.rc.deg), unused_anc);
    } else {
        const P4 q = philox4x32_10(wlo, whi, pos, ep | kStreamStep, a.key0, a.key1);
        const uint32_t ci = (uint32_t)pick32(q.x0, w.rc.deg);
        uint64_t canc = kAnchorNone64;
        const Row cand = load_edge<MODEL, DET, RL>(a, w.rc.off + ci, canc);
        if constexpr (MODEL == kDeepWalk) {
            accepts++;   // weights are all 1: sample() always accepts
            nx = cand;
        } else {
            // metropolis_hastings_sampler.h:118-122: accept iff w(a) < w(c) or
            // u <= w(c) / w(a).  A non-return candidate weighs 1 (triangle) or
            // 1/q (outward); when both weights give the same decision the
            // class, and so the has_edge probe, cannot matter (on sparse-
            // triangle graphs the anchor is mostly outward, and an outward
            // anchor accepts every candidate).
            const double u = u01(q.x1, q.x2);
            auto accept = [&](float wc, float wa) { return (wa < wc) || (u <= (double)wc / (double)wa); };
            uint32_t acls = 0, ai = 0;
            bool need, noret;
            anchor_lookup(a, w.rc, w.rp, w.ac, w.anc, ai, acls, need, noret);
            // The decision falls monotonically with w(a) and rises with w(c): a
            // candidate accepted against the heaviest class with its lightest
            // possible weight is accepted whatever the anchor is, so an anchor
            // that is not cached yet is not computed for it (exact; the entry
            // stays empty for a later walker that needs it).  In the sparse
            // re-walks of configs[4] 79 % of the steps enter a state with no
            // cached anchor; p = .5, q = 2 settles a quarter of them here.
            const bool sure = need && !a.no_sure &&
                              accept(cand.v == w.rp.v ? a.inv_p : w_lightest_nonreturn(a), w_heaviest(a));
            const bool init = need && !sure;
            bool resolved = true;
            uint32_t ccls = 3;   // the candidate's class once probed, 3 = not probed
            if constexpr (PARK) {
                if (init) {
                    *parked = true;
                    return 0;
                }
            } else {
                // Return-first (ret_first: the return 1/p is the unique heaviest class, WEIGHT
                // inits).  The candidate's own class is probed first; when it is accepted against
                // every non-return anchor (max(1, 1/q)), only a return among the 21 proposals could
                // reject it, and a return needs no has_edge: the init reads its proposals' targets
                // and none of prev's filter words or edge-hash buckets.  Exact (the decision falls
                // monotonically with the anchor's weight).  When no proposal returns, the entry
                // keeps that fact (kClassNoReturn), so the next walker whose candidate is settled
                // by it needs no init at all.  (A return candidate is sure-accepted under ret_first.)
                bool tonly = false, fill = init;
                if (RF && a.ret_first && init) {
                    ccls = cand.v == w.rp.v ? 0u : (has_edge(a, w.rp, cand.v) ? 1u : 2u);
                    tonly = accept(class_weight(a, ccls), fmaxf(1.0f, a.inv_q));
                    if (tonly && noret) fill = false;   // settled by the cached fact alone
                }
                ai = anchor_fill(a, fill, w.rc, w.rp, w.ac, w.anc, ai, acls, inits, tonly && !noret, resolved);
                if (init && !fill) resolved = false;
            }
            bool ok = true;   // proposing the anchor itself is always accepted (and an unresolved
                              // targets-only init: the candidate wins against any non-return anchor)
            if (!sure && resolved && ai != ci) {
                const float wa = class_weight(a, acls);
                if (cand.v == w.rp.v) {
                    ok = accept(a.inv_p, wa);
                } else {
                    const bool ok_tri = accept(1.0f, wa), ok_out = accept(a.inv_q, wa);
                    const bool tri = ok_tri == ok_out || (ccls != 3 ? ccls == 1 : has_edge(a, w.rp, cand.v));
                    ok = tri ? ok_tri : ok_out;
                }
            }
            accepts += ok;
            w.ac = a.anchor + (w.rc.off + (ok ? ci : ai)) * kAnchorStride;
            if (ok) {
                nx = cand;
                w.anc = canc;
            } else {
                nx = load_edge<MODEL, DET>(a, w.rc.off + ai, w.anc);
            }
        }
    }
    w.rp = w.rc;
    w.rc = nx;
    return nx.v;
}

// Re-walk start states (node2vec MH).  A re-walk starts at a batch source x
// with the walk's previous vertex prev; the anchor of state (x, prev) is
// cached on the edge prev -> x, a slot of prev's row found by a binary search
// (~log2 deg(prev) dependent loads, and prev is degree-biased).  Walks share
// start states (configs[2]: ~28 M re-walks over far fewer (x, prev) pairs),
// so the re-walk keeps a per-batch table keyed by (x, prev) whose value is
// the state's anchor entry: one 64-B bucket read finds it (a CAS claims a
// new key).  It caches the same pure function of the snapshot as the edge
// entry (x's row was reset in this epoch, so only this epoch's entries are
// valid in either place), so the corpus does not change.  Buckets of four
// {key, entry} pairs, linear probing over kStabProbes buckets; null when
// they are full (the caller searches prev's row).
constexpr uint32_t kStabProbes = 4;
__device__ __forceinline__ uint64_t* stab_entry(const WalkArgs& a, uint32_t x, uint32_t prev)
{
    typedef unsigned long long ull;
    const uint64_t key = ((uint64_t)x << 32) | prev;   // ids < 2^32 - 2: ~0 is no key
    uint64_t b = edge_hash(key) & a.stab_mask;
    for (uint32_t probe = 0; probe < kStabProbes; probe++, b = (b + 1) & a.stab_mask) {
        uint64_t* e = a.stab + b * 8;
        const ulonglong2 q0 = *reinterpret_cast<const ulonglong2*>(e), q1 = *reinterpret_cast<const ulonglong2*>(e + 2);
        const ulonglong2 q2 = *reinterpret_cast<const ulonglong2*>(e + 4), q3 = *reinterpret_cast<const ulonglong2*>(e + 6);
        const uint64_t k[4] = {q0.x, q1.x, q2.x, q3.x};
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            if (k[i] == key) return e + 2 * i + 1;
            if (k[i] == kStabEmpty) {   // (the read may be stale: the CAS decides)
                const ull old = atomicCAS(reinterpret_cast<ull*>(e + 2 * i), (ull)kStabEmpty, (ull)key);
                if (old == kStabEmpty || old == key) return e + 2 * i + 1;
            }
        }
    }
    return nullptr;
}

// Walker state at position p of walk wid (cur = its vertex): the rows of cur
// and prev and, for node2vec MH, the slot of the edge prev -> cur.
template <int MODEL, bool DET>
__device__ __forceinline__ void walk_state(const WalkArgs& a, uint32_t cur, uint32_t prev, uint32_t p, uint32_t wlo,
                                           uint32_t whi, uint32_t ep, Walker& w)
{
    w.rc = load_rec(a.vrec, cur);
    w.rp = w.rc;
    w.ac = nullptr;
    w.anc = kAnchorNone64;
    if constexpr (MODEL == kNode2Vec && !DET) {
        if (p > 0) {
            w.rp = load_rec(a.vrec, prev);
        } else if (w.rc.deg) {
            // Node2Vec::initial_state: prev = random neighbour (node2vec.h:42-50)
            const P4 q = philox4x32_10(wlo, whi, 0, ep | kStreamPrev, a.key0, a.key1);
            uint64_t unused;
            w.rp = load_edge<MODEL, DET>(a, w.rc.off + pick32(q.x0, w.rc.deg), unused);
        }
        // (At a re-walk start cur is a batch source reset in this epoch, so the
        // entry found here is one another walker initialised in this epoch;
        // skipping the search and initialising instead gives the same corpus but
        // many more inits: configs[2] node2vec re-walk 73 -> 93 ms.)
        if (w.rc.deg) {
            // a re-walk start: the start-state table (one bucket read); otherwise,
            // or when its neighbourhood is full, the edge prev -> cur in prev's row
            if (p > 0 && a.stab) w.ac = stab_entry(a, w.rc.v, w.rp.v);
            if (!w.ac) {
                const int64_t ein = row_find(a.adj, w.rp, w.rc.v);
                if (ein >= 0) w.ac = a.anchor + (uint64_t)ein * kAnchorStride;
            }
            if (w.ac) w.anc = *w.ac;
        }
    }
}

// Anchor pre-init after an update batch (node2vec MH).  A batch invalidates
// the anchors of two families of states around each source x: (y, x) — the
// entries of x's rebuilt row, slot x -> y — and (x, y) — x's samplers were
// reset (wharfmh.h:504,539), entries on the in-edges y -> x.  The re-walk
// visits nearly all of them (configs[2]: ~9.5 M inits per batch, 1.0-1.1 per
// state), and lazily each init stalls its lock-step wave for rounds of
// dependent loads while most lanes have none.  Measured on configs[2]: the
// sorted re-walk 55.8 -> 54.0 ms plus 1.1 ms here (profiles/r02/n2v_preinit).
// Here one lane per (source, slot) pair computes both states' anchors with
// every lane of the wave initialising (anchor_init_wave at full occupancy),
// and writes them where the walkers look: the edge entries, and for (x, y) —
// the re-walk start states — the start-state table too.  The anchor is a
// pure function of the snapshot, so the corpus is unchanged (entries the
// pre-init does not reach, e.g. in-edges of a directed graph without a
// reverse edge, are initialised lazily as before).
// preoff[i] = sum of the new degrees of sources < i, preoff[k] = pairs.
#ifndef WHARF_PREINIT_ROUNDS
#define WHARF_PREINIT_ROUNDS 4   // proposals per lane in flight in the pre-init kernels (full waves)
#endif
__device__ __forceinline__ void anchor_compute(const WalkArgs& a, bool need, const Row& rc, const Row& rp,
                                               uint32_t& an, uint32_t& cls, uint32_t& inits)
{
    inits += need;
    if (a.init == kInitWeight) anchor_init_wave<WHARF_PREINIT_ROUNDS>(a, need, rc, rp, an, cls);
    else if (need) an = anchor_init(a, rc, rp, cls);
}

__global__ __launch_bounds__(256) void k_anchor_preinit(WalkArgs a, const uint64_t* __restrict__ preoff, uint64_t k)
{
    const uint64_t total = preoff[k];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t inits = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        uint64_t lo = 0, hi = k;   // the source i with preoff[i] <= t < preoff[i + 1]
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (preoff[mid] <= t) lo = mid; else hi = mid;
        }
        const uint32_t x = a.runs[lo].src;
        const Row rx = load_rec(a.vrec, x);
        const uint64_t e = rx.off + (t - preoff[lo]);
        const uint32_t y = a.adj[e];
        const Row ry = load_rec(a.vrec, y);
        uint32_t an = 0, cls = 0;
        // (y, x): entry of slot x -> y (a walker that crosses it and stays at y needs y's row);
        // an entry carried through the batch (anchor carry) is still valid
        const uint64_t ca = a.anchor[e * kAnchorStride];
        const bool carried = ca != kAnchorNone64 && ((uint32_t)(ca >> 32) & 0x3FFFFFFFu) >= ry.epoch &&
                             (uint32_t)(ca >> 62) != kClassNoReturn;
        const bool need_a = ry.deg != 0 && !carried;
        anchor_compute(a, need_a, ry, rx, an, cls, inits);
        if (need_a) a.anchor[e * kAnchorStride] = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
        // (x, y): entry of slot y -> x, and the start-state table
        const int64_t ein = row_find(a.adj, ry, x);
        const bool need_b = ein >= 0;
        anchor_compute(a, need_b, rx, ry, an, cls, inits);
        if (need_b) {
            const uint64_t v = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
            a.anchor[(uint64_t)ein * kAnchorStride] = v;
            if (a.stab) {
                uint64_t* se = stab_entry(a, x, y);
                if (se) *se = v;
            }
        }
    }
    wave_add(a.counters + 7, inits);
}

// Generation with a cold anchor cache (node2vec MH, the first generation of a
// handle): when the walks take many more steps than there are states, nearly
// every state (cur, prev) — one per CSR slot prev -> cur — is entered, and
// lazily each first entry stalls its lock-step wave for an init.  Instead the
// anchors of all slots are computed up front, one lane per slot, every lane of
// a wave initialising; the same pure function of the snapshot, so the corpus
// is unchanged.  owner[e] = (row owner of slot e) + 1, written row by row (one
// wave per row, lanes over its slots: no scan over the pool, whose ~4.1 G slots
// at configs[4] are past 2^31); slack slots keep 0 and are skipped.
__global__ __launch_bounds__(256) void k_slot_owner_fill(const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ deg, uint64_t n,
                                                         uint32_t* __restrict__ owner)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t v = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); v < n; v += waves) {
        const uint64_t o = off[v];
        const uint32_t d = deg[v];
        for (uint32_t i = lane; i < d; i += 64) owner[o + i] = (uint32_t)v + 1;
    }
}

// The up-front inits in two orders (round 6, undirected graphs with the reverse-slot index).  A
// state (y, x) -- cur y, prev x, its entry on slot x -> y -- costs random 128-B lines on one side:
// in prev order (lanes over x's row, x's filter words and row record shared by the wave) the 21
// proposals' targets land in y's row, ~min(21, lines of y's row) distinct lines; in cur order
// (lanes over y's row, y's row shared) they are x's filter words, ~min(21, lines of x's filter),
// plus x's filter descriptor and the entry written at the reverse slot.  Each state goes to the
// cheaper side by InitOrder (a table the host fills from that model): cur order iff y's row spans
// at least t[filt_log2_words(deg x)] lines.  Prev-order lanes read y's row record from the slot's
// own edge record (coalesced, 32-B node2vec records) instead of vrec[y] (one random line each);
// cur-order lanes read x's record from the slot y -> x likewise.  XCD-aware: a window of the
// grid-stride loop is dealt to the 8 XCDs in contiguous eighths, so each row's lines are fetched
// into one XCD's L2.  Same anchors, one init per state.
#ifndef WHARF_INIT_XCD_SPAN
#define WHARF_INIT_XCD_SPAN 0   // A/B: 1 = each XCD takes one contiguous eighth of all slots, 2 = plain order
#endif
struct SlotLoop {
    uint64_t i, end, step;
};
__device__ __forceinline__ SlotLoop init_slot_loop(uint64_t slots)
{
    const uint32_t nb = gridDim.x, b = blockIdx.x;   // dispatch deals blocks to XCDs round-robin
    if (nb % 8 || WHARF_INIT_XCD_SPAN == 2) return SlotLoop{(uint64_t)b * blockDim.x + threadIdx.x, slots, (uint64_t)nb * blockDim.x};
    if (WHARF_INIT_XCD_SPAN == 1) {
        const uint64_t part = (slots + 7) / 8, lo = min(slots, (uint64_t)(b % 8) * part);
        return SlotLoop{lo + (uint64_t)(b / 8) * blockDim.x + threadIdx.x, min(slots, lo + part),
                        (uint64_t)(nb / 8) * blockDim.x};
    }
    return SlotLoop{((uint64_t)(b % 8) * (nb / 8) + b / 8) * blockDim.x + threadIdx.x, slots,
                    (uint64_t)nb * blockDim.x};
}
__device__ __forceinline__ bool init_in_cur_order(const InitOrder& ord, uint32_t dcur, uint32_t dprev)
{
    const uint32_t lg = min(filt_log2_words(dprev), kInitOrderLg - 1);
    return ((uint64_t)dcur + 31) / 32 >= ord.t[lg];
}

// by_cur_y / by_cur_x (round 5, undirected graphs): the states (y, x) with deg(y) > by_cur_y and
// deg(x) <= by_cur_x are left to k_anchor_init_by_cur (0: none are).  hybrid: the states
// init_in_cur_order selects are left to k_anchor_init_cur.
__global__ __launch_bounds__(256) void k_anchor_init_all(WalkArgs a, const uint32_t* __restrict__ owner, uint64_t slots,
                                                         uint32_t by_cur_y, uint32_t by_cur_x, bool hybrid,
                                                         InitOrder ord)
{
    uint32_t inits = 0;
    for (SlotLoop l = init_slot_loop(slots); l.i < l.end; l.i += l.step) {
        const uint64_t e = l.i;
        const uint32_t y = a.adj[e], o = owner[e];
        bool need = y != kGap && o != 0;
        Row rx{}, ry{};
        if (need) {
            rx = load_rec(a.vrec, o - 1);
            ry = load_rec(a.erec, e * 2);   // y's row: slot e's own (32-B) record
            need = e < rx.off + rx.deg && ry.deg != 0;   // (slots past a row's end are kGap; the test is cheap)
            if (by_cur_y && ry.deg > by_cur_y && rx.deg <= by_cur_x) need = false;
            if (hybrid && init_in_cur_order(ord, ry.deg, rx.deg)) need = false;
        }
        uint32_t an = 0, cls = 0;
        anchor_compute(a, need, ry, rx, an, cls, inits);
        if (need) a.anchor[e * kAnchorStride] = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
    }
    wave_add(a.counters + 7, inits);
}

// The states init_in_cur_order selects, in cur order: one lane per slot f = y -> x of y's row (the
// state (y, x)); x's row from f's own record; the entry written at slot x -> y = off(x) + ridx[f].
// VERIFY (tests, WHARF_REV_VERIFY): the reverse slot is checked first, and a stale one is found by
// a search instead.
template <bool VERIFY>
__global__ __launch_bounds__(256) void k_anchor_init_cur(WalkArgs a, const uint32_t* __restrict__ owner, uint64_t slots,
                                                         const uint32_t* __restrict__ ridx, InitOrder ord)
{
    uint32_t inits = 0;
    for (SlotLoop l = init_slot_loop(slots); l.i < l.end; l.i += l.step) {
        const uint64_t f = l.i;
        const uint32_t x = a.adj[f], o = owner[f];
        bool need = x != kGap && o != 0;
        Row ry{}, rx{};
        int64_t ein = -1;
        if (need) {
            ry = load_rec(a.vrec, o - 1);   // cur: the row this slot belongs to (shared by the wave)
            rx = load_rec(a.erec, f * 2);   // prev: slot f's own record
            need = f < ry.off + ry.deg && rx.deg != 0 && init_in_cur_order(ord, ry.deg, rx.deg);
            if (need) {
                const uint32_t r = ridx[f];
                ein = r == kNoRidx ? -1 : (int64_t)(rx.off + r);
                if (VERIFY && ein >= 0 && (r >= rx.deg || a.adj[ein] != ry.v)) ein = -1;
                if (ein < 0) ein = row_find(a.adj, rx, ry.v);
                need = ein >= 0;   // (an undirected graph always has the slot x -> y)
            }
        }
        uint32_t an = 0, cls = 0;
        anchor_compute(a, need, ry, rx, an, cls, inits);
        if (need) a.anchor[(uint64_t)ein * kAnchorStride] = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
    }
    wave_add(a.counters + 7, inits);
}

// The same anchors, for the states (y, x) whose cur y is a hub (deg > by_cur_y) and
// whose prev x is small (deg <= by_cur_x), computed in cur order: one lane per slot
// y -> x of y's row, so a wave's states share cur's row and the 21 proposals of each
// land in one row the wave keeps in L2, while the small prev's filter words (one
// line) and the search for slot x -> y in x's short row (where the entry lives) are
// the random part.  In prev order (k_anchor_init_all, lanes of one prev's row) a
// hub cur's proposals are ~21 random lines per state.  Line model on RMAT at
// configs[4]'s density (scale 20): 8.46 lines per state in prev order,
// 6.66 with the states of hub y >= 256 and x <= 256 taken here.  Undirected graphs
// only: the state (y, x) of slot x -> y is reached through slot y -> x.  (Round 5; without
// the reverse-slot index only.)
__global__ __launch_bounds__(256) void k_anchor_init_by_cur(WalkArgs a, const uint32_t* __restrict__ owner,
                                                            uint64_t slots, uint32_t by_cur_y, uint32_t by_cur_x)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t inits = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < slots; e += stride) {
        const uint32_t x = a.adj[e], o = owner[e];
        bool need = x != kGap && o != 0;
        Row rx{}, ry{};
        if (need) {
            ry = load_rec(a.vrec, o - 1);   // cur: the row this slot belongs to
            rx = load_rec(a.vrec, x);
            need = e < ry.off + ry.deg && ry.deg > by_cur_y && rx.deg <= by_cur_x && rx.deg != 0;
        }
        uint32_t an = 0, cls = 0;
        anchor_compute(a, need, ry, rx, an, cls, inits);
        if (need) {
            const int64_t ein = row_find(a.adj, rx, ry.v);   // slot x -> y: the state's entry
            if (ein >= 0) a.anchor[(uint64_t)ein * kAnchorStride] = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
        }
    }
    wave_add(a.counters + 7, inits);
}

void launch_slot_owner_fill(const uint64_t* off, const uint32_t* deg, uint64_t n, uint32_t* owner, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_slot_owner_fill, cu_count() * 32, 256, 0, s, off, deg, n, owner);
}

void launch_anchor_init_all(const WalkArgs& a, const uint32_t* owner, uint64_t slots, uint32_t by_cur_y,
                            uint32_t by_cur_x, const uint32_t* ridx, const InitOrder& ord, bool verify, hipStream_t s)
{
    if (!slots) return;
    const bool hybrid = ridx != nullptr;
    if (hybrid) by_cur_y = 0;
    hipLaunchKernelGGL(k_anchor_init_all, cu_count() * 8, 256, 0, s, a, owner, slots, by_cur_y, by_cur_x, hybrid, ord);
    if (hybrid) {
        if (verify) hipLaunchKernelGGL(k_anchor_init_cur<true>, cu_count() * 8, 256, 0, s, a, owner, slots, ridx, ord);
        else hipLaunchKernelGGL(k_anchor_init_cur<false>, cu_count() * 8, 256, 0, s, a, owner, slots, ridx, ord);
    } else if (by_cur_y) {
        hipLaunchKernelGGL(k_anchor_init_by_cur, cu_count() * 8, 256, 0, s, a, owner, slots, by_cur_y, by_cur_x);
    }
}

__global__ void k_source_degrees(const RunInfo* __restrict__ runs, uint64_t k, const ERec* __restrict__ vrec,
                                 uint64_t* __restrict__ out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= k; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = i < k ? vrec[runs[i].src].deg : 0;
}

void launch_source_degrees(const RunInfo* runs, uint64_t k, const ERec* vrec, uint64_t* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_source_degrees, grid_for(k + 1, 256), 256, 0, s, runs, k, vrec, out);
}

void launch_anchor_preinit(const WalkArgs& a, const uint64_t* preoff, uint64_t k, hipStream_t s)
{
    if (k) hipLaunchKernelGGL(k_anchor_preinit, cu_count() * 8, 256, 0, s, a, preoff, k);
}

// Generation (wharfmh.h:275-326): every lane of a wave writes the same
// position at the same time -> one contiguous 256-B store per step.
// BLK: the handle holds a block shard (ShardMap); a contiguous one maps j -> lo + j
// in its own instantiation, which compiles to round 3's code (the generic map in
// the sweep's prologue changed its loop's code layout: configs[2] re-walk 43.4 ->
// 48.6 ms on one box, profiles/r04/sweep_map/)
template <bool BLK>
__device__ __forceinline__ uint32_t start_vertex(const WalkArgs& a, uint64_t j)
{
    if constexpr (BLK) return (uint32_t)shard_map(a).vertex(j);
    return (uint32_t)(a.lo + j);
}

// The walk matrix written (k_walk, k_rewalk_sweep) and scanned (k_rewalk_sweep) with non-temporal
// stores and loads (round 6), so the streamed matrix displaces fewer of the edge-record lines the
// gathers hit in the Infinity Cache: same-box A/B, 3 reps, headline +0.4 %, configs[2] DeepWalk MH
// re-walk -3 % (profiles/r06/nt_walks/).  0 / 0 restores plain accesses (A/B).
#ifndef WHARF_NT_WALK_STORES
#define WHARF_NT_WALK_STORES 1
#endif
#ifndef WHARF_NT_SWEEP_LOADS
#define WHARF_NT_SWEEP_LOADS 1
#endif
__device__ __forceinline__ void put_walk(uint32_t* p, uint32_t v)
{
    if (WHARF_NT_WALK_STORES) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ uint32_t get_walk(const uint32_t* p)
{
    if (WHARF_NT_SWEEP_LOADS) return __builtin_nontemporal_load(p);
    return *p;
}

template <int MODEL, bool DET, bool BLK = false, int RL = -1>
__global__ __launch_bounds__(256) void k_walk(WalkArgs a)
{
    uint32_t steps = 0, accepts = 0, inits = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W;
    for (uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; li < W; li += stride) {
        const uint64_t r = li / a.n_loc;
        const uint32_t v = start_vertex<BLK>(a, li - r * a.n_loc);
        const uint64_t wid = r * a.n + v;
        const uint32_t ep = a.epoch << 4, wlo = (uint32_t)wid, whi = (uint32_t)(wid >> 32);
        const uint64_t* __restrict__ rt = DET ? a.rtab + r * a.L : nullptr;
        walks[li] = v;
        Walker w;
        walk_state<MODEL, DET>(a, v, v, 0, wlo, whi, ep, w);
        uint32_t pos = 0;
        for (; pos + 1 < a.L; pos++) {
            if (w.rc.deg == 0) break;   // dead end: the walk stops (reference: lrand() % 0)
            put_walk(walks + (uint64_t)(pos + 1) * W + li,
                     walk_step<MODEL, DET, false, false, RL>(a, w, rt, pos, wlo, whi, ep, accepts, inits));
            steps++;
        }
        for (pos = pos + 1; pos < a.L; pos++) walks[(uint64_t)pos * W + li] = kSent;
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// Fused rewalk-point scan + suffix re-walk (wharfmh.h:519-537 + 761-859),
// DeepWalk and deterministic mode.  The rewalk point of a walk is the first
// position holding a batch source; positions after it are re-sampled on the
// updated graph.  Rewalk points differ from lane to lane, so a
// lane-at-its-own-pace loop would make every store of a wave hit 64 different
// rows (4-B partial-line writes, measured 1.4x slower).  Instead each wave
// sweeps positions in lock step, scan and walk interleaved: at position pos a
// lane is still scanning (reads the old value, checks the bitmap), walking
// (writes a new vertex) or done; whenever any lane of the wave writes, all
// lanes write (scanning lanes their old value), so each row of a wave is one
// full 256-B store.  A lane starting its walk costs the wave one 16-B gather,
// so the scan of late-starting lanes hides behind the walking of the others.
enum : uint32_t { kLaneScan = 0, kLaneWalk = 1, kLaneDone = 2 };

// Batch-source test of the rewalk-point scan: a 16-KiB Bloom filter of the
// batch sources (two hashes, 2^17 bits: ~2 % false positives at 10 k sources)
// in LDS answers most positions; only its positives read the exact bitmap.
// Without it every scanned position is a random L2 read of the n-bit bitmap
// (1.6 G per configs[2] batch, the re-walk kernel's only extra cost over
// generation).
__device__ __forceinline__ void bloom_to_lds(const WalkArgs& a, uint32_t* s_bloom)
{
    for (uint32_t i = threadIdx.x; i < kBloomWords; i += blockDim.x) s_bloom[i] = a.bloom[i];
    __syncthreads();
}

__device__ __forceinline__ bool is_source(const WalkArgs& a, const uint32_t* s_bloom, uint32_t x)
{
    if (!bloom_test(s_bloom, x)) return false;
    return (a.bitmap[x >> 5] >> (x & 31)) & 1u;
}

template <int MODEL, bool DET, bool BLK = false, int RL = -1>
__global__ __launch_bounds__(256) void k_rewalk_sweep(WalkArgs a)
{
    __shared__ uint32_t s_bloom[kBloomWords];
    bloom_to_lds(a, s_bloom);
    uint32_t steps = 0, accepts = 0, inits = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W;
    const uint32_t L = a.L;
    for (uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; li < W; li += stride) {
        const uint64_t r = li / a.n_loc;
        // the start vertex: the walk's position 0 (no re-walk moves it) under a block
        // shard; lo + j otherwise (round 3's code: the generic map in this prologue changed
        // the loop's code layout, configs[2] re-walk 43.4 -> 48.6 ms, profiles/r04/sweep_map/)
        const uint32_t v = BLK ? walks[li] : start_vertex<false>(a, li - r * a.n_loc);
        const uint64_t wid = r * a.n + v;
        const uint32_t ep = a.epoch << 4, wlo = (uint32_t)wid, whi = (uint32_t)(wid >> 32);
        const uint64_t* __restrict__ rt = DET ? a.rtab + r * L : nullptr;
        uint32_t mode = kLaneScan, p = kNoRewalk;
        uint32_t x = v, xprev = v;                       // old value at pos, at pos - 1
        uint32_t xn = L > 1 ? walks[W + li] : kSent;     // old value at pos + 1 (prefetched)
        Walker w;
        w.rc.deg = 0;
        for (uint32_t pos = 0; pos < L; pos++) {
            uint32_t val = kSent;
            bool fresh = false;
            if (mode == kLaneWalk) {
                if (w.rc.deg) {
                    val = walk_step<MODEL, DET, false, false, RL>(a, w, rt, DET ? pos - 1 - p : pos - 1, wlo, whi, ep,
                                                                  accepts, inits);
                    steps++;
                }
                fresh = true;
            } else if (mode == kLaneScan) {
                if (pos > 0) {
                    xprev = x;
                    x = xn;
                    if (pos + 1 < L && x != kSent) xn = get_walk(walks + (uint64_t)(pos + 1) * W + li);
                }
                val = x;
                if (x == kSent) {
                    mode = kLaneDone;   // old walk ended: no batch source on it
                } else if (is_source(a, s_bloom, x)) {
                    p = pos;
                    mode = a.scan_only ? kLaneDone : kLaneWalk;
                    if (!a.scan_only) walk_state<MODEL, DET>(a, x, xprev, p, wlo, whi, ep, w);
                }
            }
            if (!a.scan_only && __any(fresh)) {
                // kLaneDone lanes: unaffected (their old walk is kSent from
                // here on) — the same value is rewritten
                put_walk(walks + (uint64_t)pos * W + li, val);
            }
            if (!__any(mode != kLaneDone)) break;
        }
        a.aff[li] = (uint8_t)p;
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// Deterministic re-walk by suffix table.  In deterministic mode a re-walk
// from (vertex s, position p) of a round-r walk draws Random(r) from draw 0
// again (wharfmh.h:813-840), so its suffix depends only on (r, s): it is the
// first L-1-p steps of a walk STARTING at s in round r on the new graph.  The
// rewalk vertex is always a batch source, so k_det_suffix walks the wpv x k
// suffixes once (k <= 10 k distinct sources per batch) and k_rewalk_chunked
// copies them: the re-walk of ~34 M walks becomes a streaming pass over the
// walk matrix plus reads of a small, cache-resident table, instead of one
// random graph gather per re-walked position.  Same values, same step count.
constexpr uint32_t kXcds = 8;   // MI355X: 8 XCDs, workgroups dispatched round-robin

__global__ __launch_bounds__(256) void k_det_suffix(WalkArgs a)
{
    const uint64_t total = (uint64_t)a.wpv * a.memo_k;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = t / a.memo_k, i = t - r * a.memo_k;
        const uint32_t src = a.runs[i].src;
        uint32_t* __restrict__ out = a.memo + t * a.memo_stride;
        const uint64_t* __restrict__ rt = a.rtab + r * a.L;
        Walker w;
        walk_state<kDeepWalk, true>(a, src, src, 0, 0, 0, 0, w);
        out[0] = src;
        uint32_t unused = 0;
        for (uint32_t j = 1; j < a.memo_stride; j++) {
            uint32_t val = kSent;
            if (j < a.L && w.rc.deg) val = walk_step<kDeepWalk, true>(a, w, rt, j - 1, 0, 0, 0, unused, unused);
            out[j] = val;
        }
    }
}

// Chunked rewalk-point scan (and the suffix-table copy of the deterministic
// re-walk).  The sweeps above read a lane's old walk one position at a time
// with one row prefetched: a wave has one 256-B row in flight, so the scan is
// latency-bound (configs[2]: 6.7 GB in 5.4 ms, 1.2 TB/s).  Here a wave reads
// kScanChunk rows per round trip: the next chunk's rows are loaded while the
// current one is tested (Bloom filter in LDS, then the exact bitmap for the
// positives in ascending order), and in the copy the chunk's rows are
// written whole — the suffix-table value for walking lanes, the old value
// (still in registers) for the others.
#ifndef WHARF_SCAN_CHUNK
#define WHARF_SCAN_CHUNK 16
#endif
#ifndef WHARF_CHUNK_NT
#define WHARF_CHUNK_NT 3   // bit 0: non-temporal walk loads, bit 1: stores (A/B: -2..-3 % on the copy)
#endif
// Non-temporal row loads pay when most walks re-walk (configs[2], 81 %: copy
// 7.9 -> 7.3 ms, scan 3.25 -> 3.14 ms) and cost when few do (configs[3] 1/8
// shard, 32 %: copy 7.8 -> 10.7 ms), so the chunked scans are instantiated both
// ways and the host picks per batch (WalkArgs::nt_rows; profiles/r02/nt_rows).
constexpr uint32_t kScanChunk = WHARF_SCAN_CHUNK;
#ifndef WHARF_COPY_GROUP
#define WHARF_COPY_GROUP 64   // lanes whose row segment the suffix copy writes together
#endif
constexpr uint32_t kCopyGroup = WHARF_COPY_GROUP;
template <bool NTL = (WHARF_CHUNK_NT & 1) != 0>
__device__ __forceinline__ uint32_t walk_load(const uint32_t* p)
{
    if (NTL) return __builtin_nontemporal_load(p);
    return *p;
}
__device__ __forceinline__ void walk_store(uint32_t* p, uint32_t v)
{
    if (WHARF_CHUNK_NT & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// One walk-matrix row of a wave through a buffer resource: the row base (wave
// uniform) sits in SGPRs and the lane adds its 32-bit byte offset, so the
// address costs no VALU (a global access pays a 64-bit VALU add per row; the
// chunked scans are VALU-bound).  aux 2 = non-temporal.
#ifndef WHARF_ROW_BUFFER
#define WHARF_ROW_BUFFER 0   // A/B (profiles/r02/chunked_scan): same scan time, copy 1-3 % slower
#endif
constexpr int kRowRsrcFlags = 0x00020000;   // gfx9 buffer descriptor word 3 (32-bit raw access)
template <bool NTL = (WHARF_CHUNK_NT & 1) != 0>
__device__ __forceinline__ uint32_t row_load(const uint32_t* row, uint32_t lane)
{
    if (!WHARF_ROW_BUFFER) return walk_load<NTL>(row + lane);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, 0x7FFFFFFF, kRowRsrcFlags);
    return __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, 0, NTL ? 2 : 0);
}
__device__ __forceinline__ void row_store(uint32_t* row, uint32_t lane, uint32_t v)
{
    if (!WHARF_ROW_BUFFER) { walk_store(row + lane, v); return; }
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, 0x7FFFFFFF, kRowRsrcFlags);
    __builtin_amdgcn_raw_buffer_store_b32(v, r, lane * 4, 0, (WHARF_CHUNK_NT & 2) ? 2 : 0);
}
static_assert(kMemoPad >= kScanChunk, "suffix table padding");
static_assert(kScanChunk % 4 == 0 && kScanChunk <= 32, "chunk positions live in a 32-bit mask");

__device__ __forceinline__ uint32_t chunk_pick(const uint32_t (&x)[kScanChunk], uint32_t j)
{
    // and/or, not a select chain: LLVM folds selects over an array into a
    // dynamically indexed load, which puts the array in scratch memory
    uint32_t v = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanChunk; i++) v |= x[i] & (0u - (uint32_t)(j == i));
    return v;
}

// Batch-source test of one chunk, in two halves so a caller can put the next
// chunk's row loads between them.  chunk_issue: the Bloom test of every
// position (LDS), then the exact bitmap word of every positive, all loads
// independent (one round trip per chunk; the first version settled the
// positives one dependent load at a time: ~3-4 round trips per chunk for a
// wave, a third of the configs[2] scan's time).  chunk_resolve: the first
// position whose bit is set, or kScanChunk (then `ended` tells whether the
// old walk ended inside the chunk).
#ifndef WHARF_SCAN_BATCH
#define WHARF_SCAN_BATCH 1   // A/B: 0 = one dependent bitmap read per positive
#endif
struct ChunkTest {
    uint32_t mask, end;
    uint32_t w[kScanChunk];
};

// FB: the filter in LDS has 4096 << FB words (FB 0: the 16-KiB filter, 1: 32 KiB
// folded from the 64-KiB one, 2: the 64-KiB one); a key's word is hash >> (20 - FB)
template <int FB>
__device__ __forceinline__ bool bloom_test_fb(const uint32_t* f, uint32_t x)
{
    const uint32_t h = bloom_mix(x), b = bloom_bits(h);
    return (f[h >> (20 - FB)] & b) == b;
}
static_assert(kBigBloomWords == (kBloomWords << 2), "the big filter is the 16-KiB one at 4x the words");

// the filter of 4096 << FB words into LDS (FB 1: word i = big[2i] | big[2i + 1],
// a superset filter: keys of either big word share its bit positions)
template <int FB>
__device__ __forceinline__ void filter_to_lds(const WalkArgs& a, uint32_t* s_bloom)
{
    if constexpr (FB == 0) {
        for (uint32_t i = threadIdx.x; i < kBloomWords; i += blockDim.x) s_bloom[i] = a.bloom[i];
    } else if constexpr (FB == 1) {
        const uint2* big = reinterpret_cast<const uint2*>(a.bloom + kBloomWords);
        for (uint32_t i = threadIdx.x; i < 2 * kBloomWords; i += blockDim.x) {
            const uint2 w = big[i];
            s_bloom[i] = w.x | w.y;
        }
    } else {
        for (uint32_t i = threadIdx.x; i < kBigBloomWords; i += blockDim.x) s_bloom[i] = a.bloom[kBloomWords + i];
    }
    __syncthreads();
}

// LEAN (round 3, profiles/r03/scan_kernels): the filter bits tested as shifts of the
// word and the walk's end found from the chunk's last position (kSent fills the
// rest of a row once its walk ends): ~11 instead of ~17 VALU per position
#ifndef WHARF_CHUNK_LEAN
#define WHARF_CHUNK_LEAN 1
#endif
// IDX (the deterministic copy, round 3): the positives' source indices
// (a.src_idx, kNoSource for every vertex that is not a batch source) instead
// of their bitmap words: one read both settles a positive and names its
// suffix-table row (the copy read the bitmap word, then the index)
template <int FB = 0, bool LEAN = WHARF_CHUNK_LEAN != 0, bool IDX = false>
__device__ __forceinline__ void chunk_issue(const WalkArgs& a, const uint32_t* s_bloom, const uint32_t (&x)[kScanChunk],
                                            uint32_t cnt, ChunkTest& t)
{
    t.mask = 0;
    t.end = cnt;
    if constexpr (LEAN) {
#pragma unroll
        for (uint32_t j = 0; j < kScanChunk; j++) {
            const uint32_t h = bloom_mix(x[j]), fw = s_bloom[h >> (20 - FB)];
            uint32_t b = (fw >> ((h >> 13) & 31u)) & (fw >> ((h >> 8) & 31u));
            if (WHARF_BLOOM_K > 2) b &= fw >> ((h >> 3) & 31u);
            t.mask |= (b & 1u) << j;
        }
        if ((cnt == kScanChunk ? x[kScanChunk - 1] : chunk_pick(x, cnt - 1)) == kSent) {
#pragma unroll
            for (int j = (int)kScanChunk - 1; j >= 0; j--)
                if (x[j] == kSent && (uint32_t)j < cnt) t.end = (uint32_t)j;
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < kScanChunk; j++) {
            t.mask |= (uint32_t)bloom_test_fb<FB>(s_bloom, x[j]) << j;
            if (x[j] == kSent && j < t.end) t.end = j;
        }
    }
    if (t.end < 32) t.mask &= (1u << t.end) - 1u;
#if WHARF_SCAN_BATCH
#pragma unroll
    for (uint32_t j = 0; j < kScanChunk; j++) {
        if constexpr (IDX) t.w[j] = ((t.mask >> j) & 1u) ? a.src_idx[x[j]] : kNoSource;
        else t.w[j] = ((t.mask >> j) & 1u) ? a.bitmap[x[j] >> 5] : 0u;
    }
#endif
}

template <bool IDX = false>
__device__ __forceinline__ uint32_t chunk_resolve(const WalkArgs& a, const uint32_t (&x)[kScanChunk], uint32_t cnt,
                                                  const ChunkTest& t, bool& ended)
{
#if WHARF_SCAN_BATCH
    uint32_t hit = 0;
#pragma unroll
    for (uint32_t j = 0; j < kScanChunk; j++) {
        if constexpr (IDX) hit |= (uint32_t)(t.w[j] != kNoSource) << j;
        else hit |= ((t.w[j] >> (x[j] & 31u)) & 1u) << j;
    }
    hit &= t.mask;
    if (hit) return (uint32_t)__builtin_ctz(hit);
#else
    for (uint32_t mask = t.mask; mask; mask &= mask - 1u) {
        const uint32_t j = (uint32_t)__builtin_ctz(mask);
        const uint32_t v = chunk_pick(x, j);
        if ((a.bitmap[v >> 5] >> (v & 31)) & 1u) return j;
    }
#endif
    ended = t.end < cnt;
    return kScanChunk;
}

// a wave-uniform 64-bit value (from the first active lane) in SGPRs
__device__ __forceinline__ uint64_t uniform64(uint64_t x)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// XCD-aware walk ranges: workgroup b runs on XCD b % 8, which takes the
// (b % 8)-th eighth of the walks (whole 256-walk blocks, so rows stay aligned).
struct XcdRange {
    uint64_t first, end, stride;
};
__device__ __forceinline__ XcdRange xcd_range(uint64_t W)
{
    const uint32_t xcd = blockIdx.x % kXcds, slot = blockIdx.x / kXcds, per = gridDim.x / kXcds;
    const uint64_t part = (((W + kXcds - 1) / kXcds) + 255) & ~255ull;
    const uint64_t c0 = min(W, (uint64_t)xcd * part);
    return {c0 + (uint64_t)slot * blockDim.x + threadIdx.x, min(W, c0 + part), (uint64_t)per * blockDim.x};
}

// COPY = false: rewalk points only (apply_walk_updates = false, any model).
// COPY = true: deterministic re-walk from the suffix table (k_det_suffix).
#ifndef WHARF_SCAN_WAVES_EU
#define WHARF_SCAN_WAVES_EU 0   // A/B: force this many waves per SIMD on the scans (0 = compiler's choice)
#endif
#if WHARF_SCAN_WAVES_EU
#define WHARF_SCAN_WAVES __attribute__((amdgpu_waves_per_eu(WHARF_SCAN_WAVES_EU, WHARF_SCAN_WAVES_EU)))
#else
#define WHARF_SCAN_WAVES
#endif

// The scan alone holds no copy state (mv[], the table row): forcing 8 waves per
// SIMD costs it a few spilled VGPRs and hides more of the bitmap round trips
// (configs[2] scan 3.3 -> 3.15 ms); the copy keeps the compiler's choice (81
// VGPRs, 5 waves) — forced to more waves it spills and slows (7.6 -> 15 ms),
// and even the same kernel body moved into a device function compiles to 100
// VGPRs and runs 25 % slower (profiles/r02/scan_waves).
#ifndef WHARF_SCAN_ONLY_WAVES_EU
#define WHARF_SCAN_ONLY_WAVES_EU 8
#endif
#ifndef WHARF_COPY_EARLY_ROWS
#define WHARF_COPY_EARLY_ROWS 0   // A/B: the copy issues the next chunk's rows before its source-index wait
#endif
#ifndef WHARF_COPY_WAVES
#define WHARF_COPY_WAVES 1   // A/B: minimum waves/SIMD of the copy (1 = the compiler's choice; the 32-KiB
                             // filter caps it at 5 by LDS; 16-KiB filter forced to 6: 100 B spilled, 16 vs
                             // 7.2 ms, profiles/r03/copy_lean/copy_waves.txt)
#endif
template <bool COPY, bool NTL, int FB = 0, bool IDX = false>
__global__ __launch_bounds__(256, COPY ? WHARF_COPY_WAVES : WHARF_SCAN_ONLY_WAVES_EU) WHARF_SCAN_WAVES void k_rewalk_chunked(WalkArgs a)
{
    constexpr uint32_t C = kScanChunk;
    __shared__ uint32_t s_bloom[kBloomWords << FB];
    filter_to_lds<FB>(a, s_bloom);
    uint32_t steps = 0;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W;
    const uint32_t L = a.L;
    const XcdRange xr = xcd_range(W);
    const uint32_t lane = __lane_id();
    for (uint64_t li = xr.first; li < xr.end; li += xr.stride) {
        const uint64_t r = li / a.n_loc;
        uint32_t p = kNoRewalk;
        bool scanning = true;
        const uint32_t* __restrict__ row = nullptr;   // suffix row shifted by -p: the new value at pos is row[pos]
        // the wave's columns start at a uniform base: row addresses live in
        // SGPRs, the lane adds a 32-bit offset (no 64-bit VALU address math)
        uint32_t* __restrict__ wb = walks + uniform64(li - lane);
        uint32_t cur[C], nxt[C];
#pragma unroll
        for (uint32_t j = 0; j < C; j++) cur[j] = j < L ? row_load<NTL>(wb + (uint64_t)j * W, lane) : kSent;
        for (uint32_t c0 = 0; c0 < L; c0 += C) {
            const uint32_t cnt = min(C, L - c0);
            const bool was_scanning = scanning;
            const bool more = c0 + C < L;
            ChunkTest ct;
            if (scanning) chunk_issue<FB, WHARF_CHUNK_LEAN != 0, COPY && IDX>(a, s_bloom, cur, cnt, ct);
            if ((!COPY || WHARF_COPY_EARLY_ROWS) && more && scanning) {
                // scan only: the next chunk's rows go out before the bitmap words
                // are waited for (loads complete in order: the wait leaves them in flight)
#pragma unroll
                for (uint32_t j = 0; j < C; j++)
                    nxt[j] = c0 + C + j < L ? row_load<NTL>(wb + (uint64_t)(c0 + C + j) * W, lane) : kSent;
            }
            if (scanning) {
                bool ended = false;
                const uint32_t j = chunk_resolve<COPY && IDX>(a, cur, cnt, ct, ended);
                if (j < C) {
                    p = c0 + j;
                    scanning = false;
                    if (COPY) {
                        const uint32_t sx = (COPY && IDX) ? chunk_pick(ct.w, j) : a.src_idx[chunk_pick(cur, j)];
                        row = a.memo + (r * a.memo_k + sx) * a.memo_stride - p;
                    }
                } else if (ended) {
                    scanning = false;
                }
            }
            uint32_t mv[C];
            if (COPY) {
                const bool walking = p < c0 + cnt - 1;   // new values inside this chunk
                if (walking) {
#pragma unroll
                    for (uint32_t q = 0; q < C; q += 4) {
                        uint4 t;
                        __builtin_memcpy(&t, row + c0 + q, 16);
                        mv[q] = t.x, mv[q + 1] = t.y, mv[q + 2] = t.z, mv[q + 3] = t.w;
                    }
                }
            }
            // next chunk's rows, in flight while this chunk is written
            if (COPY && !WHARF_COPY_EARLY_ROWS && more && scanning) {
#pragma unroll
                for (uint32_t j = 0; j < C; j++)
                    nxt[j] = c0 + C + j < L ? row_load<NTL>(wb + (uint64_t)(c0 + C + j) * W, lane) : kSent;
            }
            if (COPY) {
#pragma unroll
                for (uint32_t j = 0; j < C; j++) {
                    const uint32_t pos = c0 + j;
                    // a row segment is written when one of its lanes re-walks this
                    // position: whole 256-B rows (kCopyGroup 64) or 64-B quarters
                    const uint64_t need = __ballot(p < pos);
                    const uint32_t sh = (__lane_id() / kCopyGroup) * kCopyGroup;
                    const uint64_t gm = (~0ull >> (64 - kCopyGroup)) << sh;
                    if (j < cnt && (need & gm)) {
                        uint32_t val = was_scanning ? cur[j] : kSent;
                        if (p < pos) {
                            val = mv[j];
                            steps += val != kSent;
                        }
                        row_store(wb + (uint64_t)pos * W, lane, val);
                    }
                }
            }
            if (!__any(scanning || (COPY && p != kNoRewalk))) break;
            if (more && (COPY ? scanning : was_scanning)) {
#pragma unroll
                for (uint32_t j = 0; j < C; j++) cur[j] = nxt[j];
            }
        }
        a.aff[li] = (uint8_t)p;
    }
    if (COPY) wave_add(a.counters + 0, steps);
}

// The rewalk-point scan alone with the 64-KiB Bloom filter of the in-edge scan
// (kBigBloomWords, ~0.02 % false positives at 10 k sources instead of ~3 %):
// with the 16-KiB filter, ~40 % of the 16-position chunks of a walk that does
// not meet a source carry a false positive whose exact bitmap word costs the
// wave a round trip — ~1 ms of the 3 ms configs[2] scan
// (profiles/r02/chunked_scan).  64 KiB of LDS per workgroup: 1024-thread
// workgroups, two per CU, 8 waves per SIMD as before.
template <bool NTL>
__global__ __launch_bounds__(1024, 8) void k_rewalk_scan_big(WalkArgs a)
{
    constexpr uint32_t C = kScanChunk;
    __shared__ uint32_t s_bloom[kBigBloomWords];
    filter_to_lds<2>(a, s_bloom);
    const uint64_t W = a.W;
    const uint32_t L = a.L;
    const XcdRange xr = xcd_range(W);
    const uint32_t lane = __lane_id();
    for (uint64_t li = xr.first; li < xr.end; li += xr.stride) {
        uint32_t p = kNoRewalk;
        bool scanning = true;
        const uint32_t* __restrict__ wb = a.walks + uniform64(li - lane);
        uint32_t cur[C], nxt[C];
#pragma unroll
        for (uint32_t j = 0; j < C; j++) cur[j] = j < L ? row_load<NTL>(wb + (uint64_t)j * W, lane) : kSent;
        for (uint32_t c0 = 0; c0 < L; c0 += C) {
            const uint32_t cnt = min(C, L - c0);
            const bool more = c0 + C < L, was_scanning = scanning;
            ChunkTest ct;
            if (scanning) chunk_issue<2>(a, s_bloom, cur, cnt, ct);
            if (more && scanning) {
#pragma unroll
                for (uint32_t j = 0; j < C; j++)
                    nxt[j] = c0 + C + j < L ? row_load<NTL>(wb + (uint64_t)(c0 + C + j) * W, lane) : kSent;
            }
            if (scanning) {
                bool ended = false;
                const uint32_t j = chunk_resolve(a, cur, cnt, ct, ended);
                if (j < C) {
                    p = c0 + j;
                    scanning = false;
                } else if (ended) {
                    scanning = false;
                }
            }
            if (!__any(scanning)) break;
            if (more && was_scanning) {
#pragma unroll
                for (uint32_t j = 0; j < C; j++) cur[j] = nxt[j];
            }
        }
        a.aff[li] = (uint8_t)p;
    }
}

// The rewalk-point scan with the fewest instructions per position (round 3).
// SQ counters of k_rewalk_scan_big on configs[2] (profiles/r03/scan_kernels):
// 29.5 VALU + 8.6 SALU per walk position, issue stalls 31 % and waitcnt
// stalls 43 % of wave cycles: the scan is bound by instruction issue as much
// as by HBM.  Here, per position: the filter hash (3), its LDS word (1), the
// three bit tests as shifts of the word (7) and the mask bit (2); per chunk:
// the walk-end test on the last position only (a walk that ends leaves kSent
// in the rest of its row), the bitmap word of the first positive only, and
// the 16 row loads from two buffer descriptors per chunk with the row offsets
// in SGPRs (1 SALU + 1 load per row, no per-row branch), issued after that
// word's load so the wait for it leaves the rows in flight.  A false
// positive (~0.1 % of positions with the 64-KiB filter) falls back to the
// chunk's next positive, re-read from HBM.  Needs 7 * 4 * W < 2^32 (the host
// uses k_rewalk_scan_big / k_rewalk_plan beyond).
constexpr uint64_t kLeanMaxW = ((1ull << 32) - 1) / 28;
template <bool NTL>
__device__ __forceinline__ void lean_chunk(const uint32_t* wb, uint32_t r0, uint32_t L, uint64_t W, uint32_t voff,
                                           uint32_t (&Y)[kScanChunk])
{
    // always 16 loads and no branch (the compiler can then count them); rows
    // past the walk length re-read the last row (only a partial last chunk).
    // Rows r0..r0+7 and r0+8..r0+15 from one descriptor each (offsets < 7 rows)
    const uint32_t w4 = (uint32_t)W * 4u, last = L - 1;
    const uint32_t b1 = min(r0 + 8, last);
    const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)(wb + (uint64_t)r0 * W), 0, 0xFFFFFFFF,
                                                                         kRowRsrcFlags);
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)(wb + (uint64_t)b1 * W), 0, 0xFFFFFFFF,
                                                                         kRowRsrcFlags);
#pragma unroll
    for (uint32_t j = 0; j < kScanChunk; j++) {
        const uint32_t row = min(r0 + j, last);
        if (j < 8) Y[j] = __builtin_amdgcn_raw_buffer_load_b32(rs0, voff, (row - r0) * w4, NTL ? 2 : 0);
        else Y[j] = __builtin_amdgcn_raw_buffer_load_b32(rs1, voff, (row - b1) * w4, NTL ? 2 : 0);
    }
}

// The rewalk point of the lane's walk (column `lane` of the wave's 64 columns at wb).
template <bool NTL>
__device__ __forceinline__ uint32_t lean_point(const WalkArgs& a, const uint32_t* s_bloom, const uint32_t* wb,
                                               uint32_t lane)
{
    constexpr uint32_t C = kScanChunk;
    const uint64_t W = a.W;
    const uint32_t L = a.L;
    // one chunk buffer: the chunk is dead once its first positive is picked,
    // so the next chunk's loads reuse its registers
    uint32_t X[C];
    lean_chunk<NTL>(wb, 0, L, W, lane * 4, X);
    uint32_t p = kNoRewalk;
    bool scanning = true;
    uint32_t mask, x0, j0, w0;
    bool ended;
    // the filter test of chunk c0 and the bitmap word of its first positive
    auto test = [&](uint32_t c0) {
        const uint32_t cnt = min(C, L - c0);
        mask = 0;
        ended = false;
        if (scanning) {
#pragma unroll
            for (uint32_t j = 0; j < C; j++) {
                const uint32_t h = bloom_mix(X[j]);
                const uint32_t fw = s_bloom[h >> 18];
                // bloom_bits(h) all set in fw: the three bits tested in place
                uint32_t t = (fw >> ((h >> 13) & 31u)) & (fw >> ((h >> 8) & 31u));
                if (WHARF_BLOOM_K > 2) t &= fw >> ((h >> 3) & 31u);
                mask |= (t & 1u) << j;
            }
            if (cnt < C) mask &= (1u << cnt) - 1u;
            const uint32_t last = cnt == C ? X[C - 1] : chunk_pick(X, cnt - 1);
            if (last == kSent) {   // the walk ends in this chunk: positives stop at its end
                ended = true;
                uint32_t e = cnt;
#pragma unroll
                for (int j = (int)C - 1; j >= 0; j--)
                    if (X[j] == kSent) e = (uint32_t)j;
                mask &= (1u << e) - 1u;
            }
        }
        x0 = 0, j0 = 0, w0 = 0;
        if (mask) {
            j0 = (uint32_t)__builtin_ctz(mask);
            x0 = chunk_pick(X, j0);
            w0 = a.bitmap[x0 >> 5];
        }
    };
    // settle chunk c0 from its first positive's word
    auto settle = [&](uint32_t c0) {
        if (mask) {
            bool hit = (w0 >> (x0 & 31u)) & 1u;
            while (!hit) {   // a false positive: the next one, re-read from HBM (rare)
                mask &= mask - 1u;
                if (!mask) break;
                j0 = (uint32_t)__builtin_ctz(mask);
                x0 = walk_load<false>(wb + (uint64_t)(c0 + j0) * W + lane);
                hit = (a.bitmap[x0 >> 5] >> (x0 & 31u)) & 1u;
            }
            if (hit) {
                p = c0 + j0;
                scanning = false;
            }
        }
        if (ended) scanning = false;
    };
    uint32_t c0 = 0;
    for (; c0 + C < L; c0 += C) {   // chunks with a successor: its 16 loads, unconditional
        test(c0);
        lean_chunk<NTL>(wb, c0 + C, L, W, lane * 4, X);
        settle(c0);
        if (!__any(scanning)) return p;
    }
    test(c0);   // the last chunk
    settle(c0);
    return p;
}

template <bool NTL>
__global__ __launch_bounds__(1024, 8) void k_rewalk_scan_lean(WalkArgs a)
{
    __shared__ uint32_t s_bloom[kBigBloomWords];
    filter_to_lds<2>(a, s_bloom);
    const XcdRange xr = xcd_range(a.W);
    const uint32_t lane = __lane_id();
    const uint32_t xend = (uint32_t)xr.end, xstride = (uint32_t)xr.stride;
    for (uint32_t li = (uint32_t)xr.first; li < xend; li += xstride) {
        const uint32_t* __restrict__ wb = a.walks + __builtin_amdgcn_readfirstlane(li - lane);
        a.aff[li] = (uint8_t)lean_point<NTL>(a, s_bloom, wb, lane);
    }
}

// k_rewalk_plan on the lean scan (round 3): 1024-thread workgroups (the 64-KiB
// filter, two per CU), four 256-walk blocks per step, each binned and listed
// exactly as k_rewalk_plan does it.  FROM_AFF (round 6, A/B: WHARF_PLAN_SPLIT=1):
// the points come from k_rewalk_scan_lean's aff[] instead, in a binning pass that
// reads one byte per walk.  The idea was that the fused scan's binning barriers
// hold each workgroup to its slowest wave.  The scan alone was measured as slow
// as the fused plan (configs[4]: 5.75 vs 5.9 ms), so the split is not the default.
template <bool NTL, bool FROM_AFF = false>
__global__ __launch_bounds__(1024, 8) void k_rewalk_plan_lean(WalkArgs a)
{
    __shared__ uint32_t s_bloom[FROM_AFF ? 1 : kBigBloomWords];
    __shared__ uint32_t s_bin[4][256];                     // count, then cursor, per rewalk point (255: none)
    __shared__ uint32_t s_wsum[4][kWavesPerBlock];
    __shared__ unsigned long long s_ticket[4];
    if constexpr (!FROM_AFF) filter_to_lds<2>(a, s_bloom);
    if (blockDim.x != 1024) __builtin_trap();              // four 256-walk blocks, one bin per thread
    const uint64_t W = a.W;
    const uint32_t L = a.L, t = threadIdx.x, sb = t >> 8, tl = t & 255, lane = __lane_id(), wv = tl >> 6;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024; base < W; base += (uint64_t)gridDim.x * 1024) {
        const uint64_t li = base + t;
        uint32_t p = kNoRewalk;
        if constexpr (FROM_AFF) {
            if (li < W) p = a.aff[li];
        } else {
            if (li < W) p = lean_point<NTL>(a, s_bloom, a.walks + uniform64(li - lane), lane);
            if (li < W) a.aff[li] = (uint8_t)p;
        }
        if (a.scan_only) continue;
        const uint32_t key = (li < W && p + 1 < L) ? p : 255u;   // re-walking: something after the point
        // plan_group (A/B): the workgroup's 1024 walks binned as one group (bins of block 0; the
        // others stay empty and scan to zeros), so a wave's 64 entries span a narrower range of
        // rewalk points over 4 KB of row instead of 1 KB
        const uint32_t gb = a.plan_group ? 0u : sb;
        s_bin[sb][tl] = 0;
        __syncthreads();
        atomicAdd(&s_bin[gb][key], 1u);
        __syncthreads();
        const uint32_t c = s_bin[sb][tl];
        uint32_t incl = c;                                 // exclusive scan of the block's 256 bins
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
            if ((int)lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[sb][wv] = incl;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += s_wsum[sb][w];
        s_bin[sb][tl] = before + incl - c;
        __syncthreads();
        const uint32_t nact = s_bin[gb][255];              // entries ranked before the "none" bin
        if constexpr (FROM_AFF) {
            // one list ticket per workgroup step (4 blocks) instead of one per block: without the
            // scan in front, the same-address atomics were this pass's bound (3.9 ms at configs[4]).
            // Bit 40 of a block's ticket, which picks its listing direction, alternates by block.
            if (t == 0) {
                uint32_t c[4], tot = 0;
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) tot += (c[b] = s_bin[b][255]);   // (plan_group: blocks 1-3 stay empty)
                uint64_t o = tot ? (atomicAdd(a.counters + 2, (4ull << 40) | tot) & kListMask) : 0ull;
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) {
                    s_ticket[b] = o | ((uint64_t)(b & 1u) << 40);
                    o += c[b];
                }
            }
        } else {
            if (tl == 0 && gb == sb) s_ticket[sb] = nact ? atomicAdd(a.counters + 2, (1ull << 40) | nact) : 0ull;
        }
        __syncthreads();
        const uint64_t blk = (base >> 8) + sb;
        if (tl == 0 && a.bdesc && (blk << 8) < W) a.bdesc[blk] = (s_ticket[sb] & kListMask) | ((uint64_t)nact << 40);
        if (key != 255u) {
            const uint32_t rank = atomicAdd(&s_bin[gb][key], 1u);
            const uint64_t tk = s_ticket[gb];
            const uint32_t at = ((tk >> 40) & 1u) ? nact - 1 - rank : rank;
            a.defer[(tk & kListMask) + at] = li | ((uint64_t)p << 56);
        }
        __syncthreads();                                   // s_bin / s_ticket are reused
    }
}

__global__ void k_src_index(const RunInfo* __restrict__ runs, uint64_t k, uint32_t* __restrict__ src_idx)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (uint64_t)gridDim.x * blockDim.x)
        src_idx[runs[i].src] = (uint32_t)i;
}

void launch_src_index(const RunInfo* runs, uint64_t k, uint32_t* src_idx, hipStream_t s)
{
    if (k) hipLaunchKernelGGL(k_src_index, grid_for(k, 256), 256, 0, s, runs, k, src_idx);
}

// node2vec MH re-walk, two kernels.  Setting up a node2vec walker is a chain
// of dependent loads (rows of cur and prev, the binary search for the
// anchor-cache slot of prev -> cur) and its steps carry wave-cooperative
// anchor inits, so the re-walk is bound by dependent-gather latency times the
// lanes that have work: idle lanes are lost throughput.
//
// k_rewalk_plan: per block of 256 walks, the rewalk-point scan (coalesced row
// reads, Bloom filter in LDS + bitmap), then a counting sort of the block's
// re-walking walks by rewalk point in LDS, appended to one compacted list
// {li | p << 56} (a packed atomic hands each block its offset and a ticket;
// odd tickets store their run descending, so two blocks that meet inside a
// wave meet at similar rewalk points).
//
// k_rewalk_sorted: each wave takes 64 consecutive list entries — walks of one
// block (their stores share the block's 1 KB row segments in L2) at nearly the
// same rewalk point — and sweeps positions in lock step from the smallest.
// Replaces a fused per-wave sweep over the walk matrix (each wave swept 64
// consecutive walks from their smallest rewalk point: ~58 % of lane-steps
// idle on configs[2], and sparse waves had to be deferred to the flattened
// list kernel): configs[2] node2vec batch 73.7 -> 63.6 ms, configs[4]-shaped
// (scale 24, wpv 1) re-walk 51.7 / 43.9 -> 39.1 / 31.5 ms; the flattened
// kernel over the same sorted list: 104 ms / 47.9 ms (scattered stores).

// The rewalk point of lane li's walk by the chunked scan of k_rewalk_chunked<false>
// (kScanChunk rows per round trip, the next chunk's rows in flight while this
// one's bitmap words are read).  Every lane of the wave calls it; lanes
// without a walk (li >= W) with active = false.
__device__ __forceinline__ uint32_t chunked_point(const WalkArgs& a, const uint32_t* s_bloom, uint64_t li, bool active)
{
    constexpr uint32_t C = kScanChunk;
    const uint32_t L = a.L, lane = __lane_id();
    const uint64_t W = a.W;
    const uint32_t* __restrict__ wb = a.walks + uniform64(li - lane);
    uint32_t p = kNoRewalk;
    bool scanning = active;
    uint32_t cur[C], nxt[C];
#pragma unroll
    for (uint32_t j = 0; j < C; j++) cur[j] = (scanning && j < L) ? row_load(wb + (uint64_t)j * W, lane) : kSent;
    for (uint32_t c0 = 0; c0 < L; c0 += C) {
        const uint32_t cnt = min(C, L - c0);
        const bool more = c0 + C < L, was_scanning = scanning;
        ChunkTest ct;
        if (scanning) chunk_issue(a, s_bloom, cur, cnt, ct);
        if (more && scanning) {
#pragma unroll
            for (uint32_t j = 0; j < C; j++)
                nxt[j] = c0 + C + j < L ? row_load(wb + (uint64_t)(c0 + C + j) * W, lane) : kSent;
        }
        if (scanning) {
            bool ended = false;
            const uint32_t j = chunk_resolve(a, cur, cnt, ct, ended);
            if (j < C) {
                p = c0 + j;
                scanning = false;
            } else if (ended) {
                scanning = false;
            }
        }
        if (!__any(scanning)) break;
        if (more && was_scanning) {
#pragma unroll
            for (uint32_t j = 0; j < C; j++) cur[j] = nxt[j];
        }
    }
    return p;
}

__global__ __launch_bounds__(256) WHARF_SCAN_WAVES void k_rewalk_plan(WalkArgs a)
{
    __shared__ uint32_t s_bloom[kBloomWords];
    __shared__ uint32_t s_bin[256];                        // count, then cursor, per rewalk point (255: none)
    __shared__ uint32_t s_wsum[kWavesPerBlock];
    __shared__ unsigned long long s_ticket;
    bloom_to_lds(a, s_bloom);
    if (blockDim.x != 256) __builtin_trap();               // one histogram bin per thread
    const uint64_t W = a.W;
    const uint32_t L = a.L, t = threadIdx.x, lane = __lane_id();
    for (uint64_t base = (uint64_t)blockIdx.x * 256; base < W; base += (uint64_t)gridDim.x * 256) {
        const uint64_t li = base + t;
        // chunked scan (round 2: the one-row-prefetch scan it replaces was
        // latency-bound, 7.5 ms per configs[2] node2vec batch)
        const uint32_t p = chunked_point(a, s_bloom, li, li < W);
        if (li < W) a.aff[li] = (uint8_t)p;
        if (a.scan_only) continue;
        const uint32_t key = (li < W && p + 1 < L) ? p : 255u;   // re-walking: something after the point
        s_bin[t] = 0;
        __syncthreads();
        atomicAdd(&s_bin[key], 1u);
        __syncthreads();
        const uint32_t c = s_bin[t];
        uint32_t incl = c;                                 // exclusive scan of the 256 bins
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
            if ((int)lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[t >> 6] = incl;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t w = 0; w < (t >> 6); w++) before += s_wsum[w];
        s_bin[t] = before + incl - c;
        __syncthreads();
        const uint32_t nact = s_bin[255];                  // entries ranked before the "none" bin
        if (t == 0) s_ticket = nact ? atomicAdd(a.counters + 2, (1ull << 40) | nact) : 0ull;
        __syncthreads();
        if (t == 0 && a.bdesc) a.bdesc[base >> 8] = (s_ticket & kListMask) | ((uint64_t)nact << 40);
        if (key != 255u) {
            const uint32_t rank = atomicAdd(&s_bin[key], 1u);
            const uint64_t tk = s_ticket;
            const uint32_t at = ((tk >> 40) & 1u) ? nact - 1 - rank : rank;
            a.defer[(tk & kListMask) + at] = li | ((uint64_t)p << 56);
        }
        __syncthreads();                                   // s_bin / s_ticket are reused
    }
}

// An entry of the node2vec re-walk list names an owned walk (li < W) and a
// rewalk point with a step after it (p + 1 < L), which k_rewalk_plan* always
// write.  Anything else — a list that was corrupted or mis-sized between the
// plan and its consumer (round 3: a global sort of the list faulted its first
// GPU run) — is never dereferenced: the consumer skips it and
// reports it through a.err, and the host fails the update with WHARF_E_STATE.
__device__ __forceinline__ bool list_entry_ok(const WalkArgs& a, uint64_t li, uint32_t p)
{
    if (li < a.W && p + 1 < a.L) return true;
    atomicOr(a.err, 1ull);
    return false;
}

// Sort a wave's 64 re-walk list entries (walk | point << 56; ~0 = none) by walk
// (column), ascending, so the nones end up last: bitonic over the lanes.
__device__ __forceinline__ uint64_t wave_sort_entries(uint64_t ent)
{
    const uint32_t lane = __lane_id();
    // key: the walk in the high bits, the point in the low byte (a none stays the largest)
    uint64_t key = ent == ~0ull ? ~0ull : ((ent & ((1ull << 56) - 1)) << 8) | (ent >> 56);
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(key >> 32), (int)j, 64) << 32) |
                                   (uint32_t)__shfl_xor((int)(uint32_t)key, (int)j, 64);
            const bool up = (lane & k) == 0, low = (lane & j) == 0;
            key = (up == low) ? (key < other ? key : other) : (key < other ? other : key);
        }
    }
    return key == ~0ull ? ~0ull : (key >> 8) | ((key & 0xFFull) << 56);
}

// (105 VGPRs, 4 waves/SIMD; forcing 5 spills 12 B and measured no faster:
// configs[2] node2vec batch 65.4 vs 63.6 ms)
template <int MODEL, bool DET, bool RF = false>   // RF: return-first inits (WalkArgs::ret_first, A/B)
__global__ __launch_bounds__(256) void k_rewalk_sorted(WalkArgs a)
{
    uint32_t steps = 0, accepts = 0, inits = 0;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W, cnt = a.counters[2] & kListMask;
    const uint32_t L = a.L, ep = a.epoch << 4;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c0 = wave * 64; c0 < cnt; c0 += nwaves * 64) {
        const uint64_t e = c0 + __lane_id();
        // the wave's 64 entries (walks of one block at nearly the same rewalk point) in
        // column order (round 3): lane order does not change what a wave computes (each
        // walk's draws depend only on its id), but ascending columns let the row stores of
        // neighbouring lanes merge; a bitonic sort over the wave, 21 shuffle steps
        uint64_t ent = e < cnt ? a.defer[e] : ~0ull;
        if (a.lane_sort) ent = wave_sort_entries(ent);
        const bool active = ent != ~0ull && list_entry_ok(a, ent & ((1ull << 56) - 1), (uint32_t)(ent >> 56));
        uint64_t li = 0;
        uint32_t p = L, wlo = 0, whi = 0;
        const uint64_t* __restrict__ rt = nullptr;
        Walker w;
        w.rc.deg = 0;
        if (active) {
            li = ent & ((1ull << 56) - 1);
            p = (uint32_t)(ent >> 56);
            const uint64_t r = li / a.n_loc;
            const uint64_t wid = r * a.n + a.walks[li];
            wlo = (uint32_t)wid;
            whi = (uint32_t)(wid >> 32);
            if constexpr (DET) rt = a.rtab + r * L;
            const uint32_t x = walks[(uint64_t)p * W + li];
            const uint32_t xprev = p ? walks[(uint64_t)(p - 1) * W + li] : x;
            walk_state<MODEL, DET>(a, x, xprev, p, wlo, whi, ep, w);
        }
        uint32_t first = active ? p + 1 : L;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) first = min(first, (uint32_t)__shfl_xor((int)first, o, 64));
#ifdef WHARF_INIT_STATS
        if (__lane_id() == 0 && first < L) atomicAdd(a.counters + 6, 64ull * (L - first));   // lane-slots swept
#endif
        for (uint32_t pos = first; pos < L; pos++) {
            uint32_t val = kSent;
            if (active && pos > p && w.rc.deg) {
                val = walk_step<MODEL, DET, false, RF>(a, w, rt, DET ? pos - 1 - p : pos - 1, wlo, whi, ep, accepts, inits);
                steps++;
            }
            // the lanes are walks scattered over a block (sorted by rewalk point),
            // so these are partial-line stores: 446 M write requests for 5.3 GB of
            // values on configs[2] (~12-17 ms of the ~60 ms re-walk: a timing
            // probe without them).  Non-temporal: -1.7 %.  A compact [L][list]
            // buffer written in whole rows plus a merge pass that rewrites the
            // matrix rows whole cost as much (sorted 57 -> 47 ms, merge 9.8 ms;
            // profiles/r02/n2v_rewalk2)
#ifndef WHARF_PROBE_NO_REWALK_STORE   // timing probe only (tools/ab_build.sh): the walks are not written
            if (active && pos > p) __builtin_nontemporal_store(val, walks + (uint64_t)pos * W + li);
#else
            steps += val == 0xFFFFFFFDu;   // keeps val live; never true for a vertex id < 2^32 - 2
#endif
        }
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// Block-staged alternative to k_rewalk_sorted (WHARF_N2V_REWALK=block): a
// workgroup takes one 256-walk block's run of the list (k_rewalk_plan's
// bdesc), wave w its entries [64 w, 64 w + 64), and sweeps positions in chunks
// of kTileRows; the new values go to an LDS tile [kTileRows][256] and each
// position of the chunk leaves as ONE full 1-KiB row segment of the walk
// matrix — the columns that are not re-walked there (walks of the block that do
// not re-walk, or are still before their rewalk point) read their old value back
// (a coalesced row read).  k_rewalk_sorted's lanes are walks scattered over a
// block, so its stores are partial lines (446 M write requests for 5.3 GB of
// values per configs[2] batch; a timing probe without them ran 43 vs 55 ms).
constexpr uint32_t kTileRows = 16;

template <int MODEL>
__global__ __launch_bounds__(256) void k_rewalk_block(WalkArgs a)
{
    __shared__ uint32_t tile[kTileRows][256];
    __shared__ uint32_t pcol[256];   // rewalk point of each column of the block, or kNoRewalk
    __shared__ uint32_t s_first;
    if (blockDim.x != 256) __builtin_trap();   // one column per thread
    uint32_t steps = 0, accepts = 0, inits = 0;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W, nblk = (W + 255) >> 8;
    const uint32_t L = a.L, ep = a.epoch << 4, t = threadIdx.x;
    for (uint64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint64_t d = a.bdesc[b];
        const uint32_t cnt = (uint32_t)(d >> 40);
        if (cnt == 0) continue;   // (uniform over the workgroup)
        const uint64_t base = b << 8;
        pcol[t] = kNoRewalk;
        if (t == 0) s_first = L;
        __syncthreads();
        const uint64_t ent = t < cnt ? a.defer[(d & kListMask) + t] : 0ull;
        // (also within this workgroup's 256-walk block: pcol is indexed by li - base)
        const bool active = t < cnt && list_entry_ok(a, ent & ((1ull << 56) - 1), (uint32_t)(ent >> 56)) &&
                            (ent & ((1ull << 56) - 1)) - base < 256;
        uint64_t li = 0;
        uint32_t p = L, wlo = 0, whi = 0;
        Walker w;
        w.rc.deg = 0;
        if (t < cnt && !active && list_entry_ok(a, ent & ((1ull << 56) - 1), (uint32_t)(ent >> 56)))
            atomicOr(a.err, 2ull);   // a valid walk outside the block: not this kernel's list
        if (active) {
            li = ent & ((1ull << 56) - 1);
            p = (uint32_t)(ent >> 56);
            const uint64_t r = li / a.n_loc;
            const uint64_t wid = r * a.n + a.walks[li];
            wlo = (uint32_t)wid;
            whi = (uint32_t)(wid >> 32);
            pcol[li - base] = p;
            atomicMin(&s_first, p + 1);
            const uint32_t x = walks[(uint64_t)p * W + li];
            const uint32_t xprev = p ? walks[(uint64_t)(p - 1) * W + li] : x;
            walk_state<MODEL, false>(a, x, xprev, p, wlo, whi, ep, w);
        }
        __syncthreads();
        const uint32_t first = s_first, pc = pcol[t];
        const uint64_t col = base + t;
        for (uint32_t c0 = first; c0 < L; c0 += kTileRows) {
            const uint32_t rows = min(kTileRows, L - c0);
            for (uint32_t j = 0; j < rows; j++) {
                const uint32_t pos = c0 + j;
                if (active && pos > p) {
                    uint32_t val = kSent;
                    if (w.rc.deg) {
                        val = walk_step<MODEL, false>(a, w, nullptr, pos - 1, wlo, whi, ep, accepts, inits);
                        steps++;
                    }
                    tile[j][li - base] = val;
                }
            }
            __syncthreads();
            if (col < W) {
                for (uint32_t j = 0; j < rows; j++) {
                    const uint64_t at = (uint64_t)(c0 + j) * W + col;
                    const uint32_t v = (pc != kNoRewalk && c0 + j > pc) ? tile[j][t] : walks[at];
                    __builtin_nontemporal_store(v, walks + at);
                }
            }
            __syncthreads();
        }
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// Flattened alternative to k_rewalk_sorted over the same list
// (WHARF_N2V_REWALK=flat): lanes at their own pace.  One flattened loop — a lane whose walk is done
// takes its next list entry in the same iteration instead of waiting for the
// rest of its wave.  Stores land in scattered rows (partial lines), the price
// of keeping every lane busy; results are identical to the lock-step sweep
// (each walk's draws depend only on its id, positions and the epoch).
template <int MODEL, bool DET>
__global__ __launch_bounds__(256) void k_rewalk_list(WalkArgs a)
{
    uint32_t steps = 0, accepts = 0, inits = 0;
    const uint64_t cnt = a.counters[2] & kListMask;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W;
    const uint32_t L = a.L, ep = a.epoch << 4;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t li = 0;
    uint32_t p = 0, pos = L, wlo = 0, whi = 0;
    const uint64_t* __restrict__ rt = nullptr;
    Walker w;
    w.rc.deg = 0;
    for (;;) {
        while (pos >= L && i < cnt) {   // next walk of this lane (an entry out of range is skipped)
            const uint64_t e = a.defer[i];
            i += stride;
            li = e & ((1ull << 56) - 1);
            p = (uint32_t)(e >> 56);
            if (!list_entry_ok(a, li, p)) continue;
            const uint64_t r = li / a.n_loc;
            const uint64_t wid = r * a.n + a.walks[li];
            wlo = (uint32_t)wid;
            whi = (uint32_t)(wid >> 32);
            if constexpr (DET) rt = a.rtab + r * L;
            const uint32_t x = walks[(uint64_t)p * W + li];
            const uint32_t xprev = p ? walks[(uint64_t)(p - 1) * W + li] : x;
            walk_state<MODEL, DET>(a, x, xprev, p, wlo, whi, ep, w);
            pos = p + 1;
        }
        if (!__any(pos < L)) break;
#ifdef WHARF_INIT_STATS
        if (__lane_id() == 0) atomicAdd(a.counters + 6, 64ull);
#endif
        if (pos < L) {
            uint32_t val = kSent;
            if (w.rc.deg) {
                val = walk_step<MODEL, DET>(a, w, rt, DET ? pos - 1 - p : pos - 1, wlo, whi, ep, accepts, inits);
                steps++;
            }
            walks[(uint64_t)pos * W + li] = val;
            pos++;
        }
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// node2vec MH re-walk by passes (sparse walks: configs[4]'s 1/8 shard, where
// 79 % of the re-walk steps enter a state whose anchor was never computed).
// In the lock-step kernels above each such init stalls its wave for rounds of
// dependent proposal loads while few lanes have one.  Here a walker that needs
// an anchor PARKS instead: k_rewalk_park advances every walker of its input
// list (lanes at their own pace, a lane whose walker parks or ends takes the
// next entry) and appends the parked ones {walk | pos, cur, prev, cache entry}
// to an output list (one atomic per wave, ballot + prefix rank); k_park_init
// then computes the anchors of the whole list with every lane of every wave
// initialising (anchor_init_wave over full waves, as k_anchor_init_all), and
// the next pass resumes the walkers.  Anchors are a pure function of the
// snapshot, so the corpus, step and acceptance counts equal the lock-step
// kernels' (the parity suite forces this path).  The host runs passes until the
// list is short, then finishes it with lazy inits (PARK = false).
struct ParkRec {
    uint64_t lp;         // walk column | next position << 56
    uint32_t cur, prev;  // the walker's state
    uint64_t* ac;        // its anchor cache entry (edge record or start-state table), or null:
    uint64_t own;        //   a state without one (a re-walk start whose edge prev -> cur is gone)
                         //   gets its anchor here, for the walker that resumes from this record
};

template <int MODEL, bool FRESH, bool PARK>
__global__ __launch_bounds__(256) void k_rewalk_park(WalkArgs a, const ParkRec* in,
                                                     const unsigned long long* __restrict__ in_cnt,
                                                     ParkRec* __restrict__ out, unsigned long long* __restrict__ out_cnt)
{
    uint32_t steps = 0, accepts = 0, inits = 0;
    const uint64_t cnt = FRESH ? (a.counters[2] & kListMask) : *in_cnt;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t* __restrict__ walks = a.walks;
    const uint64_t W = a.W;
    const uint32_t L = a.L, ep = a.epoch << 4;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t li = 0;
    uint32_t pos = L, wlo = 0, whi = 0;
    Walker w;
    w.rc.deg = 0;
    bool has = false;
    for (;;) {
        while (!has && i < cnt) {   // this lane's next walker (a fresh entry out of range is skipped)
            if constexpr (FRESH) {
                const uint64_t e = a.defer[i];
                li = e & ((1ull << 56) - 1);
                const uint32_t p = (uint32_t)(e >> 56);
                if (!list_entry_ok(a, li, p)) {
                    i += stride;
                    continue;
                }
                pos = p + 1;
                const uint64_t r = li / a.n_loc;
                const uint64_t wid = r * a.n + a.walks[li];
                wlo = (uint32_t)wid;
                whi = (uint32_t)(wid >> 32);
                const uint32_t x = walks[(uint64_t)p * W + li];
                const uint32_t xprev = p ? walks[(uint64_t)(p - 1) * W + li] : x;
                walk_state<MODEL, false>(a, x, xprev, p, wlo, whi, ep, w);
            } else {
                const ParkRec pr = in[i];
                li = pr.lp & ((1ull << 56) - 1);
                pos = (uint32_t)(pr.lp >> 56);
                const uint64_t r = li / a.n_loc;
                const uint64_t wid = r * a.n + a.walks[li];
                wlo = (uint32_t)wid;
                whi = (uint32_t)(wid >> 32);
                w.rc = load_rec(a.vrec, pr.cur);
                w.rp = load_rec(a.vrec, pr.prev);
                w.ac = pr.ac ? pr.ac : const_cast<uint64_t*>(&in[i].own);   // (k_park_init filled it)
                w.anc = *w.ac;
            }
            has = pos < L;
            i += stride;
        }
        if (!__any(has)) break;
        bool park = false;
        if (has) {
            uint32_t val = kSent;
            const bool live = w.rc.deg != 0;   // a walk at a vertex without out-edges ends
            if (live) val = walk_step<MODEL, false, PARK>(a, w, nullptr, pos - 1, wlo, whi, ep, accepts, inits, &park);
            if (!park) {
                steps += live;
                walks[(uint64_t)pos * W + li] = val;
                has = ++pos < L;
            }
        }
        if constexpr (PARK) {
            const uint64_t pm = __ballot(park);
            if (pm) {
                unsigned long long base = 0;
                if (__lane_id() == 0) base = atomicAdd(out_cnt, (unsigned long long)__popcll(pm));
                base = __shfl(base, 0, 64);
                if (park) {
                    out[base + __popcll(pm & ((1ull << __lane_id()) - 1))] =
                        ParkRec{li | ((uint64_t)pos << 56), w.rc.v, w.rp.v, w.ac, kAnchorNone64};
                    has = false;
                }
            }
        }
    }
    wave_add(a.counters + 0, steps);
    wave_add(a.counters + 1, accepts);
    wave_add(a.counters + 7, inits);
}

// The anchors of the parked states, one per lane over full waves.
__global__ __launch_bounds__(256) void k_park_init(WalkArgs a, ParkRec* in, const unsigned long long* __restrict__ in_cnt)
{
    const uint64_t cnt = *in_cnt;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t inits = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += stride) {
        const ParkRec pr = in[t];
        const Row rc = load_rec(a.vrec, pr.cur), rp = load_rec(a.vrec, pr.prev);
        uint32_t an = 0, cls = 0;
        anchor_compute(a, true, rc, rp, an, cls, inits);
        *(pr.ac ? pr.ac : &in[t].own) = ((uint64_t)cls << 62) | ((uint64_t)a.epoch << 32) | an;
    }
    wave_add(a.counters + 7, inits);
}

void launch_rewalk_park(const WalkArgs& a, int fresh, int park, const void* in, const unsigned long long* in_cnt,
                        void* out, unsigned long long* out_cnt, hipStream_t s)
{
    const dim3 grid(cu_count() * 8), block(256);   // resident lanes (8 blocks of 256 per CU)
    const ParkRec* pin = reinterpret_cast<const ParkRec*>(in);
    ParkRec* pout = reinterpret_cast<ParkRec*>(out);
    if (fresh && park) hipLaunchKernelGGL((k_rewalk_park<kNode2Vec, true, true>), grid, block, 0, s, a, pin, in_cnt, pout, out_cnt);
    else if (fresh) hipLaunchKernelGGL((k_rewalk_park<kNode2Vec, true, false>), grid, block, 0, s, a, pin, in_cnt, pout, out_cnt);
    else if (park) hipLaunchKernelGGL((k_rewalk_park<kNode2Vec, false, true>), grid, block, 0, s, a, pin, in_cnt, pout, out_cnt);
    else hipLaunchKernelGGL((k_rewalk_park<kNode2Vec, false, false>), grid, block, 0, s, a, pin, in_cnt, pout, out_cnt);
}

void launch_park_init(const WalkArgs& a, const void* in, const unsigned long long* in_cnt, hipStream_t s)
{
    hipLaunchKernelGGL(k_park_init, cu_count() * 8, 256, 0, s, a, reinterpret_cast<ParkRec*>(const_cast<void*>(in)),
                       in_cnt);
}

// Blocks for the walk kernels: one walk per lane by default; a smaller grid of
// lanes each looping over several walks with WHARF_WALK_BLOCKS_PER_CU=k
// (k blocks of 256 per CU; 0 = one walk per lane).
unsigned cu_count()
{
    static int cus = -1;
    if (cus < 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    return (unsigned)cus;
}


static unsigned walk_grid(uint64_t W)
{
    static int per_cu = -1;
    if (per_cu < 0) {
        const char* e = getenv("WHARF_WALK_BLOCKS_PER_CU");
        per_cu = e ? std::max(0, atoi(e)) : 0;
    }
    const uint64_t full = (W + 255) / 256;
    if (per_cu <= 0) return (unsigned)full;
    return (unsigned)std::min<uint64_t>(full, (uint64_t)cu_count() * per_cu);
}

// resident lanes for the node2vec re-walk list kernels (8 blocks of 256 per CU)
static unsigned list_grid() { return cu_count() * 8; }

// WHARF_N2V_REWALK=flat: the flattened list kernel instead of the sorted lock-step one (A/B, tests)
static bool flat_list()
{
    const char* e = getenv("WHARF_N2V_REWALK");
    return e && std::string(e) == "flat";
}

void launch_walk(const WalkArgs& a, bool rewalk, hipStream_t s)
{
    if (a.W == 0) return;
    // re-walks: persistent blocks (8 per CU, 16 KiB of Bloom filter each), so
    // the filter is copied to LDS once per block, not once per 256 walks
    const dim3 grid(rewalk ? std::min<uint64_t>((a.W + 255) / 256, (uint64_t)cu_count() * 8) : walk_grid(a.W)),
        block(256);
    const dim3 lgrid(list_grid());
    // node2vec plan on the lean scan (WHARF_PLAN_KERNEL=chunked: k_rewalk_plan, round 2)
    const char* pk = getenv("WHARF_PLAN_KERNEL");
    const bool plan_lean = !(pk && std::string(pk) == "chunked") && a.W <= kLeanMaxW;
    const dim3 pgrid((unsigned)std::min<uint64_t>((a.W + 1023) / 1024, (uint64_t)cu_count() * 2));
    // the lean scan's grid: a multiple of 8 workgroups (xcd_range)
    const dim3 bgrid((std::max<unsigned>(std::min<uint64_t>((a.W + 1023) / 1024, (uint64_t)cu_count() * 2), kXcds) /
                      kXcds) * kXcds);
    // the node2vec plan fused (default) or as the per-wave lean scan + a binning pass (WHARF_PLAN_SPLIT=1,
    // A/B: same-session traces, profiles/r06/plan_split: configs[4] shard 38.0 / 37.5 vs 37.0 / 37.4 ms of
    // plan + re-walk kernels per batch, configs[2] 50.1 / 49.5 vs 49.5 / 53.9; the scan alone is as slow
    // as the fused plan, 5.75 vs 5.9 ms at configs[4], so the extra pass does not pay)
    const char* ps = getenv("WHARF_PLAN_SPLIT");
    const bool plan_split = ps && *ps && atoi(ps) != 0;
    const bool cr = a.rf.compact != 0;   // compact 8-B edge records (never with node2vec MH's anchors)
#define WHARF_LAUNCH(M, D)                                                                   \
    do {                                                                                     \
        if (rewalk && M == kNode2Vec) {                                                      \
            if (a.stage == 2) {                                                              \
            } else if (plan_lean && plan_split) {                                            \
                if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_scan_lean<true>), bgrid, dim3(1024), 0, s, a); \
                else hipLaunchKernelGGL((k_rewalk_scan_lean<false>), bgrid, dim3(1024), 0, s, a); \
                hipLaunchKernelGGL((k_rewalk_plan_lean<false, true>), pgrid, dim3(1024), 0, s, a); \
            } else if (plan_lean) {                                                          \
                if (a.nt_rows) hipLaunchKernelGGL(k_rewalk_plan_lean<true>, pgrid, dim3(1024), 0, s, a); \
                else hipLaunchKernelGGL(k_rewalk_plan_lean<false>, pgrid, dim3(1024), 0, s, a);  \
            } else {                                                                         \
                hipLaunchKernelGGL(k_rewalk_plan, grid, block, 0, s, a);                     \
            }                                                                                \
            /* park: the host runs the passes; stage 1: the host reorders the list first */  \
            if (!a.scan_only && !a.park && a.stage != 1) {                                   \
                if (a.bdesc) hipLaunchKernelGGL((k_rewalk_block<M>), lgrid, block, 0, s, a);     \
                else if (flat_list()) hipLaunchKernelGGL((k_rewalk_list<M, D>), lgrid, block, 0, s, a); \
                else if (a.ret_first) hipLaunchKernelGGL((k_rewalk_sorted<M, D, M == kNode2Vec>), lgrid, block, 0, s, a); \
                else hipLaunchKernelGGL((k_rewalk_sorted<M, D>), lgrid, block, 0, s, a);     \
            }                                                                                \
        } else if (rewalk) {                                                                 \
            if (cr && a.sh_parts > 1) hipLaunchKernelGGL((k_rewalk_sweep<M, D, true, 1>), grid, block, 0, s, a); \
            else if (cr) hipLaunchKernelGGL((k_rewalk_sweep<M, D, false, 1>), grid, block, 0, s, a); \
            else if (a.sh_parts > 1) hipLaunchKernelGGL((k_rewalk_sweep<M, D, true, 0>), grid, block, 0, s, a); \
            else hipLaunchKernelGGL((k_rewalk_sweep<M, D, false, 0>), grid, block, 0, s, a);     \
        } else {                                                                             \
            if (cr && a.sh_parts > 1) hipLaunchKernelGGL((k_walk<M, D, true, 1>), grid, block, 0, s, a); \
            else if (cr) hipLaunchKernelGGL((k_walk<M, D, false, 1>), grid, block, 0, s, a); \
            else if (a.sh_parts > 1) hipLaunchKernelGGL((k_walk<M, D, true, 0>), grid, block, 0, s, a); \
            else hipLaunchKernelGGL((k_walk<M, D, false, 0>), grid, block, 0, s, a);         \
        }                                                                                    \
    } while (0)
    // a multiple of 8 workgroups: every XCD gets the same number
    const dim3 mgrid((std::max<unsigned>(grid.x, kXcds) / kXcds) * kXcds);
    const char* nc = getenv("WHARF_NO_CHUNKED_SCAN");   // A/B and tests: scan-only by the sweeps
    const bool chunked = !(nc && atoi(nc));
    if (rewalk && a.det && a.memo && !a.scan_only) {
        hipLaunchKernelGGL(k_det_suffix, grid_for((uint64_t)a.wpv * a.memo_k, 256), 256, 0, s, a);
        // the 32-KiB filter (5 workgroups of 256 per CU still fit the 160 KiB of LDS);
        // WHARF_COPY_SMALL_BLOOM=1 (A/B): the 16-KiB one
        const char* cb = getenv("WHARF_COPY_SMALL_BLOOM");
        if (cb && atoi(cb) && a.src_exact) {
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_chunked<true, true, 0, true>), mgrid, block, 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_chunked<true, false, 0, true>), mgrid, block, 0, s, a);
        } else if (cb && atoi(cb)) {
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_chunked<true, true, 0>), mgrid, block, 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_chunked<true, false, 0>), mgrid, block, 0, s, a);
        } else if (a.src_exact) {   // the source index settles the positives (IDX)
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_chunked<true, true, 1, true>), mgrid, block, 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_chunked<true, false, 1, true>), mgrid, block, 0, s, a);
        } else {
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_chunked<true, true, 1>), mgrid, block, 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_chunked<true, false, 1>), mgrid, block, 0, s, a);
        }
        return;
    }
    if (rewalk && a.scan_only && chunked) {
        // WHARF_SCAN_KERNEL (A/B and tests): lean (default) = k_rewalk_scan_lean, 64-KiB
        // filter, where 7 * 4 * W fits 32 bits; big = k_rewalk_scan_big (round 2, also lean's
        // fallback); WHARF_SCAN_SMALL_BLOOM=1: k_rewalk_chunked<false> with the 16-KiB filter
        const char* sb = getenv("WHARF_SCAN_SMALL_BLOOM");
        const char* sk = getenv("WHARF_SCAN_KERNEL");
        const bool small = sb && atoi(sb), big = sk && std::string(sk) == "big";
        if (!small && !big && a.W <= kLeanMaxW) {
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_scan_lean<true>), bgrid, dim3(1024), 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_scan_lean<false>), bgrid, dim3(1024), 0, s, a);
            return;
        }
        if (!small) {
            if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_scan_big<true>), bgrid, dim3(1024), 0, s, a);
            else hipLaunchKernelGGL((k_rewalk_scan_big<false>), bgrid, dim3(1024), 0, s, a);
            return;
        }
        if (a.nt_rows) hipLaunchKernelGGL((k_rewalk_chunked<false, true>), mgrid, block, 0, s, a);
        else hipLaunchKernelGGL((k_rewalk_chunked<false, false>), mgrid, block, 0, s, a);
        return;
    }
    if (a.det) WHARF_LAUNCH(kDeepWalk, true);
    else if (a.model == kDeepWalk) WHARF_LAUNCH(kDeepWalk, false);
    else WHARF_LAUNCH(kNode2Vec, false);
#undef WHARF_LAUNCH
}

// ---------------------------------------------------------------------------
// graph construction / maintenance
// ---------------------------------------------------------------------------
__global__ void k_rmat_keys(RmatParams p, uint64_t M, int directed, uint64_t* __restrict__ keys)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t s, d;
        rmat_edge(p, (uint32_t)i, s, d);
        keys[i] = ((uint64_t)s << 32) | d;
        if (!directed) keys[M + i] = ((uint64_t)d << 32) | s;
    }
}

__global__ void k_pairs_to_keys(const uint32_t* __restrict__ pairs, uint64_t m, uint64_t n,
                                uint64_t* __restrict__ keys, unsigned long long* __restrict__ err)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = pairs[2 * i], d = pairs[2 * i + 1];
        if (s >= n || d >= n) atomicOr(err, 1ull);
        keys[i] = ((uint64_t)s << 32) | d;
    }
}

// insert every (u, v) of the CSR into the edge hash set (4-key buckets, linear probing)
__global__ void k_edge_hash_build(const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg, uint64_t n,
                                  const uint32_t* __restrict__ adj, unsigned long long* __restrict__ table, uint64_t mask)
{
    const uint64_t v0 = (uint64_t)blockIdx.x * 64;
    for (uint64_t u = v0 + threadIdx.x / 64; u < min(v0 + 64, n); u += blockDim.x / 64) {
        const uint64_t b0 = off[u], e0 = b0 + deg[u];
        for (uint64_t j = b0 + (threadIdx.x & 63); j < e0; j += 64) {
            const unsigned long long key = (u << 32) | adj[j];
            uint64_t b = (edge_hash(key) & mask) & ~3ull;
            for (bool done = false; !done; b = (b + 4) & mask) {
                for (int k = 0; k < 4 && !done; k++) {
                    const unsigned long long old = atomicCAS(table + b + k, (unsigned long long)kEmptyKey, key);
                    done = old == kEmptyKey || old == key;
                }
            }
        }
    }
}

// apply a batch to the edge set: insert the new edges / tombstone the deleted ones
__global__ void k_edge_hash_update(const uint64_t* __restrict__ bkeys, uint64_t mb, const uint32_t* __restrict__ chg,
                                   int insert, unsigned long long* __restrict__ table, uint64_t mask)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < mb; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!chg[i]) continue;
        const unsigned long long key = bkeys[i];
        uint64_t b = (edge_hash(key) & mask) & ~3ull;
        for (bool done = false; !done; b = (b + 4) & mask) {
            for (int k = 0; k < 4 && !done; k++) {
                if (insert) {
                    const unsigned long long old = atomicCAS(table + b + k, (unsigned long long)kEmptyKey, key);
                    done = old == kEmptyKey || old == key;
                } else {
                    const unsigned long long cur = table[b + k];
                    if (cur == key) { table[b + k] = kTombKey; done = true; }
                    else if (cur == kEmptyKey) done = true;   // not present
                }
            }
        }
    }
}

void launch_edge_hash_update(const uint64_t* bkeys, uint64_t mb, const uint32_t* chg, int insert, uint64_t* table,
                             uint64_t mask, hipStream_t s)
{
    if (mb) hipLaunchKernelGGL(k_edge_hash_update, grid_for(mb, 256), 256, 0, s, bkeys, mb, chg, insert,
                               (unsigned long long*)table, mask);
}

void launch_edge_hash_build(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* adj, uint64_t* table,
                            uint64_t mask, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_edge_hash_build, (unsigned)((n + 63) / 64), 256, 0, s, off, deg, n, adj,
                              (unsigned long long*)table, mask);
}

// ---------------------------------------------------------------------------
// Neighbour filters (see has_edge_filtered): sizes, directory, fill; per batch
// only the source rows are rebuilt (a row that outgrows its words gets new
// ones at the end of the pool)
// ---------------------------------------------------------------------------
__global__ void k_filter_sizes(const uint32_t* __restrict__ deg, uint64_t n, uint64_t* __restrict__ words)
{
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= n; u += (uint64_t)gridDim.x * blockDim.x)
        words[u] = u < n ? 1ull << filt_log2_words(deg[u]) : 0;
}

__global__ void k_filter_pack(const uint32_t* __restrict__ deg, uint64_t n, uint64_t* __restrict__ fdir)
{
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (uint64_t)gridDim.x * blockDim.x)
        fdir[u] |= (uint64_t)filt_log2_words(deg[u]) << kFiltOffBits;
}

__device__ __forceinline__ void filter_set(uint32_t* pool, uint64_t fd, uint32_t c)
{
    const uint64_t h = filt_hash(c);
    atomicOr(pool + filt_word(fd, h), filt_bits(h));
}

// one wave per row, lanes sweep the row's targets (as k_edge_hash_build)
__global__ void k_filter_fill(const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg, uint64_t n,
                              const uint32_t* __restrict__ adj, const uint64_t* __restrict__ fdir,
                              uint32_t* __restrict__ pool)
{
    const uint64_t v0 = (uint64_t)blockIdx.x * 64;
    for (uint64_t u = v0 + threadIdx.x / 64; u < min(v0 + 64, n); u += blockDim.x / 64) {
        const uint64_t b0 = off[u], e0 = b0 + deg[u], fd = fdir[u];
        for (uint64_t j = b0 + (threadIdx.x & 63); j < e0; j += 64) filter_set(pool, fd, adj[j]);
    }
}

// per batch source: words its new row needs when it outgrew its old ones, else 0
__global__ void k_filter_plan(const RunInfo* __restrict__ runs, uint64_t k, const uint32_t* __restrict__ deg,
                              const uint64_t* __restrict__ fdir, uint64_t* __restrict__ need)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= k; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i == k) { need[i] = 0; continue; }
        const uint32_t u = runs[i].src;
        const uint32_t lg = filt_log2_words(deg[u]);
        need[i] = lg > (uint32_t)(fdir[u] >> kFiltOffBits) ? 1ull << lg : 0;
    }
}

// one block per batch source: (re)place, clear and refill its filter from the new row
__global__ void k_filter_rows(const RunInfo* __restrict__ runs, const uint64_t* __restrict__ noff,
                              const uint32_t* __restrict__ deg, const uint32_t* __restrict__ adj, const uint64_t* __restrict__ need,
                              const uint64_t* __restrict__ gofs, uint64_t base, uint64_t* __restrict__ fdir,
                              uint32_t* __restrict__ pool)
{
    const uint64_t i = blockIdx.x;
    const uint32_t u = runs[i].src;
    uint64_t fd = fdir[u];
    if (need[i]) {
        const uint32_t lg = filt_log2_words(deg[u]);
        fd = (base + gofs[i]) | ((uint64_t)lg << kFiltOffBits);
        __syncthreads();   // every thread has read the old descriptor
        if (threadIdx.x == 0) fdir[u] = fd;
    }
    const uint64_t w0 = fd & kFiltOffMask, nw = 1ull << (fd >> kFiltOffBits);
    for (uint64_t j = threadIdx.x; j < nw; j += blockDim.x) pool[w0 + j] = 0;
    __threadfence();
    __syncthreads();
    for (uint64_t j = noff[u] + threadIdx.x; j < noff[u] + deg[u]; j += blockDim.x) filter_set(pool, fd, adj[j]);
}

void launch_filter_sizes(const uint32_t* deg, uint64_t n, uint64_t* words, hipStream_t s)
{
    hipLaunchKernelGGL(k_filter_sizes, grid_for(n + 1, 256), 256, 0, s, deg, n, words);
}

void launch_filter_pack(const uint32_t* deg, uint64_t n, uint64_t* fdir, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_filter_pack, grid_for(n, 256), 256, 0, s, deg, n, fdir);
}

void launch_filter_fill(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* adj, const uint64_t* fdir,
                        uint32_t* pool, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_filter_fill, (unsigned)((n + 63) / 64), 256, 0, s, off, deg, n, adj, fdir, pool);
}

void launch_filter_plan(const RunInfo* runs, uint64_t k, const uint32_t* deg, const uint64_t* fdir, uint64_t* need,
                        hipStream_t s)
{
    hipLaunchKernelGGL(k_filter_plan, grid_for(k + 1, 256), 256, 0, s, runs, k, deg, fdir, need);
}


__global__ void k_csr_to_keys(const uint64_t* __restrict__ off, uint64_t n, const uint32_t* __restrict__ tgt,
                              uint64_t* __restrict__ keys, unsigned long long* __restrict__ err)
{
    // one block per 64 rows: lanes sweep a row's targets contiguously
    const uint64_t v0 = (uint64_t)blockIdx.x * 64;
    for (uint64_t v = v0 + threadIdx.x / 64; v < min(v0 + 64, n); v += blockDim.x / 64) {
        const uint64_t b = off[v], e = off[v + 1];
        for (uint64_t j = b + (threadIdx.x & 63); j < e; j += 64) {
            const uint32_t d = tgt[j];
            if (d >= n) atomicOr(err, 1ull);
            keys[j] = (v << 32) | d;
        }
    }
}

// keep[i]: first of its run of equal keys, and not a self loop when asked
__global__ void k_unique_flags(const uint64_t* __restrict__ keys, uint64_t m, int drop_loops, uint8_t* __restrict__ keep)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        bool ok = i == 0 || keys[i - 1] != k;
        if (drop_loops && (uint32_t)(k >> 32) == (uint32_t)k) ok = false;
        keep[i] = ok;
    }
}

// off[v] = lower_bound(keys, v << 32) for v in [0, n]
__global__ void k_offsets_from_keys(const uint64_t* __restrict__ keys, uint64_t m, uint64_t n, uint64_t* __restrict__ off)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = v << 32;
        uint64_t lo = 0, hi = m;
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            if (keys[mid] < t) lo = mid + 1; else hi = mid;
        }
        off[v] = lo;
    }
}

__global__ void k_low32(const uint64_t* __restrict__ keys, uint64_t m, uint32_t* __restrict__ out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)keys[i];
}

__global__ void k_vrec(const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg, uint64_t n,
                       const uint32_t* __restrict__ row_epoch, ERec* __restrict__ vrec)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        vrec[v] = make_rec((uint32_t)v, deg[v], off[v], row_epoch ? row_epoch[v] : 0u);
}

// erec[e] = vrec[adj[e]] for every live slot of the pool: each slot carries
// its target's row (rs = 2: 32-B records whose anchor entry starts empty,
// unless keep_anchors: a repack copied them along)
__global__ void k_erec(const uint32_t* __restrict__ adj, uint64_t slots, const ERec* __restrict__ vrec,
                       ERec* __restrict__ erec, uint32_t rs, int keep_anchors, RecFmt rf)
{
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < slots; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t t = adj[e];
        if (t == kGap) continue;
        store_erec(erec, e, rs, vrec[t], rf);
        if (rs == 2 && !keep_anchors) reinterpret_cast<uint64_t*>(erec)[e * kAnchorStride + 2] = kAnchorNone64;
    }
}

void launch_vrec(const uint64_t* off, const uint32_t* deg, uint64_t n, const uint32_t* row_epoch, ERec* vrec,
                 hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_vrec, grid_for(n, 256), 256, 0, s, off, deg, n, row_epoch, vrec);
}

void launch_erec(const uint32_t* adj, uint64_t slots, const ERec* vrec, ERec* erec, uint32_t rs, int keep_anchors,
                 RecFmt rf, hipStream_t s)
{
    if (slots)
        hipLaunchKernelGGL(k_erec, grid_for(slots, 256), 256, 0, s, adj, slots, vrec, erec, rs, keep_anchors, rf);
}

// Per batch edge (sorted, unique): does it change its source row?
//   insert: dst not yet in adj(src)  (tree_plus::uniont, wharfmh.h:511)
//   delete: dst present in adj(src)  (tree_plus::difference, wharfmh.h:659)
__global__ void k_batch_change(const uint64_t* __restrict__ bkeys, uint64_t mb, const uint64_t* __restrict__ off,
                               const uint32_t* __restrict__ deg, const uint32_t* __restrict__ adj, int insert,
                               uint32_t* __restrict__ chg)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < mb; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(bkeys[i] >> 32), d = (uint32_t)bkeys[i];
        uint64_t lo = off[s], hi = lo + deg[s];
        const uint64_t end = hi;
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            if (adj[mid] < d) lo = mid + 1; else hi = mid;
        }
        const bool present = lo < end && adj[lo] == d;
        chg[i] = insert ? !present : present;
    }
}

// run starts of equal sources -> flag
__global__ void k_run_flags(const uint64_t* __restrict__ bkeys, uint64_t mb, uint8_t* __restrict__ f)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < mb; i += (uint64_t)gridDim.x * blockDim.x)
        f[i] = i == 0 || (bkeys[i] >> 32) != (bkeys[i - 1] >> 32);
}

// per source run j: src, old row [off, end), batch run [rs, re)
__global__ void k_run_info(const uint64_t* __restrict__ bkeys, const uint32_t* __restrict__ run_start, uint64_t k,
                           uint64_t mb, const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg,
                           RunInfo* __restrict__ runs, uint32_t* __restrict__ bitmap, uint32_t* __restrict__ bloom)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t rs = run_start[j];
        const uint32_t re = j + 1 < k ? run_start[j + 1] : (uint32_t)mb;
        const uint32_t s = (uint32_t)(bkeys[rs] >> 32);
        RunInfo ri;
        ri.src = s; ri.rs = rs; ri.re = re; ri.off = off[s]; ri.end = off[s] + deg[s];
        runs[j] = ri;
        atomicOr(bitmap + (s >> 5), 1u << (s & 31));
        const uint32_t h = bloom_mix(s);
        atomicOr(bloom + bloom_word(h), bloom_bits(h));
        atomicOr(bloom + kBloomWords + bloom_word_big(h), bloom_bits(h));
    }
}

// batch_walk_update with a caller-given vertex set: the same bitmap, Bloom
// filter and source table (src only) as k_run_info, no sampler reset
__global__ void k_mark_sources(const uint32_t* __restrict__ src, uint64_t k, RunInfo* __restrict__ runs,
                               uint32_t* __restrict__ bitmap, uint32_t* __restrict__ bloom)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[j];
        RunInfo ri{};
        ri.src = s;
        runs[j] = ri;
        atomicOr(bitmap + (s >> 5), 1u << (s & 31));
        const uint32_t h = bloom_mix(s);
        atomicOr(bloom + bloom_word(h), bloom_bits(h));
        atomicOr(bloom + kBloomWords + bloom_word_big(h), bloom_bits(h));
    }
}

// ---------------------------------------------------------------------------
// Slack-row CSR: a batch touches only the rows of its sources.
//
// Row v lives at slots [off[v], off[v] + deg[v]) of the slot pool (adj and
// the edge records erec share the slot index), with cap[v] >= deg[v] slots
// reserved; unused slots hold kGap.  An update merges each source's batch
// edges into its row in place when the row's slack holds them, else moves the
// row to fresh slots at the end of the pool (its old slots become kGap); the
// pool is repacked with fresh slack only when its headroom runs out.  Every
// record caches its target's row, so the records of slots whose target is a
// batch source (the in-edges of a changed row, whatever the graph's
// symmetry) are rewritten by one streaming scan of the pool's targets with
// the batch-source Bloom filter in LDS: 4 B per slot instead of moving every
// slot's target and record (40 or 72 B) as a contiguous CSR requires.
// ---------------------------------------------------------------------------

// from a contiguous CSR: deg, the initial capacity and the capacity as u64
// for the layout scan (capw[n] = 0)
__global__ void k_row_degrees(const uint64_t* __restrict__ coff, uint64_t n, uint32_t* __restrict__ deg,
                              uint32_t* __restrict__ cap, uint64_t* __restrict__ capw, int slack)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (uint64_t)gridDim.x * blockDim.x) {
        if (v == n) { capw[n] = 0; continue; }
        const uint32_t d = (uint32_t)(coff[v + 1] - coff[v]);
        const uint32_t c = slack ? row_cap_initial(d) : d;
        deg[v] = d;
        cap[v] = c;
        capw[v] = c;
    }
}

// repack: fresh capacities from the current degrees (capw as above)
__global__ void k_row_recap(const uint32_t* __restrict__ deg, uint64_t n, uint32_t* __restrict__ cap,
                            uint64_t* __restrict__ capw, int slack)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (uint64_t)gridDim.x * blockDim.x) {
        if (v == n) { capw[n] = 0; continue; }
        const uint32_t c = slack ? row_cap_initial(deg[v]) : deg[v];
        cap[v] = c;
        capw[v] = c;
    }
}

// deg as u64 with a trailing 0 (the scan of a compacted export)
__global__ void k_deg_u64(const uint32_t* __restrict__ deg, uint64_t n, uint64_t* __restrict__ out)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (uint64_t)gridDim.x * blockDim.x)
        out[v] = v < n ? deg[v] : 0;
}

// dst[doff[v] + i] = src[soff[v] + i] for i < deg[v], one wave per row; with
// sanc, the 8-B anchor entries travel along (stride kAnchorStride)
__global__ void k_copy_rows(const uint64_t* __restrict__ soff, const uint32_t* __restrict__ deg,
                            const uint32_t* __restrict__ src, const uint64_t* __restrict__ doff, uint64_t n,
                            uint32_t* __restrict__ dst, const uint64_t* __restrict__ sanc, uint64_t* __restrict__ danc)
{
    const uint64_t v0 = (uint64_t)blockIdx.x * 64;
    for (uint64_t v = v0 + threadIdx.x / 64; v < min(v0 + 64, n); v += blockDim.x / 64) {
        const uint64_t b = soff[v], o = doff[v];
        const uint32_t d = deg[v];
        for (uint32_t j = threadIdx.x & 63; j < d; j += 64) {
            dst[o + j] = src[b + j];
            if (sanc) danc[(o + j) * kAnchorStride] = sanc[(b + j) * kAnchorStride];
        }
    }
}

// per run: the source's new degree and, when it outgrows the row's slots,
// the capacity of its new place (need), and its old degree (save: the
// scratch copy the merge reads)
__global__ void k_plan_rows(const RunInfo* __restrict__ runs, uint64_t k, const uint32_t* __restrict__ cap,
                            const uint32_t* __restrict__ cf, int insert, int slack, uint64_t* __restrict__ need,
                            uint64_t* __restrict__ save, RowPlan* __restrict__ plan, unsigned long long* __restrict__ dead)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= k; j += (uint64_t)gridDim.x * blockDim.x) {
        if (j == k) { need[k] = 0; save[k] = 0; continue; }
        const RunInfo ri = runs[j];
        const uint32_t d = (uint32_t)(ri.end - ri.off), c = cap[ri.src];
        const uint32_t delta = cf[ri.re] - cf[ri.rs];
        const uint32_t nd = insert ? d + delta : d - delta;
        const bool reloc = nd > c;
        const uint32_t nc = reloc ? (slack ? row_cap_grown(nd) : nd) : c;
        need[j] = reloc ? nc : 0;
        save[j] = d;
        plan[j] = RowPlan{reloc ? kRelocate : ri.off, nd, nc, c};
        if (reloc && c) atomicAdd(dead, (unsigned long long)c);   // the row's old place becomes kGap
    }
}

// block per run: the old row, copied aside (the merge may overwrite it in place);
// with sanc, its anchor entries too (anchor carry, k_anchor_invalidate)
__global__ void k_save_rows(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ adj,
                            const uint64_t* __restrict__ sofs, uint32_t* __restrict__ scratch,
                            const uint64_t* __restrict__ anc, uint64_t* __restrict__ sanc,
                            const uint32_t* __restrict__ rev, uint32_t* __restrict__ srev)
{
    const RunInfo ri = runs[blockIdx.x];
    uint32_t* __restrict__ out = scratch + sofs[blockIdx.x];
    for (uint64_t i = threadIdx.x; i < ri.end - ri.off; i += blockDim.x) {
        out[i] = adj[ri.off + i];
        if (sanc) sanc[sofs[blockIdx.x] + i] = anc[(ri.off + i) * kAnchorStride];
        if (srev) srev[sofs[blockIdx.x] + i] = rev[ri.off + i];
    }
}

// first index in a[0, n) with a[i] >= x (ascending u32)
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}
// the same over the low words of sorted (src, dst) keys
__device__ __forceinline__ uint32_t lower_bound_dst(const uint64_t* __restrict__ k, uint32_t n, uint32_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint32_t)k[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Block per run: write the source's new row, ascending (tree_plus::uniont /
// difference, wharfmh.h:511,659).  Insert: old element i lands at i + (new
// batch edges below it), new edge t at (new edges before t) + (old elements
// below it).  Delete: old element i, unless deleted, lands at i - (deleted
// edges below it).  Slots left over become kGap: the tail of a shrunk row,
// or the whole old place of a moved row and the slack of its new one.
__global__ void k_merge_rows(const RunInfo* __restrict__ runs, const uint64_t* __restrict__ bkeys,
                             const uint32_t* __restrict__ chg, const uint32_t* __restrict__ cf,
                             const uint32_t* __restrict__ scratch, const uint64_t* __restrict__ sofs,
                             const uint64_t* __restrict__ relofs, uint64_t pool_end, int insert,
                             RowPlan* __restrict__ plan, uint32_t* __restrict__ adj,
                             const uint64_t* __restrict__ sanc, uint64_t* __restrict__ anc,
                             const uint32_t* __restrict__ srev, uint32_t* __restrict__ rev)
{
    const uint64_t j = blockIdx.x;
    const RunInfo ri = runs[j];
    const RowPlan p = plan[j];
    const bool reloc = p.noff == kRelocate;
    const uint64_t noff = reloc ? pool_end + relofs[j] : ri.off;
    const uint32_t d = (uint32_t)(ri.end - ri.off), nb = ri.re - ri.rs, base = cf[ri.rs];
    const uint32_t* __restrict__ old = scratch + sofs[j];
    const uint64_t* __restrict__ bk = bkeys + ri.rs;
    for (uint32_t i = threadIdx.x; i < d; i += blockDim.x) {
        const uint32_t x = old[i];
        const uint32_t lb = lower_bound_dst(bk, nb, x);
        const uint32_t below = cf[ri.rs + lb] - base;
        uint64_t at = ~0ull;
        if (insert) at = noff + i + below;
        else if (!(lb < nb && (uint32_t)bk[lb] == x && chg[ri.rs + lb])) at = noff + i - below;
        if (at != ~0ull) {
            adj[at] = x;
            if (sanc) anc[at * kAnchorStride] = sanc[sofs[j] + i];   // the entry travels with its edge
            if (srev) rev[at] = srev[sofs[j] + i];
        }
    }
    if (insert) {
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) {
            if (!chg[ri.rs + t]) continue;
            const uint32_t x = (uint32_t)bk[t];
            const uint64_t at = noff + (cf[ri.rs + t] - base) + lower_bound_u32(old, d, x);
            adj[at] = x;
            if (sanc) anc[at * kAnchorStride] = kAnchorNone64;
            if (srev) rev[at] = kNoRidx;
        }
    }
    if (reloc) {
        for (uint32_t i = threadIdx.x; i < p.ocap; i += blockDim.x) adj[ri.off + i] = kGap;
        for (uint32_t i = p.ndeg + threadIdx.x; i < p.ncap; i += blockDim.x) adj[noff + i] = kGap;
    } else {
        for (uint32_t i = p.ndeg + threadIdx.x; i < d; i += blockDim.x) adj[ri.off + i] = kGap;
    }
    __syncthreads();   // every thread has read plan[j] before it is resolved
    if (threadIdx.x == 0) plan[j].noff = noff;
}

// ---------------------------------------------------------------------------
// Source rows in chunks (round 4).  The kernels above take one workgroup per
// batch source; a hub source's row (10^5-10^6 slots on the configs[3] / [4]
// graphs) then runs on one CU while the rest of the chip idles: in the
// configs[4] shard's update, save / merge / records / filters took 0.6 / 0.7 /
// 0.76 / 1.47 ms, nearly all of it the few hub rows' workgroups
// (profiles/r04/update_rows).  Here every run is cut into kRowChunk-slot
// chunks of its longest range (old row, old and new capacity), the chunk counts
// are prefix-summed on the device, and a persistent grid deals the chunks, so a
// hub row spreads over the chip.  Every element's work is independent (the
// merge reads the saved copy of the old row, so its writes may land in any
// order), and the one write that ordered them — the move target resolved into
// plan[j].noff at the end of k_merge_rows — is a separate kernel after it.
// ---------------------------------------------------------------------------
#ifndef WHARF_ROW_CHUNKED
#define WHARF_ROW_CHUNKED 1   // A/B: 0 = a workgroup per source row (round 3)
#endif
constexpr uint32_t kRowChunk = 4096;

__global__ void k_run_chunks(const RunInfo* __restrict__ runs, const RowPlan* __restrict__ plan, uint64_t k,
                             uint32_t* __restrict__ cnt)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= k; j += (uint64_t)gridDim.x * blockDim.x) {
        if (j == k) { cnt[k] = 0; continue; }
        const uint64_t d = runs[j].end - runs[j].off;
        const uint64_t len = max(max(d, (uint64_t)plan[j].ocap), max((uint64_t)plan[j].ncap, (uint64_t)1));
        cnt[j] = (uint32_t)((len + kRowChunk - 1) / kRowChunk);
    }
}

// chunk t of the prefix `pre` (pre[k] = total): its run j and the run's chunk c
__device__ __forceinline__ bool run_chunk(const uint32_t* __restrict__ pre, uint64_t k, uint64_t t, uint64_t& j,
                                          uint32_t& c)
{
    if (t >= pre[k]) return false;
    uint64_t lo = 0, hi = k;   // the last run with pre[run] <= t
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (pre[mid] <= t) lo = mid; else hi = mid;
    }
    j = lo;
    c = (uint32_t)(t - pre[lo]);
    return true;
}

__global__ void k_save_rows_c(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                              const uint32_t* __restrict__ adj, const uint64_t* __restrict__ sofs,
                              uint32_t* __restrict__ scratch, const uint64_t* __restrict__ anc, uint64_t* __restrict__ sanc,
                              const uint32_t* __restrict__ rev, uint32_t* __restrict__ srev)
{
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const RunInfo ri = runs[j];
        const uint64_t d = ri.end - ri.off, hi = min(d, lo + kRowChunk);
        uint32_t* __restrict__ out = scratch + sofs[j];
        for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
            out[i] = adj[ri.off + i];
            if (sanc) sanc[sofs[j] + i] = anc[(ri.off + i) * kAnchorStride];
            if (srev) srev[sofs[j] + i] = rev[ri.off + i];
        }
    }
}

__global__ void k_merge_rows_c(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                               const uint64_t* __restrict__ bkeys, const uint32_t* __restrict__ chg,
                               const uint32_t* __restrict__ cf, const uint32_t* __restrict__ scratch,
                               const uint64_t* __restrict__ sofs, const uint64_t* __restrict__ relofs, uint64_t pool_end,
                               int insert, const RowPlan* __restrict__ plan, uint32_t* __restrict__ adj,
                               const uint64_t* __restrict__ sanc, uint64_t* __restrict__ anc,
                               const uint32_t* __restrict__ srev, uint32_t* __restrict__ rev)
{
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const RunInfo ri = runs[j];
        const RowPlan p = plan[j];   // (noff is resolved by k_resolve_plan, after every chunk)
        const bool reloc = p.noff == kRelocate;
        const uint64_t noff = reloc ? pool_end + relofs[j] : ri.off;
        const uint32_t d = (uint32_t)(ri.end - ri.off), nb = ri.re - ri.rs, base = cf[ri.rs];
        const uint32_t* __restrict__ old = scratch + sofs[j];
        const uint64_t* __restrict__ bk = bkeys + ri.rs;
        const uint64_t hi = lo + kRowChunk;
        for (uint64_t i = lo + threadIdx.x; i < min(hi, (uint64_t)d); i += blockDim.x) {
            const uint32_t x = old[i];
            const uint32_t lb = lower_bound_dst(bk, nb, x);
            const uint32_t below = cf[ri.rs + lb] - base;
            uint64_t at = ~0ull;
            if (insert) at = noff + i + below;
            else if (!(lb < nb && (uint32_t)bk[lb] == x && chg[ri.rs + lb])) at = noff + i - below;
            if (at != ~0ull) {
                adj[at] = x;
                if (sanc) anc[at * kAnchorStride] = sanc[sofs[j] + i];   // the entry travels with its edge
                if (srev) rev[at] = srev[sofs[j] + i];
            }
        }
        if (insert && c == 0) {
            for (uint32_t e = threadIdx.x; e < nb; e += blockDim.x) {
                if (!chg[ri.rs + e]) continue;
                const uint32_t x = (uint32_t)bk[e];
                const uint64_t at = noff + (cf[ri.rs + e] - base) + lower_bound_u32(old, d, x);
                adj[at] = x;
                if (sanc) anc[at * kAnchorStride] = kAnchorNone64;
                if (srev) rev[at] = kNoRidx;
            }
        }
        if (reloc) {
            for (uint64_t i = lo + threadIdx.x; i < min(hi, (uint64_t)p.ocap); i += blockDim.x) adj[ri.off + i] = kGap;
            for (uint64_t i = max(lo, (uint64_t)p.ndeg) + threadIdx.x; i < min(hi, (uint64_t)p.ncap); i += blockDim.x)
                adj[noff + i] = kGap;
        } else {
            for (uint64_t i = max(lo, (uint64_t)p.ndeg) + threadIdx.x; i < min(hi, (uint64_t)d); i += blockDim.x)
                adj[ri.off + i] = kGap;
        }
    }
}

__global__ void k_resolve_plan(const RunInfo* __restrict__ runs, uint64_t k, const uint64_t* __restrict__ relofs,
                               uint64_t pool_end, RowPlan* __restrict__ plan)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (uint64_t)gridDim.x * blockDim.x)
        plan[j].noff = plan[j].noff == kRelocate ? pool_end + relofs[j] : runs[j].off;
}

__global__ void k_erec_rows_c(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                              const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg,
                              const uint32_t* __restrict__ adj, const ERec* __restrict__ vrec, ERec* __restrict__ erec,
                              uint32_t rs, int keep_anc, RecFmt rf)
{
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const uint32_t s = runs[j].src;
        const uint64_t b = off[s], e = b + deg[s];
        for (uint64_t q = b + lo + threadIdx.x; q < min(e, b + lo + kRowChunk); q += blockDim.x) {
            store_erec(erec, q, rs, vrec[adj[q]], rf);
            if (rs == 2 && !keep_anc) reinterpret_cast<uint64_t*>(erec)[q * kAnchorStride + 2] = kAnchorNone64;
        }
    }
}

// per batch source: its neighbour filter's new descriptor (rows that outgrew their words)
__global__ void k_filter_desc(const RunInfo* __restrict__ runs, uint64_t k, const uint32_t* __restrict__ deg,
                              const uint64_t* __restrict__ need, const uint64_t* __restrict__ gofs, uint64_t base,
                              uint64_t* __restrict__ fdir)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (uint64_t)gridDim.x * blockDim.x)
        if (need[i]) fdir[runs[i].src] = (base + gofs[i]) | ((uint64_t)filt_log2_words(deg[runs[i].src]) << kFiltOffBits);
}

__global__ void k_filter_clear_c(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                                 const uint64_t* __restrict__ fdir, uint32_t* __restrict__ pool)
{
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const uint64_t fd = fdir[runs[j].src], w0 = fd & kFiltOffMask, nw = 1ull << (fd >> kFiltOffBits);
        // the run's last chunk clears every word left: a filter sized by an earlier, larger degree
        // (deletions never shrink it) can have more words than the chunks of the rows cover
        const uint64_t hi = c + 1 == pre[j + 1] - pre[j] ? nw : min(nw, lo + kRowChunk);
        for (uint64_t q = lo + threadIdx.x; q < hi; q += blockDim.x) pool[w0 + q] = 0;
    }
}

__global__ void k_filter_fill_c(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                                const uint64_t* __restrict__ noff, const uint32_t* __restrict__ deg,
                                const uint32_t* __restrict__ adj, const uint64_t* __restrict__ fdir,
                                uint32_t* __restrict__ pool)
{
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const uint32_t u = runs[j].src;
        const uint64_t fd = fdir[u], b = noff[u];
        for (uint64_t q = lo + threadIdx.x; q < min((uint64_t)deg[u], lo + kRowChunk); q += blockDim.x)
            filter_set(pool, fd, adj[b + q]);
    }
}

static unsigned chunk_grid() { return cu_count() * 4; }

// per run: the source's new row and record, and its row epoch: the source's
// samplers are reset (wharfmh.h:504,539).  Runs after the last point where the
// batch can fail (the pool planning), so a failed batch leaves no epoch behind.
__global__ void k_commit_rows(const RunInfo* __restrict__ runs, uint64_t k, const RowPlan* __restrict__ plan,
                              uint32_t epoch, uint64_t* __restrict__ off, uint32_t* __restrict__ deg,
                              uint32_t* __restrict__ cap, ERec* __restrict__ vrec, uint32_t* __restrict__ row_epoch)
{
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = runs[j].src;
        const RowPlan p = plan[j];
        off[s] = p.noff;
        deg[s] = p.ndeg;
        cap[s] = p.ncap;
        vrec[s] = make_rec(s, p.ndeg, p.noff, epoch);
        if (row_epoch) row_epoch[s] = epoch;
    }
}

// records of the rebuilt source rows: erec[slot] = vrec[adj[slot]] (block per
// run); their anchor entries (states (target, source), whose anchors read the
// source's row) start empty: see anchor_lookup and DESIGN.md §4
__global__ void k_erec_rows(const RunInfo* __restrict__ runs, const uint64_t* __restrict__ off,
                            const uint32_t* __restrict__ deg, const uint32_t* __restrict__ adj,
                            const ERec* __restrict__ vrec, ERec* __restrict__ erec, uint32_t rs, int keep_anc,
                            RecFmt rf)
{
    const uint32_t s = runs[blockIdx.x].src;
    const uint64_t b = off[s], e = b + deg[s];
    for (uint64_t j = b + threadIdx.x; j < e; j += blockDim.x) {
        store_erec(erec, j, rs, vrec[adj[j]], rf);
        if (rs == 2 && !keep_anc) reinterpret_cast<uint64_t*>(erec)[j * kAnchorStride + 2] = kAnchorNone64;
    }
}

// Anchor carry (node2vec MH, undirected graphs).  The entry of slot x -> y holds
// the anchor of state (y, x): 21 proposals from y's row, classed by
// has_edge(x, proposal).  A batch that changes x's row by the edges (x, c)
// changes only the classes of proposals equal to some c, so the anchor can
// differ only where c is in y's row: y in N(x) and N(c).  Those entries are
// reset; every other entry of x's row is carried through the merge
// (k_save_rows / k_merge_rows) and equals what a re-initialisation would give
// (the anchor is a pure function of the two rows).  One wave per
// changed batch edge.  With the neighbour filters (fdir / fpool, refilled for
// the new rows), x's row is walked and each y tested against c's filter: one
// independent load per element, and a false positive only resets an entry
// that did not need it.  Without them the smaller row's elements are searched
// in the larger row.
__global__ __launch_bounds__(256) void k_anchor_invalidate(const uint64_t* __restrict__ bkeys, uint64_t mb,
                                                           const uint32_t* __restrict__ chg,
                                                           const uint64_t* __restrict__ off,
                                                           const uint32_t* __restrict__ deg,
                                                           const uint32_t* __restrict__ adj, uint64_t* __restrict__ anc,
                                                           const uint64_t* __restrict__ fdir,
                                                           const uint32_t* __restrict__ fpool)
{
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t lane = __lane_id();
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < mb; i += nw) {
        const uint64_t key = bkeys[i];
        const uint32_t x = (uint32_t)(key >> 32), c = (uint32_t)key;
        if (!chg[i] || x == c) continue;   // (wave-uniform)
        const Row rx{x, deg[x], 0u, off[x]}, rcv{c, deg[c], 0u, off[c]};
        if (fpool) {
            // the smaller row's elements against the other row's filter; a positive found in c's
            // row is located in x's row by a search (positives are few: N(x) and N(c) rarely meet)
            const bool walk_x = rx.deg <= rcv.deg;
            const Row& rw = walk_x ? rx : rcv;
            const uint64_t fd = fdir[walk_x ? c : x];
            for (uint32_t j = lane; j < rw.deg; j += 64) {
                const uint32_t y = adj[rw.off + j];
                const uint64_t h = filt_hash(y);
                const uint32_t b = filt_bits(h);
                if ((fpool[filt_word(fd, h)] & b) != b) continue;
                const int64_t e = walk_x ? (int64_t)(rx.off + j) : row_find(adj, rx, y);
                if (e >= 0) anc[(uint64_t)e * kAnchorStride] = kAnchorNone64;
            }
        } else if (rx.deg <= rcv.deg) {
            for (uint32_t j = lane; j < rx.deg; j += 64)
                if (row_find(adj, rcv, adj[rx.off + j]) >= 0) anc[(rx.off + j) * kAnchorStride] = kAnchorNone64;
        } else {
            for (uint32_t j = lane; j < rcv.deg; j += 64) {
                const int64_t e = row_find(adj, rx, adj[rcv.off + j]);
                if (e >= 0) anc[(uint64_t)e * kAnchorStride] = kAnchorNone64;
            }
        }
    }
}

// keys sorted ascending: any key whose reverse (v, u) is missing sets *asym
__global__ void k_keys_symmetric(const uint64_t* __restrict__ keys, uint64_t m, unsigned long long* __restrict__ asym)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i], r = (k << 32) | (k >> 32);
        uint64_t lo = 0, hi = m;
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            if (keys[mid] < r) lo = mid + 1; else hi = mid;
        }
        if (lo >= m || keys[lo] != r) *asym = 1ull;   // (a plain store: every writer writes 1)
    }
}

// In-edge records of the batch sources: every slot whose target is a source
// gets the source's new row record (the anchor entry stays: its epoch tag is
// checked against the new row epoch, anchor_lookup).  One streaming pass over
// the pool's targets, four slots per 16-B load; the Bloom filter of the
// sources sits in LDS and only its positives read the exact bitmap.
__device__ __forceinline__ void patch_slot(uint32_t t, uint64_t e, const uint32_t* bitmap, const ERec* vrec, ERec* erec,
                                           uint32_t rs, RecFmt rf)
{
    if (t != kGap && ((bitmap[t >> 5] >> (t & 31)) & 1u)) store_erec(erec, e, rs, vrec[t], rf);
}

// 1024-thread workgroups, two per CU (the 64-KiB filter in LDS), 32 waves per CU (8 per SIMD: 64 VGPRs)
#ifndef WHARF_INEDGE_LOADS
#define WHARF_INEDGE_LOADS 4
#endif
constexpr uint32_t kInEdgeLoads = WHARF_INEDGE_LOADS;
#ifndef WHARF_INEDGE_NT
#define WHARF_INEDGE_NT 1   // A/B: non-temporal pool loads (the pool is read once per batch)
#endif
// Round 3: the filter test of the thread's four 16-B loads first, then one
// wave-uniform branch to the positives (round 2 branched per load: configs[3]
// pass 2.65-2.73 -> 2.32-2.38 ms with the lean test).  A two-pass form that
// listed the positives' slots and settled them after the stream was slower
// (2.93-3.03 vs 2.52-2.56 ms, profiles/r03/in_edge_scan).
__global__ __launch_bounds__(1024, 8) void k_patch_in_edges(const uint32_t* __restrict__ adj, uint64_t slots,
                                                        const uint32_t* __restrict__ bitmap,
                                                        const uint32_t* __restrict__ bloom_big,
                                                        const ERec* __restrict__ vrec, ERec* __restrict__ erec,
                                                        uint32_t rs, RecFmt rf)
{
    __shared__ uint32_t s_bloom[kBigBloomWords];
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (uint32_t i = threadIdx.x; i < kBigBloomWords / 4; i += blockDim.x)
        reinterpret_cast<u32x4*>(s_bloom)[i] = reinterpret_cast<const u32x4*>(bloom_big)[i];
    __syncthreads();
    // 32-bit 16-B-group indices (a pool of < 2^34 slots); the Bloom test as shifts of the
    // filter word (the lean scan's form: ~11 VALU per slot instead of ~15)
    const uint32_t n4 = (uint32_t)(slots / 4), stride = gridDim.x * blockDim.x;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const u32x4* __restrict__ a4 = reinterpret_cast<const u32x4*>(adj);
    auto lean_test = [&](uint32_t x) -> uint32_t {
        const uint32_t h = bloom_mix(x), fw = s_bloom[h >> 18];
        uint32_t t = (fw >> ((h >> 13) & 31u)) & (fw >> ((h >> 8) & 31u));
        if (WHARF_BLOOM_K > 2) t &= fw >> ((h >> 3) & 31u);
        return t & 1u;
    };
    // kInEdgeLoads 16-B loads per thread in flight (one left the pass latency-bound at 8 MB in flight;
    // configs[3] pool, 10.2 GB: 1 / 2 / 4 loads 3.00 / 2.75 / 2.65 ms, profiles/r02/in_edge_scan)
    for (uint32_t q0 = g; q0 < n4; q0 += kInEdgeLoads * stride) {
        u32x4 tv[kInEdgeLoads];
#pragma unroll
        for (uint32_t u = 0; u < kInEdgeLoads; u++) {
            const uint32_t q = q0 + u * stride;
#if WHARF_INEDGE_NT
            tv[u] = q < n4 ? __builtin_nontemporal_load(a4 + q) : u32x4{kGap, kGap, kGap, kGap};
#else
            tv[u] = q < n4 ? a4[q] : u32x4{kGap, kGap, kGap, kGap};
#endif
        }
        uint32_t hits = 0;   // 4 bits per load
#pragma unroll
        for (uint32_t u = 0; u < kInEdgeLoads; u++) {
            const u32x4 t = tv[u];
            hits |= (lean_test(t.x) | lean_test(t.y) << 1 | lean_test(t.z) << 2 | lean_test(t.w) << 3) << (4 * u);
        }
        if (!__any(hits != 0)) continue;
        for (uint32_t m = hits; m; m &= m - 1u) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            patch_slot(tv[b >> 2][b & 3u], 4 * (uint64_t)(q0 + (b >> 2) * stride) + (b & 3u), bitmap, vrec, erec, rs, rf);
        }
    }
    if (g < slots - 4 * (uint64_t)n4) {   // the pool's last < 4 slots
        const uint64_t e = 4 * (uint64_t)n4 + g;
        const uint32_t x = adj[e];
        if (bloom_test_big(s_bloom, x)) patch_slot(x, e, bitmap, vrec, erec, rs, rf);
    }
}

// ---------------------------------------------------------------------------
// Reverse-slot index (round 5; the survey's optional rev[e]).  On
// an undirected graph the in-edges of a batch source s are the reverses of its
// out-edges: the slot of (y -> s) in y's row, for y in N(s).  ridx[e] (u32, one
// per pool slot) holds, for slot e = (x -> y), the index of x in y's row, so the
// reverse slot is y.off + ridx[e], with y's row offset read from e's own edge
// record (erec[e] caches the target's row): no random read.  With it the records
// of the sources' in-edges are patched from the sources' own rows — Σ deg(s)
// direct record writes — instead of the streaming scan of every pool slot
// (k_patch_in_edges, 4 B per slot: 10.9 GB per batch at configs[3]).  An index
// relative to the target's row survives that row moving; it changes only when
// the row's content does, i.e. when the target is itself a batch source.  Kept
// valid through a batch:
//  * the entries of the sources' rows travel through k_save_rows / k_merge_rows
//    with their edges (a new edge starts kNoRidx);
//  * k_patch_rev recomputes an entry whose target is itself a batch source (its
//    row was rebuilt) or new, by a search of s in the target's new row, and
//    writes the reverse slot's entry with its record (ridx[r] = q - s.off);
//  * a repack or compaction moves the rows but not their ridx entries: the
//    index is rebuilt from scratch (k_rev_owner + k_rev_build, one search per
//    slot), as at its first build.
// Directed graphs (or batches) keep the scan.  Same records either way, so no
// result changes (the parity suite runs both: WHARF_REV=0 / 1).
// ---------------------------------------------------------------------------
// pass 1 of a build: ridx[e] = the owner row of slot e (one wave per row; slack slots stay kNoRidx)
__global__ void k_rev_owner(const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg, uint64_t n,
                            uint32_t* __restrict__ ridx)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t v = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); v < n; v += waves) {
        const uint64_t o = off[v];
        const uint32_t d = deg[v];
        for (uint32_t i = lane; i < d; i += 64) ridx[o + i] = (uint32_t)v;
    }
}

// pass 2, in place: owner x of slot e = (x -> y) -> the index of x in y's row (a search)
__global__ void k_rev_build(const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg,
                            const uint32_t* __restrict__ adj, uint64_t slots, uint32_t* __restrict__ ridx,
                            unsigned long long* __restrict__ miss)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < slots; e += stride) {
        const uint32_t x = ridx[e];
        if (x == kNoRidx) continue;
        const uint32_t y = adj[e];
        const uint64_t yo = off[y];
        const int64_t r = row_find(adj, Row{y, deg[y], 0u, yo}, x);
        if (r < 0) *miss = 1ull;   // (a plain store: every writer writes 1) the graph is not symmetric
        ridx[e] = r < 0 ? kNoRidx : (uint32_t)((uint64_t)r - yo);
    }
}

// Per batch, after the sources' rows and records are committed (k_commit_rows,
// k_erec_rows): slot q = (s -> y) of source s's new row gives its reverse r, whose
// record becomes s's new row and whose entry points back at q.  y's row (offset,
// degree) comes from q's own record, just rewritten by k_erec_rows.  Chunks of the
// sources' rows dealt as in k_erec_rows_c (a hub source's row spreads over the chip).
template <bool VERIFY>
__global__ void k_patch_rev(const RunInfo* __restrict__ runs, const uint32_t* __restrict__ pre, uint64_t k,
                            const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg,
                            const uint32_t* __restrict__ adj, const uint32_t* __restrict__ bitmap,
                            const ERec* __restrict__ vrec, ERec* __restrict__ erec, uint32_t rs, RecFmt rf,
                            uint32_t* __restrict__ ridx, unsigned long long* __restrict__ miss)
{
    // (pieces of 256 slots — one per thread — instead of the 4096-slot chunks were slower: the
    // chunk lookup's dependent loads then run once per 256 slots; configs[3] 0.9 -> 1.55 ms)
    for (uint64_t t = blockIdx.x;; t += gridDim.x) {   // chunk t: run j's chunk c, slots [lo, lo + kRowChunk)
        uint64_t j;
        uint32_t c;
        if (!run_chunk(pre, k, t, j, c)) break;
        const uint64_t lo = (uint64_t)c * kRowChunk;
        const uint32_t s = runs[j].src;
        const uint64_t b = off[s], e = b + deg[s];
        const ERec rec = vrec[s];
        for (uint64_t q = b + lo + threadIdx.x; q < min(e, b + lo + kRowChunk); q += blockDim.x) {
            const Row ry = load_erec(erec, q, rs, rf, deg);   // the target y and its (new) row
            uint32_t x = ridx[q];
            // a source target's row was rebuilt (and so was its entry for s): search it; a new edge too
            bool search = x == kNoRidx || ((bitmap[ry.v >> 5] >> (ry.v & 31)) & 1u);
            // a carried entry is checked before anything is written through it: outside y's row (always
            // checked: the degree is in hand), or -- VERIFY, on in the test suite (WHARF_REV_VERIFY=1,
            // tests/conftest.py): +0.25 ms per configs[4] batch -- not at s, it is stale (an index bug):
            // repaired by the search, and flagged so the host drops the index and the scan rewrites
            if (!search && (x >= ry.deg || (VERIFY && adj[ry.off + x] != s))) {
                *miss = 2ull;
                search = true;
            }
            if (search) {
                const int64_t f = row_find(adj, ry, s);
                if (f < 0) {
                    *miss = 1ull;
                    continue;
                }
                x = (uint32_t)((uint64_t)f - ry.off);
                ridx[q] = x;
            }
            const uint64_t r = ry.off + x;
            store_erec(erec, r, rs, rec, rf);   // the row part (node2vec: the anchor entry behind it stays)
            ridx[r] = (uint32_t)(q - b);
        }
    }
}

void launch_rev_build(const uint64_t* off, const uint32_t* deg, const uint32_t* adj, uint64_t n, uint64_t slots,
                      uint32_t* ridx, unsigned long long* miss, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_rev_owner, cu_count() * 32, 256, 0, s, off, deg, n, ridx);
    if (slots) hipLaunchKernelGGL(k_rev_build, cu_count() * 16, 256, 0, s, off, deg, adj, slots, ridx, miss);
}

void launch_patch_rev(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* off, const uint32_t* deg,
                      const uint32_t* adj, const uint32_t* bitmap, const ERec* vrec, ERec* erec, uint32_t rs,
                      RecFmt rf, uint32_t* ridx, unsigned long long* miss, hipStream_t s)
{
    // workgroups per CU (each deals 4096-slot chunks of the sources' rows; A/B: WHARF_PATCH_REV_WG)
    static const int per_cu = [] {
        const char* e = getenv("WHARF_PATCH_REV_WG");
        return e && *e ? std::max(1, atoi(e)) : 16;
    }();
    static const bool verify = [] {
        const char* e = getenv("WHARF_REV_VERIFY");
        return e && *e && atoi(e) != 0;
    }();
    if (k) {
        if (verify)
            hipLaunchKernelGGL(k_patch_rev<true>, cu_count() * per_cu, 256, 0, s, runs, pre, k, off, deg, adj, bitmap,
                               vrec, erec, rs, rf, ridx, miss);
        else
            hipLaunchKernelGGL(k_patch_rev<false>, cu_count() * per_cu, 256, 0, s, runs, pre, k, off, deg, adj, bitmap,
                               vrec, erec, rs, rf, ridx, miss);
    }
}

// ---------------------------------------------------------------------------
// walk export / index
// ---------------------------------------------------------------------------
// [L][W] -> [W][L] through a 64x64 LDS tile (+1 pad against bank conflicts)
__global__ void k_transpose(const uint32_t* __restrict__ in, uint64_t W, uint32_t L, uint32_t* __restrict__ out)
{
    __shared__ uint32_t tile[64][65];
    const uint64_t w0 = (uint64_t)blockIdx.x * 64;
    const uint32_t p0 = blockIdx.y * 64;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 256 threads: 4 rows per pass
    for (uint32_t r = ty; r < 64; r += 4) {
        const uint32_t p = p0 + r;
        const uint64_t w = w0 + tx;
        if (p < L && w < W) tile[r][tx] = in[(uint64_t)p * W + w];
    }
    __syncthreads();
    for (uint32_t r = ty; r < 64; r += 4) {
        const uint64_t w = w0 + r;
        const uint32_t p = p0 + tx;
        if (p < L && w < W) out[w * L + p] = tile[tx][r];
    }
}

// rows out[i][p] = walks[p][li(i)], li(i) = list ? list[i] : base + i
__global__ void k_gather_rows(const uint32_t* __restrict__ walks, uint64_t W, uint32_t L, const uint64_t* __restrict__ list,
                              uint64_t base, uint64_t count, uint32_t* __restrict__ out)
{
    const uint64_t total = count * L;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = t / count, i = t - p * count;   // consecutive threads: consecutive walks of one position
        const uint64_t li = list ? list[i] : base + i;
        out[i * L + p] = walks[p * W + li];
    }
}

void launch_gather_rows(const uint32_t* walks, uint64_t W, uint32_t L, const uint64_t* list, uint64_t base,
                        uint64_t count, uint32_t* out, hipStream_t s)
{
    if (count) hipLaunchKernelGGL(k_gather_rows, grid_for(count * L, 256), 256, 0, s, walks, W, L, list, base, count, out);
}

// entries: sort key = (vertex << kb) | (wid*L + pos), value = next
// Index entries of the vertices in the window [v0, v1): sort key
// (v - v0) << kb | (wid * L + p) (64-bit: n * wpv * L may exceed 2^32),
// value = the next vertex.  The whole index is the window [0, n).
__global__ void k_index_entries(const uint32_t* __restrict__ walks, uint64_t W, uint32_t L, ShardMap sm, int kb,
                                uint32_t v0, uint32_t v1, const uint64_t* __restrict__ col_base,
                                uint64_t* __restrict__ skeys, uint32_t* __restrict__ vals)
{
    for (uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; li < W; li += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t wid = sm.wid(li);
        uint64_t at = col_base[li];
        for (uint32_t p = 0; p < L; p++) {
            const uint32_t v = walks[(uint64_t)p * W + li];
            if (v == kSent) break;
            if (v < v0 || v >= v1) continue;
            const uint32_t nx = p + 1 < L ? walks[(uint64_t)(p + 1) * W + li] : kSent;
            skeys[at] = ((uint64_t)(v - v0) << kb) | (wid * L + p);
            vals[at] = nx;
            at++;
        }
    }
}

// per walk: its positions holding a vertex of [v0, v1)
__global__ void k_walk_lengths(const uint32_t* __restrict__ walks, uint64_t W, uint32_t L, uint32_t v0, uint32_t v1,
                               uint64_t* __restrict__ len)
{
    for (uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; li < W; li += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        for (uint32_t p = 0; p < L; p++) {
            const uint32_t v = walks[(uint64_t)p * W + li];
            if (v == kSent) break;
            c += v >= v0 && v < v1;
        }
        len[li] = c;
    }
}

__global__ void k_index_split(const uint64_t* __restrict__ skeys, uint64_t E, int kb, unsigned long long* __restrict__ counts,
                              uint64_t* __restrict__ keys)
{
    const uint64_t mask = kb >= 64 ? ~0ull : ((1ull << kb) - 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = skeys[i];
        keys[i] = k & mask;
        atomicAdd(counts + (k >> kb), 1ull);
    }
}

// Affected walk ids, ascending, as a two-pass stream compaction of aff[]
// (1 B per owned walk, kNoRewalk = unaffected): 16 walks per thread (one
// 16-B load), 4096 per block.  Pass 1 counts per block; an exclusive scan
// of the block counts; pass 2 writes each affected walk's id (wid, not the
// local column) at its rank.
constexpr uint32_t kAffPerThread = 16, kAffPerBlock = 256 * kAffPerThread;

__device__ __forceinline__ uint32_t aff_count16(const uint8_t* __restrict__ aff, uint64_t W, uint64_t base)
{
    uint32_t c = 0;
    if (base + kAffPerThread <= W) {
        const uint4 q = *reinterpret_cast<const uint4*>(aff + base);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int b = 0; b < 4; b++) c += ((w[k] >> (8 * b)) & 0xFFu) != kNoRewalk;
    } else {
        for (uint64_t i = base; i < W; i++) c += aff[i] != kNoRewalk;
    }
    return c;
}

__global__ __launch_bounds__(256) void k_aff_count(const uint8_t* __restrict__ aff, uint64_t W, uint32_t* __restrict__ counts)
{
    const uint64_t base = (uint64_t)blockIdx.x * kAffPerBlock + (uint64_t)threadIdx.x * kAffPerThread;
    uint32_t c = base < W ? aff_count16(aff, W, base) : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ uint32_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void k_aff_write(const uint8_t* __restrict__ aff, uint64_t W, const uint32_t* __restrict__ offs,
                                                   ShardMap sm, uint32_t* __restrict__ out)
{
    const uint64_t base = (uint64_t)blockIdx.x * kAffPerBlock + (uint64_t)threadIdx.x * kAffPerThread;
    const uint32_t c = base < W ? aff_count16(aff, W, base) : 0;
    // block-exclusive prefix of the per-thread counts
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    __shared__ uint32_t part[4];
    if (lane == 63) part[wv] = x;
    __syncthreads();
    uint32_t pre = x - c;
    for (uint32_t k = 0; k < wv; k++) pre += part[k];
    uint64_t at = (uint64_t)offs[blockIdx.x] + pre;
    if (!c) return;
    const uint64_t end = base + kAffPerThread < W ? base + kAffPerThread : W;
    for (uint64_t l = base; l < end; l++) {
        if (aff[l] == kNoRewalk) continue;
        out[at++] = (uint32_t)sm.wid(l);
    }
}

unsigned aff_blocks(uint64_t W) { return (unsigned)((W + kAffPerBlock - 1) / kAffPerBlock); }
void launch_aff_count(const uint8_t* aff, uint64_t W, uint32_t* counts, hipStream_t s)
{ if (W) hipLaunchKernelGGL(k_aff_count, aff_blocks(W), 256, 0, s, aff, W, counts); }
void launch_aff_write(const uint8_t* aff, uint64_t W, const uint32_t* offs, const ShardMap& sm, uint32_t* out,
                      hipStream_t s)
{ if (W) hipLaunchKernelGGL(k_aff_write, aff_blocks(W), 256, 0, s, aff, W, offs, sm, out); }

__global__ void k_fill_u64(uint64_t* __restrict__ p, uint64_t cnt, uint64_t v)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_fill_u32(uint32_t* __restrict__ p, uint64_t cnt, uint32_t v)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// Szudzik pairing (walks/pairings.h:124-210); exact isqrt for 64-bit unpair
__device__ __forceinline__ uint64_t isqrt64(uint64_t z)
{
    uint64_t s = (uint64_t)sqrt((double)z);
    while (s * s > z) s--;
    while ((s + 1) * (s + 1) <= z && (s + 1) < 0x100000000ull) s++;
    return s;
}

__global__ void k_szudzik64(int op, uint64_t cnt, uint64_t* __restrict__ x, uint64_t* __restrict__ y, uint64_t* __restrict__ z)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x) {
        if (op == 0) {
            const uint64_t a = x[i], b = y[i];
            z[i] = b >= a ? b * (b + 1) + a : a * a + b;
        } else {
            const uint64_t v = z[i];
            const uint64_t s = isqrt64(v);
            const uint64_t t = v - s * s;
            if (t < s) { x[i] = s; y[i] = t; } else { x[i] = t - s; y[i] = s; }
        }
    }
}

// CompressedWalks entries (walks/compressed_walks.h:49-66): Szudzik(wid*L+pos, next)
__global__ void k_index_pair(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ nexts, uint64_t E,
                             uint64_t* __restrict__ out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = keys[i], b = nexts[i];
        out[i] = b >= a ? b * (b + 1) + a : a * a + b;
    }
}

// offsets of vertices [v0, v0 + cnt] relative to off[v0] (segmented-sort chunk)
__global__ void k_rel_offsets(const uint64_t* __restrict__ off, uint64_t v0, uint64_t cnt, uint32_t* __restrict__ rel)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cnt; i += (uint64_t)gridDim.x * blockDim.x)
        rel[i] = (uint32_t)(off[v0 + i] - off[v0]);
}

void launch_index_pair(const uint64_t* keys, const uint32_t* nexts, uint64_t E, uint64_t* out, hipStream_t s)
{ if (E) hipLaunchKernelGGL(k_index_pair, grid_for(E, 256), 256, 0, s, keys, nexts, E, out); }
void launch_rel_offsets(const uint64_t* off, uint64_t v0, uint64_t cnt, uint32_t* rel, hipStream_t s)
{ hipLaunchKernelGGL(k_rel_offsets, grid_for(cnt + 1, 256), 256, 0, s, off, v0, cnt, rel); }

unsigned grid_for(uint64_t work, unsigned block)
{
    const uint64_t g = (work + block - 1) / block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 256 * 64));
}

void launch_rmat_keys(const RmatParams& p, uint64_t M, int directed, uint64_t* keys, hipStream_t s)
{ hipLaunchKernelGGL(k_rmat_keys, grid_for(M, 256), 256, 0, s, p, M, directed, keys); }
void launch_pairs_to_keys(const uint32_t* pairs, uint64_t m, uint64_t n, uint64_t* keys, unsigned long long* err, hipStream_t s)
{ hipLaunchKernelGGL(k_pairs_to_keys, grid_for(m, 256), 256, 0, s, pairs, m, n, keys, err); }
void launch_csr_to_keys(const uint64_t* off, uint64_t n, const uint32_t* tgt, uint64_t* keys, unsigned long long* err, hipStream_t s)
{ if (n) hipLaunchKernelGGL(k_csr_to_keys, (unsigned)((n + 63) / 64), 256, 0, s, off, n, tgt, keys, err); }
void launch_unique_flags(const uint64_t* keys, uint64_t m, int drop_loops, uint8_t* keep, hipStream_t s)
{ hipLaunchKernelGGL(k_unique_flags, grid_for(m, 256), 256, 0, s, keys, m, drop_loops, keep); }
void launch_offsets_from_keys(const uint64_t* keys, uint64_t m, uint64_t n, uint64_t* off, hipStream_t s)
{ hipLaunchKernelGGL(k_offsets_from_keys, grid_for(n + 1, 256), 256, 0, s, keys, m, n, off); }
void launch_low32(const uint64_t* keys, uint64_t m, uint32_t* out, hipStream_t s)
{ hipLaunchKernelGGL(k_low32, grid_for(m, 256), 256, 0, s, keys, m, out); }
void launch_batch_change(const uint64_t* bkeys, uint64_t mb, const uint64_t* off, const uint32_t* deg, const uint32_t* adj,
                         int insert, uint32_t* chg, hipStream_t s)
{ hipLaunchKernelGGL(k_batch_change, grid_for(mb, 256), 256, 0, s, bkeys, mb, off, deg, adj, insert, chg); }
void launch_run_flags(const uint64_t* bkeys, uint64_t mb, uint8_t* f, hipStream_t s)
{ hipLaunchKernelGGL(k_run_flags, grid_for(mb, 256), 256, 0, s, bkeys, mb, f); }
void launch_run_info(const uint64_t* bkeys, const uint32_t* run_start, uint64_t k, uint64_t mb, const uint64_t* off,
                     const uint32_t* deg, RunInfo* runs, uint32_t* bitmap, uint32_t* bloom, hipStream_t s)
{ hipLaunchKernelGGL(k_run_info, grid_for(k, 256), 256, 0, s, bkeys, run_start, k, mb, off, deg, runs, bitmap, bloom); }

void launch_mark_sources(const uint32_t* src, uint64_t k, RunInfo* runs, uint32_t* bitmap, uint32_t* bloom, hipStream_t s)
{
    if (k) hipLaunchKernelGGL(k_mark_sources, grid_for(k, 256), 256, 0, s, src, k, runs, bitmap, bloom);
}
void launch_row_degrees(const uint64_t* coff, uint64_t n, uint32_t* deg, uint32_t* cap, uint64_t* capw, int slack,
                        hipStream_t s)
{ hipLaunchKernelGGL(k_row_degrees, grid_for(n + 1, 256), 256, 0, s, coff, n, deg, cap, capw, slack); }
void launch_row_recap(const uint32_t* deg, uint64_t n, uint32_t* cap, uint64_t* capw, int slack, hipStream_t s)
{ hipLaunchKernelGGL(k_row_recap, grid_for(n + 1, 256), 256, 0, s, deg, n, cap, capw, slack); }
void launch_deg_u64(const uint32_t* deg, uint64_t n, uint64_t* out, hipStream_t s)
{ hipLaunchKernelGGL(k_deg_u64, grid_for(n + 1, 256), 256, 0, s, deg, n, out); }
void launch_copy_rows(const uint64_t* soff, const uint32_t* deg, const uint32_t* src, const uint64_t* doff, uint64_t n,
                      uint32_t* dst, const uint64_t* sanc, uint64_t* danc, hipStream_t s)
{ if (n) hipLaunchKernelGGL(k_copy_rows, (unsigned)((n + 63) / 64), 256, 0, s, soff, deg, src, doff, n, dst, sanc, danc); }
void launch_plan_rows(const RunInfo* runs, uint64_t k, const uint32_t* cap, const uint32_t* cf, int insert, int slack,
                      uint64_t* need, uint64_t* save, RowPlan* plan, unsigned long long* dead, hipStream_t s)
{ hipLaunchKernelGGL(k_plan_rows, grid_for(k + 1, 256), 256, 0, s, runs, k, cap, cf, insert, slack, need, save, plan, dead); }

// In-place pool compaction (the repack that needs no second pool): rows keep
// their capacities and are packed in slot order, so every row's new start is at
// or below its old one and the dead slots of moved rows disappear.  The pool is
// rewritten window by window in ascending order: the slots bound for window
// [D, D + C) all come from at or above D, which no earlier window has written,
// so they are first gathered into a staging buffer, then written.
// order[i] = the row with the i-th smallest start; noff its new start.
__global__ void k_slot_order_keys(const uint64_t* __restrict__ off, const uint32_t* __restrict__ cap, uint64_t n,
                                  uint64_t* __restrict__ keys, uint32_t* __restrict__ vals)
{
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        keys[v] = off[v];
        vals[v] = (uint32_t)v;
    }
}

__global__ void k_ordered_caps(const uint32_t* __restrict__ order, const uint32_t* __restrict__ cap, uint64_t n,
                               uint64_t* __restrict__ capw)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x)
        capw[i] = i < n ? cap[order[i]] : 0;
}

// one wave per row of the window's row range [r0, r1) (rows in slot order)
__global__ void k_compact_gather(const uint32_t* __restrict__ order, const uint64_t* __restrict__ snoff, uint64_t r0,
                                 uint64_t r1, const uint64_t* __restrict__ off, const uint32_t* __restrict__ deg,
                                 const uint32_t* __restrict__ adj, const uint64_t* __restrict__ anc, uint64_t D,
                                 uint64_t C, uint32_t* __restrict__ sadj, uint64_t* __restrict__ sanc)
{
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t i = r0 + (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); i < r1; i += waves) {
        const uint32_t v = order[i];
        const uint64_t no = snoff[i], o = off[v], d = deg[v];
        const uint64_t j0 = D > no ? D - no : 0, j1 = min(d, D + C > no ? D + C - no : 0);
        for (uint64_t j = j0 + (threadIdx.x & 63); j < j1; j += 64) {
            sadj[no + j - D] = adj[o + j];
            if (anc) sanc[no + j - D] = anc[(o + j) * kAnchorStride];
        }
    }
}

__global__ void k_compact_put(const uint32_t* __restrict__ sadj, const uint64_t* __restrict__ sanc, uint64_t cnt,
                              uint64_t D, uint32_t* __restrict__ adj, uint64_t* __restrict__ anc)
{
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += (uint64_t)gridDim.x * blockDim.x) {
        adj[D + t] = sadj[t];
        if (anc) anc[(D + t) * kAnchorStride] = sanc[t];
    }
}

__global__ void k_scatter_offsets(const uint32_t* __restrict__ order, const uint64_t* __restrict__ snoff, uint64_t n,
                                  uint64_t* __restrict__ off)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x)
        off[i < n ? order[i] : n] = snoff[i];
}

void launch_slot_order_keys(const uint64_t* off, const uint32_t* cap, uint64_t n, uint64_t* keys, uint32_t* vals,
                            hipStream_t s)
{ if (n) hipLaunchKernelGGL(k_slot_order_keys, grid_for(n, 256), 256, 0, s, off, cap, n, keys, vals); }
void launch_ordered_caps(const uint32_t* order, const uint32_t* cap, uint64_t n, uint64_t* capw, hipStream_t s)
{ hipLaunchKernelGGL(k_ordered_caps, grid_for(n + 1, 256), 256, 0, s, order, cap, n, capw); }
void launch_compact_gather(const uint32_t* order, const uint64_t* snoff, uint64_t r0, uint64_t r1, const uint64_t* off,
                           const uint32_t* deg, const uint32_t* adj, const uint64_t* anc, uint64_t D, uint64_t C,
                           uint32_t* sadj, uint64_t* sanc, hipStream_t s)
{
    if (r1 > r0)
        hipLaunchKernelGGL(k_compact_gather, grid_for((r1 - r0) * 64, 256), 256, 0, s, order, snoff, r0, r1, off, deg,
                           adj, anc, D, C, sadj, sanc);
}
void launch_compact_put(const uint32_t* sadj, const uint64_t* sanc, uint64_t cnt, uint64_t D, uint32_t* adj,
                        uint64_t* anc, hipStream_t s)
{ if (cnt) hipLaunchKernelGGL(k_compact_put, grid_for(cnt, 256), 256, 0, s, sadj, sanc, cnt, D, adj, anc); }
void launch_scatter_offsets(const uint32_t* order, const uint64_t* snoff, uint64_t n, uint64_t* off, hipStream_t s)
{ hipLaunchKernelGGL(k_scatter_offsets, grid_for(n + 1, 256), 256, 0, s, order, snoff, n, off); }
void launch_run_chunks(const RunInfo* runs, const RowPlan* plan, uint64_t k, uint32_t* cnt, hipStream_t s)
{
    hipLaunchKernelGGL(k_run_chunks, grid_for(k + 1, 256), 256, 0, s, runs, plan, k, cnt);
}
void launch_save_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint32_t* adj, const uint64_t* sofs,
                      uint32_t* scratch, const uint64_t* anc, uint64_t* sanc, const uint32_t* rev, uint32_t* srev,
                      hipStream_t s)
{
    if (!k) return;
    if (WHARF_ROW_CHUNKED && pre)
        hipLaunchKernelGGL(k_save_rows_c, chunk_grid(), 256, 0, s, runs, pre, k, adj, sofs, scratch, anc, sanc, rev, srev);
    else
        hipLaunchKernelGGL(k_save_rows, (unsigned)k, 256, 0, s, runs, adj, sofs, scratch, anc, sanc, rev, srev);
}
void launch_merge_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* bkeys, const uint32_t* chg,
                       const uint32_t* cf, const uint32_t* scratch, const uint64_t* sofs, const uint64_t* relofs,
                       uint64_t pool_end, int insert, RowPlan* plan, uint32_t* adj, const uint64_t* sanc, uint64_t* anc,
                       const uint32_t* srev, uint32_t* rev, hipStream_t s)
{
    if (!k) return;
    if (WHARF_ROW_CHUNKED && pre) {
        hipLaunchKernelGGL(k_merge_rows_c, chunk_grid(), 256, 0, s, runs, pre, k, bkeys, chg, cf, scratch, sofs, relofs,
                           pool_end, insert, plan, adj, sanc, anc, srev, rev);
        hipLaunchKernelGGL(k_resolve_plan, grid_for(k, 256), 256, 0, s, runs, k, relofs, pool_end, plan);
    } else {
        hipLaunchKernelGGL(k_merge_rows, (unsigned)k, 256, 0, s, runs, bkeys, chg, cf, scratch, sofs, relofs,
                           pool_end, insert, plan, adj, sanc, anc, srev, rev);
    }
}
void launch_anchor_invalidate(const uint64_t* bkeys, uint64_t mb, const uint32_t* chg, const uint64_t* off,
                              const uint32_t* deg, const uint32_t* adj, uint64_t* anc, const uint64_t* fdir,
                              const uint32_t* fpool, hipStream_t s)
{
    if (mb) hipLaunchKernelGGL(k_anchor_invalidate, (unsigned)std::min<uint64_t>((mb + 3) / 4, (uint64_t)cu_count() * 8),
                               256, 0, s, bkeys, mb, chg, off, deg, adj, anc, fdir, fpool);
}
void launch_keys_symmetric(const uint64_t* keys, uint64_t m, unsigned long long* asym, hipStream_t s)
{ if (m) hipLaunchKernelGGL(k_keys_symmetric, grid_for(m, 256), 256, 0, s, keys, m, asym); }
void launch_commit_rows(const RunInfo* runs, uint64_t k, const RowPlan* plan, uint32_t epoch, uint64_t* off,
                        uint32_t* deg, uint32_t* cap, ERec* vrec, uint32_t* row_epoch, hipStream_t s)
{ if (k) hipLaunchKernelGGL(k_commit_rows, grid_for(k, 256), 256, 0, s, runs, k, plan, epoch, off, deg, cap, vrec, row_epoch); }
void launch_erec_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* off, const uint32_t* deg,
                      const uint32_t* adj, const ERec* vrec, ERec* erec, uint32_t rs, int keep_anc, RecFmt rf,
                      hipStream_t s)
{
    if (!k) return;
    if (WHARF_ROW_CHUNKED && pre)
        hipLaunchKernelGGL(k_erec_rows_c, chunk_grid(), 256, 0, s, runs, pre, k, off, deg, adj, vrec, erec, rs, keep_anc,
                           rf);
    else
        hipLaunchKernelGGL(k_erec_rows, (unsigned)k, 256, 0, s, runs, off, deg, adj, vrec, erec, rs, keep_anc, rf);
}
void launch_filter_rows(const RunInfo* runs, uint64_t k, const uint32_t* pre, const uint64_t* noff, const uint32_t* deg,
                        const uint32_t* adj, const uint64_t* need, const uint64_t* gofs, uint64_t base, uint64_t* fdir,
                        uint32_t* pool, hipStream_t s)
{
    if (!k) return;
    if (WHARF_ROW_CHUNKED && pre) {   // descriptors, then every row's words cleared, then filled
        hipLaunchKernelGGL(k_filter_desc, grid_for(k, 256), 256, 0, s, runs, k, deg, need, gofs, base, fdir);
        hipLaunchKernelGGL(k_filter_clear_c, chunk_grid(), 256, 0, s, runs, pre, k, fdir, pool);
        hipLaunchKernelGGL(k_filter_fill_c, chunk_grid(), 256, 0, s, runs, pre, k, noff, deg, adj, fdir, pool);
    } else {
        hipLaunchKernelGGL(k_filter_rows, (unsigned)k, 256, 0, s, runs, noff, deg, adj, need, gofs, base, fdir, pool);
    }
}
void launch_patch_in_edges(const uint32_t* adj, uint64_t slots, const uint32_t* bitmap, const uint32_t* bloom,
                           const ERec* vrec, ERec* erec, uint32_t rs, RecFmt rf, hipStream_t s)
{
    if (!slots) return;
    const unsigned grid = (unsigned)std::min<uint64_t>((slots / 4 + 1023) / 1024 + 1, (uint64_t)cu_count() * 2);
    hipLaunchKernelGGL(k_patch_in_edges, grid, 1024, 0, s, adj, slots, bitmap, bloom + kBloomWords, vrec, erec, rs, rf);
}
void launch_transpose(const uint32_t* in, uint64_t W, uint32_t L, uint32_t* out, hipStream_t s)
{
    if (!W) return;
    const dim3 g((unsigned)((W + 63) / 64), (L + 63) / 64);
    hipLaunchKernelGGL(k_transpose, g, 256, 0, s, in, W, L, out);
}
void launch_walk_lengths(const uint32_t* walks, uint64_t W, uint32_t L, uint32_t v0, uint32_t v1, uint64_t* len,
                         hipStream_t s)
{ hipLaunchKernelGGL(k_walk_lengths, grid_for(W, 256), 256, 0, s, walks, W, L, v0, v1, len); }
void launch_index_entries(const uint32_t* walks, uint64_t W, uint32_t L, const ShardMap& sm, int kb,
                          uint32_t v0, uint32_t v1, const uint64_t* col_base, uint64_t* skeys, uint32_t* vals,
                          hipStream_t s)
{ hipLaunchKernelGGL(k_index_entries, grid_for(W, 256), 256, 0, s, walks, W, L, sm, kb, v0, v1, col_base, skeys, vals); }
void launch_index_split(const uint64_t* skeys, uint64_t E, int kb, unsigned long long* counts, uint64_t* keys, hipStream_t s)
{ hipLaunchKernelGGL(k_index_split, grid_for(E, 256), 256, 0, s, skeys, E, kb, counts, keys); }
void launch_fill_u64(uint64_t* p, uint64_t cnt, uint64_t v, hipStream_t s)
{ if (cnt) hipLaunchKernelGGL(k_fill_u64, grid_for(cnt, 256), 256, 0, s, p, cnt, v); }
void launch_fill_u32(uint32_t* p, uint64_t cnt, uint32_t v, hipStream_t s)
{ if (cnt) hipLaunchKernelGGL(k_fill_u32, grid_for(cnt, 256), 256, 0, s, p, cnt, v); }
void launch_szudzik64(int op, uint64_t cnt, uint64_t* x, uint64_t* y, uint64_t* z, hipStream_t s)
{ if (cnt) hipLaunchKernelGGL(k_szudzik64, grid_for(cnt, 256), 256, 0, s, op, cnt, x, y, z); }

}  // namespace wharf
