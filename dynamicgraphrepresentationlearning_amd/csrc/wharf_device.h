// Device-side building blocks of the WharfMH walk engine (gfx950 / CDNA4).
//
//   - xoroshiro128+ with the reference's arithmetic-shift seeding
//     (utils/utility.h:152-223) — host side, used to fill the per-round draw
//     table of deterministic mode;
//   - Philox4x32-10 counter-based RNG for MH mode (one independent stream per
//     (walk, position, epoch), no shared state: replaces the racy global
//     config::random of metropolis_hastings_sampler.h:121 / deepwalk.h:82);
//   - the reference's RMAT edge recursion (rmat_util.h:250-271) and pbbs hashes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wharf {

constexpr uint32_t kSent = 0xFFFFFFFEu;        // wharfmh.h:282 (uint32 max - 1)
constexpr uint32_t kAnchorNone = 0xFFFFFFFFu;  // MH anchor slot not initialised yet
constexpr uint32_t kNoRewalk = 0xFFu;          // rewalk position "none"
constexpr uint32_t kNoSource = 0xFFFFFFFFu;    // src_idx of a vertex that is not a batch source
constexpr uint32_t kBloomWords = 4096;         // batch-source Bloom filter: 2^17 bits (16 KiB, LDS)
constexpr uint32_t kGap = 0xFFFFFFFFu;         // unused slot of the slack-row pool (not a vertex id)

// Slack-row CSR capacities: a row starts with 1/16 slack (at least 2 slots);
// a row that outgrew its slots moves to a place with 1/8 slack (at least 4).
__host__ __device__ __forceinline__ uint32_t row_cap_initial(uint32_t d)
{
    return d ? d + ((d >> 4) > 2u ? (d >> 4) : 2u) : 0u;
}
__host__ __device__ __forceinline__ uint32_t row_cap_grown(uint32_t d) { return d + ((d >> 3) > 4u ? (d >> 3) : 4u); }

// Blocked Bloom filter of the batch sources (kBloomWords 32-bit words, held
// in LDS by the scans): a key sets two bits of ONE word, so a test is one LDS
// read (~2-3 % false positives at 10 k sources).  The scans are VALU-bound, so
// the hash is one full-rate 24-bit multiply (v_mul_u32_u24; a 32-bit multiply
// is quarter rate) of the id with its high bits folded in; the word comes from
// the product's top bits, the two bit positions from bits 8-12 and 13-17.
__device__ __forceinline__ uint32_t bloom_mix(uint32_t x) { return __umul24(x ^ (x >> 15), 0x9E3779u); }
__device__ __forceinline__ uint32_t bloom_word(uint32_t h) { return h >> 20; }
#ifndef WHARF_BLOOM_K
#define WHARF_BLOOM_K 3   // bits per key, the third from bits 3-7 (2: scan 3.2-3.4 vs 3.2-3.3 ms, profiles/r02/chunked_scan)
#endif
__device__ __forceinline__ uint32_t bloom_bits(uint32_t h)
{
    uint32_t b = (1u << ((h >> 13) & 31u)) | (1u << ((h >> 8) & 31u));
    if (WHARF_BLOOM_K > 2) b |= 1u << ((h >> 3) & 31u);
    return b;
}
__device__ __forceinline__ bool bloom_test(const uint32_t* f, uint32_t x)
{
    const uint32_t h = bloom_mix(x), b = bloom_bits(h);
    return (f[bloom_word(h)] & b) == b;
}
static_assert(kBloomWords == 4096, "bloom_word yields 12 bits");
// The same scheme over 4x the words (64 KiB) for the in-edge scan, whose
// positives each cost a random bitmap read: ~0.2 % false positives
constexpr uint32_t kBigBloomWords = 16384;
__device__ __forceinline__ uint32_t bloom_word_big(uint32_t h) { return h >> 18; }
__device__ __forceinline__ bool bloom_test_big(const uint32_t* f, uint32_t x)
{
    const uint32_t h = bloom_mix(x), b = bloom_bits(h);
    return (f[bloom_word_big(h)] & b) == b;
}
// bitmap buffer: [exact bitmap][kBloomWords][kBigBloomWords]
constexpr uint32_t kFilterWords = kBloomWords + kBigBloomWords;

// Philox counter word 3 = (epoch << 4) | stream
enum : uint32_t { kStreamStep = 0, kStreamAnchor = 1, kStreamBurnin = 2, kStreamPrev = 3 };

// Row record: a vertex and its CSR row.  vrec[v] = {v, deg(v), off(v), epoch(v)};
// erec[e] = vrec[adj[e]], so a walk step reads its next vertex AND that
// vertex's row with one aligned 16-B load.  In memory the row offset (40 bits)
// and the epoch of the row's last sampler reset (24 bits) share one word.
struct alignas(16) ERec {
    uint32_t v, deg;
    uint64_t oe;
};
struct Row {          // unpacked, in registers
    uint32_t v, deg, epoch;
    uint64_t off;
};
constexpr uint64_t kOffBits = 40;
constexpr uint64_t kOffMask = (1ull << kOffBits) - 1;
constexpr uint32_t kEpochBits = 64 - kOffBits;   // row epoch: the record's top 24 bits
constexpr uint64_t kAnchorNone64 = ~0ull;
constexpr uint64_t kStabEmpty = ~0ull;         // re-walk start table: no key (its entries start as kAnchorNone64)
constexpr uint64_t kAnchorStride = 4;         // u64 words between anchor entries (32-B node2vec edge records)
constexpr uint64_t kEmptyKey = ~0ull;         // empty slot of the edge hash set
constexpr uint64_t kTombKey = ~0ull - 1;      // deleted edge (probing continues past it)
constexpr uint64_t kFiltOffBits = 48;         // neighbour-filter directory: word offset | log2(words) << 48
constexpr uint64_t kFiltOffMask = (1ull << kFiltOffBits) - 1;

// 32-bit words of a row's neighbour filter: the power of two >= deg / 4 (8-16 bits per neighbour)
__host__ __device__ __forceinline__ uint32_t filt_log2_words(uint64_t deg)
{
    const uint64_t w = (deg + 3) / 4;
    uint32_t lg = 0;
    while ((1ull << lg) < w) lg++;
    return lg;
}

// Which walks a handle owns.  Walk id wid = r * n + v (round r,
// start vertex v, wharfmh.h:275-292); the handle's local column li = r * n_loc + j,
// where the j-th owned start vertex is
//   contiguous shard [lo, hi):  v = lo + j                       (parts = 1)
//   block shard (part of parts): the part's blocks of 2^bits vertices, dealt
//     round-robin: v = ((j >> bits) * parts + part) << bits | (j & (2^bits - 1))
// Both are increasing in j, so ascending columns are ascending walk ids.
struct ShardMap {
    uint64_t n, n_loc, lo;
    uint32_t part, parts, bits;
    __host__ __device__ __forceinline__ uint64_t vertex(uint64_t j) const
    {
        return lo + ((((j >> bits) * parts + part) << bits) | (j & ((1ull << bits) - 1)));
    }
    __host__ __device__ __forceinline__ uint64_t wid(uint64_t li) const
    {
        const uint64_t r = li / n_loc;
        return r * n + vertex(li - r * n_loc);
    }
};

__host__ __device__ __forceinline__ ERec make_rec(uint32_t v, uint32_t deg, uint64_t off, uint32_t epoch)
{
    ERec r;
    r.v = v;
    r.deg = deg;
    r.oe = (off & kOffMask) | ((uint64_t)epoch << kOffBits);
    return r;
}

__device__ __forceinline__ Row load_rec(const ERec* p, uint64_t i)
{
    const uint4 q = *reinterpret_cast<const uint4*>(p + i);   // one global_load_dwordx4
    const uint64_t oe = ((uint64_t)q.w << 32) | q.z;
    Row r;
    r.v = q.x;
    r.deg = q.y;
    r.off = oe & kOffMask;
    r.epoch = (uint32_t)(oe >> kOffBits);
    return r;
}

// Compact 8-B edge records (round 6).  A DeepWalk or deterministic handle needs no
// row epoch in its edge records (only node2vec MH anchors read it), and when its
// vertex ids and pool offsets leave enough bits, a slot's record packs into one
// u64: v | off << vb | deg << (vb + ob).  A degree of 2^db - 1 or more (db = 64 -
// vb - ob) is stored as the escape 2^db - 1 and read from deg[v] (RMAT hubs: at
// configs[1], db = 14 and ~2 % of steps land on an escaped row).  Half the bytes
// per slot halve the table the walk's random gathers land in, and more of it stays
// in L2 and the Infinity Cache (tools/gather_roof: a 1.74-GiB table gathers ~10 %
// faster than 3.48 GiB).  compact = 0: the 16-B ERec layout.
struct RecFmt {
    uint32_t compact, vb, ob;
};
constexpr uint32_t kMinCompactDegBits = 12;

__host__ __device__ __forceinline__ uint64_t pack_rec8(const ERec& r, RecFmt f)
{
    const uint32_t db = 64 - f.vb - f.ob;
    const uint64_t dmax = (db >= 32 ? 0xFFFFFFFFull : ((1ull << db) - 1));
    const uint64_t d = r.deg < dmax ? r.deg : dmax;
    return (uint64_t)r.v | ((r.oe & kOffMask) << f.vb) | (d << (f.vb + f.ob));
}

__device__ __forceinline__ Row unpack_rec8(uint64_t q, RecFmt f, const uint32_t* __restrict__ deg)
{
    const uint32_t db = 64 - f.vb - f.ob;
    const uint64_t dmax = (db >= 32 ? 0xFFFFFFFFull : ((1ull << db) - 1));
    Row r;
    r.v = (uint32_t)(q & ((1ull << f.vb) - 1));
    r.off = (q >> f.vb) & ((1ull << f.ob) - 1);
    const uint64_t d = q >> (f.vb + f.ob);
#ifdef WHARF_PROBE_NO_ESCAPE   // timing probe only (hub degrees clipped: wrong walks)
    r.deg = (uint32_t)d;
#else
    r.deg = d == dmax ? deg[r.v] : (uint32_t)d;   // the escape: a hub's degree from its row
#endif
    r.epoch = 0;
    return r;
}

// slot e's record in either layout (rs: 16-B units per slot of the 16-B layout)
__device__ __forceinline__ Row load_erec(const ERec* __restrict__ erec, uint64_t e, uint32_t rs, RecFmt f,
                                         const uint32_t* __restrict__ deg)
{
    if (f.compact) return unpack_rec8(reinterpret_cast<const uint64_t*>(erec)[e], f, deg);
    return load_rec(erec, e * rs);
}

__device__ __forceinline__ void store_erec(ERec* __restrict__ erec, uint64_t e, uint32_t rs, const ERec& r, RecFmt f)
{
    if (f.compact) reinterpret_cast<uint64_t*>(erec)[e] = pack_rec8(r, f);
    else erec[e * rs] = r;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Random123); 10 rounds, key bumped between rounds.
// ---------------------------------------------------------------------------
struct P4 { uint32_t x0, x1, x2, x3; };

__device__ __forceinline__ P4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; r++) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    return P4{c0, c1, c2, c3};
}

// uniform index in [0, deg): multiply-high (Lemire, no rejection)
__device__ __forceinline__ uint64_t pick32(uint32_t r, uint32_t deg) { return __umulhi(r, deg); }
__device__ __forceinline__ uint64_t pick64(uint32_t r, uint64_t deg)
{
    // (r * deg) >> 32 for deg up to 2^64 with a 64x32 -> 96-bit product
    const uint64_t lo = (uint64_t)r * (uint32_t)deg;
    const uint64_t hi = (uint64_t)r * (uint32_t)(deg >> 32);
    return hi + (lo >> 32);
}

// drand-like uniform in [0,1) from 53 bits
__device__ __forceinline__ double u01(uint32_t hi, uint32_t lo)
{
    return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1.0p-53;
}

// x % d for a 64-bit x and 32-bit d (utility.h:220 irand: lrand() % max)
__device__ __forceinline__ uint32_t umod64_32(uint64_t x, uint32_t d) { return (uint32_t)(x % (uint64_t)d); }

// ---------------------------------------------------------------------------
// pbbs hashes (pbbslib/utilities.h:108-146) and the RMAT recursion
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t hash32(uint32_t a)
{
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

__host__ __device__ __forceinline__ uint64_t hash64(uint64_t u)
{
    uint64_t v = u * 3935559000370003845ull + 2691343689449507681ull;
    v ^= v >> 21;
    v ^= v << 37;
    v ^= v >> 4;
    v *= 4768777513237032717ull;
    v ^= v << 20;
    v ^= v >> 41;
    v ^= v << 5;
    return v;
}

struct RmatParams { double a, ab, abc; uint32_t n, h; };

// rMat<unsigned int>::operator() (rmat_util.h:255-271): level t of the
// recursion (quadrant size n >> (t+1)) reads hashDouble(randStart + t*randStride).
__device__ __forceinline__ void rmat_edge(const RmatParams& p, uint32_t i, uint32_t& src, uint32_t& dst)
{
    const uint32_t start = hash32((uint32_t)(2u * i) * p.h);
    const uint32_t stride = hash32((uint32_t)(2u * i + 1u) * p.h);
    uint32_t x = 0, y = 0, nn = p.n, t = 0;
    while (nn > 1) {
        const double d = (double)hash32(start + t * stride) / 4294967295.0;
        const uint32_t half = nn >> 1;
        if (d < p.a) {
        } else if (d < p.ab) {
            y += half;
        } else if (d < p.abc) {
            x += half;
        } else {
            x += half;
            y += half;
        }
        nn = half;
        t++;
    }
    src = x;
    dst = y;
}

// ---------------------------------------------------------------------------
// host: utility::Random (utils/utility.h:157-206).  The seed word is a signed
// long long, so the splitmix shifts are arithmetic.
// ---------------------------------------------------------------------------
struct XoroHost {
    uint64_t s0, s1;
    explicit XoroHost(uint64_t seed)
    {
        for (int i = 0; i < 2; i++) {
            seed += 0x9E3779B97F4A7C15ull;
            int64_t z = (int64_t)seed;
            z = (int64_t)((uint64_t)(z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull);
            z = (int64_t)((uint64_t)(z ^ (z >> 27)) * 0x94D049BB133111EBull);
            (i == 0 ? s0 : s1) = (uint64_t)(z ^ (z >> 31));
        }
    }
    uint64_t lrand()
    {
        const uint64_t a = s0;
        uint64_t b = s1;
        const uint64_t r = a + b;
        b ^= a;
        s0 = ((a << 55) | (a >> 9)) ^ b ^ (b << 14);
        s1 = (b << 36) | (b >> 28);
        return r;
    }
};

}  // namespace wharf
