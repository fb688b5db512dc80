/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the WharfMH walk path.
 * See wharf_oracle.h for what it is allowed to be used for.
 *
 * Every function names the reference lines it restates
 * (paths relative to the reference root, djordjijeK/DynamicGraphRepresentationLearning).
 */
#define _GNU_SOURCE
#include "wharf_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* RNG: utils/utility.h:152-223                                              */
/* ------------------------------------------------------------------------ */

/* utility.h:157-171: the state word is a *signed* long long, so every >> in
 * the mixing is an arithmetic shift. */
void wo_random_init(uint64_t seed, uint64_t state[2])
{
    for (int i = 0; i < 2; i++) {
        seed += UINT64_C(0x9E3779B97F4A7C15);
        int64_t z = (int64_t)seed;
        z = (int64_t)((uint64_t)(z ^ (z >> 30)) * UINT64_C(0xBF58476D1CE4E5B9));
        z = (int64_t)((uint64_t)(z ^ (z >> 27)) * UINT64_C(0x94D049BB133111EB));
        state[i] = (uint64_t)(z ^ (z >> 31));
    }
}

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* utility.h:194-206 (xoroshiro128+) */
uint64_t wo_lrand(uint64_t s[2])
{
    const uint64_t s0 = s[0];
    uint64_t s1 = s[1];
    const uint64_t result = s0 + s1;
    s1 ^= s0;
    s[0] = rotl64(s0, 55) ^ s1 ^ (s1 << 14);
    s[1] = rotl64(s1, 36);
    return result;
}

/* utility.h:208-218 */
double wo_drand(uint64_t s[2])
{
    union { uint64_t i; double d; } a;
    a.i = (UINT64_C(0x3FF) << 52) | (wo_lrand(s) >> 12);
    return a.d - 1.0;
}

/* ------------------------------------------------------------------------ */
/* hashes: libs/compressed_trees/pbbslib/utilities.h:108-146,286-291         */
/* ------------------------------------------------------------------------ */
uint32_t wo_hash32(uint32_t a)
{
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

uint64_t wo_hash64(uint64_t u)
{
    uint64_t v = u * UINT64_C(3935559000370003845) + UINT64_C(2691343689449507681);
    v ^= v >> 21;
    v ^= v << 37;
    v ^= v >> 4;
    v *= UINT64_C(4768777513237032717);
    v ^= v << 20;
    v ^= v >> 41;
    v ^= v << 5;
    return v;
}

uint32_t wo_log2_up(uint64_t i)
{
    uint32_t a = 0;
    uint64_t b = i - 1;
    while (b > 0) { b >>= 1; a++; }
    return a;
}

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Random123).                                                */
/* ------------------------------------------------------------------------ */
void wo_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* ------------------------------------------------------------------------ */
/* RMAT batches: utils/utility.h:55-146, libs/compressed_trees/rmat_util.h    */
/* ------------------------------------------------------------------------ */
typedef struct { double a, ab, abc; uint32_t n, h; } rmat_t;

/* rmat_util.h:250-253: hash32(i) / (double) UINT32_MAX (intT = unsigned int) */
static inline double rmat_hash_double(uint32_t i) { return (double)wo_hash32(i) / 4294967295.0; }

/* rmat_util.h:255-265, recursion unrolled: level t (nn = n >> t) draws
 * hashDouble(randStart + t*randStride); deeper levels decide low bits. */
static void rmat_edge(const rmat_t* r, uint32_t i, uint32_t* src, uint32_t* dst)
{
    uint32_t randStart = wo_hash32((uint32_t)(2u * i) * r->h);
    uint32_t randStride = wo_hash32((uint32_t)(2u * i + 1u) * r->h);
    uint32_t x = 0, y = 0, nn = r->n, t = 0;
    while (nn > 1) {
        double d = rmat_hash_double(randStart + t * randStride);
        uint32_t half = nn / 2;
        if (d < r->a) { }
        else if (d < r->ab) { y += half; }
        else if (d < r->abc) { x += half; }
        else { x += half; y += half; }
        nn >>= 1;
        t++;
    }
    *src = x;
    *dst = y;
}

static int cmp_pair(const void* pa, const void* pb)
{
    const uint32_t* a = (const uint32_t*)pa;
    const uint32_t* b = (const uint32_t*)pb;
    if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
    if (a[1] != b[1]) return a[1] < b[1] ? -1 : 1;
    return 0;
}

uint64_t wo_generate_batch_of_edges(uint64_t edges_number, uint64_t vertices_number, uint64_t batch_seed,
                                    int self_loops, int directed, double a, double b, double c,
                                    uint32_t* out)
{
    /* utility.h:76-80: rand = pbbs::random(batch_seed); seed = (u32) rand.ith_rand(0) */
    uint64_t pow2 = (uint64_t)1 << (wo_log2_up(vertices_number) - 1);
    rmat_t r;
    r.n = (uint32_t)pow2;
    r.a = a; r.ab = a + b; r.abc = a + b + c;
    r.h = wo_hash32((uint32_t)wo_hash64(0 + batch_seed));
    uint64_t total = directed ? edges_number : 2 * edges_number;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)edges_number; i++) {
        uint32_t s, d;
        rmat_edge(&r, (uint32_t)i, &s, &d);
        out[2 * i] = s; out[2 * i + 1] = d;
        if (!directed) { out[2 * (i + edges_number)] = d; out[2 * (i + edges_number) + 1] = s; }
    }
    /* utility.h:99-116: sort by (src, dst); 118-130: drop self loops & dups */
    qsort(out, total, 8, cmp_pair);
    uint64_t k = 0;
    for (uint64_t i = 0; i < total; i++) {
        if (!self_loops && out[2 * i] == out[2 * i + 1]) continue;
        if (i > 0 && out[2 * i] == out[2 * i - 2] && out[2 * i + 1] == out[2 * i - 1]) continue;
        out[2 * k] = out[2 * i]; out[2 * k + 1] = out[2 * i + 1];
        k++;
    }
    return k;
}

/* ------------------------------------------------------------------------ */
/* Szudzik: walks/pairings.h:124-225                                         */
/* ------------------------------------------------------------------------ */
uint32_t wo_szudzik32_pair(uint32_t x, uint32_t y) { return y >= x ? y * (y + 1) + x : x * x + y; }

void wo_szudzik32_unpair(uint32_t z, uint32_t* x, uint32_t* y)
{
    uint32_t s = (uint32_t)floor(sqrt((double)z));
    if (s * s > z) s--;
    uint32_t t = z - s * s;
    if (t < s) { *x = s; *y = t; } else { *x = t - s; *y = s; }
}

uint64_t wo_szudzik64_pair(uint64_t x, uint64_t y) { return y >= x ? y * (y + 1) + x : x * x + y; }

void wo_szudzik64_unpair(uint64_t z, uint64_t* x, uint64_t* y)
{
    uint64_t s = (uint64_t)floor(sqrt((double)z));
    if (s * s > z) s--;
    uint64_t t = z - s * s;
    if (t < s) { *x = s; *y = t; } else { *x = t - s; *y = s; }
}

/* ------------------------------------------------------------------------ */
/* Engine                                                                     */
/* ------------------------------------------------------------------------ */
#define ANCHOR_NONE UINT64_C(0xFFFFFFFFFFFFFFFF)

struct wo_engine {
    uint64_t n, m;
    uint64_t* off;        /* n+1 */
    uint32_t* adj;        /* m   */
    uint64_t* anchor;     /* m   : per edge slot (prev -> cur): frozen anchor slot | epoch tag << 32 */
    uint32_t* row_epoch;  /* n   : epoch of last sampler reset of the row */
    uint32_t wpv, L;
    int model, init, det;
    float p, q;
    uint64_t seed;
    uint32_t epoch;
    uint32_t* walks;      /* [W][L] */
    uint64_t accepts, steps;
};

static inline uint64_t deg_of(const wo_engine* e, uint32_t v) { return e->off[v + 1] - e->off[v]; }

/* std::binary_search over the ascending row (node2vec.h:112-119) */
static inline int64_t row_find(const wo_engine* e, uint32_t v, uint32_t x)
{
    uint64_t lo = e->off[v], hi = e->off[v + 1];
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (e->adj[mid] < x) lo = mid + 1; else hi = mid;
    }
    return (lo < e->off[v + 1] && e->adj[lo] == x) ? (int64_t)lo : -1;
}

/* node2vec.h:74-88 / deepwalk.h:67-70 */
static inline float weight(const wo_engine* e, uint32_t prev, uint32_t c)
{
    if (e->model == WO_DEEPWALK) return 1.0f;
    if (c == prev) return 1.0f / e->p;
    if (row_find(e, prev, c) >= 0) return 1.0f;
    return 1.0f / e->q;
}

static inline void philox_draw(const wo_engine* e, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4])
{
    uint32_t ctr[4] = {c0, c1, c2, c3};
    uint32_t key[2] = {(uint32_t)e->seed, (uint32_t)(e->seed >> 32)};
    wo_philox4x32_10(ctr, key, out);
}

static inline uint64_t pick(uint32_t r, uint64_t deg) { return (uint64_t)(((unsigned __int128)r * deg) >> 32); }
static inline double u01(uint32_t hi, uint32_t lo) { return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1.0p-53; }

enum { ST_STEP = 0, ST_ANCHOR = 1, ST_BURNIN = 2, ST_PREV = 3 };

/* metropolis_hastings_sampler.h:69-108, with the proposals drawn from the
 * counter-based stream of (cur, prev, row_epoch[cur]).  Returns a slot of
 * cur's row. */
static uint32_t anchor_init(const wo_engine* e, uint32_t cur, uint32_t prev)
{
    uint64_t d = deg_of(e, cur), o = e->off[cur];
    uint32_t ep = e->row_epoch[cur] << 4;
    uint32_t r[4];
    philox_draw(e, cur, prev, 0, ep | ST_ANCHOR, r);
    uint32_t last = (uint32_t)pick(r[0], d);
    if (e->init == WO_INIT_WEIGHT) {
        float best_w = weight(e, prev, e->adj[o + last]);
        for (uint32_t j = 1; j <= 20; j++) {
            philox_draw(e, cur, prev, j, ep | ST_ANCHOR, r);
            uint32_t cand = (uint32_t)pick(r[0], d);
            float w = weight(e, prev, e->adj[o + cand]);
            if (w > best_w) { best_w = w; last = cand; }
        }
    } else if (e->init == WO_INIT_BURNIN) {
        for (uint32_t i = 0; i < 100; i++) {
            philox_draw(e, cur, prev, i, ep | ST_BURNIN, r);
            uint32_t cand = (uint32_t)pick(r[0], d);
            float wn = weight(e, prev, e->adj[o + cand]), wl = weight(e, prev, e->adj[o + last]);
            if (wl < wn || u01(r[1], r[2]) <= (double)wn / (double)wl) last = cand;
        }
    }
    return last;
}

/* SamplerManager::find returns a copy (libcuckoo find(), cuckoohash_map.hh:596-609),
 * so a state's anchor stays frozen.  Cached on the edge prev -> cur (`ein`,
 * its CSR slot, or -1) with the epoch it was computed in; the sampler lives in
 * cur's SamplerManager (wharfmh.h:296-301), so it stays valid while cur's row
 * was not reset since (samplers of batch sources are reset, wharfmh.h:504,539);
 * its weight is re-evaluated on the current graph at every sample(). */
static uint32_t anchor_get(wo_engine* e, uint32_t cur, uint32_t prev, int64_t ein)
{
    if (ein < 0) return anchor_init(e, cur, prev);
    uint64_t a = __atomic_load_n(&e->anchor[ein], __ATOMIC_RELAXED);
    uint32_t tag = (uint32_t)(a >> 32);
    if (a != ANCHOR_NONE && tag >= e->row_epoch[cur]) return (uint32_t)a;
    uint32_t s = anchor_init(e, cur, prev);
    __atomic_store_n(&e->anchor[ein], ((uint64_t)e->epoch << 32) | s, __ATOMIC_RELAXED);
    return s;
}

/* One walk from (v at position p) to the end of the walk.
 *   det:  wharfmh.h:288-325 / 813-856 — Random(wid / n), draw j at position p+j,
 *         next = adj(v)[lrand() % deg(v)] (utility.h:220).
 *   MH:   sample() (metropolis_hastings_sampler.h:31-46) against the frozen
 *         anchor of (cur, prev), draws from Philox(seed; wid, pos, epoch).
 * A vertex with no out-edges ends the walk (the reference divides by zero). */
static void walk_from(wo_engine* e, uint64_t wid, uint32_t v, uint32_t p, uint32_t prev,
                      uint64_t* acc, uint64_t* steps)
{
    uint32_t* w = e->walks + wid * e->L;
    uint64_t st[2];
    if (e->det) wo_random_init(wid / e->n, st);
    w[p] = v;
    uint32_t cur = v;
    uint32_t ep = e->epoch << 4;
    int64_t ein = (e->model == WO_NODE2VEC && !e->det && deg_of(e, v)) ? row_find(e, prev, cur) : -1;
    for (uint32_t pos = p; pos + 1 < e->L; pos++) {
        uint64_t d = deg_of(e, cur);
        if (d == 0) { for (uint32_t k = pos + 1; k < e->L; k++) w[k] = WO_SENT; return; }
        uint32_t nxt;
        if (e->det) {
            nxt = e->adj[e->off[cur] + wo_lrand(st) % d];
        } else {
            uint32_t r[4];
            philox_draw(e, (uint32_t)wid, (uint32_t)(wid >> 32), pos, ep | ST_STEP, r);
            uint32_t ci = (uint32_t)pick(r[0], d);
            uint32_t c = e->adj[e->off[cur] + ci];
            if (e->model == WO_DEEPWALK) {
                nxt = c;
                (*acc)++;
            } else {
                uint32_t ai = anchor_get(e, cur, prev, ein);
                uint32_t a = e->adj[e->off[cur] + ai];
                float wc = weight(e, prev, c), wa = weight(e, prev, a);
                int ok = (wa < wc) || (u01(r[1], r[2]) <= (double)wc / (double)wa);
                nxt = ok ? c : a;
                *acc += ok;
                ein = (int64_t)(e->off[cur] + (ok ? ci : ai));
            }
        }
        (*steps)++;
        w[pos + 1] = nxt;
        prev = cur;
        cur = nxt;
    }
}

static uint32_t initial_prev(const wo_engine* e, uint64_t wid, uint32_t v)
{
    /* node2vec.h:42-50: prev = random neighbour of the start vertex */
    if (e->model != WO_NODE2VEC || e->det || deg_of(e, v) == 0) return v;
    uint32_t r[4];
    philox_draw(e, (uint32_t)wid, (uint32_t)(wid >> 32), 0, (e->epoch << 4) | ST_PREV, r);
    return e->adj[e->off[v] + pick(r[0], deg_of(e, v))];
}

wo_engine* wo_create(uint64_t n, uint64_t m, const uint64_t* off, const uint32_t* adj,
                     uint32_t wpv, uint32_t L, int model, float p, float q, int init,
                     int deterministic, uint64_t seed)
{
    wo_engine* e = (wo_engine*)calloc(1, sizeof(wo_engine));
    e->n = n; e->m = m;
    e->off = (uint64_t*)malloc((n + 1) * 8);
    memcpy(e->off, off, (n + 1) * 8);
    e->adj = (uint32_t*)malloc((m ? m : 1) * 4);
    if (m) memcpy(e->adj, adj, m * 4);
    e->anchor = (uint64_t*)malloc((m ? m : 1) * 8);
    /* anchors are read by node2vec MH only: the other modes leave the pages untouched */
    if (model == WO_NODE2VEC && !deterministic) memset(e->anchor, 0xFF, (m ? m : 1) * 8);
    e->row_epoch = (uint32_t*)calloc(n ? n : 1, 4);
    e->wpv = wpv; e->L = L; e->model = model; e->init = init; e->det = deterministic;
    e->p = p; e->q = q; e->seed = seed;
    e->walks = (uint32_t*)malloc(n * wpv * L * 4 + 4);
    /* Corpora above 8 GiB (the full-size GPU tests' windows of configs[3]: 107 GB)
     * are not pre-filled: generation writes every position of each walk it
     * produces (walk_from), so wo_time_generate_range + wo_get_walks_range of that
     * range need no fill, and untouched pages cost no host memory.  Only those two
     * calls are used on such engines. */
    if ((uint64_t)n * wpv * L * 4 <= (8ull << 30))
        for (uint64_t i = 0; i < n * wpv * L; i++) e->walks[i] = WO_SENT;
    return e;
}

void wo_free(wo_engine* e)
{
    if (!e) return;
    free(e->off); free(e->adj); free(e->anchor); free(e->row_epoch); free(e->walks);
    free(e);
}

/* wharfmh.h:250-356 */
void wo_generate(wo_engine* e)
{
    uint64_t W = e->n * e->wpv, acc = 0, steps = 0;
    #pragma omp parallel for schedule(dynamic, 256) reduction(+:acc, steps)
    for (int64_t wid = 0; wid < (int64_t)W; wid++) {
        uint32_t v = (uint32_t)(wid % e->n);
        walk_from(e, (uint64_t)wid, v, 0, initial_prev(e, wid, v), &acc, &steps);
    }
    e->accepts = acc;
    e->steps = steps;
}

double wo_time_generate_range(wo_engine* e, uint64_t w0, uint64_t w1, int threads)
{
    uint64_t acc = 0, steps = 0;
    if (threads > 0) omp_set_num_threads(threads);
    double t0 = omp_get_wtime();
    #pragma omp parallel for schedule(dynamic, 256) reduction(+:acc, steps)
    for (int64_t wid = (int64_t)w0; wid < (int64_t)w1; wid++) {
        uint32_t v = (uint32_t)(wid % e->n);
        walk_from(e, (uint64_t)wid, v, 0, initial_prev(e, wid, v), &acc, &steps);
    }
    double t = omp_get_wtime() - t0;
    e->accepts = acc;
    e->steps = steps;
    return t;
}

/* wharfmh.h:439-576 (insert) / 588-726 (delete) + 733-923 (re-walk) */
uint64_t wo_update(wo_engine* e, int insert, uint64_t m, const uint32_t* pairs_in, uint32_t flags,
                   uint32_t* affected_out)
{
    /* 1-3: sort by source (wharfmh.h:450-453, 1056-1104); remove self loops and
     * duplicates when asked (456-470).  The set union/difference collapses
     * duplicates either way. */
    uint32_t* b = (uint32_t*)malloc((m ? m : 1) * 8);
    memcpy(b, pairs_in, m * 8);
    qsort(b, m, 8, cmp_pair);
    uint64_t k = 0;
    for (uint64_t i = 0; i < m; i++) {
        if ((flags & WO_REMOVE_DUPS) && b[2 * i] == b[2 * i + 1]) continue;
        if (k > 0 && b[2 * k - 2] == b[2 * i] && b[2 * k - 1] == b[2 * i + 1]) continue;
        b[2 * k] = b[2 * i]; b[2 * k + 1] = b[2 * i + 1];
        k++;
    }
    m = k;
    e->accepts = e->steps = 0;
    if (m == 0) {   /* nothing to apply: no sources, no sampler reset, epoch unchanged */
        free(b);
        return 0;
    }

    /* batch sources: every distinct source, whether or not its row changes */
    uint8_t* is_src = (uint8_t*)calloc(e->n ? e->n : 1, 1);
    for (uint64_t i = 0; i < m; i++) is_src[b[2 * i]] = 1;

    /* rewalk points (wharfmh.h:519-537): min position of any batch source in
     * each walk, over the pre-update corpus */
    uint64_t W = e->n * e->wpv;
    uint8_t* pw = (uint8_t*)malloc(W ? W : 1);
    uint64_t naff = 0;
    for (uint64_t wid = 0; wid < W; wid++) {
        const uint32_t* w = e->walks + wid * e->L;
        uint32_t p = 0xFF;
        for (uint32_t pos = 0; pos < e->L; pos++) {
            if (w[pos] == WO_SENT) break;
            if (is_src[w[pos]]) { p = pos; break; }
        }
        pw[wid] = (uint8_t)p;
        if (p != 0xFF) affected_out[naff++] = (uint32_t)wid;
    }

    /* graph update: per-source union (tree_plus::uniont, wharfmh.h:511) or
     * difference (tree_plus::difference, 659) */
    uint64_t* noff = (uint64_t*)malloc((e->n + 1) * 8);
    uint64_t cap = e->m + (insert ? m : 0);
    uint32_t* nadj = (uint32_t*)malloc((cap ? cap : 1) * 4);
    uint64_t* nanc = (uint64_t*)malloc((cap ? cap : 1) * 8);
    uint64_t bi = 0, o = 0;
    noff[0] = 0;
    for (uint64_t v = 0; v < e->n; v++) {
        uint64_t a0 = e->off[v], a1 = e->off[v + 1];
        uint64_t b0 = bi;
        while (bi < m && b[2 * bi] == v) bi++;
        uint64_t b1 = bi;
        if (b0 == b1) {
            memcpy(nadj + o, e->adj + a0, (a1 - a0) * 4);
            memcpy(nanc + o, e->anchor + a0, (a1 - a0) * 8);
            o += a1 - a0;
        } else if (insert) {
            uint64_t i = a0, j = b0;
            while (i < a1 || j < b1) {
                uint32_t x;
                if (j >= b1 || (i < a1 && e->adj[i] < b[2 * j + 1])) x = e->adj[i++];
                else if (i >= a1 || b[2 * j + 1] < e->adj[i]) x = b[2 * j++ + 1];
                else { x = e->adj[i++]; j++; }
                nanc[o] = ANCHOR_NONE;
                nadj[o++] = x;
            }
        } else {
            uint64_t j = b0;
            for (uint64_t i = a0; i < a1; i++) {
                while (j < b1 && b[2 * j + 1] < e->adj[i]) j++;
                if (j < b1 && b[2 * j + 1] == e->adj[i]) continue;
                nanc[o] = ANCHOR_NONE;
                nadj[o++] = e->adj[i];
            }
        }
        noff[v + 1] = o;
    }
    free(e->off); free(e->adj); free(e->anchor);
    e->off = noff; e->adj = nadj; e->anchor = nanc; e->m = o;

    /* samplers of batch sources are replaced by fresh managers (wharfmh.h:504,539) */
    e->epoch++;
    for (uint64_t v = 0; v < e->n; v++) if (is_src[v]) e->row_epoch[v] = e->epoch;

    /* batch_walk_update (wharfmh.h:761-859) */
    uint64_t acc = 0, steps = 0;
    if (flags & WO_APPLY_WALK_UPDATES) {
        #pragma omp parallel for schedule(dynamic, 64) reduction(+:acc, steps)
        for (int64_t i = 0; i < (int64_t)naff; i++) {
            uint64_t wid = affected_out[i];
            uint32_t p = pw[wid];
            uint32_t* w = e->walks + wid * e->L;
            uint32_t v = w[p];
            uint32_t prev = v;
            if (e->model == WO_NODE2VEC && !e->det)
                prev = p > 0 ? w[p - 1] : initial_prev(e, wid, v);   /* 817-823 */
            walk_from(e, wid, v, p, prev, &acc, &steps);
        }
    }
    e->accepts = acc;
    e->steps = steps;
    free(b); free(is_src); free(pw);
    return naff;
}

uint64_t wo_num_edges(const wo_engine* e) { return e->m; }
uint64_t wo_num_walks(const wo_engine* e) { return e->n * e->wpv; }
uint64_t wo_get_accepts(const wo_engine* e) { return e->accepts; }
uint64_t wo_get_steps(const wo_engine* e) { return e->steps; }

void wo_get_csr(const wo_engine* e, uint64_t* off_out, uint32_t* adj_out)
{
    memcpy(off_out, e->off, (e->n + 1) * 8);
    if (e->m) memcpy(adj_out, e->adj, e->m * 4);
}

void wo_get_walks(const wo_engine* e, uint32_t* out)
{
    memcpy(out, e->walks, e->n * e->wpv * e->L * 4);
}

void wo_get_walks_range(const wo_engine* e, uint64_t w0, uint64_t w1, uint32_t* out)
{
    memcpy(out, e->walks + w0 * e->L, (w1 - w0) * e->L * 4);
}

/* walks/inverted_index.h:12-37: vertex walk[pos] holds key wid*L+pos -> next
 * (SENT at the last position), per vertex ascending by key. */
uint64_t wo_index_size(const wo_engine* e)
{
    uint64_t W = e->n * e->wpv, c = 0;
    for (uint64_t i = 0; i < W * e->L; i++) c += e->walks[i] != WO_SENT;
    return c;
}

void wo_export_index(const wo_engine* e, uint64_t* counts, uint64_t* keys, uint32_t* nexts)
{
    uint64_t W = e->n * e->wpv, L = e->L;
    memset(counts, 0, e->n * 8);
    for (uint64_t i = 0; i < W * L; i++) if (e->walks[i] != WO_SENT) counts[e->walks[i]]++;
    uint64_t* cur = (uint64_t*)malloc((e->n + 1) * 8);
    cur[0] = 0;
    for (uint64_t v = 0; v < e->n; v++) cur[v + 1] = cur[v] + counts[v];
    /* keys are visited in ascending order, so each vertex's list comes out sorted */
    for (uint64_t wid = 0; wid < W; wid++)
        for (uint64_t pos = 0; pos < L; pos++) {
            uint32_t v = e->walks[wid * L + pos];
            if (v == WO_SENT) break;
            uint64_t at = cur[v]++;
            keys[at] = wid * L + pos;
            nexts[at] = pos + 1 < L ? e->walks[wid * L + pos + 1] : WO_SENT;
        }
    free(cur);
}
