/*
 * TEST INFRASTRUCTURE ONLY — drives the C oracle (wharf_oracle.c) through
 * every engine path under a sanitizer build (make -C oracle asan tsan):
 * RMAT graph, generation, insert / delete batches with and without walk
 * updates, deterministic and MH DeepWalk, MH node2vec with the three sampler
 * inits, index export.  OpenMP runs the walk loops on several threads, so
 * the TSan build (clang + libomp + the Archer tool) checks the anchor cache's
 * concurrent lazy initialisation (wharf_oracle.c anchor_get) for races.
 * Exit status 0 and "sanitize OK" when every self-check passed.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wharf_oracle.h"

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                     \
        }                                                                 \
    } while (0)

static int has_edge(const uint64_t* off, const uint32_t* adj, uint32_t a, uint32_t b)
{
    uint64_t lo = off[a], hi = off[a + 1];
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (adj[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < off[a + 1] && adj[lo] == b;
}

/* every stored transition is an edge of the current graph; walks start at their vertex */
static void check_walks(wo_engine* e, uint64_t n, uint32_t wpv, uint32_t L)
{
    const uint64_t W = wo_num_walks(e), m = wo_num_edges(e);
    CHECK(W == n * wpv);
    uint64_t* off = malloc((n + 1) * 8);
    uint32_t* adj = malloc((m ? m : 1) * 4);
    uint32_t* w = malloc(W * L * 4);
    wo_get_csr(e, off, adj);
    wo_get_walks(e, w);
    for (uint64_t i = 0; i < W; i++) {
        const uint32_t* r = w + i * L;
        CHECK(r[0] == (uint32_t)(i % n));
        for (uint32_t p = 1; p < L && r[p] != WO_SENT; p++) CHECK(has_edge(off, adj, r[p - 1], r[p]));
    }
    free(off);
    free(adj);
    free(w);
}

static void run(const uint64_t* off, const uint32_t* adj, uint64_t n, uint64_t m, int model, int init, int det)
{
    const uint32_t wpv = 3, L = 24;
    wo_engine* e = wo_create(n, m, off, adj, wpv, L, model, 0.5f, 2.0f, init, det, 17);
    CHECK(e != NULL);
    wo_generate(e);
    check_walks(e, n, wpv, L);
    uint32_t* aff = malloc(n * wpv * 4);
    uint32_t* batch = malloc(2 * 2 * 400 * 4);
    for (uint64_t s = 0; s < 4; s++) {
        const uint64_t k = wo_generate_batch_of_edges(400, n, 100 + s, 0, 0, 0.5, 0.2, 0.1, batch);
        const uint32_t fl = WO_REMOVE_DUPS | (s == 2 ? 0 : WO_APPLY_WALK_UPDATES);
        const uint64_t na = wo_update(e, s % 2 == 0, k, batch, fl, aff);
        for (uint64_t i = 1; i < na; i++) CHECK(aff[i - 1] < aff[i]);
        if (fl & WO_APPLY_WALK_UPDATES) check_walks(e, n, wpv, L);
    }
    const uint64_t sz = wo_index_size(e);
    uint64_t* counts = malloc(n * 8);
    uint64_t* keys = malloc((sz ? sz : 1) * 8);
    uint32_t* nexts = malloc((sz ? sz : 1) * 4);
    wo_export_index(e, counts, keys, nexts);
    uint64_t tot = 0;
    for (uint64_t v = 0; v < n; v++) tot += counts[v];
    CHECK(tot == sz);
    free(counts);
    free(keys);
    free(nexts);
    free(aff);
    free(batch);
    wo_free(e);
}

int main(void)
{
    const uint64_t n = 1 << 11, samples = 12000;
    uint32_t* pairs = malloc(2 * 2 * samples * 4);
    const uint64_t m = wo_generate_batch_of_edges(samples, n, 3, 0, 0, 0.5, 0.2, 0.1, pairs);
    uint64_t* off = calloc(n + 1, 8);
    uint32_t* adj = malloc(m * 4);
    for (uint64_t i = 0; i < m; i++) off[pairs[2 * i] + 1]++;
    for (uint64_t v = 0; v < n; v++) off[v + 1] += off[v];
    for (uint64_t i = 0; i < m; i++) adj[i] = pairs[2 * i + 1];   /* pairs are sorted by (src, dst) */
    run(off, adj, n, m, WO_DEEPWALK, WO_INIT_WEIGHT, 1);
    run(off, adj, n, m, WO_NODE2VEC, WO_INIT_WEIGHT, 1);
    run(off, adj, n, m, WO_DEEPWALK, WO_INIT_WEIGHT, 0);
    for (int init = WO_INIT_RANDOM; init <= WO_INIT_WEIGHT; init++) run(off, adj, n, m, WO_NODE2VEC, init, 0);
    uint64_t st[2];
    wo_random_init(42, st);
    CHECK(wo_lrand(st) != wo_lrand(st));
    free(pairs);
    free(off);
    free(adj);
    if (g_fail) return 1;
    printf("sanitize OK\n");
    return 0;
}
