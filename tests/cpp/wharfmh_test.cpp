// The reference's integration tests (tests/wharfmh.cpp:56-264, tests/sampler.cpp)
// restated against include/wharfmh.hpp — the C++ drop-in — on the GPU.
// Built by __graft_entry__.build(); run by tests/test_cpp_dropin.py (-m gpu).
#include <cstdio>
#include <cstdlib>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "wharfmh.hpp"

static int g_fail = 0;
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);           \
            g_fail++;                                                          \
        }                                                                      \
    } while (0)

struct Csr {
    size_t n, m;
    std::vector<uint64_t> off;   // n entries, like the reference's uintE* offsets
    std::vector<uint32_t> adj;
};

// symmetric RMAT graph (utility::generate_batch_of_edges(..., directed=false))
static Csr rmat_graph(uint64_t samples, uint64_t n, uint64_t seed)
{
    std::vector<uint32_t> pairs(4 * samples);
    uint64_t k = 0;
    wharf::check(wharf_generate_batch_of_edges(0, samples, 2 * n, seed, 0, 0, 0.5, 0.2, 0.1, pairs.data(), &k), nullptr,
                 "generate_batch_of_edges");
    Csr g{n, k, std::vector<uint64_t>(n, 0), std::vector<uint32_t>(k)};
    std::vector<uint64_t> cnt(n + 1, 0);
    for (uint64_t i = 0; i < k; i++) cnt[pairs[2 * i] + 1]++;
    for (size_t v = 0; v < n; v++) cnt[v + 1] += cnt[v];
    for (size_t v = 0; v < n; v++) g.off[v] = cnt[v];
    for (uint64_t i = 0; i < k; i++) g.adj[i] = pairs[2 * i + 1];
    return g;
}

static std::vector<std::tuple<uint32_t, uint32_t>> batch(uint64_t samples, uint64_t n, uint64_t seed, bool directed)
{
    std::vector<uint32_t> pairs(4 * samples);
    uint64_t k = 0;
    wharf::check(wharf_generate_batch_of_edges(0, samples, n, seed, 0, directed, 0.5, 0.2, 0.1, pairs.data(), &k),
                 nullptr, "generate_batch_of_edges");
    std::vector<std::tuple<uint32_t, uint32_t>> e(k);
    for (uint64_t i = 0; i < k; i++) e[i] = std::make_tuple(pairs[2 * i], pairs[2 * i + 1]);
    // hand it over unsorted: the drop-in sorts the caller's buffer like the reference
    std::reverse(e.begin(), e.end());
    return e;
}

static bool walks_follow_edges(wharf::WharfMH& w, size_t walks)
{
    std::vector<uint64_t> off;
    std::vector<uint32_t> adj;
    w.flatten_graph(off, adj);
    for (size_t wid = 0; wid < walks; wid += 7) {
        std::istringstream ss(w.walk((uint32_t)wid));
        std::vector<uint32_t> v;
        uint32_t x;
        while (ss >> x) v.push_back(x);
        if (v.empty() || v[0] != wid % w.number_of_vertices()) return false;
        for (size_t i = 0; i + 1 < v.size(); i++)
            if (!std::binary_search(adj.begin() + off[v[i]], adj.begin() + off[v[i] + 1], v[i + 1])) return false;
    }
    return true;
}

// tests/wharfmh.cpp:56-99
static void test_constructor(const Csr& g)
{
    wharf::WharfMH w((long)g.n, (long)g.m, g.off.data(), g.adj.data(), false);
    EXPECT(w.number_of_vertices() == g.n);
    EXPECT(w.number_of_edges() == g.m);
    std::vector<uint64_t> off;
    std::vector<uint32_t> adj;
    w.flatten_graph(off, adj);
    bool ok = true;
    for (size_t v = 0; v < g.n && ok; v++) {
        const uint64_t b = g.off[v], e = v + 1 < g.n ? g.off[v + 1] : g.m;
        ok = (off[v + 1] - off[v] == e - b);
        std::set<uint32_t> s(g.adj.begin() + b, g.adj.begin() + e);
        for (uint64_t j = off[v]; j < off[v + 1] && ok; j++) ok = s.count(adj[j]) == 1;
    }
    EXPECT(ok);
    std::vector<uint64_t> c, k;
    std::vector<uint32_t> nx;
    w.inverted_index(c, k, nx);
    EXPECT(k.empty());   // no walks yet: empty inverted indexes
}

// tests/wharfmh.cpp:101-140
static void test_destroy(const Csr& g)
{
    wharf::WharfMH w((long)g.n, (long)g.m, g.off.data(), g.adj.data());
    w.generate_initial_random_walks();
    std::vector<uint64_t> c, k;
    std::vector<uint32_t> nx;
    w.inverted_index(c, k, nx);
    EXPECT(!k.empty());
    std::vector<uint64_t> pc, paired;   // CompressedWalks form: same counts, Szudzik(key, next) per entry
    w.compressed_walks(pc, paired);
    EXPECT(pc == c && paired.size() == k.size());
    {
        bool same = true;
        for (size_t v = 0, o = 0; v < c.size() && same; o += c[v], v++) {
            std::vector<uint64_t> z;
            for (uint64_t i = o; i < o + c[v]; i++) {
                const uint64_t a = k[i], b = nx[i];
                z.push_back(b >= a ? b * (b + 1) + a : a * a + b);
            }
            std::sort(z.begin(), z.end());
            same = std::equal(z.begin(), z.end(), paired.begin() + o);
        }
        EXPECT(same);
    }
    const wharf_memory mem = w.memory_footprint();   // memory-footprint.cpp's report
    EXPECT(mem.n == g.n && mem.m == g.m && mem.walks_bytes >= k.size() * 4 && mem.csr_bytes >= g.m * 4);
    EXPECT(mem.total_bytes >= mem.csr_bytes + mem.records_bytes + mem.walks_bytes);
    w.destroy_index();
    w.inverted_index(c, k, nx);
    EXPECT(k.empty());
    EXPECT(w.number_of_vertices() == g.n && w.number_of_edges() == g.m);
    w.destroy();
    EXPECT(w.number_of_vertices() == 0 && w.number_of_edges() == 0);
}

// tests/wharfmh.cpp:142-264
static void test_updates(const Csr& g)
{
    wharf::WharfMH w((long)g.n, (long)g.m, g.off.data(), g.adj.data());
    w.generate_initial_random_walks();
    const size_t walks = g.n * wharf::config().walks_per_vertex;
    EXPECT(walks_follow_edges(w, walks));
    const size_t start = w.number_of_edges();
    auto b = batch(100, g.n, 0, true);
    auto aff = w.insert_edges_batch(b.size(), b.data(), false, true, g.n);
    EXPECT(std::is_sorted(b.begin(), b.end()));   // caller's buffer sorted in place
    EXPECT(w.number_of_edges() >= start);
    EXPECT(!aff.empty() && std::is_sorted(aff.begin(), aff.end()));
    EXPECT(walks_follow_edges(w, walks));
    auto d = batch(100000, g.n, 0, false);
    const size_t before = w.number_of_edges();
    w.delete_edges_batch(d.size(), d.data(), false, true, g.n);
    EXPECT(w.number_of_edges() <= before);
    EXPECT(walks_follow_edges(w, walks));
}

// tests/sampler.cpp:24-35 graph; corpus pinned by the reference
static void test_six_vertex_corpus()
{
    const uint64_t off[6] = {0, 2, 5, 10, 13, 15};
    const uint32_t adj[18] = {1, 2, 0, 2, 3, 0, 1, 3, 4, 5, 1, 2, 5, 2, 5, 2, 3, 4};
    wharf_config saved = wharf::config();
    wharf::config().walks_per_vertex = 2;
    wharf::config().walk_length = 5;
    wharf::WharfMH w(6, 18, off, adj);
    w.generate_initial_random_walks();
    const char* expect[12] = {"0 1 0 1 2 ", "1 3 1 2 3 ", "2 4 5 3 2 ", "3 5 2 0 2 ", "4 2 4 2 3 ", "5 4 5 3 2 ",
                              "0 2 4 2 5 ", "1 0 2 0 2 ", "2 3 5 4 5 ", "3 1 3 5 2 ", "4 5 4 2 5 ", "5 2 4 2 5 "};
    for (uint32_t i = 0; i < 12; i++) EXPECT(w.walk(i) == expect[i]);
    EXPECT(w.vertex_at_walk(11, 3) == 2);
    wharf::config() = saved;
}

int main()
{
    int ndev = 0;
    if (wharf_device_count(&ndev) != WHARF_OK || ndev == 0) {
        std::printf("no HIP device\n");
        return 2;
    }
    const Csr g = rmat_graph(100000, 1 << 14, 3);
    test_constructor(g);
    test_destroy(g);
    test_updates(g);
    test_six_vertex_corpus();
    std::printf(g_fail ? "FAILED (%d)\n" : "OK\n", g_fail);
    return g_fail ? 1 : 0;
}
