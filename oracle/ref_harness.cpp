// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Driver for the *reference* WharfMH implementation (header-only C++17 under
// /root/reference).  It is compiled by oracle/Makefile directly against the
// reference headers where they lie (no sources are copied) and the binary is
// written to oracle/_ref/.  It is used to
//   (1) produce the golden vectors committed under tests/golden/
//       (tests/golden/make_golden.py drives it), and
//   (2) time the reference CPU path as bench.py's `cpu_baseline` leg.
//
// It only calls the reference's public API:
//   dygrl::WharfMH ctor / generate_initial_random_walks / insert_edges_batch /
//   delete_edges_batch / walk / graph_tree   (graph/wharfmh.h:26-923)
//   utility::Random, utility::generate_batch_of_edges (utils/utility.h:55-223)
//   pairings::Szudzik (walks/pairings.h:113-226)
//
// Commands are read from argv, executed in order:
//   out <dir>                                  output directory for dumps
//   cfg <wpv> <L> <deepwalk|node2vec> <p> <q> <random|burnin|weight> <det 0|1> <rngseed>
//   graph-adj <file>                           Ligra AdjacencyGraph text
//   graph-csr <file>                           raw: u64 n, u64 m, u64 off[n], u32 adj[m]
//   graph-rmat <M> <V> <seed> <n>              undirected RMAT base graph, n vertices
//   gen                                        generate_initial_random_walks, dump walks
//   ins|del <M> <seed> <directed 0|1>          RMAT batch (generate_batch_of_edges(M, n, seed,
//                                              false, directed)) then insert/delete with
//                                              sorted=false, remove_dups=true, nn=pow2
//   insf|delf <file>                           batch from raw file: u64 m, u32 pairs[2m]
//   dump-index                                 per-vertex (key,next) lists
//   dump-graph                                 flattened CSR
//   walkstr <wid>                              WharfMH::walk(wid) text to walkstr_<k>.txt
//   time-gen <reps>                            time generate_initial_random_walks
//   time-upd <M> <seed> <directed 0|1> <reps>  time insert_edges_batch of RMAT batches
//                                              (seeds seed, seed+1, ...; walk update applied,
//                                              nothing dumped)
//   kat                                        RNG / hash / Szudzik / RMAT known answers
//   batch <M> <V> <seed> <directed>            dump generate_batch_of_edges output
#include <wharfmh.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>
#include <algorithm>
#include <mutex>

namespace {

std::string g_out = ".";
int g_step = 0;
dygrl::WharfMH* g_w = nullptr;
size_t g_n = 0;

void write_raw(const std::string& name, const void* data, size_t bytes)
{
    std::string path = g_out + "/" + name;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    if (bytes && std::fwrite(data, 1, bytes, f) != bytes) { std::perror("fwrite"); std::exit(2); }
    std::fclose(f);
}

// Walk matrix [W][L] by following the inverted index exactly as WharfMH::walk
// does (wharfmh.h:365-394); positions after the sentinel are padded with SENT.
void dump_walks(const std::string& tag)
{
    const uint32_t SENT = std::numeric_limits<uint32_t>::max() - 1;
    const size_t L = config::walk_length;
    const size_t W = g_n * config::walks_per_vertex;
    std::vector<uint32_t> mat(W * L, SENT);
    parallel_for(0, W, [&](size_t wid) {
        uint32_t cur = wid % g_w->number_of_vertices();
        for (size_t pos = 0; pos < L && cur != SENT; pos++) {
            mat[wid * L + pos] = cur;
            auto node = g_w->graph_tree.find(cur);
            cur = node.value.inverted_index.find_next(wid, pos);
        }
    });
    write_raw("walks_" + tag + ".bin", mat.data(), mat.size() * 4);
}

void dump_index(const std::string& tag)
{
    // per vertex: sorted (key, next); layout: u64 n, u64 cnt[n], then (u32 key, u32 next) pairs
    size_t n = g_w->number_of_vertices();
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> per(n);
    parallel_for(0, n, [&](size_t v) {
        auto node = g_w->graph_tree.find(v);
        if (!node.valid) return;
        auto& idx = node.value.inverted_index;
        std::vector<std::pair<uint32_t, uint32_t>> e(idx.size());
        dygrl::InvertedIndex::entries(idx, e.data());
        per[v] = std::move(e);
    });
    std::vector<uint64_t> head;
    head.push_back(n);
    for (auto& p : per) head.push_back(p.size());
    std::vector<uint32_t> body;
    for (auto& p : per) for (auto& kv : p) { body.push_back(kv.first); body.push_back(kv.second); }
    std::vector<char> buf(head.size() * 8 + body.size() * 4);
    std::memcpy(buf.data(), head.data(), head.size() * 8);
    if (!body.empty()) std::memcpy(buf.data() + head.size() * 8, body.data(), body.size() * 4);
    write_raw("index_" + tag + ".bin", buf.data(), buf.size());
}

void dump_graph(const std::string& tag)
{
    auto flat = g_w->flatten_graph();
    size_t n = g_w->number_of_vertices();
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t v = 0; v < n; v++) off[v + 1] = off[v] + flat[v].degree;
    std::vector<uint32_t> adj(off[n]);
    for (size_t v = 0; v < n; v++)
        for (size_t j = 0; j < flat[v].degree; j++) adj[off[v] + j] = flat[v].neighbors[j];
    std::vector<char> buf(8 + (n + 1) * 8 + adj.size() * 4);
    uint64_t nn = n;
    std::memcpy(buf.data(), &nn, 8);
    std::memcpy(buf.data() + 8, off.data(), (n + 1) * 8);
    if (!adj.empty()) std::memcpy(buf.data() + 8 + (n + 1) * 8, adj.data(), adj.size() * 4);
    write_raw("graph_" + tag + ".bin", buf.data(), buf.size());
}

void build_from_csr(size_t n, size_t m, const std::vector<uint64_t>& off, const std::vector<uint32_t>& adj)
{
    // the ctor takes ownership of pbbs arrays (wharfmh.h:99-103) -> hand it copies
    uintE* o = pbbs::new_array_no_init<uintE>(n);
    uintV* e = pbbs::new_array_no_init<uintV>(std::max<size_t>(m, 1));
    for (size_t i = 0; i < n; i++) o[i] = off[i];
    for (size_t i = 0; i < m; i++) e[i] = adj[i];
    g_w = new dygrl::WharfMH(n, m, o, e, true);
    g_n = n;
}

// CSR from a sorted, deduplicated edge list (the form generate_batch_of_edges returns).
void build_from_edges(size_t n, std::tuple<uintV, uintV>* E, size_t m)
{
    std::vector<uint64_t> off(n + 1, 0);
    std::vector<uint32_t> adj(m);
    for (size_t i = 0; i < m; i++) off[std::get<0>(E[i]) + 1]++;
    for (size_t v = 0; v < n; v++) off[v + 1] += off[v];
    for (size_t i = 0; i < m; i++) adj[i] = std::get<1>(E[i]);
    build_from_csr(n, m, off, adj);
}

void dump_batch(const std::string& tag, std::tuple<uintV, uintV>* E, size_t m)
{
    std::vector<uint32_t> b(2 * m);
    for (size_t i = 0; i < m; i++) { b[2 * i] = std::get<0>(E[i]); b[2 * i + 1] = std::get<1>(E[i]); }
    write_raw("batch_" + tag + ".bin", b.data(), b.size() * 4);
}

void run_update(bool insert, std::tuple<uintV, uintV>* E, size_t m, const std::string& tag)
{
    size_t n = g_w->number_of_vertices();
    size_t pow2 = 1ul << (pbbs::log2_up(n) - 1);
    dump_batch(tag + "_in", E, m);
    auto t0 = std::chrono::steady_clock::now();
    auto aff = insert ? g_w->insert_edges_batch(m, E, false, true, pow2)
                      : g_w->delete_edges_batch(m, E, false, true, pow2);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<uint32_t> a(aff.begin(), aff.end());
    std::sort(a.begin(), a.end());
    write_raw("affected_" + tag + ".bin", a.data(), a.size() * 4);
    // the reference sorts the caller's buffer in place (wharfmh.h:450-453)
    dump_batch(tag + "_sorted", E, m);
    std::printf("%s %s m=%zu affected=%zu seconds=%.6f\n", insert ? "insert" : "delete", tag.c_str(), m, a.size(), s);
}

void do_kat()
{
    std::string path = g_out + "/kat.txt";
    FILE* f = std::fopen(path.c_str(), "w");
    for (uint64_t seed : {0ull, 1ull, 2ull, 9ull, 12345ull, 0xFFFFFFFFFFFFFFFFull, 0x8000000000000000ull}) {
        utility::Random r(seed);
        std::fprintf(f, "random %llu state %llu %llu lrand", (unsigned long long)seed,
                     (unsigned long long)r.rng_seed0, (unsigned long long)r.rng_seed1);
        for (int i = 0; i < 8; i++) std::fprintf(f, " %llu", (unsigned long long)r.lrand());
        std::fprintf(f, "\n");
        utility::Random d(seed);
        std::fprintf(f, "drand %llu", (unsigned long long)seed);
        for (int i = 0; i < 4; i++) std::fprintf(f, " %.17g", d.drand());
        std::fprintf(f, "\n");
        utility::Random q(seed);
        std::fprintf(f, "irand %llu", (unsigned long long)seed);
        for (int mx : {1, 2, 3, 7, 80, 1000, 65537, 2147483647}) std::fprintf(f, " %d", q.irand(mx));
        std::fprintf(f, "\n");
    }
    for (uint64_t x : {0ull, 1ull, 2ull, 7ull, 123456789ull, 0xFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull})
        std::fprintf(f, "hash64 %llu %llu\n", (unsigned long long)x, (unsigned long long)pbbs::hash64(x));
    for (uint32_t x : {0u, 1u, 2u, 7u, 123456789u, 0xFFFFFFFFu})
        std::fprintf(f, "hash32 %u %u\n", x, pbbs::hash32(x));
    using SZ = pairings::Szudzik<uint32_t>;
    using SZ64 = pairings::Szudzik<uint64_t>;
    std::fprintf(f, "szudzik32 65535 65535 %u\n", SZ::pair({65535u, 65535u}));
    std::fprintf(f, "szudzik32 10 3 %u\n", SZ::pair({10u, 3u}));
    std::fprintf(f, "szudzik32 3 10 %u\n", SZ::pair({3u, 10u}));
    std::fprintf(f, "szudzik32_triplet 123 25 200 %u\n", SZ::pair_triplet({123u, 25u, 200u}));
    auto up = SZ::unpair(4294967295u);
    std::fprintf(f, "szudzik32_unpair 4294967295 %u %u\n", up.first, up.second);
    auto ut = SZ::unpair_triplet(229643916u);
    std::fprintf(f, "szudzik32_unpair_triplet 229643916 %u %u %u\n", std::get<0>(ut), std::get<1>(ut), std::get<2>(ut));
    std::fprintf(f, "szudzik64 4000000000 3999999999 %llu\n", (unsigned long long)SZ64::pair({4000000000ull, 3999999999ull}));
    std::fprintf(f, "szudzik64 3999999999 4000000000 %llu\n", (unsigned long long)SZ64::pair({3999999999ull, 4000000000ull}));
    auto u64p = SZ64::unpair(SZ64::pair({123456789ull, 987654321ull}));
    std::fprintf(f, "szudzik64_roundtrip 123456789 987654321 %llu %llu\n", (unsigned long long)u64p.first, (unsigned long long)u64p.second);
    std::fclose(f);
}

}  // namespace

int main(int argc, char** argv)
{
    std::vector<std::string> a(argv + 1, argv + argc);
    for (size_t i = 0; i < a.size();) {
        const std::string& c = a[i++];
        if (c == "out") {
            g_out = a[i++];
        } else if (c == "cfg") {
            config::walks_per_vertex = std::stoi(a[i++]);
            config::walk_length = std::stoi(a[i++]);
            std::string model = a[i++];
            config::random_walk_model = model == "node2vec" ? types::NODE2VEC : types::DEEPWALK;
            config::paramP = std::stof(a[i++]);
            config::paramQ = std::stof(a[i++]);
            std::string init = a[i++];
            config::sampler_init_strategy = init == "random" ? types::RANDOM : init == "burnin" ? types::BURNIN : types::WEIGHT;
            config::deterministic_mode = std::stoi(a[i++]) != 0;
            config::random.reinit(std::stoull(a[i++]));
        } else if (c == "graph-adj") {
            size_t n, m; uintE* off; uintV* e;
            std::tie(n, m, off, e) = read_unweighted_graph(a[i++].c_str(), true, false);
            g_w = new dygrl::WharfMH(n, m, off, e, true);
            g_n = n;
        } else if (c == "graph-csr") {
            std::ifstream in(a[i++], std::ios::binary);
            uint64_t n, m;
            in.read((char*)&n, 8); in.read((char*)&m, 8);
            std::vector<uint64_t> off(n); std::vector<uint32_t> adj(m);
            in.read((char*)off.data(), n * 8); in.read((char*)adj.data(), m * 4);
            build_from_csr(n, m, off, adj);
        } else if (c == "graph-rmat") {
            size_t M = std::stoull(a[i++]), V = std::stoull(a[i++]), seed = std::stoull(a[i++]), n = std::stoull(a[i++]);
            auto b = utility::generate_batch_of_edges(M, V, seed, false, false);
            build_from_edges(n, b.first, b.second);
            pbbs::free_array(b.first);
        } else if (c == "gen") {
            auto t0 = std::chrono::steady_clock::now();
            g_w->generate_initial_random_walks();
            double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::printf("gen seconds=%.6f\n", s);
            dump_walks(std::to_string(g_step++) + "_gen");
        } else if (c == "ins" || c == "del") {
            size_t M = std::stoull(a[i++]), seed = std::stoull(a[i++]);
            bool directed = std::stoi(a[i++]) != 0;
            auto b = utility::generate_batch_of_edges(M, g_n, seed, false, directed);
            std::string tag = std::to_string(g_step++) + "_" + c;
            run_update(c == "ins", b.first, b.second, tag);
            pbbs::free_array(b.first);
            dump_walks(tag);
        } else if (c == "insf" || c == "delf") {
            std::ifstream in(a[i++], std::ios::binary);
            uint64_t m; in.read((char*)&m, 8);
            std::vector<uint32_t> p(2 * m); in.read((char*)p.data(), 8 * m);
            auto* E = pbbs::new_array_no_init<std::tuple<uintV, uintV>>(std::max<size_t>(m, 1));
            for (size_t k = 0; k < m; k++) E[k] = std::make_tuple(p[2 * k], p[2 * k + 1]);
            std::string tag = std::to_string(g_step++) + "_" + c;
            run_update(c == "insf", E, m, tag);
            pbbs::free_array(E);
            dump_walks(tag);
        } else if (c == "dump-index") {
            dump_index(std::to_string(g_step - 1));
        } else if (c == "dump-graph") {
            dump_graph(std::to_string(g_step - 1));
        } else if (c == "walkstr") {
            uint32_t wid = std::stoul(a[i++]);
            std::string s = g_w->walk(wid);
            write_raw("walkstr_" + std::to_string(wid) + ".txt", s.data(), s.size());
        } else if (c == "time-gen") {
            int reps = std::stoi(a[i++]);
            for (int r = 0; r < reps; r++) {
                g_w->destroy_index();
                auto t0 = std::chrono::steady_clock::now();
                g_w->generate_initial_random_walks();
                double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::printf("time-gen seconds=%.6f walks=%zu L=%d workers=%d\n", s,
                            g_n * (size_t)config::walks_per_vertex, (int)config::walk_length, (int)num_workers());
                std::fflush(stdout);
            }
        } else if (c == "time-upd") {
            size_t M = std::stoull(a[i++]), seed = std::stoull(a[i++]);
            bool directed = std::stoi(a[i++]) != 0;
            int reps = std::stoi(a[i++]);
            size_t pow2 = 1ul << (pbbs::log2_up(g_n) - 1);
            for (int r = 0; r < reps; r++) {
                auto b = utility::generate_batch_of_edges(M, g_n, seed + r, false, directed);
                auto t0 = std::chrono::steady_clock::now();
                auto aff = g_w->insert_edges_batch(b.second, b.first, false, true, pow2);
                double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::printf("time-upd seconds=%.6f edges=%zu affected=%zu workers=%d\n", s, b.second, aff.size(),
                            (int)num_workers());
                std::fflush(stdout);
                pbbs::free_array(b.first);
            }
        } else if (c == "kat") {
            do_kat();
        } else if (c == "batch") {
            size_t M = std::stoull(a[i++]), V = std::stoull(a[i++]), seed = std::stoull(a[i++]);
            bool directed = std::stoi(a[i++]) != 0;
            auto b = utility::generate_batch_of_edges(M, V, seed, false, directed);
            dump_batch("gen_" + std::to_string(M) + "_" + std::to_string(V) + "_" + std::to_string(seed) + "_" + std::to_string(directed), b.first, b.second);
            pbbs::free_array(b.first);
        } else {
            std::fprintf(stderr, "unknown command %s\n", c.c_str());
            return 2;
        }
    }
    return 0;
}
