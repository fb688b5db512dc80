// Host IO (csrc/wharf_io.cpp) and the compat layer's host helpers
// (include/compat/wharfmh.h: commandLine, timer, pbbs::, read_unweighted_graph)
// under ASan + UBSan: well-formed, truncated and malformed AdjacencyGraph
// files, SNAP edge lists with comments / duplicates / self loops, empty and
// appended corpora.  `make -C tests/cpp sanitize` builds it from the sources
// (no GPU involved); tests/test_sanitizers.py runs it.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <wharfmh.h>   // the compat layer (include/compat)

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                     \
        }                                                                 \
    } while (0)

// the compat header's read_unweighted_graph reports errors through the
// library's wharf_last_error, which lives in the GPU part of libwharf_gpu.so
extern "C" const char* wharf_last_error(const wharf_handle*) { return "io error"; }

static std::string dir;
static std::string put(const std::string& name, const std::string& text)
{
    const std::string p = dir + "/" + name;
    std::ofstream(p) << text;
    return p;
}
static std::string slurp(const std::string& p)
{
    std::stringstream s;
    s << std::ifstream(p).rdbuf();
    return s.str();
}

int main()
{
    char tmpl[] = "/tmp/wharf_io_XXXXXX";
    dir = mkdtemp(tmpl);

    // AdjacencyGraph: size query, then contents
    const std::string g = put("g.adj", "AdjacencyGraph\n4\n5\n0\n2\n3\n5\n1\n2\n0\n3\n1\n");
    uint64_t n = 0, m = 0;
    CHECK(wharf_read_adjacency_graph(g.c_str(), &n, &m, nullptr, nullptr) == WHARF_OK && n == 4 && m == 5);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> adj(m);
    CHECK(wharf_read_adjacency_graph(g.c_str(), &n, &m, off.data(), adj.data()) == WHARF_OK);
    CHECK(off[3] == 5 && adj[4] == 1);
    // truncated, malformed, out-of-range target, missing file, empty file, no trailing newline
    for (const char* bad : {"AdjacencyGraph\n4\n5\n0\n2\n3\n", "AdjacencyGrap\n1\n0\n0\n", "AdjacencyGraph\n2\n1\n0\n1\n7\n",
                            "AdjacencyGraph\n2\n1\n0\nx\n1\n", "", "AdjacencyGraph"}) {
        const std::string p = put("bad.adj", bad);
        uint64_t nn = 0, mm = 0;
        std::vector<uint64_t> o(8);
        std::vector<uint32_t> a(8);
        const int rc = wharf_read_adjacency_graph(p.c_str(), &nn, &mm, o.data(), a.data());
        CHECK(rc == WHARF_E_INVALID);
    }
    {
        const std::string p = put("tail.adj", "AdjacencyGraph 2 1 0 1 1");   // last token at EOF
        uint64_t o[2];
        uint32_t a[1];
        CHECK(wharf_read_adjacency_graph(p.c_str(), &n, &m, o, a) == WHARF_OK && a[0] == 1);
    }
    CHECK(wharf_read_adjacency_graph((dir + "/missing").c_str(), &n, &m, nullptr, nullptr) == WHARF_E_INVALID);

    // SNAP -> AdjacencyGraph: comments, duplicates, self loop, symmetrised
    const std::string snap = put("s.txt", "# FromNodeId ToNodeId\n% other\n0 1\n1 0\n2 2\n0 3\n0 1\n");
    const std::string out = dir + "/s.adj";
    CHECK(wharf_snap_to_adj(snap.c_str(), out.c_str(), 1) == WHARF_OK);
    CHECK(slurp(out) == "AdjacencyGraph\n4\n4\n0\n2\n3\n3\n1\n3\n0\n0\n");
    CHECK(wharf_snap_to_adj(put("odd.txt", "0 1\n2\n").c_str(), out.c_str(), 1) == WHARF_E_INVALID);
    CHECK(wharf_snap_to_adj(put("empty.txt", "").c_str(), out.c_str(), 0) == WHARF_OK);
    CHECK(slurp(out) == "AdjacencyGraph\n0\n0\n");

    // corpus text: SENT-padded rows, empty corpus, append
    const uint32_t rows[6] = {3, 1, WHARF_SENTINEL, 4294967293u, 0, 2};
    const std::string c = dir + "/c.txt";
    CHECK(wharf_format_corpus(rows, 2, 3, c.c_str(), 0) == WHARF_OK);
    CHECK(wharf_format_corpus(nullptr, 0, 3, c.c_str(), 1) == WHARF_OK);
    CHECK(wharf_format_corpus(rows, 1, 3, c.c_str(), 1) == WHARF_OK);
    CHECK(slurp(c) == "3 1 \n4294967293 0 2 \n3 1 \n");
    CHECK(wharf_format_corpus(nullptr, 1, 3, c.c_str(), 0) == WHARF_E_INVALID);

    // compat helpers
    size_t gn, gm;
    uintE* goff;
    uintV* gadj;
    std::tie(gn, gm, goff, gadj) = read_unweighted_graph(g.c_str(), true);
    CHECK(gn == 4 && gm == 5 && goff[2] == 3 && gadj[0] == 1);
    pbbs::free_array(goff);
    pbbs::free_array(gadj);
    const char* argv[] = {"prog", "-f", "x.adj", "-s", "-w", "7", "-paramP", "0.25", "-det"};
    commandLine P(9, (char**)argv, "");
    CHECK(P.getOptionValue("-f", default_file_name) == "x.adj" && P.getOption("-s") && !P.getOption("-m"));
    CHECK(P.getOptionLongValue("-w", 10) == 7 && P.getOptionLongValue("-l", 80) == 80);
    CHECK(P.getOptionDoubleValue("-paramP", 4.0) == 0.25 && P.getOptionValue("-det", "true") == "true");
    CHECK(pbbs::log2_up(1) == 0 && pbbs::log2_up(2) == 1 && pbbs::log2_up(5) == 3 && pbbs::log2_up(1024) == 10);
    auto seq = pbbs::sequence<size_t>(3);
    seq[2] = 9;
    size_t* arr = seq.to_array();
    CHECK(arr[2] == 9 && seq.empty());
    pbbs::free_array(arr);
    timer t("t", false);
    t.add(0.5);
    CHECK(t.get_total() == 0.5);
    t.reset();
    CHECK(t.get_total() == 0.0);

    for (const char* f : {"g.adj", "bad.adj", "tail.adj", "s.txt", "s.adj", "odd.txt", "empty.txt", "c.txt"})
        std::remove((dir + "/" + f).c_str());
    rmdir(dir.c_str());
    if (g_fail) return 1;
    std::printf("io sanitize OK\n");
    return 0;
}
