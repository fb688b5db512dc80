// Host-side graph and corpus IO of the walk engine:
//   - Ligra AdjacencyGraph text reader (libs/compressed_trees/common/IO.h:67-106),
//   - SNAP edge list -> AdjacencyGraph converter (replaces the prebuilt
//     experiments/bin/SNAPtoAdj: symmetrise, sort, drop duplicates and self loops),
//   - the yskip text corpus writer (vertex-classification.cpp:142-150,
//     WharfMH::walk format wharfmh.h:365-394: "v0 v1 ... \n").
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "wharf_gpu.h"

namespace wharf_io {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    explicit Mapped(const char* path)
    {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return;
        struct stat st;
        if (fstat(fd, &st) != 0) return;
        n = (size_t)st.st_size;
        if (n) {
            void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            p = m == MAP_FAILED ? nullptr : (const char*)m;
        }
    }
    ~Mapped()
    {
        if (p) munmap((void*)p, n);
        if (fd >= 0) ::close(fd);
    }
    bool ok() const { return fd >= 0 && (p || n == 0); }
};

// whitespace-separated unsigned tokens; '#' / '%' start a comment line (SNAP headers)
struct Tokens {
    const char* p;
    const char* e;
    Tokens(const char* b, size_t n) : p(b), e(b + n) {}
    bool next(uint64_t& v)
    {
        for (;;) {
            while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
            if (p < e && (*p == '#' || *p == '%')) {
                while (p < e && *p != '\n') p++;
                continue;
            }
            break;
        }
        if (p >= e || *p < '0' || *p > '9') return false;
        uint64_t x = 0;
        while (p < e && *p >= '0' && *p <= '9') x = x * 10 + (uint64_t)(*p++ - '0');
        v = x;
        return true;
    }
    bool word(const char* w)
    {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
        const size_t l = std::strlen(w);
        if ((size_t)(e - p) < l || std::memcmp(p, w, l) != 0) return false;
        p += l;
        return true;
    }
};

static char* utoa(char* o, uint32_t v)
{
    char t[12];
    int k = 0;
    do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) *o++ = t[--k];
    return o;
}

}  // namespace wharf_io

using namespace wharf_io;

extern "C" {

int wharf_read_adjacency_graph(const char* path, uint64_t* n_out, uint64_t* m_out, uint64_t* offsets, uint32_t* targets)
{
    if (!path || !n_out || !m_out) return WHARF_E_INVALID;
    Mapped f(path);
    if (!f.ok()) return WHARF_E_INVALID;
    Tokens t(f.p, f.n);
    uint64_t n = 0, m = 0;
    if (!t.word("AdjacencyGraph") || !t.next(n) || !t.next(m)) return WHARF_E_INVALID;   // IO.h:86-90
    *n_out = n;
    *m_out = m;
    if (!offsets) return WHARF_OK;   // size query
    for (uint64_t i = 0; i < n; i++)
        if (!t.next(offsets[i])) return WHARF_E_INVALID;
    for (uint64_t i = 0; i < m; i++) {
        uint64_t x;
        if (!t.next(x) || x >= n) return WHARF_E_INVALID;
        targets[i] = (uint32_t)x;
    }
    return WHARF_OK;
}

int wharf_snap_to_adj(const char* snap_path, const char* adj_path, int symmetric)
{
    if (!snap_path || !adj_path) return WHARF_E_INVALID;
    Mapped f(snap_path);
    if (!f.ok()) return WHARF_E_INVALID;
    Tokens t(f.p, f.n);
    std::vector<uint64_t> e;
    uint64_t a, b, n = 0;
    while (t.next(a)) {
        if (!t.next(b)) return WHARF_E_INVALID;
        if (a > 0xFFFFFFFDull || b > 0xFFFFFFFDull) return WHARF_E_INVALID;
        n = std::max(n, std::max(a, b) + 1);
        if (a == b) continue;
        e.push_back(a << 32 | b);
        if (symmetric) e.push_back(b << 32 | a);
    }
    std::sort(e.begin(), e.end());
    e.erase(std::unique(e.begin(), e.end()), e.end());
    FILE* o = std::fopen(adj_path, "w");
    if (!o) return WHARF_E_INVALID;
    std::fprintf(o, "AdjacencyGraph\n%llu\n%llu\n", (unsigned long long)n, (unsigned long long)e.size());
    std::vector<char> buf(1 << 20);
    size_t at = 0;
    auto flush = [&] {
        std::fwrite(buf.data(), 1, at, o);
        at = 0;
    };
    uint64_t j = 0;
    for (uint64_t v = 0; v < n; v++) {
        while (j < e.size() && (e[j] >> 32) < v) j++;
        if (at + 24 > buf.size()) flush();
        at += std::snprintf(buf.data() + at, 24, "%llu\n", (unsigned long long)j);
    }
    for (uint64_t k = 0; k < e.size(); k++) {
        if (at + 16 > buf.size()) flush();
        char* q = utoa(buf.data() + at, (uint32_t)e[k]);
        *q++ = '\n';
        at = (size_t)(q - buf.data());
    }
    flush();
    return std::fclose(o) == 0 ? WHARF_OK : WHARF_E_INVALID;
}

// Corpus text: walk-major rows (SENT-padded) -> "v0 v1 ... \n" per walk.
int wharf_format_corpus(const uint32_t* rows, uint64_t count, uint32_t L, const char* path, int append)
{
    if (!path || (count && !rows)) return WHARF_E_INVALID;
    FILE* o = std::fopen(path, append ? "a" : "w");
    if (!o) return WHARF_E_INVALID;
    const uint64_t chunk = 1 << 16;
    std::vector<char> buf(chunk * (size_t)L * 11 + chunk);
    for (uint64_t c0 = 0; c0 < count; c0 += chunk) {
        const uint64_t c1 = std::min(count, c0 + chunk);
        char* q = buf.data();
        for (uint64_t w = c0; w < c1; w++) {
            const uint32_t* r = rows + w * L;
            for (uint32_t pos = 0; pos < L && r[pos] != WHARF_SENTINEL; pos++) {
                q = utoa(q, r[pos]);
                *q++ = ' ';
            }
            *q++ = '\n';
        }
        if (std::fwrite(buf.data(), 1, (size_t)(q - buf.data()), o) != (size_t)(q - buf.data())) {
            std::fclose(o);
            return WHARF_E_INVALID;
        }
    }
    return std::fclose(o) == 0 ? WHARF_OK : WHARF_E_INVALID;
}

}  // extern "C"
