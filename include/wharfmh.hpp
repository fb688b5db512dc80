// wharfmh.hpp — header-only C++17 mirror of dygrl::WharfMH (graph/wharfmh.h)
// over the C ABI of include/wharf_gpu.h.
//
// Drop-in for driver code of the reference (experiments/src/*.cpp,
// tests/wharfmh.cpp): same class shape, method names and argument order.
//
//     #include <wharfmh.hpp>                       // instead of <wharfmh.h>
//     wharf::WharfMH w(n, m, offsets, edges);      // dygrl::WharfMH(n, m, offsets, edges)
//     w.generate_initial_random_walks();
//     auto affected = w.insert_edges_batch(m_b, batch, false, true, nn);
//
// The reference's mutable globals (config::walks_per_vertex, walk_length,
// random_walk_model, paramP, paramQ, sampler_init_strategy, deterministic_mode)
// are read from wharf::config at construction, like the reference reads its
// globals at each call.  Errors throw wharf::Error (the reference exits).
#pragma once

#include <algorithm>
#include <cstdint>
#include <iostream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "wharf_gpu.h"

namespace wharf {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc, const wharf_handle* h, const char* what)
{
    if (rc != WHARF_OK) throw Error(rc, std::string(what) + ": " + wharf_last_error(h));
}

// config::* (config/globals.h:7-29); edit before constructing a WharfMH.
inline wharf_config& config()
{
    static wharf_config c = [] {
        wharf_config d;
        wharf_config_default(&d);
        return d;
    }();
    return c;
}

class WharfMH {
public:
    using Edge = std::tuple<uint32_t, uint32_t>;

    // WharfMH(long n, long m) (wharfmh.h:26): n isolated vertices
    WharfMH(long graph_vertices, long graph_edges, int device = 0)
    {
        (void)graph_edges;
        check(wharf_create_empty(&config(), (uint64_t)graph_vertices, device, &h_), nullptr, "WharfMH");
    }

    // WharfMH(long n, long m, uintE* offsets, uintV* edges, bool free_memory) (wharfmh.h:58).
    // The arrays are copied and the caller keeps ownership here; free_memory is
    // accepted for source compatibility.  include/compat/wharfmh.h's
    // dygrl::WharfMH takes ownership and frees them, as the reference does
    // with pbbs::free_array (wharfmh.h:99-103).
    WharfMH(long graph_vertices, long graph_edges, const uint64_t* offsets, const uint32_t* edges,
            bool free_memory = true, int device = 0)
    {
        (void)free_memory;
        check(wharf_create(&config(), (uint64_t)graph_vertices, (uint64_t)graph_edges, offsets, edges, device, &h_),
              nullptr, "WharfMH");
    }

    WharfMH(const WharfMH&) = delete;
    WharfMH& operator=(const WharfMH&) = delete;
    WharfMH(WharfMH&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    ~WharfMH() { destroy(); }

    // number_of_vertices / number_of_edges (wharfmh.h:117-133)
    size_t number_of_vertices() const
    {
        uint64_t n = 0;
        if (h_) check(wharf_number_of_vertices(h_, &n), h_, "number_of_vertices");
        return n;
    }
    size_t number_of_edges() const
    {
        uint64_t m = 0;
        if (h_) check(wharf_number_of_edges(h_, &m), h_, "number_of_edges");
        return m;
    }

    // generate_initial_random_walks (wharfmh.h:250)
    void generate_initial_random_walks() { check(wharf_generate(h_), h_, "generate_initial_random_walks"); }

    // insert_edges_batch / delete_edges_batch (wharfmh.h:439, 588).  Like the
    // reference, an unsorted batch is sorted by source in the caller's buffer.
    std::vector<uint32_t> insert_edges_batch(size_t m, Edge* edges, bool sorted = false, bool remove_dups = false,
                                             size_t nn = SIZE_MAX, bool apply_walk_updates = true,
                                             bool run_seq = false)
    {
        return update(true, m, edges, sorted, remove_dups, nn, apply_walk_updates, run_seq);
    }
    std::vector<uint32_t> delete_edges_batch(size_t m, Edge* edges, bool sorted = false, bool remove_dups = false,
                                             size_t nn = SIZE_MAX, bool apply_walk_updates = true,
                                             bool run_seq = false)
    {
        return update(false, m, edges, sorted, remove_dups, nn, apply_walk_updates, run_seq);
    }

    // batch_walk_update (wharfmh.h:733) over a vertex set (wharf_batch_walk_update)
    std::vector<uint32_t> batch_walk_update(const std::vector<uint32_t>& sources)
    {
        uint64_t walks = 0;
        check(wharf_shard(h_, nullptr, nullptr, &walks), h_, "shard");
        std::vector<uint32_t> affected(std::max<uint64_t>(walks, 1));
        uint64_t na = 0;
        check(wharf_batch_walk_update(h_, sources.data(), sources.size(), 0, affected.data(), &na), h_,
              "batch_walk_update");
        affected.resize(na);
        return affected;
    }

    // walk (wharfmh.h:365): "v0 v1 ... " with a trailing space
    std::string walk(uint32_t walk_id)
    {
        size_t len = 0;
        check(wharf_walk_string(h_, walk_id, nullptr, 0, &len), h_, "walk");
        std::string s(len + 1, '\0');
        check(wharf_walk_string(h_, walk_id, &s[0], s.size(), &len), h_, "walk");
        s.resize(len);
        return s;
    }

    // vertex_at_walk (wharfmh.h:404)
    uint32_t vertex_at_walk(uint32_t walk_id, uint32_t position)
    {
        uint32_t v = 0;
        check(wharf_vertex_at_walk(h_, walk_id, position, &v), h_, "vertex_at_walk");
        return v;
    }

    // flatten_graph (wharfmh.h:175) as CSR: offsets (n+1), targets (m)
    void flatten_graph(std::vector<uint64_t>& offsets, std::vector<uint32_t>& targets)
    {
        offsets.resize(number_of_vertices() + 1);
        targets.resize(number_of_edges());
        check(wharf_get_graph(h_, offsets.data(), targets.data()), h_, "flatten_graph");
    }

    // inverted index (walks/inverted_index.h): per-vertex counts, (key, next)
    void inverted_index(std::vector<uint64_t>& counts, std::vector<uint64_t>& keys, std::vector<uint32_t>& nexts)
    {
        uint64_t sz = 0;
        check(wharf_index_size(h_, &sz), h_, "index_size");
        counts.resize(number_of_vertices());
        keys.resize(sz);
        nexts.resize(sz);
        check(wharf_export_index(h_, counts.data(), keys.data(), nexts.data()), h_, "export_index");
    }

    // the pairing-encoded CompressedWalks form (walks/compressed_walks.h): per vertex,
    // Szudzik(wid * L + pos, next) ascending, 64-bit
    void compressed_walks(std::vector<uint64_t>& counts, std::vector<uint64_t>& paired)
    {
        uint64_t sz = 0;
        check(wharf_index_size(h_, &sz), h_, "index_size");
        counts.resize(number_of_vertices());
        paired.resize(sz);
        check(wharf_export_index_paired(h_, counts.data(), paired.data()), h_, "export_index_paired");
    }

    // destroy / destroy_index (wharfmh.h:228, 237)
    void destroy()
    {
        if (h_) wharf_destroy(h_);
        h_ = nullptr;
    }
    void destroy_index() { check(wharf_destroy_index(h_), h_, "destroy_index"); }

    wharf_stats stats() const
    {
        wharf_stats s{};
        check(wharf_get_stats(h_, &s), h_, "stats");
        return s;
    }
    // WharfMH::memory_footprint (wharfmh.h:928-998): prints the device bytes by role
    wharf_memory memory_footprint() const
    {
        wharf_memory r{};
        check(wharf_memory_footprint(h_, &r), h_, "memory_footprint");
        auto mb = [](uint64_t b) { return std::to_string(b / 1048576.0) + " MB = " + std::to_string(b / 1073741824.0) + " GB"; };
        std::cout << "\nGraph: \n\tVertices: " << r.n << ", Edges: " << r.m << "\n"
                  << "CSR: \n\tMemory usage: " << mb(r.csr_bytes) << "\n"
                  << "Row records: \n\tMemory usage: " << mb(r.records_bytes) << "\n"
                  << "Walks: \n\tMemory usage: " << mb(r.walks_bytes) << "\n"
                  << "Samplers: \n\tMemory usage: " << mb(r.samplers_bytes) << "\n"
                  << "Edge hash: \n\tMemory usage: " << mb(r.edge_hash_bytes) << "\n"
                  << "Total memory used: \n\t" << mb(r.total_bytes) << "\n"
                  << std::endl;
        return r;
    }
    wharf_handle* handle() const { return h_; }

private:
    std::vector<uint32_t> update(bool insert, size_t m, Edge* edges, bool sorted, bool remove_dups, size_t nn,
                                 bool apply, bool run_seq)
    {
        (void)nn;
        (void)run_seq;
        if (!sorted) std::sort(edges, edges + m);   // wharfmh.h:450-453 sorts the caller's buffer
        std::vector<uint32_t> pairs(2 * m);
        for (size_t i = 0; i < m; i++) {
            pairs[2 * i] = std::get<0>(edges[i]);
            pairs[2 * i + 1] = std::get<1>(edges[i]);
        }
        uint64_t walks = 0;
        check(wharf_shard(h_, nullptr, nullptr, &walks), h_, "shard");
        std::vector<uint32_t> affected(walks);
        uint64_t na = 0;
        const uint32_t flags = (sorted ? WHARF_SORTED : 0) | (remove_dups ? WHARF_REMOVE_DUPS : 0) |
                               (apply ? WHARF_APPLY_WALK_UPDATES : 0);
        check(insert ? wharf_insert_edges(h_, m, pairs.data(), flags, affected.data(), &na)
                     : wharf_delete_edges(h_, m, pairs.data(), flags, affected.data(), &na),
              h_, insert ? "insert_edges_batch" : "delete_edges_batch");
        affected.resize(na);
        return affected;
    }

    wharf_handle* h_ = nullptr;
};

}  // namespace wharf
