// Corpus readout through the C ABI, the way the reference's own exporter does it:
// WharfMH::walk(i) once per walk, in order (experiments/src/vertex-classification.cpp:145-148).
// Times wharf_walk_string over the first `n_old` walks with a device read per call
// (WHARF_WALK_NO_SNAPSHOT=1, round 2's path) and over the first `n_new` walks through
// the host snapshot, on configs[1]'s graph (RMAT scale 22, 117 M samples, wpv 10, L 80).
// Then the reference's incremental pattern (vertex-classification.cpp:171-176):
// after an insert batch of the throughput driver's sizes (5 / 50 / 500 directed
// edges between low-degree vertices, throughput-latency.cpp:87-93), walk(i) of
// the affected walks only.  Every mode reads the SAME batch's affected walks
// (round 5: each mode gets a fresh handle over the same graph, generation and
// batch, so the update and its affected set are identical): the default (all
// the update's affected rows gathered with one list gather on the first read of
// one of them, round 4), without that stage (WHARF_WALK_NO_STAGE=1: the snapshot
// chunk taken once 32 of its walks were read, single rows before), the chunk
// taken on the first read (+ WHARF_WALK_FILL_AFTER=0, round 3), and a device
// read per call (WHARF_WALK_NO_SNAPSHOT=1).
//
//   tools/walk_readout [n_old=20000] [n_new=41943040]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "wharf_gpu.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv)
{
    const uint64_t n_old = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000;
    uint64_t n_new = argc > 2 ? strtoull(argv[2], nullptr, 10) : 41943040;
    wharf_config cfg;
    wharf_config_default(&cfg);
    cfg.deterministic = 0;
    cfg.model = WHARF_DEEPWALK;   // configs[1]'s model (the default is globals.h's NODE2VEC)
    wharf_handle* h = nullptr;
    const uint64_t n = 1ull << 22;
    if (wharf_create_rmat(&cfg, n, 117185083, 2 * n, 2, 0.5, 0.2, 0.1, 0, &h) || wharf_generate(h)) {
        fprintf(stderr, "setup failed: %s\n", wharf_last_error(h));
        return 1;
    }
    uint64_t W = 0;
    wharf_shard(h, nullptr, nullptr, &W);
    if (n_new > W) n_new = W;
    std::vector<char> buf(80 * 11 + 1);
    size_t len = 0, total = 0;
    setenv("WHARF_WALK_NO_SNAPSHOT", "1", 1);
    double t0 = now();
    for (uint64_t i = 0; i < n_old; i++) {
        if (wharf_walk_string(h, i, buf.data(), buf.size(), &len)) return 2;
        total += len;
    }
    const double t_old = now() - t0;
    printf("per-call device reads: %llu walks in %.3f s\n", (unsigned long long)n_old, t_old);
    fflush(stdout);
    unsetenv("WHARF_WALK_NO_SNAPSHOT");
    t0 = now();
    for (uint64_t i = 0; i < n_new; i++) {
        if (wharf_walk_string(h, i, buf.data(), buf.size(), &len)) return 3;
        total += len;
    }
    const double t_new = now() - t0;
    printf("host snapshot: %llu walks in %.3f s\n", (unsigned long long)n_new, t_new);
    fflush(stdout);
    wharf_destroy(h);
    h = nullptr;
    // sparse: the affected walks of small batches, every mode on the same batch
    std::vector<uint32_t> aff(W), pairs;
    std::string sparse = "[";
    const char* modes[4] = {"default_stage", "no_stage_fill_after_32", "no_stage_fill_on_first_read",
                            "device_read_per_call"};
    for (uint64_t bs : {5ull, 50ull, 500ull}) {
        std::string rec = "{\"batch_edges\": " + std::to_string(bs);
        // edges between low-degree vertices (RMAT's upper id half), so the affected walks are a
        // sparse set: an RMAT batch of any size touches hubs that most walks visit
        pairs.assign(2 * bs, 0);
        uint64_t x = 88172645463325252ull + bs * 7;
        for (uint64_t i = 0; i < 2 * bs; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            pairs[i] = (uint32_t)(n / 2 + x % (n / 2));
        }
        uint64_t naff_first = 0;
        for (int m = 0; m < 4; m++) {
            wharf_handle* hm = nullptr;
            uint64_t naff = 0;
            std::vector<uint32_t> p(pairs);   // the call may reorder its input
            if (wharf_create_rmat(&cfg, n, 117185083, 2 * n, 2, 0.5, 0.2, 0.1, 0, &hm) || wharf_generate(hm) ||
                wharf_insert_edges(hm, bs, p.data(), WHARF_REMOVE_DUPS | WHARF_APPLY_WALK_UPDATES, aff.data(), &naff)) {
                fprintf(stderr, "sparse setup failed: %s\n", wharf_last_error(hm));
                return 4;
            }
            if (m == 0) naff_first = naff;
            if (naff != naff_first) {   // same graph, generation and batch: the same affected walks
                fprintf(stderr, "mode %s: %llu affected walks, first mode %llu\n", modes[m], (unsigned long long)naff,
                        (unsigned long long)naff_first);
                return 5;
            }
            if (m >= 1) setenv("WHARF_WALK_NO_STAGE", "1", 1);
            if (m == 2) setenv("WHARF_WALK_FILL_AFTER", "0", 1);
            if (m == 3) setenv("WHARF_WALK_NO_SNAPSHOT", "1", 1);
            t0 = now();
            for (uint64_t i = 0; i < naff; i++) {
                if (wharf_walk_string(hm, aff[i], buf.data(), buf.size(), &len)) return 6;
                total += len;
            }
            const double t = now() - t0;
            unsetenv("WHARF_WALK_NO_STAGE");
            unsetenv("WHARF_WALK_FILL_AFTER");
            unsetenv("WHARF_WALK_NO_SNAPSHOT");
            wharf_destroy(hm);
            char part[200];
            snprintf(part, sizeof part, ", \"%s\": {\"affected\": %llu, \"ms\": %.3f, \"us_per_walk\": %.3f}",
                     modes[m], (unsigned long long)naff, 1e3 * t, naff ? 1e6 * t / naff : 0.0);
            rec += part;
            printf("batch of %llu edges, %s: %llu affected walks read in %.3f ms\n", (unsigned long long)bs, modes[m],
                   (unsigned long long)naff, 1e3 * t);
            fflush(stdout);
        }
        sparse += (sparse.size() > 1 ? ", " : "") + rec + "}";
    }
    sparse += "]";
    printf("{\"walks\": %llu, \"per_call_device_read\": {\"calls\": %llu, \"seconds\": %.3f, \"us_per_call\": %.2f, "
           "\"all_walks_seconds_extrapolated\": %.1f}, \"host_snapshot\": {\"calls\": %llu, \"seconds\": %.3f, "
           "\"us_per_call\": %.3f, \"all_walks_seconds\": %.1f}, \"affected_walks_of_small_batches\": %s, \"chars\": %zu}\n",
           (unsigned long long)W, (unsigned long long)n_old, t_old, 1e6 * t_old / n_old, t_old / n_old * W,
           (unsigned long long)n_new, t_new, 1e6 * t_new / n_new, t_new / n_new * W, sparse.c_str(), total);
    return 0;
}
