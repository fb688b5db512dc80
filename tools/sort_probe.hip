// Probe of the rocPRIM radix sort the node2vec re-walk list's global order uses
// (wharf_api.hip walk_update, WHARF_N2V_LIST_ORDER=global): entries
// {li | p << 56} sorted by their top 8 bits only (begin_bit 56, end_bit 64).
// Checks that the output is a permutation of the input (every entry once) and
// ascending in the point, for several sizes, against a full-width sort and a
// pairs sort keyed by the point byte.  Prints one JSON line per case.
//   tools/sort_probe
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHK(x)                                                                       \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void k_point_of(const uint64_t* in, size_t n, uint8_t* key)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        key[i] = (uint8_t)(in[i] >> 56);
}

static int check(const char* what, size_t n, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
                 uint64_t W)
{
    std::vector<uint64_t> a(in), b(out);
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    size_t bad_range = 0, unsorted = 0, first_bad = ~0ull;
    for (size_t i = 0; i < n; i++) {
        if ((out[i] & ((1ull << 56) - 1)) >= W || (out[i] >> 56) >= 80) {
            bad_range++;
            if (first_bad == ~0ull) first_bad = i;
        }
        if (i && (out[i] >> 56) < (out[i - 1] >> 56)) unsorted++;
    }
    const bool perm = a == b;
    std::printf("{\"case\": \"%s\", \"n\": %zu, \"permutation\": %s, \"out_of_range\": %zu, \"first_bad_index\": %lld, "
                "\"first_bad_value\": \"0x%016llx\", \"descents\": %zu}\n",
                what, n, perm ? "true" : "false", bad_range, first_bad == ~0ull ? -1ll : (long long)first_bad,
                first_bad == ~0ull ? 0ull : (unsigned long long)out[first_bad], unsorted);
    return perm && !bad_range && !unsorted ? 0 : 1;
}

// keys sorted on bits [b0, b1) only must come out as a permutation of the input,
// ascending in those bits
static int check_bits(const char* what, int b0, int b1, size_t n, const std::vector<uint64_t>& in,
                      const std::vector<uint64_t>& out)
{
    std::vector<uint64_t> a(in), b(out);
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    const uint64_t mask = (b1 - b0 == 64) ? ~0ull : ((1ull << (b1 - b0)) - 1);
    size_t descents = 0;
    for (size_t i = 1; i < n; i++)
        if (((out[i] >> b0) & mask) < ((out[i - 1] >> b0) & mask)) descents++;
    const bool perm = a == b;
    std::printf("{\"case\": \"%s\", \"bits\": [%d, %d], \"n\": %zu, \"permutation\": %s, \"descents\": %zu}\n", what, b0,
                b1, n, perm ? "true" : "false", descents);
    return perm && !descents ? 0 : 1;
}

int main()
{
    int fails = 0;
    std::mt19937_64 rng(7);
    // 1. the list order of round 3: entries {li | p << 56} by their top byte, keys only, against a
    //    full-width sort and a pairs sort keyed by the point byte
    for (size_t n : {1ul, 100ul, 3000ul, 12288ul, 100000ul, 1ul << 20, 13000000ul}) {
        const uint64_t W = n * 3 + 5;
        std::vector<uint64_t> h(n);
        for (auto& x : h) x = (rng() % W) | ((rng() % 79) << 56);
        uint64_t *din, *dout;
        uint8_t *k1, *k2;
        CHK(hipMalloc(&din, n * 8));
        CHK(hipMalloc(&dout, n * 8));
        CHK(hipMalloc(&k1, n));
        CHK(hipMalloc(&k2, n));
        std::vector<uint64_t> o(n);
        for (int mode = 0; mode < 3; mode++) {
            CHK(hipMemcpy(din, h.data(), n * 8, hipMemcpyHostToDevice));
            CHK(hipMemset(dout, 0xEE, n * 8));
            size_t bytes = 0;
            void* tmp = nullptr;
            if (mode == 0) {   // the list-order call: keys only, top byte
                CHK(rocprim::radix_sort_keys(nullptr, bytes, din, dout, n, 56u, 64u));
                CHK(hipMalloc(&tmp, bytes));
                CHK(rocprim::radix_sort_keys(tmp, bytes, din, dout, n, 56u, 64u));
            } else if (mode == 1) {   // full width
                CHK(rocprim::radix_sort_keys(nullptr, bytes, din, dout, n, 0u, 64u));
                CHK(hipMalloc(&tmp, bytes));
                CHK(rocprim::radix_sort_keys(tmp, bytes, din, dout, n, 0u, 64u));
            } else {   // pairs: the point byte as key, the entry as value
                hipLaunchKernelGGL(k_point_of, 1024, 256, 0, 0, din, n, k1);
                CHK(rocprim::radix_sort_pairs(nullptr, bytes, k1, k2, din, dout, n, 0u, 8u));
                CHK(hipMalloc(&tmp, bytes));
                CHK(rocprim::radix_sort_pairs(tmp, bytes, k1, k2, din, dout, n, 0u, 8u));
            }
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost));
            CHK(hipFree(tmp));
            const char* names[3] = {"keys_bits_56_64", "keys_bits_0_64", "pairs_point_byte"};
            fails += check(names[mode], n, h, o, W);
        }
        CHK(hipFree(din));
        CHK(hipFree(dout));
        CHK(hipFree(k1));
        CHK(hipFree(k2));
    }
    // 2. the bit ranges the library sorts on (begin 0: batch keys to 32 + log2 n bits, pool
    //    compaction, index export) and other begin bits, keys only, at the sizes of a batch
    int ranges[][2] = {{0, 44}, {0, 48}, {0, 56}, {0, 64}, {8, 64}, {32, 64}, {48, 64}, {56, 64}, {4, 44}};
    for (size_t n : {3000ul, 20000ul, 300000ul}) {
        for (auto& r : ranges) {
            std::vector<uint64_t> h(n);
            for (auto& x : h) x = rng() & (r[1] == 64 ? ~0ull : ((1ull << r[1]) - 1));
            uint64_t *din, *dout;
            CHK(hipMalloc(&din, n * 8));
            CHK(hipMalloc(&dout, n * 8));
            CHK(hipMemcpy(din, h.data(), n * 8, hipMemcpyHostToDevice));
            size_t bytes = 0;
            void* tmp = nullptr;
            CHK(rocprim::radix_sort_keys(nullptr, bytes, din, dout, n, (unsigned)r[0], (unsigned)r[1]));
            CHK(hipMalloc(&tmp, bytes));
            CHK(rocprim::radix_sort_keys(tmp, bytes, din, dout, n, (unsigned)r[0], (unsigned)r[1]));
            CHK(hipDeviceSynchronize());
            std::vector<uint64_t> o(n);
            CHK(hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost));
            fails += check_bits("keys_u64", r[0], r[1], n, h, o);
            CHK(hipFree(tmp));
            CHK(hipFree(din));
            CHK(hipFree(dout));
        }
    }
    std::printf("{\"fails\": %d}\n", fails);
    return fails ? 1 : 0;
}
