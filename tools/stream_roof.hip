// Streaming roof on MI355X for the update path's streaming kernels: what a
// pass over a large u32 array reaches with the access shapes they use.
//
//   hipcc --offload-arch=gfx950 -O3 tools/stream_roof.hip -o tools/stream_roof && tools/stream_roof
//
//   sum      16-B loads per lane, grid-strided (U loads in flight per lane), XOR-reduced
//   bloom    the same with the batch-source Bloom test of every element (LDS,
//            k_patch_in_edges / scan_chunk): one LDS read + compare per element
//   copy     16-B loads and stores (the det re-walk copy's byte budget)
//   rows16   position-major [80][W] matrix, one lane per walk, 16 rows of a
//            chunk loaded per round trip (k_rewalk_chunked<false>'s shape)
//   rows16x  the same with k_rewalk_chunked's XCD-partitioned walk ranges
//   scan16   rows16x + the rewalk-point scan: Bloom test per position (LDS),
//            exact bitmap for positives, a lane stops at its first source
//            (~2.5 % of positions hold one of 10 k sources), the wave stops
//            when all its lanes did
// Each line: GB/s over the bytes moved, for workgroups-per-CU x U x non-temporal.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                   \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kWords = 4096;

__device__ __forceinline__ uint32_t bword(uint32_t x) { return (x * 2654435761u) >> 20; }
__device__ __forceinline__ uint32_t bbits(uint32_t x)
{
    const uint32_t h = (x ^ 0x5bd1e995u) * 0x9E3779B1u + 0x7f4a7c15u;
    return (1u << (h >> 27)) | (1u << ((h >> 22) & 31u));
}

__global__ void k_init(uint32_t* a, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = (uint32_t)((i * 0x9E3779B97F4A7C15ull) >> 40);   // vertex-like ids < 2^24
}

template <int U, bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int U, bool NT, bool BLOOM>
__global__ __launch_bounds__(256) void k_read(const uint32_t* __restrict__ a, uint64_t n, const uint32_t* __restrict__ f,
                                              uint32_t* __restrict__ out)
{
    __shared__ uint32_t s[kWords];
    if (BLOOM) {
        for (uint32_t i = threadIdx.x; i < kWords; i += blockDim.x) s[i] = f[i];
        __syncthreads();
    }
    const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const u32x4* a4 = reinterpret_cast<const u32x4*>(a);
    uint32_t acc = 0;
    for (uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += stride * U) {
        u32x4 t[U];
#pragma unroll
        for (int u = 0; u < U; u++) t[u] = q0 + u * stride < n4 ? ld<U, NT>(a4 + q0 + u * stride) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (BLOOM) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t x = t[u][j], b = bbits(x);
                    acc += (s[bword(x)] & b) == b;
                }
            } else {
                acc ^= t[u].x ^ t[u].y ^ t[u].z ^ t[u].w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads alive
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint32_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ b)
{
    const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const u32x4* a4 = reinterpret_cast<const u32x4*>(a);
    u32x4* b4 = reinterpret_cast<u32x4*>(b);
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
        const u32x4 t = NT ? __builtin_nontemporal_load(a4 + q) : a4[q];
        if (NT) __builtin_nontemporal_store(t, b4 + q);
        else b4[q] = t;
    }
}

// [L][W] position-major, lane = walk, C rows per round trip
template <int C, bool NT>
__global__ __launch_bounds__(256) void k_rows(const uint32_t* __restrict__ a, uint64_t W, uint32_t L,
                                              uint32_t* __restrict__ out)
{
    uint32_t acc = 0;
    for (uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; li < W; li += (uint64_t)gridDim.x * blockDim.x) {
        for (uint32_t c0 = 0; c0 < L; c0 += C) {
            uint32_t x[C];
#pragma unroll
            for (int j = 0; j < C; j++)
                x[j] = c0 + j < L ? (NT ? __builtin_nontemporal_load(a + (uint64_t)(c0 + j) * W + li)
                                        : a[(uint64_t)(c0 + j) * W + li])
                                  : 0u;
#pragma unroll
            for (int j = 0; j < C; j++) acc ^= x[j];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

struct Xr { uint64_t first, end, stride; };
__device__ __forceinline__ Xr xcd_range(uint64_t W)
{
    const uint32_t xcd = blockIdx.x % 8, slot = blockIdx.x / 8, per = gridDim.x / 8;
    const uint64_t part = (((W + 7) / 8) + 255) & ~255ull;
    const uint64_t c0 = min(W, (uint64_t)xcd * part);
    return {c0 + (uint64_t)slot * blockDim.x + threadIdx.x, min(W, c0 + part), (uint64_t)per * blockDim.x};
}

template <int C>
__global__ __launch_bounds__(256) void k_rows_x(const uint32_t* __restrict__ a, uint64_t W, uint32_t L,
                                                uint32_t* __restrict__ out)
{
    uint32_t acc = 0;
    const Xr xr = xcd_range(W);
    for (uint64_t li = xr.first; li < xr.end; li += xr.stride) {
        for (uint32_t c0 = 0; c0 < L; c0 += C) {
            uint32_t x[C];
#pragma unroll
            for (int j = 0; j < C; j++)
                x[j] = c0 + j < L ? __builtin_nontemporal_load(a + (uint64_t)(c0 + j) * W + li) : 0u;
#pragma unroll
            for (int j = 0; j < C; j++) acc ^= x[j];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// the walk matrix of the scan: ~2.5 % of positions hold one of 10 k source ids
__device__ __forceinline__ uint32_t srcid(uint32_t k) { return (k * 1637u) & 0xFFFFFFu; }
__global__ void k_init_scan(uint32_t* a, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h = (uint32_t)((i * 0x9E3779B97F4A7C15ull) >> 32);
        a[i] = h % 40 == 0 ? srcid(h % 10000) : ((h >> 8) | 1u) & 0xFFFFFFu;
    }
}
__global__ void k_init_filters(uint32_t* bitmap, uint32_t* bloom)
{
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < 10000; k += gridDim.x * blockDim.x) {
        const uint32_t s = srcid(k);
        atomicOr(bitmap + (s >> 5), 1u << (s & 31));
        const uint32_t h = __umul24(s ^ (s >> 15), 0x9E3779u);
        atomicOr(bloom + (h >> 20), (1u << ((h >> 13) & 31u)) | (1u << ((h >> 8) & 31u)));
    }
}

__global__ __launch_bounds__(256) void k_scan16(const uint32_t* __restrict__ a, uint64_t W, uint32_t L,
                                                const uint32_t* __restrict__ bitmap, const uint32_t* __restrict__ bloom,
                                                uint8_t* __restrict__ aff)
{
    constexpr int C = 16;
    __shared__ uint32_t s[4096];
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) s[i] = bloom[i];
    __syncthreads();
    const Xr xr = xcd_range(W);
    for (uint64_t li = xr.first; li < xr.end; li += xr.stride) {
        uint32_t p = 0xFF;
        bool scanning = true;
        uint32_t cur[C], nxt[C];
#pragma unroll
        for (int j = 0; j < C; j++) cur[j] = __builtin_nontemporal_load(a + (uint64_t)j * W + li);
        for (uint32_t c0 = 0; c0 < L; c0 += C) {
            if (scanning) {
                uint32_t mask = 0;
#pragma unroll
                for (int j = 0; j < C; j++) {
                    const uint32_t x = cur[j], h = __umul24(x ^ (x >> 15), 0x9E3779u);
                    const uint32_t b = (1u << ((h >> 13) & 31u)) | (1u << ((h >> 8) & 31u));
                    mask |= (uint32_t)((s[h >> 20] & b) == b) << j;
                }
                while (mask) {
                    const uint32_t j = (uint32_t)__builtin_ctz(mask);
                    uint32_t v = 0;
#pragma unroll
                    for (int i = 0; i < C; i++) v |= cur[i] & (0u - (uint32_t)(j == (uint32_t)i));
                    if ((bitmap[v >> 5] >> (v & 31)) & 1u) { p = c0 + j; scanning = false; break; }
                    mask &= mask - 1u;
                }
            }
            const bool more = c0 + C < L;
            if (more && scanning) {
#pragma unroll
                for (int j = 0; j < C; j++)
                    nxt[j] = c0 + C + j < L ? __builtin_nontemporal_load(a + (uint64_t)(c0 + C + j) * W + li) : 0u;
            }
            if (!__any(scanning)) break;
            if (more && scanning) {
#pragma unroll
                for (int j = 0; j < C; j++) cur[j] = nxt[j];
            }
        }
        aff[li] = (uint8_t)p;
    }
}

int main(int argc, char** argv)
{
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2560000000ull;   // configs[3] pool slots
    const uint64_t W = 41943040;
    const uint32_t L = 80;
    uint32_t *a, *b, *f, *out;
    CHK(hipMalloc(&a, n * 4));
    CHK(hipMalloc(&b, W * L * 4 > n * 4 ? W * L * 4 : n * 4));
    CHK(hipMalloc(&f, kWords * 4));
    CHK(hipMalloc(&out, 64));
    hipLaunchKernelGGL(k_init, 4096, 256, 0, 0, a, n);
    hipLaunchKernelGGL(k_init, 4096, 256, 0, 0, b, W * L);
    CHK(hipMemset(f, 0x11, kWords * 4));   // ~12 % of bits set (a 10 k-source filter has ~14 %)
    CHK(hipDeviceSynchronize());
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto time = [&](const char* what, int bpc, int u, int nt, double bytes, auto launch) {
        float best = 1e30f, first = 0;
        for (int rep = 0; rep < 3; rep++) {
            // between launches, touch 4 GB elsewhere (as the update pipeline does), so
            // the first timed launch also meets cold TLBs and caches
            if (rep == 0) hipLaunchKernelGGL(k_init, 4096, 256, 0, 0, a, (uint64_t)1 << 30);
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 0) first = ms;
            if (ms < best) best = ms;
        }
        std::printf("{\"kernel\": \"%s\", \"wg_per_cu\": %d, \"U\": %d, \"nt\": %d, \"ms\": %.3f, \"GBps\": %.1f, "
                    "\"first_ms\": %.3f}\n", what, bpc, u, nt, best, bytes / best / 1e6, first);
    };
    {
        uint32_t *bm, *bl;
        uint8_t* aff;
        CHK(hipMalloc(&bm, (1u << 24) / 8));
        CHK(hipMalloc(&bl, 4096 * 4));
        CHK(hipMalloc(&aff, W));
        CHK(hipMemset(bm, 0, (1u << 24) / 8));
        CHK(hipMemset(bl, 0, 4096 * 4));
        hipLaunchKernelGGL(k_init_filters, 40, 256, 0, 0, bm, bl);
        for (int bpc : {8, 16}) {
            const unsigned g = (unsigned)(cus * bpc);
            hipLaunchKernelGGL(k_init, 4096, 256, 0, 0, b, W * L);
            CHK(hipDeviceSynchronize());
            time("rows16", bpc, 16, 1, W * L * 4.0, [&] { hipLaunchKernelGGL((k_rows<16, true>), g, 256, 0, 0, b, W, L, out); });
            time("rows16x", bpc, 16, 1, W * L * 4.0, [&] { hipLaunchKernelGGL((k_rows_x<16>), g, 256, 0, 0, b, W, L, out); });
            hipLaunchKernelGGL(k_init_scan, 4096, 256, 0, 0, b, W * L);
            CHK(hipDeviceSynchronize());
            time("scan16 (matrix bytes)", bpc, 16, 1, W * L * 4.0,
                 [&] { hipLaunchKernelGGL(k_scan16, g, 256, 0, 0, b, W, L, bm, bl, aff); });
        }
        if (argc > 2) return 0;   // scan shapes only
    }
    for (int bpc : {4, 8, 16, 32}) {
        const unsigned g = (unsigned)(cus * bpc);
#define READ(U, NT, BL)                                                                                   \
    time(BL ? "bloom" : "sum", bpc, U, NT, n * 4.0,                                                       \
         [&] { hipLaunchKernelGGL((k_read<U, NT, BL>), g, 256, 0, 0, a, n, f, out); })
        READ(1, true, false); READ(2, true, false); READ(4, true, false); READ(1, false, false); READ(4, false, false);
        READ(1, true, true); READ(2, true, true); READ(4, true, true); READ(1, false, true);
        time("copy", bpc, 1, 1, n * 8.0, [&] { hipLaunchKernelGGL(k_copy<true>, g, 256, 0, 0, a, n, b); });
        time("copy", bpc, 1, 0, n * 8.0, [&] { hipLaunchKernelGGL(k_copy<false>, g, 256, 0, 0, a, n, b); });
        time("rows16", bpc, 16, 1, W * L * 4.0, [&] { hipLaunchKernelGGL((k_rows<16, true>), g, 256, 0, 0, b, W, L, out); });
        time("rows16", bpc, 16, 0, W * L * 4.0, [&] { hipLaunchKernelGGL((k_rows<16, false>), g, 256, 0, 0, b, W, L, out); });
        time("rows8", bpc, 8, 1, W * L * 4.0, [&] { hipLaunchKernelGGL((k_rows<8, true>), g, 256, 0, 0, b, W, L, out); });
    }
    return 0;
}
