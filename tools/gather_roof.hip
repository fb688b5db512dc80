// Random-gather roof on MI355X: the ceiling the walk kernel is judged against.
//
//   hipcc --offload-arch=gfx950 -O3 tools/gather_roof.hip -o tools/gather_roof && tools/gather_roof [GiB [kind [mode]]]
//
// A table of 16-B records (size like the edge-record array of the com-orkut-sized
// graph, 3.7 GB) is gathered at uniformly random slots, one lane per "walk",
// 79 gathers per lane, 4-B coalesced store per gather (the walk kernel's shape):
//   dep    next slot depends on the loaded record (pointer chasing, like a walk)
//   indep  slots from a counter hash (no dependency: max memory-level parallelism)
//   stream the same bytes read sequentially (HBM streaming ceiling)
//   dep_64B_block / dep_128B_block: each gather reads the whole aligned 64-B /
//   128-B block around its slot (calibrates what one 16-B gather fetches)
//   dep_store2B / dep_store1B: a 2-B / 1-B store per step (does the store cost scale with bytes?)
//   dep_store_at_end: the lane's 79 steps held in VGPRs, written after its last gather
//
// Second argument: table memory kind — "coarse" (hipMalloc, default),
// "uncached" (hipDeviceMallocUncached: requests bypass L2 line fills) or
// "fine" (hipDeviceMallocFinegrained).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                   \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void k_init(uint4* t, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        t[i] = make_uint4(mix((uint32_t)i), mix((uint32_t)i ^ 0x9e3779b9u), (uint32_t)i, 0);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ t, uint64_t n, uint32_t* __restrict__ out,
                                                uint64_t W, int L)
{
    const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= W) return;   // W is a multiple of 256: whole blocks (modes 11/12 synchronise)
    uint32_t x = mix((uint32_t)li);
    uint32_t b0 = 0, b1 = 0, b2 = 0;   // mode 8: 4-step store buffer
    __shared__ uint32_t tile[16 * 256];   // modes 11/12: 16 steps x 256 lanes staged in LDS
    uint32_t hold[MODE == 16 ? 79 : 1];   // mode 16: the walk in registers (L = 79, fully unrolled)
#pragma unroll
    for (int p = 0; p < (MODE == 16 ? 79 : L); p++) {
        uint64_t slot;
        if (MODE == 4) {                                                          // dep + Philox4x32-10 per step
            uint32_t c0 = (uint32_t)li, c1 = x, c2 = (uint32_t)p, c3 = 0, k0 = 0x5EED, k1 = 0;
#pragma unroll
            for (int rr = 0; rr < 10; rr++) {
                if (rr) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
                const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
                const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
                const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
                c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
            }
            x = c0;
        }
        if (MODE == 0 || MODE >= 4) slot = __umulhi(x, (uint32_t)n);             // dep
        else if (MODE == 1) slot = __umulhi(mix((uint32_t)(li * 131 + p)), (uint32_t)n);   // indep
        else if (MODE == 2) slot = (li + (uint64_t)p * W) % n;                    // stream
        else slot = __umulhi(x, (uint32_t)n);                                     // dep, nt load
        uint4 r;
        if (MODE == 5) {          // dep, 4-B loads anywhere in the table
            const uint32_t* t4 = reinterpret_cast<const uint32_t*>(t);
            const uint32_t q = t4[__umulhi(x, (uint32_t)n) * 4 + (x & 3)];
            r = make_uint4(q, q ^ 0x9e3779b9u, 0, 0);
        } else if (MODE == 6) {   // dep, 8-B loads
            const uint2* t2 = reinterpret_cast<const uint2*>(t);
            const uint2 q = t2[__umulhi(x, (uint32_t)n) * 2 + (x & 1)];
            r = make_uint4(q.x, q.y, 0, 0);
        } else if (MODE == 13 || MODE == 14) {   // dep, a whole 64-B / 128-B aligned block per gather
            const int k = MODE == 13 ? 4 : 8;
            const uint4* b = t + (slot & ~(uint64_t)(k - 1));
            r = b[0];
            for (int j = 1; j < k; j++) { const uint4 q = b[j]; r.x ^= q.x; r.y ^= q.y; }
        } else if (MODE == 3) {
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(t + slot));
            r = make_uint4(q.x, q.y, q.z, q.w);
        } else {
            r = t[slot];
        }
        if (MODE == 16) {         // dep, the lane's whole walk kept in VGPRs, written after its last gather
            hold[p] = r.x;   // written after the loop
        } else if (MODE == 15) {  // dep, a 2-B store per step (half the write bytes)
            reinterpret_cast<uint16_t*>(out)[(uint64_t)p * W + li] = (uint16_t)r.x;
        } else if (MODE == 17) {  // dep, a 1-B store per step
            reinterpret_cast<uint8_t*>(out)[(uint64_t)p * W + li] = (uint8_t)r.x;
        } else if (MODE == 8) {          // dep, one 16-B store per 4 steps ([p/4][W] x uint4 layout)
            if ((p & 3) == 0) b0 = r.x;
            else if ((p & 3) == 1) b1 = r.x;
            else if ((p & 3) == 2) b2 = r.x;
            else reinterpret_cast<uint4*>(out)[(uint64_t)(p >> 2) * W + li] = make_uint4(b0, b1, b2, r.x);
        } else if (MODE == 9) {   // dep, a store per step into one L2-resident row
            out[li] = r.x;
        } else if (MODE == 10) {  // dep, non-temporal store
            __builtin_nontemporal_store(r.x, out + (uint64_t)p * W + li);
        } else if (MODE == 11 || MODE == 12) {   // dep, 16 steps staged in LDS, then one burst per block
            tile[(p & 15) * 256 + threadIdx.x] = r.x;
            if ((p & 15) == 15 || p == L - 1) {
                __syncthreads();
                const int rows = (p & 15) + 1, p0 = p & ~15;
                if (MODE == 11) {   // [p/16][W][16]: the block's 16 KB chunk is contiguous
                    uint4* o = reinterpret_cast<uint4*>(out + (uint64_t)p0 * W + (uint64_t)blockIdx.x * 256 * 16);
                    for (int k = threadIdx.x; k < 256 * 4; k += 256) {
                        const int lane = k >> 2, q = (k & 3) * 4;
                        o[k] = make_uint4(tile[q * 256 + lane], tile[(q + 1) * 256 + lane], tile[(q + 2) * 256 + lane],
                                          tile[(q + 3) * 256 + lane]);
                    }
                } else {            // position-major as the walk matrix, written 16 rows at once
                    for (int k = 0; k < rows; k++)
                        out[(uint64_t)(p0 + k) * W + (uint64_t)blockIdx.x * 256 + threadIdx.x] = tile[k * 256 + threadIdx.x];
                }
                __syncthreads();
            }
        } else if (MODE != 7 || r.x == 0xFFFFFFFFu) {
            out[(uint64_t)p * W + li] = r.x;   // 7: dep without the store
        }
        x = (MODE == 0 || MODE >= 3) ? mix(r.y ^ x) : x + r.y;
    }
    if (MODE == 16) {
        __asm__ volatile("" ::: "memory");   // keep the compiler from moving the stores back between the gathers
#pragma unroll
        for (int k = 0; k < 79; k++) out[(uint64_t)k * W + li] = hold[k];
    }
}

int main(int argc, char** argv)
{
    const double gib = argc > 1 ? std::atof(argv[1]) : 3.48;
    const uint64_t n = (uint64_t)(gib * (1ull << 30) / 16);
    const uint64_t W = 41943040;
    const int L = 79;
    uint4* t;
    uint32_t* out;
    const char* kind = argc > 2 ? argv[2] : "coarse";
    const char* only = argc > 3 ? argv[3] : nullptr;   // one mode by name (bench.py: "dep")
    if (!std::strcmp(kind, "uncached")) CHK(hipExtMallocWithFlags((void**)&t, n * 16, hipDeviceMallocUncached));
    else if (!std::strcmp(kind, "fine")) CHK(hipExtMallocWithFlags((void**)&t, n * 16, hipDeviceMallocFinegrained));
    else CHK(hipMalloc(&t, n * 16));
    CHK(hipMalloc(&out, W * ((L + 15) / 16 * 16) * 4));   // mode 11 writes whole 16-step chunks
    hipLaunchKernelGGL(k_init, 4096, 256, 0, 0, t, n);
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const char* names[18] = {"dep", "indep", "stream", "dep_nt", "dep_philox", "dep_4B", "dep_8B", "dep_nostore",
                             "dep_store16B_per_4", "dep_store_same_row", "dep_store_nt",
                             "dep_store_lds16_tiled", "dep_store_lds16_rows", "dep_64B_block", "dep_128B_block",
                             "dep_store2B", "dep_store_at_end", "dep_store1B"};
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 18; mode++) {
            if (only && std::strcmp(only, names[mode]) != 0) continue;
            CHK(hipEventRecord(a));
            if (mode == 0) hipLaunchKernelGGL(k_gather<0>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 1) hipLaunchKernelGGL(k_gather<1>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 2) hipLaunchKernelGGL(k_gather<2>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 4) hipLaunchKernelGGL(k_gather<4>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 3) hipLaunchKernelGGL(k_gather<3>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 5) hipLaunchKernelGGL(k_gather<5>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 6) hipLaunchKernelGGL(k_gather<6>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 7) hipLaunchKernelGGL(k_gather<7>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 8) hipLaunchKernelGGL(k_gather<8>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 9) hipLaunchKernelGGL(k_gather<9>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 10) hipLaunchKernelGGL(k_gather<10>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 11) hipLaunchKernelGGL(k_gather<11>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 12) hipLaunchKernelGGL(k_gather<12>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 13) hipLaunchKernelGGL(k_gather<13>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 14) hipLaunchKernelGGL(k_gather<14>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 15) hipLaunchKernelGGL(k_gather<15>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 16) hipLaunchKernelGGL(k_gather<16>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            if (mode == 17) hipLaunchKernelGGL(k_gather<17>, (unsigned)((W + 255) / 256), 256, 0, 0, t, n, out, W, L);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            const double g = (double)W * L;
            if (rep == 1)
                std::printf("{\"mode\": \"%s\", \"mem\": \"%s\", \"table_GiB\": %.2f, \"ms\": %.3f, \"Ggathers_per_s\": %.2f, "
                            "\"useful_GBps_16B\": %.1f}\n",
                            names[mode], kind, gib, ms, g / ms / 1e6, g * 20 / ms / 1e6);
        }
    return 0;
}
