// probe.hip -- diagnostic microbenchmarks for the classify traffic shape
// (not part of the product).  Build: hipcc -O3 --offload-arch=gfx950 -o probe probe.hip
// Prints achieved GB/s for:
//   copy     : float4 read+write of the slab size (calibration, like the guide's 6.29 TB/s)
//   read     : tile-pattern read of 16M x 64-B slots, one u32 per wave written
//   rw10     : tile read + 10 B/pkt SoA writes (u32, u32, u16) of values derived from the frames
//   rw10lane : the same traffic with per-lane strided frame loads (bytes 0..39 of each slot)
//   rw10lds  : rw10 with the frames staged through a swizzled LDS tile (the classify layout)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, uint64_t n)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        out[i] = in[i];
}

template <int MODE>
__global__ __launch_bounds__(256) void k_tile(const uint8_t *slab, uint64_t n_tiles, uint32_t *o32a,
                                              uint32_t *o32b, uint16_t *o16, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    uint32_t acc = 0;
    const uint64_t wstep = (uint64_t)gridDim.x * 4;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < n_tiles; t += wstep) {
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        u32x4 r0 = g[lane], r1 = g[64 + lane], r2 = g[128 + lane], r3 = g[192 + lane];
        if (MODE == 0) {
            acc ^= r0.x ^ r1.y ^ r2.z ^ r3.w;
            continue;
        }
        uint32_t w3, w5, w6, w7, w8;
        if (MODE == 1) {
            // lane holds chunks of 4 different frames: use all of them (no dead loads)
            w3 = r0.w ^ r3.x; w5 = r1.y ^ r3.y; w6 = r1.z ^ r3.z; w7 = r1.w ^ r3.w; w8 = r2.x;
        } else {
            const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t f = 16u * k + fr_in_k;
                const u32x4 v = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
                tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v;
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t sw = (lane >> 2) & 3u;
            const u32x4 p0 = tile[lane * 4u + (0u ^ sw)];
            const u32x4 p1 = tile[lane * 4u + (1u ^ sw)];
            const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
            __builtin_amdgcn_wave_barrier();
            w3 = p0.w; w5 = p1.y; w6 = p1.z; w7 = p1.w; w8 = p2.x;
        }
        const uint64_t i = t * 64u + lane;
        o32a[i] = w3 ^ w8;
        o32b[i] = w5 + w6 * 3u + w7;
        o16[i] = (uint16_t)(w7 >> 3);
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// per-lane strided pattern: each lane loads its own frame's bytes 0..39
__global__ __launch_bounds__(256) void k_lane(const uint8_t *slab, uint64_t n, uint32_t *o32a,
                                              uint32_t *o32b, uint16_t *o16)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint8_t *p = slab + i * 64u;
        const u32x4 q0 = *(const u32x4 *)p, q1 = *(const u32x4 *)(p + 16);
        const uint2 q2 = *(const uint2 *)(p + 32);
        o32a[i] = q0.w ^ q2.x;
        o32b[i] = q1.y + q1.z * 3u + q1.w;
        o16[i] = (uint16_t)(q1.w >> 3);
    }
}

int main()
{
    const uint64_t n = 1ull << 24;
    uint8_t *slab;
    uint32_t *a, *b, *sink;
    uint16_t *q;
    u32x4 *cp;
    CK(hipMalloc(&slab, n * 64));
    CK(hipMalloc(&cp, n * 64));
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&q, n * 2));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(slab, 1, n * 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 256;
    auto timeit = [&](auto launch, double bytes, const char *name) {
        for (int w = 0; w < 3; w++)
            launch();
        std::vector<float> ts;
        for (int r = 0; r < 20; r++) {
            hipEventRecord(e0, 0);
            launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-28s %.4f ms  %7.1f GB/s\n", name, ts[10], bytes / (ts[10] * 1e-3) / 1e9);
    };
    for (int bpc : {4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL(k_copy, dim3(cus * bpc), dim3(256), 0, 0, (const u32x4 *)slab, cp, n * 4); },
               2.0 * n * 64, nm);
    }
    const uint64_t tiles = n / 64;
    for (int bpc : {2, 4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "read bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL(k_tile<0>, dim3(cus * bpc), dim3(256), 0, 0, slab, tiles, a, b, q, sink); },
               64.0 * n, nm);
        snprintf(nm, sizeof nm, "rw10 bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL(k_tile<1>, dim3(cus * bpc), dim3(256), 0, 0, slab, tiles, a, b, q, sink); },
               74.0 * n, nm);
        snprintf(nm, sizeof nm, "rw10lane bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL(k_lane, dim3(cus * bpc), dim3(256), 0, 0, slab, n, a, b, q); },
               74.0 * n, nm);
        snprintf(nm, sizeof nm, "rw10lds bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL(k_tile<2>, dim3(cus * bpc), dim3(256), 0, 0, slab, tiles, a, b, q, sink); },
               74.0 * n, nm);
    }
    return 0;
}
