// probe2.hip -- which part of the frame-tile read costs bandwidth (diagnostic, not product).
// Build: hipcc -O3 --offload-arch=gfx950 -o probe2 probe2.hip
// 16M x 64-B slots (1 GiB), wave tiles of 64 frames (4 KiB), 10 B/frame written.
//   full     : 4 x dwordx4 per lane, XOR of all 16 dwords (read only, full return to VGPRs)
//   part3    : 3 x dwordx4, the lanes holding bytes 48..63 of a frame masked off
//   lds      : register staging into a swizzled LDS tile + 10-B writes (the classify layout)
//   lds3     : lds with chunk 3 of every frame not loaded (classify needs bytes 12..41 only)
//   glds     : global_load_lds_dwordx4 (LDS-DMA) into the tile, vmcnt(0), 10-B writes
//   glds2    : glds with the next tile issued before the current one is consumed
//   glds3x2  : glds2 with chunk 3 not loaded (3 DMAs per tile)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ void emit(uint64_t i, u32x4 p0, u32x4 p1, u32x4 p2, uint32_t *a, uint32_t *b, uint16_t *q)
{
    a[i] = p0.w ^ p2.x;
    b[i] = p1.y + p1.z * 3u + p1.w;
    q[i] = (uint16_t)(p1.w >> 3);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_reg(const uint8_t *slab, uint64_t n_tiles, uint32_t *a, uint32_t *b,
                                             uint16_t *q, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    uint32_t acc = 0;
    const uint64_t wstep = (uint64_t)gridDim.x * 4;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < n_tiles; t += wstep) {
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        const bool need = MODE == 0 || MODE == 2 || (lane & 3u) != 3u;
        u32x4 r0 = {0, 0, 0, 0}, r1 = r0, r2 = r0, r3 = r0;
        if (need) {
            r0 = g[lane];
            r1 = g[64 + lane];
            r2 = g[128 + lane];
            r3 = g[192 + lane];
        }
        if (MODE <= 1) {
            const u32x4 x = r0 ^ r1 ^ r2 ^ r3;
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
            continue;
        }
        const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            const u32x4 v = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
            if (need)
                tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)];
        const u32x4 p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        emit(t * 64u + lane, p0, p1, p2, a, b, q);
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// LDS-DMA: slot s of the tile (s = 64k + lane for instruction k) holds frame f = s/4,
// part (s&3) ^ ((f>>2)&3): the swizzle is applied on the global (source) address.
template <int NCH>
__device__ __forceinline__ void glds_tile(const uint8_t *slab, uint64_t t, u32x4 *tile, uint32_t lane)
{
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t s = 64u * k + lane, f = s >> 2, part = (s & 3u) ^ ((f >> 2) & 3u);
        if (NCH == 3 && part == 3u)
            continue;  // keeps the LDS slot stale: never read
        const uint8_t *src = slab + t * 4096u + f * 64u + part * 16u;
        __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)(tile + 64u * k),
                                         16, 0, 0);
    }
}

template <int DEPTH, int NCH>
__global__ __launch_bounds__(256) void k_glds(const uint8_t *slab, uint64_t n_tiles, uint32_t *a, uint32_t *b,
                                              uint16_t *q)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][2][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t wstep = (uint64_t)gridDim.x * 4;
    uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
    uint32_t buf = 0;
    if (DEPTH == 2 && t < n_tiles)
        glds_tile<NCH>(slab, t, s_tile[wv][0], lane);
    for (; t < n_tiles; t += wstep) {
        u32x4 *tile = s_tile[wv][buf];
        if (DEPTH == 1) {
            glds_tile<NCH>(slab, t, tile, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            const uint64_t tn = t + wstep;
            if (tn < n_tiles) {
                glds_tile<NCH>(slab, tn, s_tile[wv][buf ^ 1u], lane);
                // wait for everything but the NCH DMAs just issued
                if (NCH == 4)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        u32x4 p0, p1, p2;
        p0 = tile[lane * 4u + (0u ^ sw)];
        p1 = tile[lane * 4u + (1u ^ sw)];
        p2 = tile[lane * 4u + (2u ^ sw)];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        emit(t * 64u + lane, p0, p1, p2, a, b, q);
        buf ^= DEPTH == 2 ? 1u : 0u;
    }
}

int main()
{
    const uint64_t n = 1ull << 24, tiles = n / 64;
    uint8_t *slab;
    uint32_t *a, *b, *sink;
    uint16_t *q;
    CK(hipMalloc(&slab, n * 64));
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&q, n * 2));
    CK(hipMalloc(&sink, 64));
    {
        std::vector<uint8_t> h(n * 64);
        for (uint64_t i = 0; i < h.size(); i++)
            h[i] = (uint8_t)(i * 2654435761u >> 13);
        CK(hipMemcpy(slab, h.data(), h.size(), hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int cus = 256;
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
        printf("%-22s %.4f ms  %7.1f GB/s\n", name, ts[10], bytes / (ts[10] * 1e-3) / 1e9);
        fflush(stdout);
    };
    // reference results for the glds variants (must equal lds)
    std::vector<uint32_t> ra(n), rb(n);
    bool first = true;
    auto check = [&](const char *name) {
        std::vector<uint32_t> xa(n), xb(n);
        hipMemcpy(xa.data(), a, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(xb.data(), b, n * 4, hipMemcpyDeviceToHost);
        if (first) {
            ra = xa;
            rb = xb;
            first = false;
            return;
        }
        if (xa != ra || xb != rb)
            printf("MISMATCH %s\n", name);
    };
    char nm[64];
    for (int bpc : {2, 4, 8}) {
        const dim3 g(cus * bpc);
        hipMemset(a, 0, n * 4);
        hipLaunchKernelGGL(k_reg<2>, g, dim3(256), 0, 0, slab, tiles, a, b, q, sink);
        hipDeviceSynchronize();
        check("lds");
#define RUN(NAME, BYTES, ...)                                                                        \
    snprintf(nm, sizeof nm, "%s bpc=%d", NAME, bpc);                                                \
    timeit([&] { hipLaunchKernelGGL(__VA_ARGS__); }, BYTES, nm)
        RUN("full", 64.0 * n, k_reg<0>, g, dim3(256), 0, 0, slab, tiles, a, b, q, sink);
        RUN("part3", 64.0 * n, k_reg<1>, g, dim3(256), 0, 0, slab, tiles, a, b, q, sink);
        RUN("lds", 74.0 * n, k_reg<2>, g, dim3(256), 0, 0, slab, tiles, a, b, q, sink);
        RUN("lds3", 74.0 * n, k_reg<3>, g, dim3(256), 0, 0, slab, tiles, a, b, q, sink);
        check("lds3");
        RUN("glds", 74.0 * n, (k_glds<1, 4>), g, dim3(256), 0, 0, slab, tiles, a, b, q);
        check("glds");
        RUN("glds2", 74.0 * n, (k_glds<2, 4>), g, dim3(256), 0, 0, slab, tiles, a, b, q);
        check("glds2");
        RUN("glds3x2", 74.0 * n, (k_glds<2, 3>), g, dim3(256), 0, 0, slab, tiles, a, b, q);
        check("glds3x2");
    }
    return 0;
}
