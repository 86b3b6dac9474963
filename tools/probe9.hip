// probe9.hip -- what the per-frame result stores cost beside the C4 / C5 window
// reads, and whether their shape matters (diagnostic, not product).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe9 tools/probe9.hip
//
// The window read of cndp_probe_windows (4 lanes a frame, 16 frames a 16-B load
// instruction, nt loads; C5: 32M frames at a 1536-B stride, C4: 16M IMIX frames
// at u64 offsets) with these result stores per frame:
//   set   nh | nh+hash+queue | +edge | +edge+t16 (the five streams k_cnet_defer writes)
//   shape direct: one nt store instruction per stream and 64-frame tile (edge: a
//                 64-B half line per tile)
//         stageS: the wave gathers S tiles' results in LDS and writes them with
//                 16-B nt stores (every stream in whole 128-B lines from S = 2)
// Times are medians of 11 launches (HIP events) after 3 warm ones.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                       \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

struct Out {
    uint32_t *a, *b;
    uint16_t *q;
    uint8_t *e;
    uint16_t *t;
};

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const u32x4 *)p); }

// S = 0: direct stores; S > 0: staged per S tiles (n_tiles a multiple of S per wave range)
template <int S>
__global__ __launch_bounds__(256) void k_w(const uint8_t *slab, uint64_t stride, const uint64_t *offs, uint64_t n,
                                           Out o)
{
    constexpr int SS = S > 0 ? S : 1;
    // per wave: SS tiles x (256 + 256 + 128 + 64 + 128) B
    __shared__ __attribute__((aligned(16))) uint8_t s_o[4][SS * 832];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t tiles = n / 64u, units = tiles / SS;
    uint8_t *so = s_o[wv];
    for (uint64_t u = (uint64_t)blockIdx.x * 4u + wv; u < units; u += (uint64_t)gridDim.x * 4u) {
#pragma unroll
        for (int j = 0; j < SS; j++) {
            const uint64_t g = u * SS + j;
            const uint64_t mine = offs ? offs[g * 64u + lane] : (g * 64u + lane) * stride;
            uint32_t res = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t fo = __shfl(mine, 16 * k + (int)(lane >> 2));
                const u32x4 w = ldnt(slab + fo + (lane & 3u) * 16u);
                uint32_t x = w.x ^ w.y ^ w.z ^ w.w;
                x ^= __shfl_xor(x, 1);
                x ^= __shfl_xor(x, 2);
                const uint32_t src = __shfl(x, (int)((lane & 15u) * 4u));
                if ((lane >> 4) == (uint32_t)k)
                    res = src;
            }
            const uint64_t i = g * 64u + lane;
            if (S == 0) {
                if (o.a)
                    __builtin_nontemporal_store(res, o.a + i);
                if (o.b)
                    __builtin_nontemporal_store(res * 2654435761u, o.b + i);
                if (o.q)
                    __builtin_nontemporal_store((uint16_t)(res >> 7), o.q + i);
                if (o.e)
                    __builtin_nontemporal_store((uint8_t)(res >> 3), o.e + i);
                if (o.t)
                    __builtin_nontemporal_store((uint16_t)(res >> 11), o.t + i);
            } else {
                ((uint32_t *)so)[j * 64 + lane] = res;
                ((uint32_t *)(so + SS * 256))[j * 64 + lane] = res * 2654435761u;
                ((uint16_t *)(so + SS * 512))[j * 64 + lane] = (uint16_t)(res >> 7);
                (so + SS * 640)[j * 64 + lane] = (uint8_t)(res >> 3);
                ((uint16_t *)(so + SS * 704))[j * 64 + lane] = (uint16_t)(res >> 11);
            }
        }
        if (S > 0) {
            __builtin_amdgcn_wave_barrier();
            const uint64_t f0 = u * SS * 64u; // the unit's first frame
            // 16-B chunks: a SS*16, b SS*16, q SS*8, e SS*4, t SS*8
            for (uint32_t c = lane; c < SS * 52u; c += 64u) {
                uint8_t *dst;
                uint32_t src;
                if (c < SS * 16u) {
                    dst = o.a ? (uint8_t *)(o.a + f0) + c * 16u : nullptr;
                    src = c * 16u;
                } else if (c < SS * 32u) {
                    dst = o.b ? (uint8_t *)(o.b + f0) + (c - SS * 16u) * 16u : nullptr;
                    src = SS * 256u + (c - SS * 16u) * 16u;
                } else if (c < SS * 40u) {
                    dst = o.q ? (uint8_t *)(o.q + f0) + (c - SS * 32u) * 16u : nullptr;
                    src = SS * 512u + (c - SS * 32u) * 16u;
                } else if (c < SS * 44u) {
                    dst = o.e ? o.e + f0 + (c - SS * 40u) * 16u : nullptr;
                    src = SS * 640u + (c - SS * 40u) * 16u;
                } else {
                    dst = o.t ? (uint8_t *)(o.t + f0) + (c - SS * 44u) * 16u : nullptr;
                    src = SS * 704u + (c - SS * 44u) * 16u;
                }
                if (dst)
                    __builtin_nontemporal_store(*(const u32x4 *)(so + src), (u32x4 *)dst);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int S>
static float run(const uint8_t *slab, uint64_t stride, const uint64_t *offs, uint64_t n, Out o, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++)
        hipLaunchKernelGGL(k_w<S>, dim3(grid), dim3(256), 0, 0, slab, stride, offs, n, o);
    std::vector<float> ts;
    for (int r = 0; r < 11; r++) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_w<S>, dim3(grid), dim3(256), 0, 0, slab, stride, offs, n, o);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ts[5];
}

__global__ void k_fill(uint32_t *p, uint64_t n32)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n32; i += (uint64_t)gridDim.x * 256)
        p[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 29);
}

int main()
{
    int dev, ncu;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t n5 = 1ull << 25, n4 = 1ull << 24, stride = 1536;
    std::vector<uint64_t> hoff(n4);
    uint64_t tot = 0;
    uint32_t x = 12345;
    for (uint64_t i = 0; i < n4; i++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t pick = (x >> 8) % 12;
        hoff[i] = tot;
        tot += pick < 7 ? 64 : pick < 11 ? 576 : 1536;
    }
    const uint64_t bytes = std::max(n5 * stride, tot) + 4096;
    uint8_t *slab;
    uint64_t *offs;
    CK(hipMalloc((void **)&slab, bytes));
    CK(hipMalloc((void **)&offs, n4 * 8));
    CK(hipMemcpy(offs, hoff.data(), n4 * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(ncu * 16), dim3(256), 0, 0, (uint32_t *)slab, bytes / 4);
    Out full{};
    CK(hipMalloc((void **)&full.a, n5 * 4));
    CK(hipMalloc((void **)&full.b, n5 * 4));
    CK(hipMalloc((void **)&full.q, n5 * 2));
    CK(hipMalloc((void **)&full.e, n5));
    CK(hipMalloc((void **)&full.t, n5 * 2));
    CK(hipDeviceSynchronize());
    struct Set {
        const char *name;
        Out o;
    } sets[4] = {{"nh", {full.a, nullptr, nullptr, nullptr, nullptr}},
                 {"nh+hash+queue", {full.a, full.b, full.q, nullptr, nullptr}},
                 {"+edge", {full.a, full.b, full.q, full.e, nullptr}},
                 {"+edge+t16", full}};
    for (int shape = 0; shape < 2; shape++) {
        const char *sn = shape == 0 ? "C5" : "C4";
        const uint64_t n = shape == 0 ? n5 : n4;
        const uint64_t *po = shape == 0 ? nullptr : offs;
        for (int bpc : {4, 8}) {
            for (auto &st : sets) {
                const int g = ncu * bpc;
                const float d = run<0>(slab, stride, po, n, st.o, g);
                const float s1 = run<1>(slab, stride, po, n, st.o, g);
                const float s2 = run<2>(slab, stride, po, n, st.o, g);
                const float s4 = run<4>(slab, stride, po, n, st.o, g);
                printf("%s bpc%d %-14s direct %.4f  stage1 %.4f  stage2 %.4f  stage4 %.4f ms\n", sn, bpc, st.name, d,
                       s1, s2, s4);
                fflush(stdout);
            }
        }
    }
    return 0;
}
