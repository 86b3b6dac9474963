// probe7.hip -- C4 / C5 access-shape probes (diagnostic, not product).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe7 tools/probe7.hip
//
// 1. Counter calibration on known byte counts (run under rocprofv3 --pmc, mode "once"):
//    k_cal_stream   dense 16-B-per-lane read of a 4 GiB buffer            (4.295 GB read)
//    k_cal_c5win    the 64-B windows of 32M frames at a 1536-B stride      (2.147 GB read)
//    k_cal_c4win    16M IMIX windows (64/576/1536-B slots, 7:4:1, shuffled,
//                   offsets read from a u64 array)                         (1.074 + 0.134 GB)
//    k_cal_c5w128   the whole first 128-B line of each 1536-B frame        (4.295 GB read)
//    Outputs: one dword per wave, so reads dominate.
// 2. C5 order sweep (mode "time"): 32M windows at the 1536-B stride, 4 lanes per frame
//    (one 16-B load each, 16 frames per wave load instruction, as k_cnet_defer loads), with
//    4 + 1 B of coalesced results per frame, in different fetch orders:
//    seq          frame = 64 g + 16 k + lane/4 (the product's order)
//    perm P       frame' = (frame * P) mod N for odd P (a bijection): consecutive frames of a
//                 wave instruction are P * 1536 B apart
//    xcd          blocks of XCD x (blockIdx % 8) walk the contiguous eighth x of the frames
//    xcdperm P    xcd, with the perm inside each eighth
//    bytes B      seq, but B bytes per frame (32 / 64 / 128 / 256): is the time per window
//                 or per byte?
//    Results are written at the logical frame index (coalesced) in every variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <random>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                       \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ u32x4 ldnt(const void *p) { return __builtin_nontemporal_load((const u32x4 *)p); }

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ __launch_bounds__(256) void k_cal_stream(const u32x4 *p, uint64_t n16, uint32_t *out)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        acc ^= fold(ldnt(p + i));
    acc ^= __shfl_xor(acc, 1);
    if ((threadIdx.x & 63u) == 0)
        out[(blockIdx.x * 256 + threadIdx.x) >> 6] = acc;
}

// 4 lanes per frame, BYTES per frame (multiple of 64: BYTES/64 loads per lane; 32: half the quads)
template <uint32_t BYTES>
__global__ __launch_bounds__(256) void k_cal_c5(const uint8_t *slab, uint64_t stride, uint64_t n, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + wv; g < n / 64; g += (uint64_t)gridDim.x * 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t f = g * 64 + 16 * k + (lane >> 2);
            const uint8_t *p = slab + f * stride + (lane & 3u) * 16u;
            if (BYTES >= 64) {
#pragma unroll
                for (uint32_t c = 0; c < BYTES / 64; c++)
                    acc ^= fold(ldnt(p + 64 * c));
            } else if ((lane & 3u) < BYTES / 16) {
                acc ^= fold(ldnt(p));
            }
        }
    }
    if (lane == 0)
        out[blockIdx.x * 4 + wv] = acc;
}

__global__ __launch_bounds__(256) void k_cal_c4win(const uint8_t *slab, const uint64_t *offs, uint64_t n, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + wv; g < n / 64; g += (uint64_t)gridDim.x * 4) {
        const uint64_t mine = offs[g * 64 + lane];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t o = __shfl(mine, 16 * k + (int)(lane >> 2));
            acc ^= fold(ldnt(slab + o + (lane & 3u) * 16u));
        }
    }
    if (lane == 0)
        out[blockIdx.x * 4 + wv] = acc;
}

// C5 order sweep.  MODE 0 seq, 1 perm, 2 xcd, 3 xcd + perm
template <int MODE>
__global__ __launch_bounds__(256) void k_c5_order(const uint8_t *slab, uint64_t n, uint64_t P, uint32_t *nh,
                                                  uint8_t *edge)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t tiles = n / 64;
    uint64_t g0, gs, gbase = 0, region = n;
    if (MODE >= 2) { // XCD x = blockIdx % 8 walks tiles [x T, (x+1) T)
        const uint64_t T = tiles / 8, x = blockIdx.x % 8, lb = blockIdx.x / 8, nlb = gridDim.x / 8;
        g0 = lb * 4 + wv;
        gs = nlb * 4;
        gbase = x * T;
        region = T * 64;
        for (uint64_t g = g0; g < T; g += gs) {
            u32x4 r[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint64_t f = g * 64 + 16 * k + (lane >> 2);
                if (MODE == 3)
                    f = (f * P) & (region - 1);
                r[k] = ldnt(slab + (gbase * 64 + f) * 1536ull + (lane & 3u) * 16u);
            }
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t x2 = fold(r[k]);
                x2 ^= __shfl_xor(x2, 1);
                x2 ^= __shfl_xor(x2, 2);
                v[k] = x2;
            }
            const uint32_t mine = __shfl(v[lane >> 4], (lane & 15u) * 4u);
            const uint64_t i = (gbase + g) * 64 + lane;
            __builtin_nontemporal_store(mine, nh + i);
            __builtin_nontemporal_store((uint8_t)mine, edge + i);
        }
        return;
    }
    g0 = (uint64_t)blockIdx.x * 4 + wv;
    gs = (uint64_t)gridDim.x * 4;
    for (uint64_t g = g0; g < tiles; g += gs) {
        u32x4 r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint64_t f = g * 64 + 16 * k + (lane >> 2);
            if (MODE == 1)
                f = (f * P) & (n - 1);
            r[k] = ldnt(slab + f * 1536ull + (lane & 3u) * 16u);
        }
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t x2 = fold(r[k]);
            x2 ^= __shfl_xor(x2, 1);
            x2 ^= __shfl_xor(x2, 2);
            v[k] = x2;
        }
        const uint32_t mine = __shfl(v[lane >> 4], (lane & 15u) * 4u);
        const uint64_t i = g * 64 + lane;
        __builtin_nontemporal_store(mine, nh + i);
        __builtin_nontemporal_store((uint8_t)mine, edge + i);
    }
}

int main(int argc, char **argv)
{
    const bool once = argc > 1 && !strcmp(argv[1], "once");
    const uint64_t n5 = 1ull << 25, stride5 = 1536, n4 = 1ull << 24, nstream = 4ull << 30;
    std::vector<uint64_t> offs(n4);
    uint64_t total4 = 0;
    {
        std::mt19937_64 rng(7);
        std::vector<uint32_t> sz(n4);
        for (uint64_t i = 0; i < n4; i++) {
            const uint32_t r = (uint32_t)(i % 12);
            sz[i] = r < 7 ? 64 : r < 11 ? 576 : 1536;
        }
        std::shuffle(sz.begin(), sz.end(), rng);
        for (uint64_t i = 0; i < n4; i++) {
            offs[i] = total4;
            total4 += sz[i];
        }
    }
    const uint64_t slab_bytes = n5 * stride5;
    uint8_t *slab, *sbuf;
    uint64_t *d_offs;
    uint32_t *out, *nh;
    uint8_t *edge;
    CK(hipMalloc(&slab, slab_bytes + 4096));
    CK(hipMemset(slab, 5, slab_bytes + 4096));
    CK(hipMalloc(&sbuf, nstream));
    CK(hipMemset(sbuf, 3, nstream));
    CK(hipMalloc(&d_offs, n4 * 8));
    CK(hipMemcpy(d_offs, offs.data(), n4 * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, 1 << 22));
    CK(hipMalloc(&nh, n5 * 4));
    CK(hipMalloc(&edge, n5));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(256 * 4), blk(256);
    auto run = [&](auto launch, const char *name, double bytes, uint64_t n) {
        if (once) { // one warm launch, then the measured one (each is one dispatch in the trace)
            launch();
            launch();
            hipDeviceSynchronize();
            printf("%-24s launched\n", name);
            fflush(stdout);
            return;
        }
        for (int w = 0; w < 3; w++)
            launch();
        std::vector<float> ts;
        for (int r = 0; r < 11; r++) {
            hipEventRecord(e0, 0);
            launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-24s %.4f ms (min %.4f)  %8.1f M frames/s  %7.1f GB/s of the named bytes\n", name, ts[5], ts[0],
               n / (ts[5] * 1e3), bytes / (ts[5] * 1e-3) / 1e9);
        fflush(stdout);
    };
    // 1. calibration
    run([&] { hipLaunchKernelGGL(k_cal_stream, grid, blk, 0, 0, (const u32x4 *)sbuf, nstream / 16, out); },
        "cal_stream_4GiB", (double)nstream, nstream / 64);
    run([&] { hipLaunchKernelGGL(k_cal_c5<64>, grid, blk, 0, 0, slab, stride5, n5, out); }, "cal_c5win_64B",
        64.0 * n5, n5);
    run([&] { hipLaunchKernelGGL(k_cal_c5<128>, grid, blk, 0, 0, slab, stride5, n5, out); }, "cal_c5w128",
        128.0 * n5, n5);
    run([&] { hipLaunchKernelGGL(k_cal_c5<32>, grid, blk, 0, 0, slab, stride5, n5, out); }, "cal_c5w32",
        32.0 * n5, n5);
    run([&] { hipLaunchKernelGGL(k_cal_c5<256>, grid, blk, 0, 0, slab, stride5, n5, out); }, "cal_c5w256",
        256.0 * n5, n5);
    run([&] { hipLaunchKernelGGL(k_cal_c4win, grid, blk, 0, 0, slab, d_offs, n4, out); }, "cal_c4win_imix",
        72.0 * n4, n4);
    if (once)
        return 0;
    // 2. C5 order sweep
    char nm[64];
    for (int bpc : {2, 4}) {
        const dim3 g(256 * bpc);
        snprintf(nm, sizeof nm, "seq bpc%d", bpc);
        run([&] { hipLaunchKernelGGL(k_c5_order<0>, g, blk, 0, 0, slab, n5, 1ull, nh, edge); }, nm, 68.0 * n5, n5);
        for (uint64_t P : {3ull, 5ull, 17ull, 255ull, 4097ull, 65537ull, 2654435761ull}) {
            snprintf(nm, sizeof nm, "perm %llu bpc%d", (unsigned long long)P, bpc);
            run([&] { hipLaunchKernelGGL(k_c5_order<1>, g, blk, 0, 0, slab, n5, P, nh, edge); }, nm, 68.0 * n5, n5);
        }
        snprintf(nm, sizeof nm, "xcd bpc%d", bpc);
        run([&] { hipLaunchKernelGGL(k_c5_order<2>, g, blk, 0, 0, slab, n5, 1ull, nh, edge); }, nm, 68.0 * n5, n5);
        for (uint64_t P : {17ull, 65537ull}) {
            snprintf(nm, sizeof nm, "xcdperm %llu bpc%d", (unsigned long long)P, bpc);
            run([&] { hipLaunchKernelGGL(k_c5_order<3>, g, blk, 0, 0, slab, n5, P, nh, edge); }, nm, 68.0 * n5, n5);
        }
    }
    return 0;
}
