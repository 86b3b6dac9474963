// probe5.hip -- streaming ceilings for the cnet configurations (diagnostic, not product).
// Build: hipcc -O3 --offload-arch=gfx950 -o probe5 probe5.hip
//   c5 : 32M frames in 1536-B slots; read the 64-B window of each, write 4 + 1 B per frame
//        lane : each lane loads its own frame's 64 B (4 x 16-B loads)
//        quad : 4 lanes per frame, one 16-B load each (a wave instruction covers 16 whole windows)
//   c4 : 16M IMIX frames (64/576/1536-B slots at 7:4:1, shuffled) addressed by a u64 offset
//        array; read offset + 64-B window, write 4 + 4 + 2 + 1 B per frame
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <random>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Out {
    uint32_t *a, *b;
    uint16_t *q;
    uint8_t *e;
};

// QUAD: 4 lanes per frame; lane part p holds bytes 16p..16p+15 of frame (16k + lane/4)
template <bool QUAD, bool OFFS, bool FULL_OUT>
__global__ __launch_bounds__(256) void k_win(const uint8_t *slab, const uint64_t *offs, uint64_t stride, uint64_t n,
                                             Out o)
{
    if (QUAD) {
        const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
        const uint64_t ng = n / 64;
        for (uint64_t g = (uint64_t)blockIdx.x * 4 + wv; g < ng; g += (uint64_t)gridDim.x * 4) {
            u32x4 r[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t f = g * 64 + 16 * k + (lane >> 2);
                const uint64_t base = OFFS ? offs[f] : f * stride;
                r[k] = *(const u32x4 *)(slab + base + (lane & 3u) * 16u);
            }
            // reduce each frame's 4 parts to lane (16k + lane/4)'s values with cross-lane xor
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t x = r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
                x ^= __shfl_xor(x, 1);
                x ^= __shfl_xor(x, 2);
                v[k] = x;
            }
            // frame of this lane: 16*(lane>>4) + (lane & 15) -> value lives in k = lane>>4, src lane (lane&15)*4
            const uint32_t src = (lane & 15u) * 4u;
            uint32_t mine = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t t = __shfl(v[k], src);
                if ((lane >> 4) == (uint32_t)k)
                    mine = t;
            }
            const uint64_t i = g * 64 + lane;
            o.a[i] = mine;
            o.e[i] = (uint8_t)mine;
            if (FULL_OUT) {
                o.b[i] = mine * 3u;
                o.q[i] = (uint16_t)(mine >> 7);
            }
        }
        return;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t base = OFFS ? offs[i] : i * stride;
        const u32x4 *p = (const u32x4 *)(slab + base);
        const u32x4 x = p[0] ^ p[1] ^ p[2] ^ p[3];
        const uint32_t m = x.x ^ x.y ^ x.z ^ x.w;
        o.a[i] = m;
        o.e[i] = (uint8_t)m;
        if (FULL_OUT) {
            o.b[i] = m * 3u;
            o.q[i] = (uint16_t)(m >> 7);
        }
    }
}

int main()
{
    const uint64_t n5 = 1ull << 25, stride5 = 1536;
    const uint64_t n4 = 1ull << 24;
    // C4 layout
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
    const uint64_t slab_bytes = std::max(n5 * stride5, total4);
    uint8_t *slab;
    uint64_t *d_offs;
    Out o;
    CK(hipMalloc(&slab, slab_bytes + 64));
    CK(hipMemset(slab, 5, slab_bytes + 64));
    CK(hipMalloc(&d_offs, n4 * 8));
    CK(hipMemcpy(d_offs, offs.data(), n4 * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&o.a, n5 * 4));
    CK(hipMalloc(&o.b, n5 * 4));
    CK(hipMalloc(&o.q, n5 * 2));
    CK(hipMalloc(&o.e, n5));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch, double bytes, uint64_t n, const char *name) {
        for (int w = 0; w < 3; w++)
            launch();
        std::vector<float> ts;
        for (int r = 0; r < 15; r++) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-22s %.4f ms  %8.1f Mpps  %7.1f GB/s(algo)\n", name, ts[7], n / (ts[7] * 1e3), bytes / (ts[7] * 1e-3) / 1e9);
        fflush(stdout);
        return 0;
    };
    char nm[64];
    for (int bpc : {2, 4, 8}) {
        const dim3 g(256 * bpc);
        snprintf(nm, sizeof nm, "c5 lane bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL((k_win<false, false, false>), g, dim3(256), 0, 0, slab, nullptr, stride5, n5, o); },
               68.0 * n5, n5, nm);
        snprintf(nm, sizeof nm, "c5 quad bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL((k_win<true, false, false>), g, dim3(256), 0, 0, slab, nullptr, stride5, n5, o); },
               68.0 * n5, n5, nm);
        snprintf(nm, sizeof nm, "c4 lane bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL((k_win<false, true, true>), g, dim3(256), 0, 0, slab, d_offs, 0, n4, o); },
               74.0 * n4, n4, nm);
        snprintf(nm, sizeof nm, "c4 quad bpc=%d", bpc);
        timeit([&] { hipLaunchKernelGGL((k_win<true, true, true>), g, dim3(256), 0, 0, slab, d_offs, 0, n4, o); },
               74.0 * n4, n4, nm);
    }
    return 0;
}
