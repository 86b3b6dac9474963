// probe4.hip -- the cost of the 10-B/frame result stores beside the 64-B/frame read
// (diagnostic, not product).  Build: hipcc -O3 --offload-arch=gfx950 -o probe4 probe4.hip
//   read      : LDS-staged tile, results XOR-ed into a register (no stores)
//   lds       : + 3 SoA stores (4 B, 4 B, 2 B per frame), grid-stride tiles
//   lds_nt    : stores non-temporal
//   lds_chunk : each block walks a contiguous range of tiles (no grid stride)
//   lds_aosoa : the 3 results of one 64-frame tile stored contiguously (640 B per tile)
//   wonly     : the 3 SoA stores alone, no frame reads
//   lds_s8    : 2 stores: (nh,hash) as one 8-B store per frame, queue 2 B
//   lds_q32   : 3 stores, the queue widened to 4 B
//   lds_qpair : queue 2 B, two frames' queues packed per dword by a lane shuffle (32 lanes store)
//   lds_2     : 2 stores (4 B, 4 B), no queue
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Out {
    uint32_t *a, *b;
    uint16_t *q;
    uint32_t *sink;
};

__device__ __forceinline__ void lds_pass(u32x4 *tile, uint32_t lane, u32x4 r0, u32x4 r1, u32x4 r2, u32x4 r3,
                                         u32x4 &p0, u32x4 &p1, u32x4 &p2)
{
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t f = 16u * k + fr_in_k;
        const u32x4 v = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
        tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v;
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t sw = (lane >> 2) & 3u;
    p0 = tile[lane * 4u + (0u ^ sw)];
    p1 = tile[lane * 4u + (1u ^ sw)];
    p2 = tile[lane * 4u + (2u ^ sw)];
    __builtin_amdgcn_wave_barrier();
}

template <int MODE>
__global__ __launch_bounds__(256) void k_v(const uint8_t *slab, uint64_t n_tiles, Out o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    uint32_t acc = 0;
    uint64_t t, t_end, wstep;
    if (MODE == 3) {
        const uint64_t per = (n_tiles + gridDim.x - 1) / gridDim.x;
        t = (uint64_t)blockIdx.x * per + wv;
        t_end = min((uint64_t)(blockIdx.x + 1) * per, n_tiles);
        wstep = 4;
    } else {
        t = (uint64_t)blockIdx.x * 4 + wv;
        t_end = n_tiles;
        wstep = (uint64_t)gridDim.x * 4;
    }
    for (; t < t_end; t += wstep) {
        const uint64_t i = t * 64u + lane;
        if (MODE == 5) {
            const uint32_t v = (uint32_t)i * 2654435761u;
            o.a[i] = v;
            o.b[i] = v ^ 7u;
            o.q[i] = (uint16_t)v;
            continue;
        }
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        const u32x4 r0 = g[lane], r1 = g[64 + lane], r2 = g[128 + lane], r3 = g[192 + lane];
        u32x4 p0, p1, p2;
        lds_pass(tile, lane, r0, r1, r2, r3, p0, p1, p2);
        const uint32_t va = p0.w ^ p2.x, vb = p1.y + p1.z * 3u + p1.w;
        const uint16_t vq = (uint16_t)(p1.w >> 3);
        if (MODE == 0) {
            acc ^= va ^ vb ^ vq;
        } else if (MODE == 1 || MODE == 3) {
            o.a[i] = va;
            o.b[i] = vb;
            o.q[i] = vq;
        } else if (MODE == 2) {
            __builtin_nontemporal_store(va, o.a + i);
            __builtin_nontemporal_store(vb, o.b + i);
            __builtin_nontemporal_store(vq, o.q + i);
        } else if (MODE == 4) {
            uint8_t *base = (uint8_t *)o.a + t * 640u;
            ((uint32_t *)base)[lane] = va;
            ((uint32_t *)(base + 256))[lane] = vb;
            ((uint16_t *)(base + 512))[lane] = vq;
        } else if (MODE == 6) {
            ((u32x2 *)o.a)[i] = (u32x2){va, vb};
            o.q[i] = vq;
        } else if (MODE == 7) {
            o.a[i] = va;
            o.b[i] = vb;
            ((uint32_t *)o.q)[i] = vq;
        } else if (MODE == 8) {
            o.a[i] = va;
            o.b[i] = vb;
            const uint32_t hi = __shfl_down((uint32_t)vq, 1);
            if ((lane & 1u) == 0)
                ((uint32_t *)o.q)[i >> 1] = (uint32_t)vq | (hi << 16);
        } else if (MODE == 9) {
            o.a[i] = va;
            o.b[i] = vb;
        }
    }
    if (acc == 0x12345678u)
        o.sink[0] = acc;
}

int main()
{
    const uint64_t n = 1ull << 24, tiles = n / 64;
    uint8_t *slab;
    Out o;
    CK(hipMalloc(&slab, n * 64));
    CK(hipMalloc(&o.a, n * 10));
    CK(hipMalloc(&o.b, n * 4));
    CK(hipMalloc(&o.q, n * 4));
    CK(hipMalloc(&o.sink, 64));
    {
        std::vector<uint32_t> h(n * 16);
        for (uint64_t i = 0; i < h.size(); i++)
            h[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
        CK(hipMemcpy(slab, h.data(), n * 64, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int cus = 256;
    auto timeit = [&](auto launch, const char *name) {
        for (int w = 0; w < 3; w++)
            launch();
        std::vector<float> ts;
        for (int r = 0; r < 20; r++) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-18s %.4f ms  %7.1f GB/s(74B)\n", name, ts[10], 74.0 * n / (ts[10] * 1e-3) / 1e9);
        fflush(stdout);
        return 0;
    };
    char nm[64];
    const char *names[] = {"read", "lds", "lds_nt", "lds_chunk", "lds_aosoa", "wonly", "lds_s8",
                           "lds_q32", "lds_qpair", "lds_2"};
    for (int bpc : {2, 4}) {
        const dim3 g(cus * bpc);
#define RUN(M)                                                                                         \
    snprintf(nm, sizeof nm, "%s bpc=%d", names[M], bpc);                                            \
    timeit([&] { hipLaunchKernelGGL(k_v<M>, g, dim3(256), 0, 0, slab, tiles, o); }, nm)
        RUN(0); RUN(1); RUN(2); RUN(4); RUN(5); RUN(6); RUN(7); RUN(8); RUN(9);
    }
    return 0;
}
