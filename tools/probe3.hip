// probe3.hip -- why does the LDS-staged frame tile + 10-B writes run at 5.1 TB/s when the
// read alone runs at 6.2-6.5?  (diagnostic, not product)
// Build: hipcc -O3 --offload-arch=gfx950 -o probe3 probe3.hip
//   rw10      : registers only, outputs mix chunks of different frames (2.5 KiB returned / tile)
//   rw10full  : registers only, every loaded dword feeds an output (4 KiB returned / tile)
//   lds       : swizzled LDS tile, per-frame outputs (the classify layout)
//   lds_nost  : lds, outputs XOR-ed into a register (no global stores)
//   lds_1st   : lds, one 4-B output array only
//   lds_pipe  : lds, next tile's loads issued before this tile's LDS pass (register double buffer)
//   lds_wide  : lds, outputs packed per wave into one 16-B-per-lane store covering 4 frames (AoS)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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
    const uint64_t wstep = (uint64_t)gridDim.x * 4;
    uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
    if (MODE == 5) {
        if (t >= n_tiles)
            return;
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        u32x4 r0 = g[lane], r1 = g[64 + lane], r2 = g[128 + lane], r3 = g[192 + lane];
        for (;;) {
            const uint64_t tn = t + wstep;
            const bool more = tn < n_tiles;
            u32x4 n0 = r0, n1 = r1, n2 = r2, n3 = r3;
            if (more) {
                const u32x4 *gn = (const u32x4 *)(slab + tn * 4096u);
                n0 = gn[lane];
                n1 = gn[64 + lane];
                n2 = gn[128 + lane];
                n3 = gn[192 + lane];
            }
            u32x4 p0, p1, p2;
            lds_pass(tile, lane, r0, r1, r2, r3, p0, p1, p2);
            const uint64_t i = t * 64u + lane;
            o.a[i] = p0.w ^ p2.x;
            o.b[i] = p1.y + p1.z * 3u + p1.w;
            o.q[i] = (uint16_t)(p1.w >> 3);
            if (!more)
                break;
            r0 = n0; r1 = n1; r2 = n2; r3 = n3;
            t = tn;
        }
        return;
    }
    for (; t < n_tiles; t += wstep) {
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        const u32x4 r0 = g[lane], r1 = g[64 + lane], r2 = g[128 + lane], r3 = g[192 + lane];
        const uint64_t i = t * 64u + lane;
        if (MODE == 0) {
            o.a[i] = r0.w ^ r3.x;
            o.b[i] = r1.y ^ r3.y + r1.z * 3u + r1.w ^ r3.z ^ r3.w;
            o.q[i] = (uint16_t)(r2.x >> 3);
        } else if (MODE == 1) {
            const u32x4 x = r0 ^ r1, y = r2 ^ r3;
            o.a[i] = x.x ^ x.y ^ y.z ^ y.w;
            o.b[i] = x.z + x.w * 3u + y.x + y.y;
            o.q[i] = (uint16_t)((x.x ^ y.w) >> 3);
        } else {
            u32x4 p0, p1, p2;
            lds_pass(tile, lane, r0, r1, r2, r3, p0, p1, p2);
            const uint32_t va = p0.w ^ p2.x, vb = p1.y + p1.z * 3u + p1.w;
            const uint16_t vq = (uint16_t)(p1.w >> 3);
            if (MODE == 2) {
                o.a[i] = va;
                o.b[i] = vb;
                o.q[i] = vq;
            } else if (MODE == 3) {
                acc ^= va ^ vb ^ vq;
            } else if (MODE == 4) {
                o.a[i] = va ^ vb ^ vq;
            } else if (MODE == 6) {
                // AoS: lane l packs frames l, l+1 (shuffled in) ... 16 B per lane per 4 frames:
                // lanes 0..15 store, each 16 B = (a,b) of two frames -> 1 KiB per wave (8 B/frame + q)
                const uint32_t a1 = __shfl_down(va, 1), b1 = __shfl_down(vb, 1);
                if ((lane & 1u) == 0)
                    *(u32x4 *)(o.a + 2 * i) = (u32x4){va, vb, a1, b1};
                o.q[i] = vq;
            }
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
    CK(hipMalloc(&o.a, n * 8));
    CK(hipMalloc(&o.b, n * 4));
    CK(hipMalloc(&o.q, n * 2));
    CK(hipMalloc(&o.sink, 64));
    CK(hipMemset(slab, 3, n * 64));
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
    const char *names[] = {"rw10", "rw10full", "lds", "lds_nost", "lds_1st", "lds_pipe", "lds_wide"};
    for (int bpc : {2, 4, 8}) {
        const dim3 g(cus * bpc);
#define RUN(M)                                                                                         \
    snprintf(nm, sizeof nm, "%s bpc=%d", names[M], bpc);                                            \
    timeit([&] { hipLaunchKernelGGL(k_v<M>, g, dim3(256), 0, 0, slab, tiles, o); }, nm)
        RUN(0); RUN(1); RUN(2); RUN(3); RUN(4); RUN(5); RUN(6);
    }
    return 0;
}
