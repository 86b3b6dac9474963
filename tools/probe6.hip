// probe6.hip -- store policy / staging / grid shape for the 64-B read + 10-B write stream
// (diagnostic, not product).  Build: hipcc -O3 --offload-arch=gfx950 -o probe6 probe6.hip
// Every variant: 16M x 64-B slots (1 GiB) read as 4 KiB wave tiles through the swizzled LDS
// tile, 3 SoA outputs (4 B, 4 B, 2 B per frame).
//   POL   store cache policy of the outputs: 0 plain, 1 nt, 2 sc1 nt, 3 sc0 sc1 nt, 4 sc1, 5 sc0 sc1
//   LPOL  tile-load policy: 0 plain, 1 nt, 2 sc1
//   STG   tiles whose outputs a wave stages in LDS before one 16-B-per-lane flush (0 = direct)
//   PF    tiles of prefetch in flight per wave (1 or 2)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int POL>
__device__ __forceinline__ void st32(uint32_t *p, uint32_t v)
{
    if (POL == 0) *p = v;
    else if (POL == 1) asm volatile("global_store_dword %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 2) asm volatile("global_store_dword %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 3) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 4) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
template <int POL>
__device__ __forceinline__ void st16(uint16_t *p, uint32_t v)
{
    if (POL == 0) *p = (uint16_t)v;
    else if (POL == 1) asm volatile("global_store_short %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 2) asm volatile("global_store_short %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 3) asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 4) asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_short %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
template <int POL>
__device__ __forceinline__ void st128(void *p, u32x4 v)
{
    if (POL == 0) *(u32x4 *)p = v;
    else if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
template <int LPOL>
__device__ __forceinline__ u32x4 ld128(const u32x4 *p)
{
    if (LPOL == 1) return __builtin_nontemporal_load(p);
    if (LPOL == 2) {
        u32x4 v;
        asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        return v;
    }
    return *p;
}

struct Out {
    uint32_t *a, *b;
    uint16_t *q;
    uint32_t *sink;
};

template <int POL, int LPOL, int STG, int PF, int ORD = 0>
__global__ __launch_bounds__(256) void k_v(const uint8_t *slab, uint64_t n_tiles, Out o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    // staged outputs: per wave STG tiles x (256 B a, 256 B b, 128 B q)
    __shared__ __attribute__((aligned(16))) uint32_t s_out[4][(STG ? STG : 1) * 160];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t S = STG ? STG : 1;
    // wave's unit = S consecutive tiles; the block's 4 waves take 4 consecutive units
    uint64_t ustep = (uint64_t)gridDim.x * 4;
    uint64_t u = (uint64_t)blockIdx.x * 4 + wv;
    uint64_t uend = n_tiles / (STG ? STG : 1);
    if (ORD == 1) { // contiguous range per wave
        const uint64_t nw = (uint64_t)gridDim.x * 4, per = (uend + nw - 1) / nw;
        u = ((uint64_t)blockIdx.x * 4 + wv) * per;
        uend = u + per < uend ? u + per : uend;
        ustep = 1;
    } else if (ORD == 2) { // contiguous range per block, its 4 waves interleaved
        const uint64_t per = (uend + gridDim.x - 1) / gridDim.x;
        u = (uint64_t)blockIdx.x * per + wv;
        uend = (uint64_t)blockIdx.x * per + per < uend ? (uint64_t)blockIdx.x * per + per : uend;
        ustep = 4;
    }
    const uint64_t n_units = uend;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    u32x4 r[PF][4];
    auto issue = [&](int slot, uint64_t tt) {
        const u32x4 *g = (const u32x4 *)(slab + tt * 4096u);
        r[slot][0] = ld128<LPOL>(g + lane);
        r[slot][1] = ld128<LPOL>(g + 64 + lane);
        r[slot][2] = ld128<LPOL>(g + 128 + lane);
        r[slot][3] = ld128<LPOL>(g + 192 + lane);
    };
    // flattened per-wave sequence of tiles: unit u, j = 0..S-1
    uint64_t cu = u;
    uint32_t cj = 0;
    auto tile_of = [&](uint64_t uu, uint32_t j) { return uu * S + j; };
    // prefetch PF tiles
    uint64_t pu = u;
    uint32_t pj = 0;
    auto adv = [&](uint64_t &uu, uint32_t &j) {
        if (++j == S) { j = 0; uu += ustep; }
    };
#pragma unroll
    for (int s = 0; s < PF; s++) {
        issue(s, tile_of(pu < n_units ? pu : u, pj));
        adv(pu, pj);
    }
    int slot = 0;
    for (; cu < n_units;) {
        u32x4 v0 = r[0][0], v1 = r[0][1], v2 = r[0][2], v3 = r[0][3];
        if (PF == 2) {
            r[0][0] = r[1][0]; r[0][1] = r[1][1]; r[0][2] = r[1][2]; r[0][3] = r[1][3];
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            const u32x4 v = k == 0 ? v0 : k == 1 ? v1 : k == 2 ? v2 : v3;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v;
        }
        __builtin_amdgcn_wave_barrier();
        issue(PF - 1, tile_of(pu < n_units ? pu : cu, pj));
        adv(pu, pj);
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)];
        const u32x4 p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        const uint32_t va = p0.w ^ p2.x, vb = p1.y + p1.z * 3u + p1.w;
        const uint32_t vq = (p1.w >> 3) & 0xffffu;
        const uint64_t t = tile_of(cu, cj);
        const uint64_t i = t * 64u + lane;
        if (STG == 0) {
            st32<POL>(o.a + i, va);
            st32<POL>(o.b + i, vb);
            st16<POL>(o.q + i, vq);
        } else {
            uint32_t *so = s_out[wv];
            so[cj * 64 + lane] = va;
            so[S * 64 + cj * 64 + lane] = vb;
            ((uint16_t *)(so + 2 * S * 64))[cj * 64 + lane] = (uint16_t)vq;
            if (cj == S - 1) {
                __builtin_amdgcn_wave_barrier();
                const uint64_t i0 = cu * S * 64u; // first frame of the unit
                // a: S*256 B = S*16 chunks of 16 B
                for (uint32_t c = lane; c < S * 16; c += 64)
                    st128<POL>((uint8_t *)(o.a + i0) + c * 16, ((const u32x4 *)so)[c]);
                for (uint32_t c = lane; c < S * 16; c += 64)
                    st128<POL>((uint8_t *)(o.b + i0) + c * 16, ((const u32x4 *)(so + S * 64))[c]);
                for (uint32_t c = lane; c < S * 8; c += 64)
                    st128<POL>((uint8_t *)(o.q + i0) + c * 16, ((const u32x4 *)(so + 2 * S * 64))[c]);
                __builtin_amdgcn_wave_barrier();
            }
        }
        adv(cu, cj);
    }
    (void)slot;
}

__global__ __launch_bounds__(256) void k_read(const uint8_t *slab, uint64_t n_tiles, Out o)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < n_tiles; t += (uint64_t)gridDim.x * 4) {
        const u32x4 *g = (const u32x4 *)(slab + t * 4096u);
        const u32x4 r0 = g[lane], r1 = g[64 + lane], r2 = g[128 + lane], r3 = g[192 + lane];
        acc ^= r0.x ^ r1.y ^ r2.z ^ r3.w ^ r0.w ^ r1.x;
    }
    if (acc == 0x12345678u)
        o.sink[0] = acc;
}

int main(int argc, char **argv)
{
    const uint64_t n = 1ull << 24, tiles = n / 64;
    const int R = 4; // slab / output sets rotated across launches (4 GiB + 4 x 160 MiB)
    uint8_t *slab[R];
    Out o[R];
    {
        std::vector<uint32_t> h(n * 16);
        for (int s = 0; s < R; s++) {
            CK(hipMalloc(&slab[s], n * 64));
            CK(hipMalloc(&o[s].a, n * 4));
            CK(hipMalloc(&o[s].b, n * 4));
            CK(hipMalloc(&o[s].q, n * 2));
            CK(hipMalloc(&o[s].sink, 64));
            for (uint64_t i = 0; i < h.size(); i++)
                h[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7) ^ (uint32_t)s;
            CK(hipMemcpy(slab[s], h.data(), n * 64, hipMemcpyHostToDevice));
        }
    }
    uint8_t *junk;
    CK(hipMalloc(&junk, 512ull << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int cus = 256;
    // rot: 1 = same slab/outputs every launch, R = rotate; flush: 512 MiB memset between launches
    auto timeit = [&](auto launch, const char *name, int rot, bool flush) {
        for (int w = 0; w < 4; w++)
            launch(w % rot);
        std::vector<float> ts;
        for (int r = 0; r < 24; r++) {
            if (flush)
                hipMemsetAsync(junk, r, 512ull << 20, 0);
            hipEventRecord(e0, 0);
            launch(r % rot);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-34s rot%d flush%d %.4f ms  %7.1f GB/s(74B)\n", name, rot, (int)flush, ts[12],
               74.0 * n / (ts[12] * 1e-3) / 1e9);
        fflush(stdout);
    };
    char nm[96];
#define RUN(POL, LPOL, STG, PF, BPC, ORD)                                                              \
    snprintf(nm, sizeof nm, "pol%d lpol%d stg%d pf%d bpc%d ord%d", POL, LPOL, STG, PF, BPC, ORD);       \
    timeit([&](int s) { hipLaunchKernelGGL((k_v<POL, LPOL, STG, PF, ORD>), dim3(cus * BPC), dim3(256), 0, 0, slab[s], tiles, o[s]); }, nm, R, 0);
    RUN(1, 1, 0, 1, 2, 0) RUN(1, 1, 0, 1, 2, 1) RUN(1, 1, 0, 1, 2, 2)
    RUN(1, 1, 0, 1, 3, 0) RUN(1, 1, 0, 1, 3, 1) RUN(1, 1, 0, 1, 3, 2)
    RUN(1, 1, 0, 2, 2, 0) RUN(1, 1, 0, 2, 2, 1) RUN(1, 1, 0, 2, 1, 1)
    RUN(1, 1, 8, 1, 2, 0) RUN(1, 1, 8, 1, 2, 1)
    return 0;
}
