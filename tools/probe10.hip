// probe10.hip -- static vs dynamic tile scheduling on the probe access shapes
// (diagnostic, not product).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe10 tools/probe10.hip
//
// The k_cnet_defer stamps (tools/cnet_stamps.py) show the waves of one launch
// ending up to 25 us (C4) / 100 us (C5) apart with equal shares of tiles.  Here
// the bench probes' shapes run with the static schedule (wave w takes tiles
// w, w + W, ...) and with chunks of C tiles handed out by a device counter
// (each wave grabs its next chunk when it starts a chunk; the last wave to
// finish resets the counters for the next launch).
//   slots : C3 -- 16M packed 64-B slots, 4 x 1 KiB nt loads a tile through the
//           LDS tile, 2 tiles in flight, nh + hash + queue stored
//   win5  : C5 -- 32M frames at a 1536-B stride, 64-B windows, nh stored
//   win4  : C4 -- 16M IMIX frames at u64 offsets, nh + hash + queue stored
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
};

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const u32x4 *)p); }

__device__ __forceinline__ void put(const Out &o, uint64_t i, uint32_t v)
{
    if (o.a)
        __builtin_nontemporal_store(v, o.a + i);
    if (o.b)
        __builtin_nontemporal_store(v * 2654435761u, o.b + i);
    if (o.q)
        __builtin_nontemporal_store((uint16_t)(v >> 7), o.q + i);
}

// A wave's tile sequence. C == 0: static (t0, t0 + W, ...); otherwise chunks
// of C tiles, the first = the wave's index, the rest from ctr[0] (+ W), the
// next chunk grabbed when a chunk starts. ~0u = the end.
struct Seq {
    uint32_t cur, pos, nx_v, done;
};

// Hybrid (C = 0x100 * R + K): tiles [0, ts) static as C == 0 (ts = nt - nt / R,
// a multiple of the wave count), then chunks of K tiles of [ts, nt) from eight
// pools, one per XCD (blockIdx % 8), each with its own counter (128 B apart);
// a wave whose pool is empty takes from the next one.
struct HSeq {
    uint32_t t, step, ts; // static: next tile, stride, end
    uint32_t pool, tried, cur, pos, K, nt, base, per;
};
__device__ __forceinline__ uint32_t hseq_grab(HSeq &h, uint32_t *ctr, uint32_t lane)
{
    while (h.tried < 8u) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(ctr + 32u * h.pool, 1u);
        g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
        if (g < h.per) { // chunk g of pool p: tiles base + (g * 8 + p) * K ...
            const uint32_t t = h.base + (g * 8u + h.pool) * h.K;
            if (t < h.nt)
                return t;
        }
        h.pool = (h.pool + 1u) & 7u;
        h.tried++;
    }
    return ~0u;
}
__device__ __forceinline__ uint32_t hseq_next(HSeq &h, uint32_t *ctr, uint32_t lane)
{
    if (h.t < h.ts) {
        const uint32_t t = h.t;
        h.t += h.step;
        return t;
    }
    if (h.cur != ~0u && h.pos < h.K && h.cur + h.pos < h.nt)
        return h.cur + h.pos++;
    h.cur = hseq_grab(h, ctr, lane);
    h.pos = 0;
    if (h.cur == ~0u)
        return ~0u;
    return h.cur + h.pos++;
}
__device__ __forceinline__ void hseq_init(HSeq &h, uint32_t C, uint32_t gw, uint32_t W, uint32_t nt)
{
    const uint32_t R = (C >> 8) & 0xffu;
    h.K = C & 0xffu;
    h.nt = nt;
    uint32_t res = nt / R;
    h.ts = (nt - res) / W * W; // the static part: whole rounds of the waves
    h.base = h.ts;
    h.per = (nt - h.ts + 8u * h.K - 1u) / (8u * h.K); // chunks per pool
    h.t = gw;
    h.step = W;
    h.pool = blockIdx.x & 7u;
    h.tried = 0;
    h.cur = ~0u;
    h.pos = 0;
}

__device__ __forceinline__ void seq_init(Seq &s, uint32_t C, uint32_t gw, uint32_t nt, uint32_t *ctr, uint32_t lane)
{
    s.cur = C ? gw * C : gw;
    s.pos = 0;
    s.done = s.cur >= nt;
    s.nx_v = 0;
    if (C && !s.done && lane == 0)
        s.nx_v = atomicAdd(ctr, 1u);
}

__device__ __forceinline__ uint32_t seq_next(Seq &s, uint32_t C, uint32_t W, uint32_t nt, uint32_t *ctr,
                                             uint32_t lane)
{
    if (s.done)
        return ~0u;
    uint32_t t;
    if (!C) {
        t = s.cur;
        s.cur += W;
    } else {
        if (s.pos == C) {
            const uint32_t nx = (uint32_t)__builtin_amdgcn_readlane((int)s.nx_v, 0) + W;
            s.cur = nx * C;
            s.pos = 0;
            if (s.cur < nt && lane == 0)
                s.nx_v = atomicAdd(ctr, 1u);
        }
        t = s.cur + s.pos++;
    }
    if (t >= nt) {
        s.done = 1;
        return ~0u;
    }
    return t;
}

__device__ __forceinline__ void hseq_fini(uint32_t *ctr, uint32_t lane)
{
    if (lane == 0) {
        __threadfence();
        const uint32_t W = gridDim.x * (blockDim.x / 64u);
        if (atomicAdd(ctr + 32u * 8u, 1u) == W - 1u)
            for (uint32_t k = 0; k < 9; k++)
                __hip_atomic_store(ctr + 32u * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ void seq_fini(uint32_t C, uint32_t *ctr, uint32_t lane)
{
    if (C && lane == 0) {
        __threadfence();
        const uint32_t W = gridDim.x * (blockDim.x / 64u);
        if (atomicAdd(ctr + 1, 1u) == W - 1u) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ __launch_bounds__(256) void k_slots(const uint8_t *slab, uint32_t nt, Out o, uint32_t C, uint32_t *ctr)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t W = gridDim.x * 4u, gw = blockIdx.x * 4u + wv;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    Seq s;
    seq_init(s, C, gw, nt, ctr, lane);
    u32x4 r[2][4];
    auto issue = [&](u32x4(&d)[4], uint32_t tt) {
        const uint8_t *g = slab + (uint64_t)(tt < nt ? tt : nt - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
    uint32_t q0 = seq_next(s, C, W, nt, ctr, lane), q1 = seq_next(s, C, W, nt, ctr, lane);
    issue(r[0], q0);
    issue(r[1], q1);
    while (q0 != ~0u) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        const uint32_t q2 = seq_next(s, C, W, nt, ctr, lane);
        issue(r[1], q2);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v[k];
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)], p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        put(o, (uint64_t)q0 * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
        q0 = q1;
        q1 = q2;
    }
    seq_fini(C, ctr, lane);
}

__global__ __launch_bounds__(256) void k_win(const uint8_t *slab, uint64_t stride, const uint64_t *offs, uint32_t nt,
                                             Out o, uint32_t C, uint32_t *ctr)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u, gw = blockIdx.x * 4u + wv;
    Seq s;
    seq_init(s, C, gw, nt, ctr, lane);
    for (uint32_t g = seq_next(s, C, W, nt, ctr, lane); g != ~0u; g = seq_next(s, C, W, nt, ctr, lane)) {
        const uint64_t i = (uint64_t)g * 64u + lane;
        const uint64_t mine = offs ? offs[i] : i * stride;
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
        put(o, i, res);
    }
    seq_fini(C, ctr, lane);
}

__global__ __launch_bounds__(256) void k_slots_h(const uint8_t *slab, uint32_t nt, Out o, uint32_t C, uint32_t *ctr)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t W = gridDim.x * 4u, gw = blockIdx.x * 4u + wv;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    HSeq h;
    hseq_init(h, C, gw, W, nt);
    u32x4 r[2][4];
    auto issue = [&](u32x4(&d)[4], uint32_t tt) {
        const uint8_t *g = slab + (uint64_t)(tt < nt ? tt : nt - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
    uint32_t q0 = hseq_next(h, ctr, lane), q1 = hseq_next(h, ctr, lane);
    issue(r[0], q0);
    issue(r[1], q1);
    while (q0 != ~0u) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        const uint32_t q2 = q1 == ~0u ? ~0u : hseq_next(h, ctr, lane);
        issue(r[1], q2);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v[k];
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)], p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        put(o, (uint64_t)q0 * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
        q0 = q1;
        q1 = q2;
    }
    hseq_fini(ctr, lane);
}

__global__ __launch_bounds__(256) void k_win_h(const uint8_t *slab, uint64_t stride, const uint64_t *offs, uint32_t nt,
                                               Out o, uint32_t C, uint32_t *ctr)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u, gw = blockIdx.x * 4u + wv;
    HSeq h;
    hseq_init(h, C, gw, W, nt);
    for (uint32_t g = hseq_next(h, ctr, lane); g != ~0u; g = hseq_next(h, ctr, lane)) {
        const uint64_t i = (uint64_t)g * 64u + lane;
        const uint64_t mine = offs ? offs[i] : i * stride;
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
        put(o, i, res);
    }
    hseq_fini(ctr, lane);
}

// static schedule, PF tiles in flight per wave (C3 shape sweep)
template <int PF>
__global__ __launch_bounds__(256) void k_slots_pf(const uint8_t *slab, uint32_t nt, Out o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t W = gridDim.x * 4u, t0 = blockIdx.x * 4u + wv;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    u32x4 r[PF][4];
    auto issue = [&](u32x4(&d)[4], uint32_t tt) {
        const uint8_t *g = slab + (uint64_t)(tt < nt ? tt : nt - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
#pragma unroll
    for (int q = 0; q < PF; q++)
        issue(r[q], t0 + q * W);
    for (uint32_t t = t0; t < nt; t += W) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
#pragma unroll
            for (int q = 0; q + 1 < PF; q++)
                r[q][k] = r[q + 1][k];
        }
        issue(r[PF - 1], t + PF * W);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v[k];
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)], p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        put(o, (uint64_t)t * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
    }
}

// NW-wave blocks; the block's tiles (blockIdx + k * gridDim) handed to its
// waves by an LDS counter (BAL) or statically (wave w takes k = w, w + NW, ...);
// 2 tiles in flight, the next index grabbed a trip before it is needed
template <int NW, bool BAL>
__global__ __launch_bounds__(NW * 64) void k_slots_bal(const uint8_t *slab, uint32_t nt, Out o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[NW][256];
    __shared__ uint32_t s_ctr;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t nk = b < nt ? (nt - b + G - 1u) / G : 0u; // the block's tiles
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    if (BAL) {
        if (threadIdx.x == 0)
            s_ctr = NW * 3u; // indices < 3 NW are taken statically below
        __syncthreads();
    }
    uint32_t ks = wv; // static: the wave's next k
    auto grab = [&]() -> uint32_t {
        uint32_t k;
        if (BAL && ks >= NW * 3u) {
            uint32_t v = 0;
            if (lane == 0)
                v = atomicAdd(&s_ctr, 1u);
            k = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        } else {
            k = ks;
            ks += NW;
        }
        return k < nk ? b + k * G : ~0u;
    };
    u32x4 r[2][4];
    auto issue = [&](u32x4(&d)[4], uint32_t tt) {
        const uint8_t *g = slab + (uint64_t)(tt < nt ? tt : nt - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
    uint32_t q0 = grab(), q1 = grab(), q2 = grab();
    issue(r[0], q0);
    issue(r[1], q1);
    while (q0 != ~0u) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        issue(r[1], q2);
        const uint32_t q3 = q2 == ~0u ? ~0u : grab();
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v[k];
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)], p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        put(o, (uint64_t)q0 * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
        q0 = q1;
        q1 = q2;
        q2 = q3;
    }
}

template <class F> static float timed(F launch)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++)
        launch();
    std::vector<float> ts;
    for (int r = 0; r < 11; r++) {
        CK(hipEventRecord(a, 0));
        launch();
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
    uint32_t *ctr;
    CK(hipMalloc((void **)&slab, bytes));
    CK(hipMalloc((void **)&offs, n4 * 8));
    CK(hipMalloc((void **)&ctr, 9 * 128));
    CK(hipMemset(ctr, 0, 9 * 128));
    CK(hipMemcpy(offs, hoff.data(), n4 * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(ncu * 16), dim3(256), 0, 0, (uint32_t *)slab, bytes / 4);
    Out full{}, nh{};
    CK(hipMalloc((void **)&full.a, n5 * 4));
    CK(hipMalloc((void **)&full.b, n5 * 4));
    CK(hipMalloc((void **)&full.q, n5 * 2));
    nh.a = full.a;
    CK(hipDeviceSynchronize());
    if (getenv("PROBE10_BAL")) { // C3 shape: static vs LDS-balanced waves inside big blocks, 4-GiB ring
        const uint32_t nt = (uint32_t)(n4 / 64);
        int k = 0;
        auto ring = [&]() { return slab + (uint64_t)(k++ & 3) * n4 * 64; };
        printf("slots C3 256-thread blocks x2/CU static %.4f\n", timed([&] {
                   hipLaunchKernelGGL(k_slots_pf<2>, dim3(ncu * 2), dim3(256), 0, 0, ring(), nt, full);
               }));
        for (int rep = 0; rep < 2; rep++) {
            printf("slots C3 balanced x1/CU: 512-thread %.4f  640-thread %.4f  768-thread %.4f  896-thread %.4f ms\n",
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<8, true>), dim3(ncu), dim3(512), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<10, true>), dim3(ncu), dim3(640), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<12, true>), dim3(ncu), dim3(768), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<14, true>), dim3(ncu), dim3(896), 0, 0, ring(), nt, full); }));
            fflush(stdout);
        }
        for (int rep = 0; rep < 2; rep++) {
            printf("slots C3 512-thread x2/CU: static %.4f balanced %.4f; 1024-thread x1/CU: static %.4f balanced %.4f; "
                   "512-thread x1/CU: static %.4f balanced %.4f ms\n",
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<8, false>), dim3(ncu * 2), dim3(512), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<8, true>), dim3(ncu * 2), dim3(512), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<16, false>), dim3(ncu), dim3(1024), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<16, true>), dim3(ncu), dim3(1024), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<8, false>), dim3(ncu), dim3(512), 0, 0, ring(), nt, full); }),
                   timed([&] { hipLaunchKernelGGL((k_slots_bal<8, true>), dim3(ncu), dim3(512), 0, 0, ring(), nt, full); }));
            fflush(stdout);
        }
        return 0;
    }
    if (getenv("PROBE10_SHAPES")) { // C3 shape sweep: tiles in flight x blocks a CU, 4 batches in a ring
        const uint32_t nt = (uint32_t)(n4 / 64);
        for (int pf : {1, 2, 3, 4}) {
            printf("slots C3 pf%d:", pf);
            for (int bpc : {1, 2, 3, 4, 6, 8}) {
                int k = 0;
                const float ms = timed([&] {
                    const uint8_t *sl = slab + (uint64_t)(k++ & 3) * n4 * 64; // a ring of 4 GiB
                    const dim3 g(ncu * bpc), b(256);
                    if (pf == 1)
                        hipLaunchKernelGGL(k_slots_pf<1>, g, b, 0, 0, sl, nt, full);
                    else if (pf == 2)
                        hipLaunchKernelGGL(k_slots_pf<2>, g, b, 0, 0, sl, nt, full);
                    else if (pf == 3)
                        hipLaunchKernelGGL(k_slots_pf<3>, g, b, 0, 0, sl, nt, full);
                    else
                        hipLaunchKernelGGL(k_slots_pf<4>, g, b, 0, 0, sl, nt, full);
                });
                printf("  bpc%d %.4f", bpc, ms);
            }
            printf(" ms\n");
            fflush(stdout);
        }
        return 0;
    }
    // C == 0: static; otherwise hybrid 0x100 * R + K (reserve 1/R, chunks of K)
    const uint32_t Hs[] = {0x0802, 0x1002, 0x1004, 0x2002};
    for (int bpc : {2, 4}) {
        printf("slots C3 bpc%d: static %.4f", bpc, timed([&] {
                   hipLaunchKernelGGL(k_slots, dim3(ncu * bpc), dim3(256), 0, 0, slab, (uint32_t)(n4 / 64), full, 0u, ctr);
               }));
        for (uint32_t C : Hs)
            printf("  h%x %.4f", C, timed([&] {
                       hipLaunchKernelGGL(k_slots_h, dim3(ncu * bpc), dim3(256), 0, 0, slab, (uint32_t)(n4 / 64), full,
                                          C, ctr);
                   }));
        printf(" ms\n");
        fflush(stdout);
    }
    for (int bpc : {4, 8}) {
        printf("win5 C5 bpc%d: static %.4f", bpc, timed([&] {
                   hipLaunchKernelGGL(k_win, dim3(ncu * bpc), dim3(256), 0, 0, slab, stride, (const uint64_t *)nullptr,
                                      (uint32_t)(n5 / 64), nh, 0u, ctr);
               }));
        for (uint32_t C : Hs)
            printf("  h%x %.4f", C, timed([&] {
                       hipLaunchKernelGGL(k_win_h, dim3(ncu * bpc), dim3(256), 0, 0, slab, stride,
                                          (const uint64_t *)nullptr, (uint32_t)(n5 / 64), nh, C, ctr);
                   }));
        printf(" ms\n");
        printf("win4 C4 bpc%d: static %.4f", bpc, timed([&] {
                   hipLaunchKernelGGL(k_win, dim3(ncu * bpc), dim3(256), 0, 0, slab, (uint64_t)0, offs,
                                      (uint32_t)(n4 / 64), full, 0u, ctr);
               }));
        for (uint32_t C : Hs)
            printf("  h%x %.4f", C, timed([&] {
                       hipLaunchKernelGGL(k_win_h, dim3(ncu * bpc), dim3(256), 0, 0, slab, (uint64_t)0, offs,
                                          (uint32_t)(n4 / 64), full, C, ctr);
                   }));
        printf(" ms\n");
        fflush(stdout);
    }
    uint32_t hc[9 * 32];
    CK(hipMemcpy(hc, ctr, sizeof(hc), hipMemcpyDeviceToHost));
    uint32_t nz = 0;
    for (uint32_t k = 0; k < 9; k++)
        nz += hc[32 * k] != 0;
    printf("counters left nonzero after the runs: %u (0 = reset by the last wave)\n", nz);
    return 0;
}
