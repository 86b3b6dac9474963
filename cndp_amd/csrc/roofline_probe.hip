// roofline_probe.hip -- same-box access-shape ceilings for bench.py (measurement
// only: nothing in the product links or calls this; libcndp_probe.so is loaded by
// bench.py beside libcndp_gpu.so).
//
// Each probe moves exactly the bytes of one config's kernel in the same access
// shape -- the frame reads, the per-frame result stores -- and does nothing
// else: no parse, no Toeplitz, no FIB gathers, no bins.  Timed in the same
// process, over the same ring of batches and outputs as the product kernel,
// its time is the ceiling that kernel's memory traffic allows on this box, so
// kernel_ms / probe_ms separates "this box's HBM" from "this kernel".
//
//   cndp_probe_slots    C2 / C3: packed 64-B slots, a wave tile of 64 frames
//                       read as 4 x 1 KiB coalesced non-temporal loads (as
//                       k_classify_stream), staged through the XOR-swizzled
//                       LDS tile, `pf` tiles in flight per wave; per frame the
//                       given 4 / 4 / 2-B outputs stored non-temporal.
//   cndp_probe_slots_bal  the same with the balanced schedule of
//                       k_classify_stream_bal (512-thread blocks, one a CU, the
//                       block's tiles shared by its waves through an LDS counter).
//   cndp_probe_windows  C4 / C5 (static, or bpc 0: k_cnet_defer's balanced
//                       schedule): the first 64 B of each frame at a stride or
//                       at u64 offsets, 4 lanes a frame, 16 frames a load
//                       instruction (as k_cnet_defer's cs_issue), the offsets
//                       read coalesced; per frame the given 4 / 4 / 2 / 1 / 2-B
//                       outputs stored non-temporal.
// Outputs are written so that the stores cannot be removed; their values mean
// nothing.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
template <typename T>
__device__ __forceinline__ void stnt(T *p, T v)
{
    __builtin_nontemporal_store(v, p);
}

struct ProbeOut {
    uint32_t *a, *b; // 4-B outputs (nh, hash)
    uint16_t *q;     // 2-B output (queue)
    uint8_t *e;      // 1-B output (edge)
    uint16_t *t;     // 2-B output (the speculation model's packet types)
};

__device__ __forceinline__ void probe_store(const ProbeOut &o, uint64_t i, uint32_t v)
{
    if (o.a)
        stnt(o.a + i, v);
    if (o.b)
        stnt(o.b + i, v * 2654435761u);
    if (o.q)
        stnt(o.q + i, (uint16_t)(v >> 7));
    if (o.e)
        stnt(o.e + i, (uint8_t)(v >> 3));
    if (o.t)
        stnt(o.t + i, (uint16_t)(v >> 11));
}

template <int PF>
__global__ __launch_bounds__(256) void k_probe_slots(const uint8_t *slab, uint64_t n_tiles, ProbeOut o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[4][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint64_t wstep = (uint64_t)gridDim.x * 4u, t0 = (uint64_t)blockIdx.x * 4u + wv;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    u32x4 r[PF][4];
    auto issue = [&](u32x4(&d)[4], uint64_t tt) {
        const uint8_t *g = slab + (tt < n_tiles ? tt : n_tiles - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
#pragma unroll
    for (int s = 0; s < PF; s++)
        issue(r[s], t0 + s * wstep);
    for (uint64_t t = t0; t < n_tiles; t += wstep) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            v[k] = r[0][k];
#pragma unroll
        for (int s = 0; s + 1 < PF; s++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                r[s][k] = r[s + 1][k];
        issue(r[PF - 1], t + PF * wstep);
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
        probe_store(o, t * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
    }
}

// the C2 / C3 kernel's balanced schedule (k_classify_stream_bal): one 512-thread
// block a CU, the block's tiles (blockIdx + k * gridDim) handed to its 8 waves
// by an LDS counter, each wave's first three static, the next index drawn a
// trip before its load; 2 tiles in flight
__global__ __launch_bounds__(512) void k_probe_slots_bal(const uint8_t *slab, uint64_t n_tiles, ProbeOut o)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[8][256];
    __shared__ uint32_t s_next;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint64_t G = gridDim.x, b = blockIdx.x, NONE = ~0ull;
    const uint64_t nk = b < n_tiles ? (n_tiles - b + G - 1) / G : 0;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    if (threadIdx.x == 0)
        s_next = 24u;
    auto tile_of = [&](uint64_t k) { return k < nk ? b + k * G : NONE; };
    auto issue = [&](u32x4(&d)[4], uint64_t tt) {
        const uint8_t *g = slab + (tt < n_tiles ? tt : n_tiles - 1u) * 4096u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = ldnt(g + (64u * k + lane) * 16u);
    };
    uint64_t q0 = tile_of(wv), q1 = tile_of(wv + 8u), q2 = tile_of(wv + 16u);
    u32x4 r[2][4];
    issue(r[0], q0);
    issue(r[1], q1);
    __syncthreads();
    auto draw = [&](uint64_t prev) -> uint32_t {
        uint32_t v = 0;
        if (prev != NONE && lane == 0)
            v = atomicAdd(&s_next, 1u);
        return v;
    };
    uint32_t kv = draw(q2);
    while (q0 != NONE) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        issue(r[1], q2);
        const uint64_t qn = q2 == NONE ? NONE : tile_of((uint32_t)__builtin_amdgcn_readfirstlane((int)kv));
        kv = draw(qn);
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
        probe_store(o, q0 * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
        q0 = q1;
        q1 = q2;
        q2 = qn;
    }
}

__global__ __launch_bounds__(256) void k_probe_windows(const uint8_t *slab, uint64_t stride, const uint64_t *offs,
                                                       uint64_t data_off, uint64_t n, ProbeOut o)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t tiles = n / 64u;
    for (uint64_t g = (uint64_t)blockIdx.x * 4u + wv; g < tiles; g += (uint64_t)gridDim.x * 4u) {
        const uint64_t mine = (offs ? offs[g * 64u + lane] : (g * 64u + lane) * stride) + data_off;
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
        probe_store(o, g * 64u + lane, res);
    }
}

// the cnet kernel's balanced schedule (k_cnet_defer with BAL): one 1024-thread
// block a CU, the block's tiles in the static schedule's round order handed to
// its 16 waves by an LDS counter (each wave's first tile static, the next
// drawn a tile ahead)
__global__ __launch_bounds__(1024) void k_probe_windows_bal(const uint8_t *slab, uint64_t stride, const uint64_t *offs,
                                                            uint64_t data_off, uint64_t n, ProbeOut o)
{
    __shared__ uint32_t s_next;
    constexpr uint32_t NW = 16;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t tiles = n / 64u, G = gridDim.x, bk = blockIdx.x, ws = G * NW, NONE = ~0ull;
    uint64_t nk = 0;
    for (uint32_t w = 0; w < NW; w++)
        nk += bk * NW + w < tiles ? (tiles - bk * NW - w + ws - 1) / ws : 0;
    auto tile_k = [&](uint64_t k) { return k < nk ? (k / NW) * ws + bk * NW + k % NW : NONE; };
    if (threadIdx.x == 0)
        s_next = NW;
    __syncthreads();
    uint64_t g = tile_k(wv);
    uint32_t kv = 0;
    if (g != NONE && lane == 0)
        kv = atomicAdd(&s_next, 1u);
    while (g != NONE) {
        const uint64_t gn = tile_k((uint32_t)__builtin_amdgcn_readfirstlane((int)kv));
        if (gn != NONE && lane == 0)
            kv = atomicAdd(&s_next, 1u);
        const uint64_t mine = (offs ? offs[g * 64u + lane] : (g * 64u + lane) * stride) + data_off;
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
        probe_store(o, g * 64u + lane, res);
        g = gn;
    }
}

static int g_cus;

static int cus()
{
    if (!g_cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_cus = 256;
    }
    return g_cus;
}

extern "C" {

// C2 / C3 shape: n frames in packed 64-B slots (whole tiles only; n % 64
// frames are not read), pf = 1 or 2 tiles in flight, bpc 256-thread blocks a CU
int cndp_probe_slots(const void *slab, uint64_t n, uint32_t *o_a, uint32_t *o_b, uint16_t *o_q, int pf, int bpc,
                     void *stream)
{
    const uint64_t nt = n / 64u;
    if (!slab || nt == 0 || bpc < 1 || bpc > 8 || (pf != 1 && pf != 2))
        return -22;
    const ProbeOut o{o_a, o_b, o_q, nullptr, nullptr};
    const dim3 grid((unsigned)(cus() * bpc)), blk(256);
    if (pf == 1)
        hipLaunchKernelGGL(k_probe_slots<1>, grid, blk, 0, (hipStream_t)stream, (const uint8_t *)slab, nt, o);
    else
        hipLaunchKernelGGL(k_probe_slots<2>, grid, blk, 0, (hipStream_t)stream, (const uint8_t *)slab, nt, o);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// C2 / C3 shape with the balanced schedule: one 512-thread block a CU
int cndp_probe_slots_bal(const void *slab, uint64_t n, uint32_t *o_a, uint32_t *o_b, uint16_t *o_q, void *stream)
{
    const uint64_t nt = n / 64u;
    if (!slab || nt == 0)
        return -22;
    const ProbeOut o{o_a, o_b, o_q, nullptr, nullptr};
    const uint32_t g = (uint64_t)cus() < nt ? (uint32_t)cus() : (uint32_t)nt;
    hipLaunchKernelGGL(k_probe_slots_bal, dim3(g), dim3(512), 0, (hipStream_t)stream, (const uint8_t *)slab, nt, o);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// C4 / C5 shape: the first 64 B of each of n frames (whole 64-frame tiles),
// frame i at offs[i] (if offs) or i * stride, plus data_off; the caller keeps
// every window inside the slab.  bpc 256-thread blocks a CU, or bpc 0: the
// balanced schedule (k_probe_windows_bal)
int cndp_probe_windows(const void *slab, uint64_t stride, const uint64_t *offs, uint64_t data_off, uint64_t n,
                       uint32_t *o_a, uint32_t *o_b, uint16_t *o_q, uint8_t *o_e, uint16_t *o_t, int bpc, void *stream)
{
    if (!slab || n < 64 || bpc < 0 || bpc > 8)
        return -22;
    const ProbeOut o{o_a, o_b, o_q, o_e, o_t};
    if (bpc == 0) // the balanced schedule: one 1024-thread block a CU
        hipLaunchKernelGGL(k_probe_windows_bal, dim3((unsigned)cus()), dim3(1024), 0, (hipStream_t)stream,
                           (const uint8_t *)slab, stride, offs, data_off, n, o);
    else
        hipLaunchKernelGGL(k_probe_windows, dim3((unsigned)(cus() * bpc)), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t *)slab, stride, offs, data_off, n, o);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
}
