// probe_drain.hip -- diagnostic (not product): how much of the C2 / C3 shape's
// time is the drain at the end of the balanced schedule, and whether handing
// tiles out across CUs at run time would recover it.
//
//   k_bal_stamp  k_probe_slots_bal (roofline_probe.hip) with each wave's end
//                time (s_memrealtime) and its XCD (HW_REG_XCC_ID) recorded
//   k_dyn        the same access shape, tiles handed out in chunks of C from
//                eight counters, one per XCD (each XCD starts on its own
//                eighth of the tiles, then takes from the others' eighths);
//                a wave draws its next chunk one chunk ahead (agent-scope
//                atomics, their round trip hidden behind the chunk's tiles);
//                the last wave to finish zeroes the counters for the next
//                launch.  Correct whatever XCD a wave reports (any XCD may
//                take from any counter); the XCD id only picks where to start.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
template <typename T>
__device__ __forceinline__ void stnt(T *p, T v)
{
    __builtin_nontemporal_store(v, p);
}

struct Out {
    uint32_t *a, *b;
    uint16_t *q;
};

__device__ __forceinline__ void store3(const Out &o, uint64_t i, uint32_t v)
{
    stnt(o.a + i, v);
    stnt(o.b + i, v * 2654435761u);
    stnt(o.q + i, (uint16_t)(v >> 7));
}

__device__ __forceinline__ uint32_t xcc_id()
{
    // HW_REG_XCC_ID (hwreg 20), bits 3:0
    return __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | ((4 - 1) << 11)) & 7u;
}

__device__ __forceinline__ void tile_work(const uint8_t *slab, uint64_t t, uint32_t lane, u32x4 *tile, const Out &o,
                                          const u32x4 (&v)[4])
{
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
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
    store3(o, t * 64u + lane, p0.w ^ p1.y ^ p1.z ^ p1.w ^ p2.x ^ p2.y);
}

__device__ __forceinline__ void issue4(const uint8_t *slab, uint64_t n_tiles, uint64_t tt, uint32_t lane,
                                       u32x4 (&d)[4])
{
    const uint8_t *g = slab + (tt < n_tiles ? tt : n_tiles - 1u) * 4096u;
#pragma unroll
    for (int k = 0; k < 4; k++)
        d[k] = ldnt(g + (64u * k + lane) * 16u);
}

// k_probe_slots_bal + per-wave end stamps {end time, xcc} at st[2 * (block * 8 + wave)]
__global__ __launch_bounds__(512) void k_bal_stamp(const uint8_t *slab, uint64_t n_tiles, Out o,
                                                   unsigned long long *st)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[8][256];
    __shared__ uint32_t s_next;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint64_t G = gridDim.x, b = blockIdx.x, NONE = ~0ull;
    const uint64_t nk = b < n_tiles ? (n_tiles - b + G - 1) / G : 0;
    if (threadIdx.x == 0)
        s_next = 24u;
    auto tile_of = [&](uint64_t k) { return k < nk ? b + k * G : NONE; };
    uint64_t q0 = tile_of(wv), q1 = tile_of(wv + 8u), q2 = tile_of(wv + 16u);
    u32x4 r[2][4];
    issue4(slab, n_tiles, q0, lane, r[0]);
    issue4(slab, n_tiles, q1, lane, r[1]);
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
        issue4(slab, n_tiles, q2, lane, r[1]);
        const uint64_t qn = q2 == NONE ? NONE : tile_of((uint32_t)__builtin_amdgcn_readfirstlane((int)kv));
        kv = draw(qn);
        tile_work(slab, q0, lane, tile, o, v);
        q0 = q1;
        q1 = q2;
        q2 = qn;
    }
    if (st && lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t w = (uint64_t)blockIdx.x * 8u + wv;
        st[2 * w] = __builtin_amdgcn_s_memrealtime();
        st[2 * w + 1] = xcc_id();
    }
}

// ctr: 8 counters 64 words apart (chunks drawn so far from each XCD's eighth),
// ctr[8 * 64]: arrivals.  C tiles a chunk.  A wave's next chunk is drawn when
// it starts a chunk and resolved when it starts the next one, so the atomic's
// round trip hides behind C tiles; an eighth found empty sends the wave on to
// the next one (synchronously, only at the end).
template <int C>
__global__ __launch_bounds__(512) void k_dyn(const uint8_t *slab, uint64_t n_tiles, Out o, uint32_t *ctr,
                                             unsigned long long *st)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[8][256];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint64_t NONE = ~0ull;
    const uint64_t nch = (n_tiles + C - 1) / C;
    const uint32_t x0 = xcc_id();
    auto lo = [&](uint32_t e8) { return nch * e8 / 8u; };
    uint32_t e = 0, xe = x0;
    auto issue_grab = [&]() -> uint32_t {
        uint32_t got = 0;
        if (lane == 0)
            got = __hip_atomic_fetch_add(&ctr[64u * xe], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return got;
    };
    auto resolve = [&](uint32_t raw) -> uint64_t {
        for (;;) {
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)raw);
            const uint64_t c = lo(xe) + r0;
            if (c < lo(xe + 1u))
                return c;
            if (++e == 8u)
                return NONE;
            xe = (x0 + e) & 7u;
            raw = issue_grab();
        }
    };
    uint64_t c0 = resolve(issue_grab());
    uint32_t pend = c0 == NONE ? 0u : issue_grab();
    uint32_t j = 0;
    auto next_tile = [&]() -> uint64_t {
        while (c0 != NONE) {
            const uint64_t t = c0 * C + j;
            if (j < (uint32_t)C && t < n_tiles) {
                j++;
                return t;
            }
            c0 = resolve(pend);
            j = 0;
            pend = c0 == NONE ? 0u : issue_grab();
        }
        return NONE;
    };
    u32x4 r[2][4];
    uint64_t a0 = next_tile();
    uint64_t a1 = next_tile();
    issue4(slab, n_tiles, a0, lane, r[0]);
    issue4(slab, n_tiles, a1, lane, r[1]);
    while (a0 != NONE) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        const uint64_t a2 = next_tile();
        issue4(slab, n_tiles, a2, lane, r[1]);
        tile_work(slab, a0, lane, tile, o, v);
        a0 = a1;
        a1 = a2;
    }
    if (lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (st) {
            const uint64_t w = (uint64_t)blockIdx.x * 8u + wv;
            st[2 * w] = __builtin_amdgcn_s_memrealtime();
            st[2 * w + 1] = x0;
        }
        // the last wave zeroes the counters for the next launch (stream order)
        const uint32_t waves = gridDim.x * 8u;
        const uint32_t t = __hip_atomic_fetch_add(&ctr[8u * 64u], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == waves - 1u) {
            for (uint32_t x = 0; x < 8u; x++)
                __hip_atomic_store(&ctr[64u * x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctr[8u * 64u], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// hybrid: the block's first ks rounds of the balanced schedule (tiles b + k G,
// k < ks, drawn from the block's LDS counter), then the tail [ks G, n_tiles) in
// chunks of C tiles handed out by eight counters in interleaved order --
// counter x gives chunks x, x + 8, x + 16, ... -- each wave drawing first from
// its XCD's counter, then from the others once that one is dry.  ks = 0:
// every tile handed out that way.
template <int C>
__global__ __launch_bounds__(512) void k_hyb(const uint8_t *slab, uint64_t n_tiles, Out o, uint32_t *ctr,
                                             uint32_t ks, unsigned long long *st)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[8][256];
    __shared__ uint32_t s_next;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *tile = s_tile[wv];
    const uint64_t NONE = ~0ull, G = gridDim.x, b = blockIdx.x;
    const uint64_t S = (uint64_t)ks * G < n_tiles ? (uint64_t)ks * G : n_tiles; // static tiles
    const uint64_t nch = (n_tiles - S + C - 1) / C;                              // tail chunks
    const uint32_t x0 = xcc_id();
    if (threadIdx.x == 0)
        s_next = 8u;
    __syncthreads();
    uint32_t e = 0, xe = x0;
    auto issue_grab = [&]() -> uint32_t {
        uint32_t got = 0;
        if (lane == 0)
            got = __hip_atomic_fetch_add(&ctr[64u * xe], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return got;
    };
    auto resolve = [&](uint32_t raw) -> uint64_t {
        for (;;) {
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)raw);
            const uint64_t c = 8ull * r0 + xe;
            if (c < nch)
                return c;
            if (++e == 8u)
                return NONE;
            xe = (x0 + e) & 7u;
            raw = issue_grab();
        }
    };
    // static phase: k from the LDS counter (wave wv starts at k = wv)
    uint32_t kcur = wv;
    bool dyn = false;
    uint64_t c0 = NONE;
    uint32_t pend = 0, j = 0;
    auto next_tile = [&]() -> uint64_t {
        if (!dyn) {
            if (kcur < ks && b + (uint64_t)kcur * G < n_tiles) {
                const uint64_t t = b + (uint64_t)kcur * G;
                uint32_t v = 0;
                if (lane == 0)
                    v = atomicAdd(&s_next, 1u);
                kcur = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
                return t;
            }
            dyn = true;
            c0 = nch ? resolve(issue_grab()) : NONE;
            pend = c0 == NONE ? 0u : issue_grab();
            j = 0;
        }
        while (c0 != NONE) {
            const uint64_t t = S + c0 * C + j;
            if (j < (uint32_t)C && t < n_tiles) {
                j++;
                return t;
            }
            c0 = resolve(pend);
            j = 0;
            pend = c0 == NONE ? 0u : issue_grab();
        }
        return NONE;
    };
    u32x4 r[2][4];
    uint64_t a0 = next_tile();
    uint64_t a1 = next_tile();
    issue4(slab, n_tiles, a0, lane, r[0]);
    issue4(slab, n_tiles, a1, lane, r[1]);
    while (a0 != NONE) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = r[0][k];
            r[0][k] = r[1][k];
        }
        const uint64_t a2 = next_tile();
        issue4(slab, n_tiles, a2, lane, r[1]);
        tile_work(slab, a0, lane, tile, o, v);
        a0 = a1;
        a1 = a2;
    }
    if (lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (st) {
            const uint64_t w = (uint64_t)blockIdx.x * 8u + wv;
            st[2 * w] = __builtin_amdgcn_s_memrealtime();
            st[2 * w + 1] = x0;
        }
        const uint32_t waves = gridDim.x * 8u;
        const uint32_t t = __hip_atomic_fetch_add(&ctr[8u * 64u], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == waves - 1u) {
            for (uint32_t x = 0; x < 8u; x++)
                __hip_atomic_store(&ctr[64u * x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctr[8u * 64u], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// scheduler wave: 8 worker waves run the balanced schedule's first ks rounds
// (LDS counter), then take chunks of C tiles of the tail [ks G, n_tiles) from
// an LDS ring that a ninth wave fills: once the workers near the end of their
// static rounds it draws a round of 8 chunks at a time, lane l from counter l
// (counter l hands out chunks l, l + 8, l + 16, ...), keeping at most one round
// ahead of the workers.  Its global atomics wait in its own vmcnt, never in a
// worker's; a round whose 8 draws all come back past the end closes the ring.
#define SR_CAP 32u
template <int C>
__global__ __launch_bounds__(576) void k_sched(const uint8_t *slab, uint64_t n_tiles, Out o, uint32_t *ctr,
                                               uint32_t ks, unsigned long long *st)
{
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[8][256];
    __shared__ uint32_t s_next, s_head, s_tail, s_read, s_done;
    __shared__ uint32_t s_ring[SR_CAP];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t NONE = ~0ull, G = gridDim.x, b = blockIdx.x;
    const uint64_t S = (uint64_t)ks * G < n_tiles ? (uint64_t)ks * G : n_tiles;
    const uint64_t nch = (n_tiles - S + C - 1) / C;
    if (threadIdx.x == 0) {
        s_next = 8u;
        s_head = s_tail = s_read = s_done = 0u;
    }
    __syncthreads();
    if (wv == 8) { // the scheduler
        // start when the workers' static draws are nearly used up
        // (k indices are the block's rounds: ks of them in all; every spin
        // here and in pop is bounded, 2 ms, a hang becomes missing outputs)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(&s_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 32u < ks &&
               __builtin_amdgcn_s_memrealtime() - t0 < 200000u)
            __builtin_amdgcn_s_sleep(8);
        for (;;) {
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(&s_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) -
                       __hip_atomic_load(&s_read, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= 8u &&
                   __builtin_amdgcn_s_memrealtime() - t1 < 200000u)
                __builtin_amdgcn_s_sleep(2);
            uint32_t got = ~0u;
            if (lane < 8u)
                got = __hip_atomic_fetch_add(&ctr[64u * lane], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t c = lane < 8u ? 8ull * got + lane : NONE;
            const bool ok = lane < 8u && c < nch;
            const unsigned long long m = __ballot(ok);
            if (!m) {
                if (lane == 0)
                    __hip_atomic_store(&s_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                break;
            }
            const uint32_t h = __hip_atomic_load(&s_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t pos = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (ok)
                s_ring[(h + pos) % SR_CAP] = (uint32_t)c;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0)
                __hip_atomic_store(&s_head, h + (uint32_t)__popcll(m), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
        u32x4 *tile = s_tile[wv];
        auto pop = [&]() -> uint64_t {
            uint32_t idx = 0;
            if (lane == 0)
                idx = atomicAdd(&s_tail, 1u);
            idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000u)
                    return NONE;
                const uint32_t h = __hip_atomic_load(&s_head, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (idx < h) {
                    const uint32_t c = s_ring[idx % SR_CAP];
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0)
                        atomicAdd(&s_read, 1u);
                    return c;
                }
                if (__hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                    idx >= __hip_atomic_load(&s_head, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
                    return NONE;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        uint32_t kcur = wv;
        bool dyn = false;
        uint64_t c0 = NONE;
        uint32_t j = 0;
        auto next_tile = [&]() -> uint64_t {
            if (!dyn) {
                if (kcur < ks && b + (uint64_t)kcur * G < n_tiles) {
                    const uint64_t t = b + (uint64_t)kcur * G;
                    uint32_t v = 0;
                    if (lane == 0)
                        v = atomicAdd(&s_next, 1u);
                    kcur = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
                    return t;
                }
                dyn = true;
                c0 = nch ? pop() : NONE;
                j = 0;
            }
            while (c0 != NONE) {
                const uint64_t t = S + c0 * C + j;
                if (j < (uint32_t)C && t < n_tiles) {
                    j++;
                    return t;
                }
                c0 = pop();
                j = 0;
            }
            return NONE;
        };
        u32x4 r[2][4];
        uint64_t a0 = next_tile();
        uint64_t a1 = next_tile();
        issue4(slab, n_tiles, a0, lane, r[0]);
        issue4(slab, n_tiles, a1, lane, r[1]);
        while (a0 != NONE) {
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                v[k] = r[0][k];
                r[0][k] = r[1][k];
            }
            const uint64_t a2 = next_tile();
            issue4(slab, n_tiles, a2, lane, r[1]);
            tile_work(slab, a0, lane, tile, o, v);
            a0 = a1;
            a1 = a2;
        }
        if (lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (st) {
                const uint64_t w = (uint64_t)blockIdx.x * 8u + wv;
                st[2 * w] = __builtin_amdgcn_s_memrealtime();
                st[2 * w + 1] = xcc_id();
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(&ctr[8u * 64u], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1u) {
            for (uint32_t x = 0; x < 8u; x++)
                __hip_atomic_store(&ctr[64u * x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctr[8u * 64u], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

static int cus()
{
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev))
        n = 256;
    return n;
}

extern "C" {
int pd_bal(const void *slab, uint64_t n, uint32_t *a, uint32_t *b, uint16_t *q, unsigned long long *st, void *s)
{
    const uint64_t nt = n / 64u;
    hipLaunchKernelGGL(k_bal_stamp, dim3((unsigned)cus()), dim3(512), 0, (hipStream_t)s, (const uint8_t *)slab, nt,
                       Out{a, b, q}, st);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int pd_hyb(const void *slab, uint64_t n, uint32_t *a, uint32_t *b, uint16_t *q, uint32_t *ctr, int chunk,
           uint32_t ks, unsigned long long *st, void *s)
{
    const uint64_t nt = n / 64u;
    const dim3 g((unsigned)cus()), blk(512);
    const Out o{a, b, q};
    const uint8_t *sl = (const uint8_t *)slab;
    switch (chunk) {
    case 2: hipLaunchKernelGGL(k_hyb<2>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 4: hipLaunchKernelGGL(k_hyb<4>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 8: hipLaunchKernelGGL(k_hyb<8>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 16: hipLaunchKernelGGL(k_hyb<16>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int pd_sched(const void *slab, uint64_t n, uint32_t *a, uint32_t *b, uint16_t *q, uint32_t *ctr, int chunk,
             uint32_t ks, unsigned long long *st, void *s)
{
    const uint64_t nt = n / 64u;
    const dim3 g((unsigned)cus()), blk(576);
    const Out o{a, b, q};
    const uint8_t *sl = (const uint8_t *)slab;
    switch (chunk) {
    case 1: hipLaunchKernelGGL(k_sched<1>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 2: hipLaunchKernelGGL(k_sched<2>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 4: hipLaunchKernelGGL(k_sched<4>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    case 8: hipLaunchKernelGGL(k_sched<8>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, ks, st); break;
    default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int pd_dyn(const void *slab, uint64_t n, uint32_t *a, uint32_t *b, uint16_t *q, uint32_t *ctr, int chunk,
           unsigned long long *st, void *s)
{
    const uint64_t nt = n / 64u;
    const dim3 g((unsigned)cus()), blk(512);
    const Out o{a, b, q};
    const uint8_t *sl = (const uint8_t *)slab;
    switch (chunk) {
    case 4: hipLaunchKernelGGL(k_dyn<4>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, st); break;
    case 8: hipLaunchKernelGGL(k_dyn<8>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, st); break;
    case 16: hipLaunchKernelGGL(k_dyn<16>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, st); break;
    case 32: hipLaunchKernelGGL(k_dyn<32>, g, blk, 0, (hipStream_t)s, sl, nt, o, ctr, st); break;
    default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
}
