// probe11.hip -- can a block whose waves split by role hide a dependent table
// walk behind the frame stream?  (diagnostic, not product)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe11 tools/probe11.hip
//
// k_cnet_defer's chain levels wait in the in-order vmcnt behind the windows the
// wave issued before them.  Here, C3-shaped data: 16M frames of
// 64 B (1 GiB), read 4 x 1 KiB a tile, and a 1 MiB table of 1024 groups x 256
// words whose entries name groups; each frame walks L levels from a key of its
// bytes and stores the last entry (4 B).
//   stream      the windows and the store, no walk: the ceiling
//   mono        one role per wave, two tiles in flight (tile t+W's windows
//               issued, then tile t walked): the walk's waits also wait for
//               t+W's windows
//   split NL/NW/G  one 1024-thread block a CU: NL loader waves (windows ->
//               keys -> an LDS ring of 64 slots), NW walker waves taking G
//               slots at once and walking their G x 64 keys level by level
//               side by side
// Every variant's outputs are compared with mono's.  Waits on the ring are
// bounded (a wave that waits too long gives up and counts it in err).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
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

#define NF (16u << 20)
#define NT (NF / 64u)
#define GRP 1024u
#define RING 64u
#define SPIN_MAX (1u << 22)

__device__ __forceinline__ u32x4 ldnt(const u32x4 *p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ void tile_load(const u32x4 *slab, uint32_t t, uint32_t lane, u32x4 (&r)[4])
{
    const u32x4 *g = slab + (uint64_t)t * 256u;
#pragma unroll
    for (int k = 0; k < 4; k++)
        r[k] = ldnt(g + 64u * k + lane);
}

__device__ __forceinline__ uint32_t key_of(const u32x4 (&r)[4])
{
    return r[0].x ^ r[1].y ^ r[2].z ^ r[3].w;
}

// one level: the group is the entry's low bits, the index a key byte; the
// first H levels read group 0's first line for every lane (C4's shallow trie
// levels: one line for all IPv6 frames)
template <int H>
__device__ __forceinline__ uint32_t lvl(const uint32_t *T, uint32_t g, uint32_t key, int l)
{
    if (l < H)
        return T[(key >> 29) + (g & 3u)];
    return T[(g & (GRP - 1u)) * 256u + ((key >> (5 * l)) & 255u)];
}

template <int L, int H = 0, bool HALF = false>
__global__ __launch_bounds__(512) void k_mono(const u32x4 *slab, const uint32_t *T, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, W = gridDim.x * 8u;
    uint32_t t = blockIdx.x * 8u + (threadIdx.x >> 6);
    u32x4 r0[4], r1[4];
    if (t < NT)
        tile_load(slab, t, lane, r0);
    for (; t < NT; t += W) {
        if (t + W < NT)
            tile_load(slab, t + W, lane, r1);
        const uint32_t key = key_of(r0);
        uint32_t e = key;
        // HALF: lanes with key bit 0 set walk one level only (IPv4 frames)
        const bool deep = !HALF || (key & 1u);
#pragma unroll
        for (int l = 0; l < L; l++)
            if (l == 0 || deep)
                e = lvl<H>(T, l == 0 ? key : e, key, l);
        __builtin_nontemporal_store(e, out + (uint64_t)t * 64u + lane);
#pragma unroll
        for (int k = 0; k < 4; k++)
            r0[k] = r1[k];
    }
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) { return *(const volatile uint32_t *)p; }
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) { *(volatile uint32_t *)p = v; }

// wait until *flag == want (wave-uniform); false after SPIN_MAX polls
__device__ __forceinline__ bool ring_wait(const uint32_t *flag, uint32_t want)
{
    for (uint32_t it = 0; it < SPIN_MAX; it++) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_ld(flag));
        if (v == want)
            return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

template <int L, int NL, int NW, int G, int H = 0, bool HALF = false>
__global__ __launch_bounds__(1024) void k_split(const u32x4 *slab, const uint32_t *T, uint32_t *out, uint32_t *err)
{
    static_assert(NL + NW == 16, "16 waves");
    static_assert(RING >= 2 * G, "ring");
    __shared__ uint32_t s_key[RING][64];
    __shared__ uint32_t s_flag[RING];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t k = threadIdx.x; k < RING; k += 1024u)
        s_flag[k] = 0u;
    __syncthreads();
    // the block's tiles: t_j = blockIdx.x + j * gridDim.x
    const uint32_t J = blockIdx.x < NT ? (NT - blockIdx.x + gridDim.x - 1u) / gridDim.x : 0u;
    uint32_t bad = 0;
    if (wv < (uint32_t)NL) {
        u32x4 r0[4], r1[4];
        uint32_t j = wv;
        if (j < J)
            tile_load(slab, blockIdx.x + j * gridDim.x, lane, r0);
        for (; j < J; j += NL) {
            if (j + NL < J)
                tile_load(slab, blockIdx.x + (j + NL) * gridDim.x, lane, r1);
            const uint32_t key = key_of(r0);
            const uint32_t s = j % RING;
            bad += !ring_wait(&s_flag[s], 0u);
            lds_st(&s_key[s][lane], key);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0)
                lds_st(&s_flag[s], j + 1u);
#pragma unroll
            for (int k = 0; k < 4; k++)
                r0[k] = r1[k];
        }
    } else {
        const uint32_t wi = wv - NL;
        for (uint32_t j0 = wi * G; j0 < J; j0 += NW * G) {
            uint32_t key[G], e[G];
#pragma unroll
            for (int k = 0; k < G; k++) {
                const uint32_t j = j0 + k;
                key[k] = 0u;
                if (j < J) {
                    bad += !ring_wait(&s_flag[j % RING], j + 1u);
                    key[k] = lds_ld(&s_key[j % RING][lane]);
                }
            }
#pragma unroll
            for (int l = 0; l < L; l++)
#pragma unroll
                for (int k = 0; k < G; k++)
                    if (l == 0 || !HALF || (key[k] & 1u))
                        e[k] = lvl<H>(T, l == 0 ? key[k] : e[k], key[k], l);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < G; k++) {
                const uint32_t j = j0 + k;
                if (j < J) {
                    __builtin_nontemporal_store(L ? e[k] : key[k],
                                                out + (uint64_t)(blockIdx.x + j * gridDim.x) * 64u + lane);
                    if (lane == 0)
                        lds_st(&s_flag[j % RING], 0u);
                }
            }
        }
    }
    if (bad && lane == 0)
        atomicAdd(err, bad);
}

static float time_it(void (*launch)(void *), void *arg, int reps = 11)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 0; k < 3; k++)
        launch(arg);
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int k = 0; k < reps; k++) {
        CK(hipEventRecord(a));
        launch(arg);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

struct Args {
    const u32x4 *slab;
    const uint32_t *T;
    uint32_t *out, *err;
    int cus;
};

template <int L, int H = 0, bool HALF = false> static void run_mono(void *p)
{
    Args *a = (Args *)p;
    hipLaunchKernelGGL((k_mono<L, H, HALF>), dim3(a->cus * 2), dim3(512), 0, 0, a->slab, a->T, a->out);
}
template <int L, int NL, int NW, int G, int H = 0, bool HALF = false> static void run_split(void *p)
{
    Args *a = (Args *)p;
    hipLaunchKernelGGL((k_split<L, NL, NW, G, H, HALF>), dim3(a->cus), dim3(1024), 0, 0, a->slab, a->T, a->out,
                       a->err);
}

int main()
{
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    u32x4 *slab;
    uint32_t *T, *ref, *out, *err;
    CK(hipMalloc(&slab, (size_t)NF * 64));
    CK(hipMalloc(&T, (size_t)GRP * 256 * 4));
    CK(hipMalloc(&ref, (size_t)NF * 4));
    CK(hipMalloc(&out, (size_t)NF * 4));
    CK(hipMalloc(&err, 4));
    {
        std::vector<uint32_t> h((size_t)GRP * 256);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto &w : h) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            w = (uint32_t)x;
        }
        CK(hipMemcpy(T, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        std::vector<uint32_t> f((size_t)1 << 24);
        for (size_t part = 0; part < 4; part++) {
            for (auto &w : f) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                w = (uint32_t)x;
            }
            CK(hipMemcpy((uint8_t *)slab + part * f.size() * 4, f.data(), f.size() * 4, hipMemcpyHostToDevice));
        }
    }
    Args a{slab, T, out, err, cus};
    const double bytes = (double)NF * 68.0;
    auto check = [&](const char *name, float ms, bool cmp) {
        uint32_t e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        bool eq = true;
        if (cmp) {
            std::vector<uint32_t> h1((size_t)NF), h2((size_t)NF);
            CK(hipMemcpy(h1.data(), ref, (size_t)NF * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), out, (size_t)NF * 4, hipMemcpyDeviceToHost));
            eq = h1 == h2;
        }
        printf("%-22s %.4f ms  %.2f TB/s  %s  ring timeouts %u\n", name, ms, bytes / (ms * 1e-3) / 1e12,
               cmp ? (eq ? "equal" : "DIFFER") : "-", e);
        CK(hipMemset(err, 0, 4));
        fflush(stdout);
    };
    CK(hipMemset(err, 0, 4));
    {
        Args r = a;
        r.out = ref;
        float ms = time_it(run_mono<0>, &r);
        check("stream (mono, L=0)", ms, false);
        ms = time_it(run_mono<5>, &r);
        check("mono L=5", ms, false);
    }
    float ms;
    ms = time_it(run_mono<5>, &a);
    check("mono L=5 (again)", ms, true);
    ms = time_it(run_split<5, 10, 6, 8>, &a);
    check("split 10/6 G8 L=5", ms, true);
    ms = time_it(run_split<0, 12, 4, 8>, &a);
    check("split 12/4 G8 L=0", ms, false);
    // C4-like: two shallow levels on one line, three deep ones, half the lanes deep
    {
        Args r = a;
        r.out = ref;
        ms = time_it(run_mono<5, 2, true>, &r);
        check("mono L5 H2 half", ms, false);
    }
    ms = time_it(run_mono<5, 2, true>, &a);
    check("mono L5 H2 half (again)", ms, true);
    ms = time_it(run_split<5, 8, 8, 4, 2, true>, &a);
    check("split 8/8 G4 L5 H2 half", ms, true);
    ms = time_it(run_split<5, 10, 6, 8, 2, true>, &a);
    check("split 10/6 G8 L5 H2 half", ms, true);
    ms = time_it(run_split<5, 12, 4, 8, 2, true>, &a);
    check("split 12/4 G8 L5 H2 half", ms, true);
    ms = time_it(run_split<5, 12, 4, 16, 2, true>, &a);
    check("split 12/4 G16 L5 H2 half", ms, true);
    ms = time_it(run_mono<3, 2, true>, &a);
    check("mono L3 H2 half", ms, false);
    ms = time_it(run_mono<2, 2, true>, &a);
    check("mono L2 H2 half", ms, false);
    return 0;
}
