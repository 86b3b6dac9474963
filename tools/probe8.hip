// probe8.hip -- does an uncached frame slab let HBM serve 64-B windows as 64-B
// requests?  (diagnostic, not product)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe8 tools/probe8.hip
//
// The C5 / C4 window read (4 lanes per frame, one 16-B load each, 16 frames per
// wave load instruction, as k_cnet_defer loads) from a frame slab allocated
//   def   hipMalloc                                   (MTYPE RW: L2 fills 128-B lines)
//   fine  hipExtMallocWithFlags(hipDeviceMallocFinegrained)
//   unc   hipExtMallocWithFlags(hipDeviceMallocUncached)
// with plain, nontemporal and sc1 (buffer aux 16) loads.  Per variant: ms per
// launch (HIP events over 10 launches) and the algorithmic window rate; under
// rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum the request sizes.
// Every variant folds the same bytes: the folds are compared.
// usage: probe8 [c5_frames_log2 (default 24)]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
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

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int LD>
__device__ __forceinline__ u32x4 ld16(const uint8_t *base, uint64_t off)
{
    if (LD == 0)
        return *(const u32x4 *)(base + off);
    if (LD == 1)
        return __builtin_nontemporal_load((const u32x4 *)(base + off));
    // buffer load, aux 16 = sc1; the resource covers 4 GiB from the 256-B-aligned
    // line of this frame (so any 64-bit offset works)
    const uint8_t *p = base + (off & ~255ull);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(off & 255u), 0, 16));
}

// C5: frame f at f * stride; results 4 + 1 B per frame written coalesced, as the product
template <int LD>
__global__ __launch_bounds__(256) void k_c5(const uint8_t *slab, uint64_t stride, uint32_t n, uint32_t *o4, uint8_t *o1,
                                            uint32_t *acc_out)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint32_t g = blockIdx.x * 4 + wv; g < n / 64; g += gridDim.x * 4) {
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t f = (uint64_t)g * 64 + 16 * k + (lane >> 2);
            const uint32_t v = fold(ld16<LD>(slab, f * stride + (lane & 3u) * 16u));
            // gather the 4 parts of frame 16k + lane/4 to its lane (xor over the quad)
            uint32_t q = v ^ __shfl_xor(v, 1) ^ __shfl_xor(v, 2);
            const uint32_t src = __shfl(q, (int)((lane & 15u) * 4u));
            if ((lane >> 4) == (uint32_t)k)
                mine = src;
        }
        o4[g * 64 + lane] = mine;
        o1[g * 64 + lane] = (uint8_t)mine;
        acc ^= mine;
    }
    acc ^= __shfl_xor(acc, 32);
    if (lane == 0)
        atomicXor(acc_out, acc);
}

// C4: IMIX windows at u64 offsets
template <int LD>
__global__ __launch_bounds__(256) void k_c4(const uint8_t *slab, const uint64_t *offs, uint32_t n, uint32_t *o4,
                                            uint32_t *acc_out)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint32_t g = blockIdx.x * 4 + wv; g < n / 64; g += gridDim.x * 4) {
        const uint64_t myoff = offs[g * 64 + lane];
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t fo = __shfl(myoff, 16 * k + (int)(lane >> 2));
            const uint32_t v = fold(ld16<LD>(slab, fo + (lane & 3u) * 16u));
            uint32_t q = v ^ __shfl_xor(v, 1) ^ __shfl_xor(v, 2);
            const uint32_t src = __shfl(q, (int)((lane & 15u) * 4u));
            if ((lane >> 4) == (uint32_t)k)
                mine = src;
        }
        o4[g * 64 + lane] = mine;
        acc ^= mine;
    }
    acc ^= __shfl_xor(acc, 32);
    if (lane == 0)
        atomicXor(acc_out, acc);
}

static const char *MEMN[3] = {"def", "fine", "unc"};
static const char *LDN[3] = {"plain", "nt", "sc1"};

template <int LD>
static float run_c5(const uint8_t *slab, uint64_t stride, uint32_t n, uint32_t *o4, uint8_t *o1, uint32_t *acc,
                    int grid, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_c5<LD>, dim3(grid), dim3(256), 0, 0, slab, stride, n, o4, o1, acc);
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(k_c5<LD>, dim3(grid), dim3(256), 0, 0, slab, stride, n, o4, o1, acc);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

template <int LD>
static float run_c4(const uint8_t *slab, const uint64_t *offs, uint32_t n, uint32_t *o4, uint32_t *acc, int grid,
                    int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_c4<LD>, dim3(grid), dim3(256), 0, 0, slab, offs, n, o4, acc);
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(k_c4<LD>, dim3(grid), dim3(256), 0, 0, slab, offs, n, o4, acc);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

__global__ void k_fill(uint32_t *p, uint64_t n32)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n32; i += (uint64_t)gridDim.x * 256)
        p[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 29);
}

int main(int argc, char **argv)
{
    const int lg = argc > 1 ? atoi(argv[1]) : 24;
    const int bpc = argc > 2 ? atoi(argv[2]) : 8;     // 256-thread blocks per CU (8 = 8 waves a SIMD)
    const int only_def = argc > 3 ? atoi(argv[3]) : 0; // 1: hipMalloc slabs, nt loads only
    const uint32_t n5 = 1u << lg, n4 = 1u << lg;
    const uint64_t stride = 1536;
    const uint64_t bytes5 = (uint64_t)n5 * stride;
    // C4 IMIX slots 64 / 576 / 1536 at 7:4:1 (pseudo-random order)
    std::vector<uint64_t> hoff(n4);
    uint64_t tot = 0;
    uint32_t x = 12345;
    for (uint32_t i = 0; i < n4; i++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t pick = (x >> 8) % 12;
        const uint64_t slot = pick < 7 ? 64 : pick < 11 ? 576 : 1536;
        hoff[i] = tot;
        tot += slot;
    }
    const uint64_t bytes = bytes5 > tot ? bytes5 : tot;
    uint64_t *offs;
    uint32_t *o4, *acc;
    uint8_t *o1;
    CK(hipMalloc((void **)&offs, n4 * 8ull));
    CK(hipMemcpy(offs, hoff.data(), n4 * 8ull, hipMemcpyHostToDevice));
    CK(hipMalloc((void **)&o4, (uint64_t)n5 * 4));
    CK(hipMalloc((void **)&o1, n5));
    CK(hipMalloc((void **)&acc, 4 * 64));
    int dev, ncu;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int grid = ncu * bpc;
    printf("C5 %u frames x %llu B (%.2f GB windows), C4 %u IMIX frames (%.2f GB slab), grid %d\n", n5,
           (unsigned long long)stride, n5 * 64.0 / 1e9, n4, tot / 1e9, grid);
    const unsigned flags[3] = {hipDeviceMallocDefault, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    uint32_t ref5 = 0, ref4 = 0;
    bool have = false;
    for (int m = 0; m < (only_def ? 1 : 3); m++) {
        uint8_t *slab = nullptr;
        hipError_t e = m == 0 ? hipMalloc((void **)&slab, bytes) : hipExtMallocWithFlags((void **)&slab, bytes, flags[m]);
        if (e != hipSuccess) {
            printf("%-5s alloc failed: %s\n", MEMN[m], hipGetErrorString(e));
            continue;
        }
        hipLaunchKernelGGL(k_fill, dim3(ncu * 16), dim3(256), 0, 0, (uint32_t *)slab, bytes / 4);
        CK(hipDeviceSynchronize());
        for (int ld = only_def ? 1 : 0; ld < (only_def ? 2 : 3); ld++) {
            for (int rep = 0; rep < 2; rep++) {
                CK(hipMemset(acc, 0, 8));
                float t5 = ld == 0 ? run_c5<0>(slab, stride, n5, o4, o1, acc, grid, 10)
                         : ld == 1 ? run_c5<1>(slab, stride, n5, o4, o1, acc, grid, 10)
                                   : run_c5<2>(slab, stride, n5, o4, o1, acc, grid, 10);
                float t4 = ld == 0 ? run_c4<0>(slab, offs, n4, o4, acc + 1, grid, 10)
                         : ld == 1 ? run_c4<1>(slab, offs, n4, o4, acc + 1, grid, 10)
                                   : run_c4<2>(slab, offs, n4, o4, acc + 1, grid, 10);
                uint32_t h[2];
                CK(hipMemcpy(h, acc, 8, hipMemcpyDeviceToHost));
                // 11 launches xor-accumulated: odd count, so the fold of one launch
                if (!have) {
                    ref5 = h[0];
                    ref4 = h[1];
                    have = true;
                }
                printf("%-5s %-5s c5 %.4f ms (%.0f GB/s of windows, %.0f with 5 B results)  c4 %.4f ms (%.0f GB/s)  %s\n",
                       MEMN[m], LDN[ld], t5, n5 * 64.0 / t5 / 1e6, n5 * 69.0 / t5 / 1e6, t4, n4 * 68.0 / t4 / 1e6,
                       h[0] == ref5 && h[1] == ref4 ? "same bytes" : "FOLD DIFFERS");
                fflush(stdout);
            }
        }
        CK(hipFree(slab));
    }
    return 0;
}
