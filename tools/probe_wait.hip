// probe_wait.hip -- request latency of a kernel launched on demand against one
// pre-enqueued behind hipStreamWaitValue32 on a signal word (diagnostic).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probe_wait tools/probe_wait.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                       \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

static double now_us()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

// one block: touch n words of host memory (as a 256-frame MAC swap would), then raise the flag
__global__ void k_req(uint32_t *hostbuf, uint32_t n, volatile uint32_t *flag, uint32_t seq)
{
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        hostbuf[i] = hostbuf[i] ^ 0x5a5a5a5au;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        *flag = seq;
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    uint32_t *hostbuf, *flag;
    CK(hipHostMalloc((void **)&hostbuf, 1 << 20, hipHostMallocMapped));
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocMapped));
    uint32_t *dbuf, *dflag;
    CK(hipHostGetDevicePointer((void **)&dbuf, hostbuf, 0));
    CK(hipHostGetDevicePointer((void **)&dflag, flag, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int dev = 0, can = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev));
    printf("CanUseStreamWaitValue %d\n", can);
    const int reps = 300;
    std::vector<double> v;
    volatile uint32_t *vf = flag;
    *vf = 0;
    // 1. launch on demand
    for (int r = 1; r <= reps; r++) {
        const double t0 = now_us();
        hipLaunchKernelGGL(k_req, dim3(1), dim3(256), 0, s, dbuf, 512, dflag, (uint32_t)r);
        while (*vf != (uint32_t)r) {
        }
        v.push_back(now_us() - t0);
    }
    printf("launch on demand: median %.1f us\n", median(v));
    CK(hipStreamSynchronize(s));
    // 2. pre-enqueued behind a wait on signal memory / on pinned host memory
    for (int kind = 0; kind < 2; kind++) {
        uint32_t *sig = nullptr;
        hipError_t e = kind == 0 ? hipExtMallocWithFlags((void **)&sig, 64, hipMallocSignalMemory)
                                 : hipHostMalloc((void **)&sig, 64, hipHostMallocMapped);
        if (e != hipSuccess) {
            printf("kind %d alloc: %s\n", kind, hipGetErrorString(e));
            continue;
        }
        volatile uint32_t *vs = sig;
        *vs = 0;
        *vf = 0;
        v.clear();
        bool ok = true;
        for (int r = 1; r <= reps && ok; r++) {
            e = hipStreamWaitValue32(s, sig, (uint32_t)r, hipStreamWaitValueGte, 0xffffffffu);
            if (e != hipSuccess) {
                printf("kind %d wait: %s\n", kind, hipGetErrorString(e));
                ok = false;
                break;
            }
            hipLaunchKernelGGL(k_req, dim3(1), dim3(256), 0, s, dbuf, 512, dflag, (uint32_t)r);
            const double tw = now_us();
            while (now_us() - tw < 50.0) { // let the CP reach the wait
            }
            const double t0 = now_us();
            *vs = (uint32_t)r;
            const double tl = now_us();
            while (*vf != (uint32_t)r) {
                if (now_us() - tl > 2e6) { // bounded: report and stop
                    printf("kind %d rep %d: no completion in 2 s\n", kind, r);
                    ok = false;
                    break;
                }
            }
            v.push_back(now_us() - t0);
        }
        if (!ok)
            *vs = 0x7fffffffu; // release any pending wait
        CK(hipStreamSynchronize(s));
        if (ok)
            printf("pre-enqueued behind a wait on %s: median %.1f us\n", kind == 0 ? "signal memory" : "pinned host memory",
                   median(v));
        if (kind == 0)
            CK(hipFree(sig));
        else
            CK(hipHostFree(sig));
    }
    return 0;
}
