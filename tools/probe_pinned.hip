// Host-side access cost of pinned memory (hipHostMalloc flag variants) vs malloc:
// the staged node path reads the records the kernels wrote and copies frames in.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void run(const char *name, uint8_t *p, size_t len, const uint8_t *src)
{
    volatile uint64_t sink = 0;
    // read 16 B records like the cnet writeback
    double t0 = now();
    for (int r = 0; r < 4; r++) {
        uint64_t s = 0;
        for (size_t i = 0; i + 16 <= len; i += 16)
            s += *(const uint32_t *)(p + i) + *(const uint32_t *)(p + i + 4) + *(const uint32_t *)(p + i + 8);
        sink += s;
    }
    double rd = (now() - t0) / 4;
    t0 = now();
    for (int r = 0; r < 4; r++)
        for (size_t i = 0; i + 128 <= len; i += 128)
            memcpy(p + i, src + i, 128);
    double wr = (now() - t0) / 4;
    printf("%-28s read16 %7.2f ns/rec  copy128 %7.2f ns/frame\n", name, rd * 1e9 / (len / 16), wr * 1e9 / (len / 128));
}

int main()
{
    const size_t len = 8u << 20;
    uint8_t *src = (uint8_t *)malloc(len);
    memset(src, 1, len);
    uint8_t *m = (uint8_t *)malloc(len);
    memset(m, 0, len);
    run("malloc", m, len, src);
    struct { const char *n; unsigned f; } v[] = {
        {"hipHostMallocDefault", hipHostMallocDefault},
        {"Mapped", hipHostMallocMapped},
        {"Mapped|NonCoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
        {"Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent},
        {"Mapped|WriteCombined", hipHostMallocMapped | hipHostMallocWriteCombined},
    };
    for (auto &x : v) {
        uint8_t *h = nullptr;
        if (hipHostMalloc((void **)&h, len, x.f) != hipSuccess) {
            printf("%s: alloc failed\n", x.n);
            continue;
        }
        memset(h, 0, len);
        run(x.n, h, len, src);
        hipHostFree(h);
    }
    return 0;
}
