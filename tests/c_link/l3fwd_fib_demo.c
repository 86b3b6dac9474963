/*
 * Test-only C program: the FIB usage of examples/cndpfwd/l3-fwd.c:78-117
 * (cne_fib_create with a DUMMY config and 48-bit default next hop,
 * cne_fib_add per rule, cne_fib_lookup_bulk per burst of up to 256 IPv4
 * addresses, next hop = tx port << 48 | MAC) compiled as plain C against
 * include/cndp_fib.h and linked to libcndp_gpu.so -- the link swap of
 * INTEGRATION.md §1 -- with every answer checked against a longest-prefix
 * match over the same rules, first in the selection a FIB is created with
 * (the host image, as cne_fib.c:86 binds the scalar lookup), then with
 * CNDP_FIB_LOOKUP_GPU.  Exit 0: all lookups right; 77: the default lookups
 * right and no GPU (the GPU lookups returned -ENODEV with the default next hop
 * filled in); 1: a wrong answer.
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "cndp_fib.h"

#define N_RULES 512
#define N_IPS 4096
#define BURST 256

struct rule {
    uint32_t ip;
    uint8_t depth;
    uint64_t nh;
};

static uint32_t rnd(uint64_t *s)
{
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 32);
}

static uint64_t lpm(const struct rule *r, int n, uint32_t ip, uint64_t dflt)
{
    int best = -1;
    for (int i = 0; i < n; i++) {
        const uint32_t m = r[i].depth ? ~0u << (32 - r[i].depth) : 0u;
        if ((ip & m) == r[i].ip && (best < 0 || r[i].depth > r[best].depth))
            best = i;
    }
    return best < 0 ? dflt : r[best].nh;
}

int main(void)
{
    struct cne_fib_conf config = {0};
    config.max_routes = 1 << 16; /* l3-fwd.c:98-101 */
    config.default_nh = 0xFFFFFFFFFFFF;
    config.type = CNE_FIB_DUMMY;
    struct cne_fib *fib = cne_fib_create("l3fwd_fib", &config);
    if (!fib) {
        fprintf(stderr, "cne_fib_create failed\n");
        return 1;
    }
    static struct rule r[N_RULES];
    uint64_t s = 42;
    for (int i = 0; i < N_RULES; i++) {
        const uint8_t d = (uint8_t)(8 + rnd(&s) % 25);
        r[i].depth = d;
        r[i].ip = rnd(&s) & (~0u << (32 - d));
        r[i].nh = ((uint64_t)(rnd(&s) % 8) << 48) | ((uint64_t)rnd(&s) << 16) | (rnd(&s) & 0xffffu);
        /* a later rule for the same prefix replaces the earlier one */
        for (int j = 0; j < i; j++)
            if (r[j].ip == r[i].ip && r[j].depth == d)
                r[j].depth = 0xFF;
        if (cne_fib_add(fib, r[i].ip, d, r[i].nh) < 0) {
            fprintf(stderr, "cne_fib_add failed\n");
            return 1;
        }
    }
    int live = 0;
    for (int i = 0; i < N_RULES; i++)
        if (r[i].depth != 0xFF)
            r[live++] = r[i];
    static uint32_t ips[N_IPS];
    for (int i = 0; i < N_IPS; i++)
        ips[i] = i % 2 ? rnd(&s) : (r[rnd(&s) % live].ip | (rnd(&s) & 0xFFu));
    int bad = 0;
    /* first as created (CNE_FIB_LOOKUP_DEFAULT: the host image, cne_fib.c:86),
     * then with the GPU extension selected */
    for (int sel = 0; sel < 2; sel++) {
        if (sel && cne_fib_select_lookup(fib, (enum cne_fib_lookup_type)CNDP_FIB_LOOKUP_GPU) != 0) {
            fprintf(stderr, "cne_fib_select_lookup(GPU) failed\n");
            return 1;
        }
        for (int b = 0; b < N_IPS; b += BURST) { /* l3fwd_fib_lookup: one call per burst */
            uint64_t nhop[BURST];
            const int rc = cne_fib_lookup_bulk(fib, ips + b, nhop, BURST);
            if (rc == -ENODEV && sel) {
                for (int i = 0; i < BURST; i++)
                    if (nhop[i] != config.default_nh)
                        return 1;
                printf("%s: default lookups right (%d wrong); no GPU: the GPU lookups returned "
                       "-ENODEV with the default next hop\n", bad ? "FAIL" : "PASS", bad);
                cne_fib_free(fib);
                return bad ? 1 : 77;
            }
            if (rc != 0) {
                fprintf(stderr, "cne_fib_lookup_bulk: %d\n", rc);
                return 1;
            }
            for (int i = 0; i < BURST; i++) {
                const uint64_t want = lpm(r, live, ips[b + i], config.default_nh);
                if (nhop[i] != want && bad++ < 4)
                    fprintf(stderr, "sel %d ip %08x: nh %llx want %llx\n", sel, ips[b + i],
                            (unsigned long long)nhop[i], (unsigned long long)want);
            }
        }
    }
    cne_fib_free(fib);
    printf("%s: %d lookups over %d rules in each selection, %d wrong\n", bad ? "FAIL" : "PASS", N_IPS, live,
           bad);
    return bad ? 1 : 0;
}
