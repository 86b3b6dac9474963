/*
 * Test/tool program: per-thread rate of cne_fib_lookup_bulk / cne_fib6_lookup_bulk
 * for the call shapes of cnet's synchronous FIB callers, in both selections of
 * cne_fib_select_lookup (the reference's default = host image, and the GPU
 * extension), compiled as plain C against include/cndp_fib.h and linked to
 * libcndp_gpu.so.  The FIBs are built as cnet builds them:
 *   rt4-fib  DIR-24-8 4 B (cnet_route4.c:180): 896 /24 + 128 /25../32 routes
 *   arp-fib  DIR-24-8 4 B (cnet_arp.c:195): 1024 /32 host entries
 *   nd6-fib  trie 4 B (cnet_nd6.c:242): 1024 /32../64 prefixes in 2001:db8::/32
 * Call shapes: 4 keys (ip4_forward.c:134-178, ip4_lookup.c:141), 1 key
 * (ip4_output.c:87,118, cnet_arp.c:77, cnet_route4.c:77), 256 keys (a graph
 * burst, examples/cndpfwd/l3-fwd.c:85).  Keys: 3 of 4 inside the routed space,
 * 1 of 4 uniform over the address space (a tbl24 miss).  Every answer of the
 * timed calls is also checked against the other selection (or, with no GPU,
 * against a brute-force LPM of the rt4 rules).
 *
 * usage: fib_rate [--gpu] [--ms MS]   prints one JSON object on stdout.
 * Exit 0 ok, 1 a wrong answer.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cndp_fib.h"

#define NKEYS 65536

static uint32_t rnd(uint64_t *s)
{
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 32);
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

static struct cne_fib *rt4, *arp;
static struct cne_fib6 *nd6;
static uint32_t keys4[NKEYS], keys_arp[NKEYS];
static uint8_t keys6[NKEYS][IPV6_ADDR_LEN];
static uint32_t r_ip[1024];
static uint8_t r_d[1024];
static uint64_t r_nh[1024];

static uint64_t lpm4(uint32_t ip)
{
    int best = -1;
    for (int i = 0; i < 1024; i++) {
        const uint32_t m = ~0u << (32 - r_d[i]);
        if ((ip & m) == r_ip[i] && (best < 0 || r_d[i] > r_d[best]))
            best = i;
    }
    return best < 0 ? 1025 : r_nh[best];
}

static void build(void)
{
    struct cne_fib_conf c = {0};
    c.type = CNE_FIB_DIR24_8;
    c.default_nh = 1025;
    c.max_routes = 1024;
    c.dir24_8.nh_sz = CNE_FIB_DIR24_8_4B;
    c.dir24_8.num_tbl8 = 256;
    rt4 = cne_fib_create("rt4-fib", &c);
    arp = cne_fib_create("arp-fib", &c);
    struct cne_fib_conf c6 = {0};
    c6.type = CNE_FIB_TRIE;
    c6.default_nh = 1025;
    c6.max_routes = 1024;
    c6.trie.nh_sz = CNE_FIB_TRIE_4B;
    c6.trie.num_tbl8 = 1 << 15;
    nd6 = cne_fib6_create("nd6-fib", &c6);
    if (!rt4 || !arp || !nd6) {
        fprintf(stderr, "create failed\n");
        exit(1);
    }
    uint64_t s = 7;
    for (int i = 0; i < 1024; i++) {
        if (i < 896) {
            r_ip[i] = (10u << 24) + ((uint32_t)i << 8);
            r_d[i] = 24;
        } else {
            const int k = i - 896;
            r_d[i] = (uint8_t)(25 + k % 8);
            r_ip[i] = ((10u << 24) | (4u << 16) | ((uint32_t)k << 8) | (rnd(&s) & 0xFF)) & (~0u << (32 - r_d[i]));
        }
        r_nh[i] = (uint64_t)(i % 64) | 1u << 24;
        if (cne_fib_add(rt4, r_ip[i], r_d[i], r_nh[i]) < 0 ||
            cne_fib_add(arp, (10u << 24) | (5u << 16) | (uint32_t)i, 32, (uint64_t)i) < 0) {
            fprintf(stderr, "add failed\n");
            exit(1);
        }
        uint8_t ip6[16] = {0x20, 0x01, 0x0d, 0xb8};
        const uint8_t d6 = (uint8_t)(i == 0 ? 32 : 33 + (i - 1) % 32);
        const uint32_t w = rnd(&s) & (d6 > 32 ? ~0u << (64 - d6) : 0u);
        ip6[4] = (uint8_t)(w >> 24);
        ip6[5] = (uint8_t)(w >> 16);
        ip6[6] = (uint8_t)(w >> 8);
        ip6[7] = (uint8_t)w;
        if (cne_fib6_add(nd6, ip6, d6, (uint64_t)i) < 0) {
            fprintf(stderr, "add6 failed\n");
            exit(1);
        }
    }
    for (int i = 0; i < NKEYS; i++) {
        keys4[i] = (i & 3) == 3 ? rnd(&s) : (10u << 24) | (rnd(&s) & 0x0004FFFFu);
        keys_arp[i] = (i & 3) == 3 ? rnd(&s) : (10u << 24) | (5u << 16) | (rnd(&s) & 0x3FF);
        for (int b = 0; b < 16; b++)
            keys6[i][b] = (uint8_t)rnd(&s);
        if ((i & 3) != 3) {
            keys6[i][0] = 0x20;
            keys6[i][1] = 0x01;
            keys6[i][2] = 0x0d;
            keys6[i][3] = 0xb8;
        }
    }
}

enum { F_RT4, F_ARP, F_ND6 };

/* run `calls` calls of n keys, walking the key array; answers to out */
static int run(int which, int n, uint64_t calls, uint64_t *out)
{
    uint64_t off = 0;
    for (uint64_t c = 0; c < calls; c++) {
        if (off + (uint64_t)n > NKEYS)
            off = 0;
        int rc;
        if (which == F_RT4)
            rc = cne_fib_lookup_bulk(rt4, keys4 + off, out + off, n);
        else if (which == F_ARP)
            rc = cne_fib_lookup_bulk(arp, keys_arp + off, out + off, n);
        else
            rc = cne_fib6_lookup_bulk(nd6, &keys6[off], out + off, n);
        if (rc < 0)
            return rc;
        off += (uint64_t)n;
    }
    return 0;
}

static int select_all(int type6, int type4)
{
    int r = cne_fib_select_lookup(rt4, type4);
    r |= cne_fib_select_lookup(arp, type4);
    r |= cne_fib6_select_lookup(nd6, type6);
    return r;
}

struct thr {
    int which, n;
    double secs;
    uint64_t calls;
    uint64_t *out;
};

static void *thr_main(void *p)
{
    struct thr *t = p;
    const double t0 = now_s();
    uint64_t calls = 0;
    while (now_s() - t0 < t->secs) {
        run(t->which, t->n, 256, t->out);
        calls += 256;
    }
    t->calls = calls;
    return NULL;
}

int main(int argc, char **argv)
{
    int gpu = 0;
    double ms = 200;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--gpu"))
            gpu = 1;
        else if (!strcmp(argv[i], "--ms") && i + 1 < argc)
            ms = atof(argv[++i]);
    }
    build();
    static uint64_t ref[3][NKEYS], got[NKEYS];
    /* reference answers: the whole key arrays once, default selection */
    if (run(F_RT4, NKEYS, 1, ref[F_RT4]) || run(F_ARP, NKEYS, 1, ref[F_ARP]) ||
        run(F_ND6, NKEYS, 1, ref[F_ND6]))
        return 1;
    int bad = 0;
    for (int i = 0; i < NKEYS; i += 61)
        if (ref[F_RT4][i] != lpm4(keys4[i]))
            bad++;
    for (int i = 0; i < NKEYS; i++) {
        const uint32_t k = keys_arp[i];
        const uint64_t want = (k >> 16) == ((10u << 8) | 5u) && (k & 0xFFFF) < 1024 ? (k & 0xFFFF) : 1025;
        if (ref[F_ARP][i] != want)
            bad++;
    }
    const char *names[3] = {"rt4", "arp", "nd6"};
    const int shapes[3] = {1, 4, 256};
    printf("{\"ms_per_point\": %.0f, \"points\": [", ms);
    int first = 1;
    for (int sel = 0; sel < 1 + gpu; sel++) {
        if (select_all(sel ? CNDP_FIB_LOOKUP_GPU : CNE_FIB_LOOKUP_DEFAULT,
                       sel ? CNDP_FIB_LOOKUP_GPU : CNE_FIB_LOOKUP_DEFAULT))
            return 1;
        for (int w = 0; w < 3; w++)
            for (int si = 0; si < 3; si++) {
                const int n = shapes[si];
                /* calibrate: how many calls fill ~ms */
                uint64_t calls = 64;
                double dt;
                for (;;) {
                    const double t0 = now_s();
                    if (run(w, n, calls, got) < 0)
                        return 1;
                    dt = now_s() - t0;
                    if (dt * 1e3 >= ms || calls > (1ull << 32))
                        break;
                    calls *= dt > 0 ? (uint64_t)(ms / 1e3 / dt * 1.2) + 2 : 16;
                }
                /* every answer of the last timed pass vs the reference */
                const uint64_t cover = calls * (uint64_t)n < NKEYS ? calls * (uint64_t)n : NKEYS;
                for (uint64_t i = 0; i < cover / (uint64_t)n * (uint64_t)n; i++)
                    if (got[i] != ref[w][i])
                        bad++;
                printf("%s{\"sel\": \"%s\", \"fib\": \"%s\", \"keys\": %d, \"ns_per_call\": %.1f, "
                       "\"Mlookups_per_s\": %.2f}",
                       first ? "" : ", ", sel ? "gpu" : "default", names[w], n, dt / calls * 1e9,
                       calls * (double)n / dt / 1e6);
                first = 0;
            }
    }
    printf("], \"threads\": [");
    /* default selection, rt4, 4-key calls, T threads on one FIB */
    select_all(CNE_FIB_LOOKUP_DEFAULT, CNE_FIB_LOOKUP_DEFAULT);
    first = 1;
    for (int T = 1; T <= 8; T *= 2) {
        pthread_t th[8];
        struct thr a[8];
        for (int k = 0; k < T; k++) {
            a[k] = (struct thr){F_RT4, 4, ms / 1e3, 0, calloc(NKEYS, sizeof(uint64_t))};
            pthread_create(&th[k], NULL, thr_main, &a[k]);
        }
        uint64_t total = 0;
        for (int k = 0; k < T; k++) {
            pthread_join(th[k], NULL);
            total += a[k].calls;
            for (int i = 0; i < NKEYS; i += 97)
                if (a[k].out[i] && a[k].out[i] != ref[F_RT4][i])
                    bad++;
            free(a[k].out);
        }
        printf("%s{\"threads\": %d, \"keys\": 4, \"Mlookups_per_s\": %.2f}", first ? "" : ", ", T,
               total * 4.0 / (ms / 1e3) / 1e6);
        first = 0;
    }
    printf("], \"wrong\": %d}\n", bad);
    cne_fib_free(rt4);
    cne_fib_free(arp);
    cne_fib6_free(nd6);
    return bad ? 1 : 0;
}
