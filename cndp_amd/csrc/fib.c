/*
 * fib.c -- host control plane of the GPU FIBs (IPv4 DIR-24-8, IPv6 trie).
 *
 * Route semantics follow the reference modify paths:
 *   IPv4  lib/usr/clib/fib/dir24_8.c:370-453 (dir24_8_modify), :456-499 create
 *   IPv6  lib/usr/clib/fib/trie.c:518-579 (trie_modify),       :581-619 create
 *   DUMMY cne_fib.c:32-71 / cne_fib6.c:34-70 (RIB-only FIBs)
 * including their return codes, the "parent already has this next hop"
 * early return, and the tbl8 reservation counters that decide -ENOSPC.
 *
 * The table build is this repository's own: a route change re-paints the
 * part of its prefix that no more-specific route covers.  That part is cut
 * into aligned prefix blocks; each block is written into tbl24 or into the
 * tbl8 group(s) under it, and a group whose 256 entries became identical is
 * folded back into its parent entry.  DUMMY FIBs use the same images with
 * 8-byte entries and a growable group pool, so the GPU serves them too.
 */
#include "fib_internal.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* entry access                                                              */
/* ------------------------------------------------------------------------ */
static inline uint64_t ent_get(const struct cndp_tbl *t, const uint8_t *base, uint64_t i)
{
    switch (t->nh_sz) {
    case 0:
        return base[i];
    case 1:
        return ((const uint16_t *)(const void *)base)[i];
    case 2:
        return ((const uint32_t *)(const void *)base)[i];
    default:
        return ((const uint64_t *)(const void *)base)[i];
    }
}

static inline void ent_set(struct cndp_tbl *t, uint8_t *base, uint64_t i, uint64_t v)
{
    switch (t->nh_sz) {
    case 0:
        base[i] = (uint8_t)v;
        break;
    case 1:
        ((uint16_t *)(void *)base)[i] = (uint16_t)v;
        break;
    case 2:
        ((uint32_t *)(void *)base)[i] = (uint32_t)v;
        break;
    default:
        ((uint64_t *)(void *)base)[i] = v;
        break;
    }
}

/* a changed range for the device painter: merged into the last one when they
 * touch (the painters walk a route's range in order), else appended; past
 * CNDP_TBL_LOG the count only marks the overflow */
static inline void log_range(struct cndp_range *log, uint32_t *n, uint64_t lo, uint64_t hi)
{
    if (*n > CNDP_TBL_LOG)
        return;
    if (*n) {
        struct cndp_range *l = &log[*n - 1];
        if (lo <= l->hi && hi >= l->lo) {
            l->lo = lo < l->lo ? lo : l->lo;
            l->hi = hi > l->hi ? hi : l->hi;
            return;
        }
    }
    if (*n < CNDP_TBL_LOG) {
        log[*n].lo = lo;
        log[*n].hi = hi;
    }
    (*n)++;
}

static inline void dirty24(struct cndp_tbl *t, uint64_t lo, uint64_t hi)
{
    if (lo < t->d24_lo)
        t->d24_lo = lo;
    if (hi > t->d24_hi)
        t->d24_hi = hi;
    log_range(t->log24, &t->n_log24, lo, hi);
}

static inline void dirty8(struct cndp_tbl *t, uint64_t lo, uint64_t hi)
{
    if (lo < t->d8_lo)
        t->d8_lo = lo;
    if (hi > t->d8_hi)
        t->d8_hi = hi;
    log_range(t->log8, &t->n_log8, lo, hi);
}

static inline uint64_t t24_get(const struct cndp_tbl *t, uint64_t i) { return ent_get(t, t->tbl24, i); }
static inline void t24_set(struct cndp_tbl *t, uint64_t i, uint64_t v)
{
    ent_set(t, t->tbl24, i, v);
    dirty24(t, i, i + 1);
}
static inline uint64_t t8_get(const struct cndp_tbl *t, uint64_t i) { return ent_get(t, t->tbl8, i); }
static inline void t8_set(struct cndp_tbl *t, uint64_t i, uint64_t v)
{
    ent_set(t, t->tbl8, i, v);
    dirty8(t, i, i + 1);
}

/* ------------------------------------------------------------------------ */
/* table lifetime + tbl8 group pool (lowest free index first)               */
/* ------------------------------------------------------------------------ */
static int tbl_init(struct cndp_tbl *t, uint32_t nh_sz, uint32_t is_trie, uint32_t num_tbl8,
                    uint64_t def_nh)
{
    memset(t, 0, sizeof(*t));
    pthread_mutex_init(&t->dev_lock, NULL);
    t->def_nh = def_nh;
    t->nh_sz = nh_sz;
    t->is_trie = is_trie;
    t->num_tbl8 = num_tbl8;
    t->cap_groups = num_tbl8 ? num_tbl8 : 64;
    t->dev_id = -1;
    size_t esz = (size_t)1 << nh_sz;
    t->tbl24 = malloc((size_t)CNDP_TBL24_ENT * esz);
    t->tbl8 = calloc((size_t)(t->cap_groups + 1) * CNDP_TBL8_GRP, esz);
    t->used = calloc((t->cap_groups + 63) / 64, sizeof(uint64_t));
    if (!t->tbl24 || !t->tbl8 || !t->used) {
        free(t->tbl24);
        free(t->tbl8);
        free(t->used);
        pthread_mutex_destroy(&t->dev_lock);
        return -ENOMEM;
    }
    uint64_t v = def_nh << 1;
    for (uint64_t i = 0; i < CNDP_TBL24_ENT; i++)
        ent_set(t, t->tbl24, i, v);
    t->d24_lo = 0;
    t->d24_hi = CNDP_TBL24_ENT;
    t->d8_lo = 0;
    t->d8_hi = (uint64_t)(t->cap_groups + 1) * CNDP_TBL8_GRP;
    return 0;
}

static void tbl_fini(struct cndp_tbl *t)
{
    cndp_tbl_dev_free(t);
    free(t->tbl24);
    free(t->tbl8);
    free(t->used);
    free(t->dir16);
    free(t->page_of);
    free(t->pages);
    free(t->page_free);
    pthread_mutex_destroy(&t->dev_lock);
    memset(t, 0, sizeof(*t));
}

static int grow_pool(struct cndp_tbl *t)
{
    uint32_t ncap = t->cap_groups * 2;
    size_t esz = (size_t)1 << t->nh_sz;
    uint8_t *n8 = realloc(t->tbl8, (size_t)(ncap + 1) * CNDP_TBL8_GRP * esz);
    if (!n8)
        return -ENOMEM;
    memset(n8 + (size_t)(t->cap_groups + 1) * CNDP_TBL8_GRP * esz, 0,
           (size_t)(ncap - t->cap_groups) * CNDP_TBL8_GRP * esz);
    t->tbl8 = n8;
    uint64_t *nu = realloc(t->used, ((ncap + 63) / 64) * sizeof(uint64_t));
    if (!nu)
        return -ENOMEM;
    memset(nu + (t->cap_groups + 63) / 64, 0,
           (((ncap + 63) / 64) - (t->cap_groups + 63) / 64) * sizeof(uint64_t));
    t->used = nu;
    dirty8(t, (uint64_t)(t->cap_groups + 1) * CNDP_TBL8_GRP, (uint64_t)(ncap + 1) * CNDP_TBL8_GRP);
    t->cap_groups = ncap;
    return 0;
}

static int group_alloc(struct cndp_tbl *t)
{
    for (;;) {
        uint32_t words = (t->cap_groups + 63) / 64;
        for (uint32_t w = 0; w < words; w++) {
            if (t->used[w] == ~0ULL)
                continue;
            uint32_t b = (uint32_t)__builtin_ctzll(~t->used[w]);
            uint32_t g = w * 64 + b;
            if (g >= t->cap_groups)
                break;
            t->used[w] |= 1ULL << b;
            t->cur_tbl8s++;
            return (int)g;
        }
        if (t->num_tbl8)
            return -ENOSPC;
        if (grow_pool(t))
            return -ENOMEM;
    }
}

static void group_free(struct cndp_tbl *t, uint64_t g)
{
    uint64_t base = g * CNDP_TBL8_GRP;
    memset(t->tbl8 + (base << t->nh_sz), 0, (size_t)CNDP_TBL8_GRP << t->nh_sz);
    dirty8(t, base, base + CNDP_TBL8_GRP);
    t->used[g / 64] &= ~(1ULL << (g % 64));
    t->cur_tbl8s--;
}

/* free every group hanging below an extended trie entry */
static void trie_free_chain(struct cndp_tbl *t, uint64_t e)
{
    if (!(e & 1u))
        return;
    uint64_t g = e >> 1;
    for (uint32_t k = 0; k < CNDP_TBL8_GRP; k++)
        trie_free_chain(t, t8_get(t, g * CNDP_TBL8_GRP + k));
    group_free(t, g);
}

/* if all 256 entries of group g are equal (and, for the trie, not extended),
 * return 1 and the common value in *v */
static int group_uniform(const struct cndp_tbl *t, uint64_t g, uint64_t *v)
{
    uint64_t base = g * CNDP_TBL8_GRP;
    uint64_t first = t8_get(t, base);
    if (t->is_trie && (first & 1u))
        return 0;
    for (uint32_t k = 1; k < CNDP_TBL8_GRP; k++)
        if (t8_get(t, base + k) != first)
            return 0;
    *v = first;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* block installers                                                          */
/* ------------------------------------------------------------------------ */
/* IPv4: write nh over the aligned block p/len (no route inside it is more
 * specific than this block, by construction of the caller). */
static int dir24_install(struct cndp_tbl *t, uint32_t p, uint32_t len, uint64_t nh)
{
    if (len <= 24) {
        uint64_t first = p >> 8, cnt = 1ull << (24 - len);
        for (uint64_t i = first; i < first + cnt; i++) {
            uint64_t e = t24_get(t, i);
            /* the entry is rewritten before its group is cleared, so a host
             * lookup running on another thread (CNE_FIB_LOOKUP_DEFAULT takes
             * no lock, as dir24_8.h's does not) never follows it into a
             * zeroed group */
            ent_set(t, t->tbl24, i, nh << 1);
            if (e & 1u) {
                __atomic_thread_fence(__ATOMIC_RELEASE);
                group_free(t, e >> 1);
            }
        }
        dirty24(t, first, first + cnt);
        return 0;
    }
    uint64_t idx = p >> 8;
    uint64_t e = t24_get(t, idx);
    if (!(e & 1u)) {
        int g = group_alloc(t);
        if (g < 0)
            return g;
        uint64_t base = (uint64_t)g * CNDP_TBL8_GRP;
        for (uint32_t k = 0; k < CNDP_TBL8_GRP; k++)
            ent_set(t, t->tbl8, base + k, e | 1u);
        dirty8(t, base, base + CNDP_TBL8_GRP);
        e = ((uint64_t)g << 1) | 1u;
        __atomic_thread_fence(__ATOMIC_RELEASE); /* group filled before it is linked */
        t24_set(t, idx, e);
    }
    uint64_t g = e >> 1;
    uint64_t first = g * CNDP_TBL8_GRP + (p & 0xffu), cnt = 1ull << (32 - len);
    for (uint64_t i = first; i < first + cnt; i++)
        ent_set(t, t->tbl8, i, (nh << 1) | 1u);
    dirty8(t, first, first + cnt);
    uint64_t v;
    if (group_uniform(t, g, &v)) { /* fold back, cf. dir24_8.c:189-247 */
        t24_set(t, idx, v & ~1ull);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        group_free(t, g);
    }
    return 0;
}

static inline uint32_t byte_at(u128 p, uint32_t k) { return (uint32_t)(p >> (120 - 8 * k)) & 0xffu; }

/* IPv6: write nh over the aligned block p/len */
static int trie_install(struct cndp_tbl *t, u128 p, uint32_t len, uint64_t nh)
{
    if (len <= 24) {
        uint64_t first = (uint64_t)(p >> 104), cnt = 1ull << (24 - len);
        for (uint64_t i = first; i < first + cnt; i++) {
            const uint64_t old = t24_get(t, i);
            ent_set(t, t->tbl24, i, nh << 1); /* unlinked before it is freed */
            __atomic_thread_fence(__ATOMIC_RELEASE);
            trie_free_chain(t, old);
        }
        dirty24(t, first, first + cnt);
        return 0;
    }
    /* walk / extend down to the group holding byte (len-1)/8 */
    uint64_t path[16];    /* entry index of each extended entry on the path */
    int in_tbl8[16];
    int depth = 0;
    uint64_t ent = (uint64_t)(p >> 104);
    int ent_in8 = 0;
    for (uint32_t k = 3; k < 16; k++) {
        uint64_t e = ent_in8 ? t8_get(t, ent) : t24_get(t, ent);
        if (!(e & 1u)) {
            int g = group_alloc(t);
            if (g < 0)
                return g;
            uint64_t base = (uint64_t)g * CNDP_TBL8_GRP;
            for (uint32_t q = 0; q < CNDP_TBL8_GRP; q++)
                ent_set(t, t->tbl8, base + q, e);
            dirty8(t, base, base + CNDP_TBL8_GRP);
            e = ((uint64_t)g << 1) | 1u;
            __atomic_thread_fence(__ATOMIC_RELEASE);
            if (ent_in8)
                t8_set(t, ent, e);
            else
                t24_set(t, ent, e);
        }
        path[depth] = ent;
        in_tbl8[depth] = ent_in8;
        depth++;
        uint64_t gbase = (e >> 1) * CNDP_TBL8_GRP;
        int rem = (int)len - 8 * (int)k;
        if (rem <= 8) {
            uint64_t first = gbase + byte_at(p, k), cnt = 1ull << (8 - rem);
            for (uint64_t i = first; i < first + cnt; i++) {
                const uint64_t old = t8_get(t, i);
                ent_set(t, t->tbl8, i, nh << 1);
                __atomic_thread_fence(__ATOMIC_RELEASE);
                trie_free_chain(t, old);
            }
            dirty8(t, first, first + cnt);
            break;
        }
        ent = gbase + byte_at(p, k);
        ent_in8 = 1;
    }
    /* fold uniform groups back up the path (trie.c:165-214 recycle) */
    for (int d = depth - 1; d >= 0; d--) {
        uint64_t e = in_tbl8[d] ? t8_get(t, path[d]) : t24_get(t, path[d]);
        uint64_t v;
        if (!(e & 1u) || !group_uniform(t, e >> 1, &v))
            break;
        if (in_tbl8[d])
            t8_set(t, path[d], v);
        else
            t24_set(t, path[d], v);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        group_free(t, e >> 1);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* paint: install nh over prefix/depth minus every more specific route       */
/* ------------------------------------------------------------------------ */
struct hole_list {
    u128 *lo, *hi; /* inclusive, in the W-bit domain */
    uint32_t n, cap;
    uint32_t width;
    int err;
};

static inline u128 key_to_u128(cndp_key128 k) { return ((u128)k.hi << 64) | k.lo; }

static inline u128 wmask(uint32_t width, uint32_t depth)
{
    /* W-bit mask with the top `depth` bits set */
    u128 all = width == 128 ? ~(u128)0 : (((u128)1 << width) - 1);
    if (depth == 0)
        return 0;
    if (depth >= width)
        return all;
    return all & ~((((u128)1) << (width - depth)) - 1);
}

static int collect_hole(const struct cndp_rnode *n, void *arg)
{
    struct hole_list *h = arg;
    if (h->n == h->cap) {
        uint32_t nc = h->cap ? h->cap * 2 : 16;
        u128 *a = realloc(h->lo, nc * sizeof(u128)), *b;
        if (!a) {
            h->err = -ENOMEM;
            return 1;
        }
        h->lo = a;
        b = realloc(h->hi, nc * sizeof(u128));
        if (!b) {
            h->err = -ENOMEM;
            return 1;
        }
        h->hi = b;
        h->cap = nc;
    }
    u128 k = key_to_u128(n->key);
    if (h->width == 32)
        k >>= 96;
    h->lo[h->n] = k;
    h->hi[h->n] = k | (~wmask(h->width, n->depth) & wmask(h->width, h->width));
    h->n++;
    return 0;
}

typedef int (*install_fn)(struct cndp_tbl *t, u128 p, uint32_t len, uint64_t nh);

static int inst4(struct cndp_tbl *t, u128 p, uint32_t len, uint64_t nh)
{
    return dir24_install(t, (uint32_t)p, len, nh);
}
static int inst6(struct cndp_tbl *t, u128 p, uint32_t len, uint64_t nh)
{
    return trie_install(t, p, len, nh);
}

/* cover [a, b] (inclusive, W-bit) with maximal aligned blocks */
static int cover_range(struct cndp_tbl *t, uint32_t width, u128 a, u128 b, uint64_t nh,
                       install_fn fn)
{
    for (;;) {
        uint32_t tz = a == 0 ? width : (uint32_t)(a & (u128)~0ULL ? __builtin_ctzll((uint64_t)a)
                                                                   : 64 + __builtin_ctzll((uint64_t)(a >> 64)));
        if (tz > width)
            tz = width;
        u128 span = b - a; /* number of addresses - 1 */
        uint32_t sb;       /* floor(log2(span + 1)) */
        if (span == wmask(width, width))
            sb = width;
        else {
            u128 s1 = span + 1;
            uint64_t hi = (uint64_t)(s1 >> 64), lo = (uint64_t)s1;
            sb = hi ? 127u - (uint32_t)__builtin_clzll(hi) : 63u - (uint32_t)__builtin_clzll(lo);
        }
        uint32_t k = tz < sb ? tz : sb;
        int r = fn(t, a, width - k, nh);
        if (r)
            return r;
        if (k == width)
            return 0;
        u128 step = (u128)1 << k;
        u128 last = a + step - 1;
        if (last >= b)
            return 0;
        a += step;
    }
}

static int paint(struct cndp_tbl *t, const struct cndp_rib *rib, uint32_t width, cndp_key128 key,
                 uint32_t depth, uint64_t nh)
{
    struct hole_list h = {0};
    h.width = width;
    cndp_rib_for_each_hole(rib, key, depth, collect_hole, &h);
    int r = h.err;
    install_fn fn = width == 32 ? inst4 : inst6;
    u128 lo = key_to_u128(key);
    if (width == 32)
        lo >>= 96;
    lo &= wmask(width, depth);
    u128 last = lo | (~wmask(width, depth) & wmask(width, width));
    u128 cur = lo;
    int done = 0;
    for (uint32_t i = 0; !r && i < h.n; i++) {
        if (h.lo[i] > cur)
            r = cover_range(t, width, cur, h.lo[i] - 1, nh, fn);
        if (h.hi[i] >= last) {
            done = 1;
            break;
        }
        cur = h.hi[i] + 1;
    }
    if (!r && !done && cur <= last)
        r = cover_range(t, width, cur, last, nh, fn);
    free(h.lo);
    free(h.hi);
    return r;
}

/* ------------------------------------------------------------------------ */
/* synchronous host lookups (the reference's CNE_FIB_LOOKUP_DEFAULT)         */
/* ------------------------------------------------------------------------ */
/* cne_fib.c:86 binds every DIR-24-8 FIB to dir24_8_get_lookup_fn(DEFAULT):
 * a scalar loop over the table image that prefetches the tbl24 entry of the
 * key `pf` positions ahead (dir24_8.h:118-148; 5/6/15/12 for 1/2/4/8-B
 * entries).  cne_fib6.c:92 does the same with trie.h:119-138.  These read the
 * host image that fib.c paints and the HBM mirror copies, so the answers are
 * the GPU lookup's by construction.  Like the reference's they take no lock:
 * the installers above link a group only after filling it and clear it only
 * after unlinking it. */
#define HOST_LK4(sfx, type, pf)                                                            \
    static void host_lookup4_##sfx(const struct cndp_tbl *t, const uint32_t *ips,         \
                                   uint64_t *nh, uint32_t n)                              \
    {                                                                                      \
        const type *t24 = (const type *)(const void *)t->tbl24;                            \
        const type *t8 = (const type *)(const void *)t->tbl8;                              \
        const uint32_t ahead = n < (pf) ? n : (pf);                                        \
        uint32_t i;                                                                        \
        for (i = 0; i < ahead; i++)                                                        \
            __builtin_prefetch(&t24[ips[i] >> 8]);                                         \
        for (i = 0; i < n; i++) {                                                          \
            if (i + ahead < n)                                                             \
                __builtin_prefetch(&t24[ips[i + ahead] >> 8]);                             \
            uint64_t e = t24[ips[i] >> 8];                                                 \
            if (__builtin_expect((e & 1u) != 0, 0))                                        \
                e = t8[(uint8_t)ips[i] + (e >> 1) * CNDP_TBL8_GRP];                        \
            nh[i] = e >> 1;                                                                \
        }                                                                                  \
    }
HOST_LK4(1b, uint8_t, 5)
HOST_LK4(2b, uint16_t, 6)
HOST_LK4(4b, uint32_t, 15)
HOST_LK4(8b, uint64_t, 12)

#define HOST_LK6(sfx, type)                                                                \
    static void host_lookup6_##sfx(const struct cndp_tbl *t, const uint8_t *ips,          \
                                   uint64_t *nh, uint32_t n)                              \
    {                                                                                      \
        const type *t24 = (const type *)(const void *)t->tbl24;                            \
        const type *t8 = (const type *)(const void *)t->tbl8;                              \
        for (uint32_t i = 0; i < n; i++) {                                                 \
            const uint8_t *a = ips + (size_t)i * 16;                                       \
            uint64_t e = t24[(uint32_t)a[0] << 16 | (uint32_t)a[1] << 8 | a[2]];           \
            for (uint32_t j = 3; (e & 1u) && j < 16; j++)                                  \
                e = t8[a[j] + (e >> 1) * CNDP_TBL8_GRP];                                   \
            nh[i] = e >> 1;                                                                \
        }                                                                                  \
    }
HOST_LK6(1b, uint8_t)
HOST_LK6(2b, uint16_t)
HOST_LK6(4b, uint32_t)
HOST_LK6(8b, uint64_t)

static void host_lookup4(const struct cndp_tbl *t, const uint32_t *ips, uint64_t *nh, uint32_t n)
{
    switch (t->nh_sz) {
    case 0:
        host_lookup4_1b(t, ips, nh, n);
        break;
    case 1:
        host_lookup4_2b(t, ips, nh, n);
        break;
    case 2:
        host_lookup4_4b(t, ips, nh, n);
        break;
    default:
        host_lookup4_8b(t, ips, nh, n);
        break;
    }
}

static void host_lookup6(const struct cndp_tbl *t, const uint8_t *ips, uint64_t *nh, uint32_t n)
{
    switch (t->nh_sz) {
    case 0:
        host_lookup6_1b(t, ips, nh, n);
        break;
    case 1:
        host_lookup6_2b(t, ips, nh, n);
        break;
    case 2:
        host_lookup6_4b(t, ips, nh, n);
        break;
    default:
        host_lookup6_8b(t, ips, nh, n);
        break;
    }
}

/* ------------------------------------------------------------------------ */
/* IPv4 API (cne_fib.h)                                                      */
/* ------------------------------------------------------------------------ */
static inline uint64_t max_nh(uint32_t nh_sz) { return (1ULL << ((8u << nh_sz) - 1)) - 1; }
static inline uint32_t mask32(uint32_t d) { return d ? (uint32_t)(0xFFFFFFFFull << (32 - d)) : 0; }

struct cne_fib *cne_fib_create(const char *name, struct cne_fib_conf *conf)
{
    /* cne_fib.c:119-167 + dir24_8.c:456-499 argument checks */
    if (!name || !conf || conf->max_routes < 0 || conf->type > CNE_FIB_DIR24_8)
        return NULL;
    if ((int64_t)conf->max_routes * 2 <= 0)
        return NULL;
    uint32_t nh_sz = 3, ntbl8 = 0;
    if (conf->type == CNE_FIB_DIR24_8) {
        if ((int)conf->dir24_8.nh_sz < CNE_FIB_DIR24_8_1B || conf->dir24_8.nh_sz > CNE_FIB_DIR24_8_8B)
            return NULL;
        nh_sz = (uint32_t)conf->dir24_8.nh_sz;
        if (conf->dir24_8.num_tbl8 > max_nh(nh_sz) || conf->dir24_8.num_tbl8 == 0 ||
            conf->default_nh > max_nh(nh_sz))
            return NULL;
        ntbl8 = (conf->dir24_8.num_tbl8 + 63u) & ~63u; /* CNE_ALIGN_CEIL(.., 64) */
    }
    struct cne_fib *f = calloc(1, sizeof(*f));
    if (!f)
        return NULL;
    snprintf(f->name, sizeof(f->name), "%s", name);
    f->type = conf->type;
    f->def_nh = conf->default_nh;
    if (cndp_rib_init(&f->rib, (uint32_t)conf->max_routes * 2u, 32) ||
        tbl_init(&f->t, nh_sz, 0, ntbl8, conf->type == CNE_FIB_DUMMY ? conf->default_nh : conf->default_nh)) {
        cndp_rib_fini(&f->rib);
        free(f);
        return NULL;
    }
    return f;
}

void cne_fib_free(struct cne_fib *fib)
{
    if (!fib)
        return;
    tbl_fini(&fib->t);
    cndp_rib_fini(&fib->rib);
    free(fib);
}

static int fib4_modify(struct cne_fib *f, uint32_t ip, uint8_t depth, uint64_t nh, int op)
{
    if (depth > CNE_FIB_MAXDEPTH)
        return -EINVAL;
    if (f->type == CNE_FIB_DUMMY) {
        /* cne_fib.c:48-71 */
        cndp_key128 k = cndp_key_from_v4(ip & mask32(depth));
        struct cndp_rnode *n = cndp_rib_lookup_exact(&f->rib, k, depth);
        if (op == CNE_FIB_ADD) {
            if (!n) {
                n = cndp_rib_insert(&f->rib, k, depth);
                if (!n)
                    return -1;
                n->nh = ~nh; /* force a repaint below */
            }
            if (n->nh != nh) {
                int r = paint(&f->t, &f->rib, 32, k, depth, nh & max_nh(3));
                if (r)
                    return r;
            }
            n->nh = nh;
            return 0;
        }
        if (!n)
            return -ENOENT;
        struct cndp_rnode *par = cndp_rib_parent(n);
        int r = paint(&f->t, &f->rib, 32, k, depth, (par ? par->nh : f->def_nh) & max_nh(3));
        if (r)
            return r;
        cndp_rib_remove(&f->rib, k, depth);
        return 0;
    }

    /* dir24_8.c:370-453 */
    if (nh > max_nh(f->t.nh_sz))
        return -EINVAL;
    ip &= mask32(depth);
    cndp_key128 k = cndp_key_from_v4(ip);
    struct cndp_rnode *n = cndp_rib_lookup_exact(&f->rib, k, depth);
    int r = 0;
    if (op == CNE_FIB_ADD) {
        if (n) {
            if (n->nh == nh)
                return 0;
            r = paint(&f->t, &f->rib, 32, k, depth, nh);
            if (r == 0)
                n->nh = nh;
            return 0; /* the reference returns 0 here whatever modify_fib said */
        }
        int had_long = 1;
        if (depth > 24) {
            had_long = cndp_rib_has_more_specific(&f->rib, cndp_key_from_v4(ip & 0xffffff00u), 24);
            if (!had_long && f->rsvd_tbl8s >= f->t.num_tbl8)
                return -ENOSPC;
        }
        n = cndp_rib_insert(&f->rib, k, depth);
        if (!n)
            return -1;
        n->nh = nh;
        struct cndp_rnode *par = cndp_rib_parent(n);
        if (par && par->nh == nh)
            return 0;
        r = paint(&f->t, &f->rib, 32, k, depth, nh);
        if (r) {
            cndp_rib_remove(&f->rib, k, depth);
            return r;
        }
        if (depth > 24 && !had_long)
            f->rsvd_tbl8s++;
        return 0;
    }
    if (op == CNE_FIB_DEL) {
        if (!n)
            return -ENOENT;
        struct cndp_rnode *par = cndp_rib_parent(n);
        if (par) {
            if (par->nh != n->nh)
                r = paint(&f->t, &f->rib, 32, k, depth, par->nh);
        } else {
            r = paint(&f->t, &f->rib, 32, k, depth, f->def_nh);
        }
        if (r == 0) {
            cndp_rib_remove(&f->rib, k, depth);
            if (depth > 24 &&
                !cndp_rib_has_more_specific(&f->rib, cndp_key_from_v4(ip & 0xffffff00u), 24))
                f->rsvd_tbl8s--;
        }
        return r;
    }
    return -EINVAL;
}

int cne_fib_add(struct cne_fib *fib, uint32_t ip, uint8_t depth, uint64_t next_hop)
{
    if (!fib || depth > CNE_FIB_MAXDEPTH)
        return -EINVAL;
    /* the host image and its dirty ranges change under dev_lock, so a device
     * sync running on a worker thread never copies a half-painted range or
     * clears the marks of a change it did not copy */
    pthread_mutex_lock(&fib->t.dev_lock);
    const int r = fib4_modify(fib, ip, depth, next_hop, CNE_FIB_ADD);
    pthread_mutex_unlock(&fib->t.dev_lock);
    return r;
}

int cne_fib_delete(struct cne_fib *fib, uint32_t ip, uint8_t depth)
{
    if (!fib || depth > CNE_FIB_MAXDEPTH)
        return -EINVAL;
    pthread_mutex_lock(&fib->t.dev_lock);
    const int r = fib4_modify(fib, ip, depth, 0, CNE_FIB_DEL);
    pthread_mutex_unlock(&fib->t.dev_lock);
    return r;
}

int cne_fib_lookup_bulk(struct cne_fib *fib, uint32_t *ips, uint64_t *next_hops, int n)
{
    if (!fib || !ips || !next_hops || n < 0)
        return -EINVAL;
    if (n == 0)
        return 0;
    if (fib->lookup_type == CNDP_FIB_LOOKUP_GPU)
        return cndp_tbl_lookup4_host(&fib->t, ips, next_hops, (uint32_t)n);
    if (fib->type == CNE_FIB_DUMMY) {
        /* cne_fib.c:32-46 walks the RIB; the image painted from it gives the
         * same answers.  Its group pool grows (realloc) on add, so this one
         * reads under the table lock */
        pthread_mutex_lock(&fib->t.dev_lock);
        host_lookup4(&fib->t, ips, next_hops, (uint32_t)n);
        pthread_mutex_unlock(&fib->t.dev_lock);
        return 0;
    }
    host_lookup4(&fib->t, ips, next_hops, (uint32_t)n);
    return 0;
}

void *cne_fib_get_dp(struct cne_fib *fib) { return fib ? &fib->t : NULL; }

struct cne_rib *cne_fib_get_rib(struct cne_fib *fib) { return fib ? (struct cne_rib *)&fib->rib : NULL; }

/* cne_fib.c:206-221: only DIR-24-8 FIBs select a lookup.  Every scalar
 * selector binds the host loop above.  CNE_FIB_LOOKUP_DIR24_8_VECTOR_AVX512 is
 * -EINVAL, as the reference answers it unless the application raised the
 * SIMD width to 512 bits (dir24_8.c:63-69: get_vector_fn is NULL at the
 * default CNE_VECT_SIMD_256, cne_cpuflags.c:24, cne_vect_generic.h:205) --
 * this library has no such knob and no AVX-512 form.  CNE_FIB_LOOKUP_GPU (an
 * extension; DUMMY FIBs accept it too) sends every cne_fib_lookup_bulk to the
 * device mirror instead. */
int cne_fib_select_lookup(struct cne_fib *fib, enum cne_fib_lookup_type type)
{
    if (fib && fib->type == CNE_FIB_DUMMY && (int)type == CNDP_FIB_LOOKUP_GPU) {
        fib->lookup_type = CNDP_FIB_LOOKUP_GPU;
        return 0;
    }
    if (!fib || fib->type != CNE_FIB_DIR24_8)
        return -EINVAL;
    switch (type) {
    case CNE_FIB_LOOKUP_DEFAULT:
    case CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO:
    case CNE_FIB_LOOKUP_DIR24_8_SCALAR_INLINE:
    case CNE_FIB_LOOKUP_DIR24_8_SCALAR_UNI:
    case CNE_FIB_LOOKUP_GPU:
        fib->lookup_type = (int)type;
        return 0;
    default:
        return -EINVAL;
    }
}

int cndp_fib_image(struct cne_fib *fib, struct cndp_fib_image *out)
{
    if (!fib || !out)
        return -EINVAL;
    out->nh_sz = fib->t.nh_sz;
    out->tbl8_groups = fib->t.cap_groups + 1;
    out->tbl24 = fib->t.tbl24;
    out->tbl8 = fib->t.tbl8;
    out->def_nh = fib->def_nh;
    return 0;
}

int cndp_fib_sync(struct cne_fib *fib, void *stream)
{
    if (!fib)
        return -EINVAL;
    return cndp_tbl_dev_sync(&fib->t, stream);
}

int cndp_fib_lookup_dev(struct cne_fib *fib, const uint32_t *ips, uint64_t *next_hops, uint32_t n,
                        void *stream)
{
    if (!fib || (n && (!ips || !next_hops)))
        return -EINVAL;
    return cndp_tbl_lookup4_dev(&fib->t, ips, next_hops, n, stream);
}

static int tbl_sync_stats(struct cndp_tbl *t, uint64_t *bytes, uint64_t *cmds)
{
    pthread_mutex_lock(&t->dev_lock);
    if (bytes)
        *bytes = t->sync_bytes;
    if (cmds)
        *cmds = t->sync_cmds;
    pthread_mutex_unlock(&t->dev_lock);
    return 0;
}

int cndp_fib_sync_stats(struct cne_fib *fib, uint64_t *bytes, uint64_t *cmds)
{
    return fib ? tbl_sync_stats(&fib->t, bytes, cmds) : -EINVAL;
}

int cndp_fib6_sync_stats(struct cne_fib6 *fib, uint64_t *bytes, uint64_t *cmds)
{
    return fib ? tbl_sync_stats(&fib->t, bytes, cmds) : -EINVAL;
}

int cndp_fib_stats(struct cne_fib *fib, uint32_t *routes, uint32_t *tbl8_used, uint32_t *rsvd)
{
    if (!fib)
        return -EINVAL;
    if (routes)
        *routes = fib->rib.routes;
    if (tbl8_used)
        *tbl8_used = fib->t.cur_tbl8s;
    if (rsvd)
        *rsvd = fib->rsvd_tbl8s;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* IPv6 API (cne_fib6.h)                                                     */
/* ------------------------------------------------------------------------ */
struct cne_fib6 *cne_fib6_create(const char *name, struct cne_fib_conf *conf)
{
    /* cne_fib6.c:119-160 + trie.c:581-619 argument checks */
    if (!name || !conf || conf->max_routes < 0 || conf->type > CNE_FIB_TRIE)
        return NULL;
    if ((int64_t)conf->max_routes * 2 <= 0)
        return NULL;
    if (conf->type == CNE_FIB_DIR24_8)
        return NULL;
    uint32_t nh_sz = 3, ntbl8 = 0;
    if (conf->type == CNE_FIB_TRIE) {
        if ((int)conf->trie.nh_sz < CNE_FIB_TRIE_2B || conf->trie.nh_sz > CNE_FIB_TRIE_8B)
            return NULL;
        nh_sz = (uint32_t)conf->trie.nh_sz;
        if (conf->trie.num_tbl8 > max_nh(nh_sz) || conf->trie.num_tbl8 == 0 ||
            conf->default_nh > max_nh(nh_sz))
            return NULL;
        ntbl8 = conf->trie.num_tbl8;
    }
    struct cne_fib6 *f = calloc(1, sizeof(*f));
    if (!f)
        return NULL;
    snprintf(f->name, sizeof(f->name), "%s", name);
    f->type = conf->type;
    f->def_nh = conf->default_nh;
    if (cndp_rib_init(&f->rib, (uint32_t)conf->max_routes * 2u, 128) ||
        tbl_init(&f->t, nh_sz, 1, ntbl8, conf->default_nh)) {
        cndp_rib_fini(&f->rib);
        free(f);
        return NULL;
    }
    return f;
}

void cne_fib6_free(struct cne_fib6 *fib)
{
    if (!fib)
        return;
    tbl_fini(&fib->t);
    cndp_rib_fini(&fib->rib);
    free(fib);
}

static inline uint32_t floor8(uint32_t d) { return d & ~7u; }
static inline uint32_t ceil8(uint32_t d) { return (d + 7u) & ~7u; }

static int fib6_modify(struct cne_fib6 *f, const uint8_t ip[16], uint8_t depth, uint64_t nh, int op)
{
    if (!ip || depth > CNE_FIB6_MAXDEPTH)
        return -EINVAL;
    cndp_key128 raw = cndp_key_from_v6(ip);
    cndp_key128 k = cndp_key_mask(raw, depth);

    if (f->type == CNE_FIB_DUMMY) {
        /* cne_fib6.c:50-70 */
        struct cndp_rnode *n = cndp_rib_lookup_exact(&f->rib, k, depth);
        if (op == CNE_FIB_ADD) {
            if (!n) {
                n = cndp_rib_insert(&f->rib, k, depth);
                if (!n)
                    return -1;
                n->nh = ~nh;
            }
            if (n->nh != nh) {
                int r = paint(&f->t, &f->rib, 128, k, depth, nh & max_nh(3));
                if (r)
                    return r;
            }
            n->nh = nh;
            return 0;
        }
        if (!n)
            return -ENOENT;
        struct cndp_rnode *par = cndp_rib_parent(n);
        int r = paint(&f->t, &f->rib, 128, k, depth, (par ? par->nh : f->def_nh) & max_nh(3));
        if (r)
            return r;
        cndp_rib_remove(&f->rib, k, depth);
        return 0;
    }

    /* trie.c:518-579.  modify_dp() rejects an oversize next hop only after
     * the RIB insert (trie.c:443-444), so the check sits at the same points */
    int nh_bad = nh > max_nh(f->t.nh_sz);
    uint32_t depth_diff = 0;
    if (depth > 24) {
        if (!cndp_rib_has_more_specific(&f->rib, k, floor8(depth))) {
            uint32_t parent_depth = 24;
            struct cndp_rnode *l = cndp_rib_lookup(&f->rib, raw);
            if (l)
                parent_depth = l->depth > 24 ? l->depth : 24;
            depth_diff = (uint8_t)(ceil8(depth) - ceil8(parent_depth)) >> 3;
        }
    }
    struct cndp_rnode *n = cndp_rib_lookup_exact(&f->rib, k, depth);
    int r = 0;
    if (op == CNE_FIB_ADD) {
        if (n) {
            if (n->nh == nh || nh_bad)
                return 0; /* modify_dp's -EINVAL is dropped here (trie.c:540-545) */
            r = paint(&f->t, &f->rib, 128, k, depth, nh);
            if (r == 0)
                n->nh = nh;
            return 0;
        }
        if (depth > 24 && f->rsvd_tbl8s >= f->t.num_tbl8 - depth_diff)
            return -ENOSPC;
        n = cndp_rib_insert(&f->rib, k, depth);
        if (!n)
            return -1;
        n->nh = nh;
        struct cndp_rnode *par = cndp_rib_parent(n);
        if (par && par->nh == nh)
            return 0;
        r = nh_bad ? -EINVAL : paint(&f->t, &f->rib, 128, k, depth, nh);
        if (r) {
            cndp_rib_remove(&f->rib, k, depth);
            return r;
        }
        f->rsvd_tbl8s += depth_diff;
        return 0;
    }
    if (op == CNE_FIB_DEL) {
        if (!n)
            return -ENOENT;
        struct cndp_rnode *par = cndp_rib_parent(n);
        if (par) {
            if (par->nh != n->nh)
                r = paint(&f->t, &f->rib, 128, k, depth, par->nh);
        } else {
            r = paint(&f->t, &f->rib, 128, k, depth, f->def_nh);
        }
        if (r)
            return r;
        cndp_rib_remove(&f->rib, k, depth);
        f->rsvd_tbl8s -= depth_diff;
        return 0;
    }
    return -EINVAL;
}

int cne_fib6_add(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth,
                 uint64_t next_hop)
{
    if (!fib || !ip || depth > CNE_FIB6_MAXDEPTH)
        return -EINVAL;
    pthread_mutex_lock(&fib->t.dev_lock); /* see cne_fib_add */
    const int r = fib6_modify(fib, ip, depth, next_hop, CNE_FIB_ADD);
    pthread_mutex_unlock(&fib->t.dev_lock);
    return r;
}

int cne_fib6_delete(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth)
{
    if (!fib || !ip || depth > CNE_FIB6_MAXDEPTH)
        return -EINVAL;
    pthread_mutex_lock(&fib->t.dev_lock);
    const int r = fib6_modify(fib, ip, depth, 0, CNE_FIB_DEL);
    pthread_mutex_unlock(&fib->t.dev_lock);
    return r;
}

int cne_fib6_lookup_bulk(struct cne_fib6 *fib, uint8_t ips[][IPV6_ADDR_LEN], uint64_t *next_hops,
                         int n)
{
    if (!fib || !ips || !next_hops || n < 0)
        return -EINVAL;
    if (n == 0)
        return 0;
    if (fib->lookup_type == CNDP_FIB_LOOKUP_GPU)
        return cndp_tbl_lookup6_host(&fib->t, &ips[0][0], next_hops, (uint32_t)n);
    if (fib->type == CNE_FIB_DUMMY) { /* cne_fib6.c:34-48, see cne_fib_lookup_bulk */
        pthread_mutex_lock(&fib->t.dev_lock);
        host_lookup6(&fib->t, &ips[0][0], next_hops, (uint32_t)n);
        pthread_mutex_unlock(&fib->t.dev_lock);
        return 0;
    }
    host_lookup6(&fib->t, &ips[0][0], next_hops, (uint32_t)n);
    return 0;
}

void *cne_fib6_get_dp(struct cne_fib6 *fib) { return fib ? &fib->t : NULL; }

/* cne_fib6.c:202-205: the build's RIB (path-compressed trie over 128-bit keys) */
struct cne_rib6 *cne_fib6_get_rib(struct cne_fib6 *fib)
{
    return fib ? (struct cne_rib6 *)&fib->rib : NULL;
}

/* cne_fib6.c:208-223, as cne_fib_select_lookup (TRIE_VECTOR_AVX512: -EINVAL
 * at the default SIMD width, trie.c:47-53) */
int cne_fib6_select_lookup(struct cne_fib6 *fib, enum cne_fib_lookup_type type)
{
    if (fib && fib->type == CNE_FIB_DUMMY && (int)type == CNDP_FIB_LOOKUP_GPU) {
        fib->lookup_type = CNDP_FIB_LOOKUP_GPU;
        return 0;
    }
    if (!fib || fib->type != CNE_FIB_TRIE)
        return -EINVAL;
    switch (type) {
    case CNE_FIB_LOOKUP_DEFAULT:
    case CNE_FIB_LOOKUP_TRIE_SCALAR:
    case CNE_FIB_LOOKUP_GPU:
        fib->lookup_type = (int)type;
        return 0;
    default:
        return -EINVAL;
    }
}

int cndp_fib6_image(struct cne_fib6 *fib, struct cndp_fib_image *out)
{
    if (!fib || !out)
        return -EINVAL;
    out->nh_sz = fib->t.nh_sz;
    out->tbl8_groups = fib->t.cap_groups + 1;
    out->tbl24 = fib->t.tbl24;
    out->tbl8 = fib->t.tbl8;
    out->def_nh = fib->def_nh;
    return 0;
}

int cndp_fib6_sync(struct cne_fib6 *fib, void *stream)
{
    if (!fib)
        return -EINVAL;
    return cndp_tbl_dev_sync(&fib->t, stream);
}

int cndp_fib6_lookup_dev(struct cne_fib6 *fib, const uint8_t *ips16, uint64_t *next_hops,
                         uint32_t n, void *stream)
{
    if (!fib || (n && (!ips16 || !next_hops)))
        return -EINVAL;
    return cndp_tbl_lookup6_dev(&fib->t, ips16, next_hops, n, stream);
}

int cndp_fib6_stats(struct cne_fib6 *fib, uint32_t *routes, uint32_t *tbl8_used, uint32_t *rsvd)
{
    if (!fib)
        return -EINVAL;
    if (routes)
        *routes = fib->rib.routes;
    if (tbl8_used)
        *tbl8_used = fib->t.cur_tbl8s;
    if (rsvd)
        *rsvd = fib->rsvd_tbl8s;
    return 0;
}
