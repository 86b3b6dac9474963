#define _GNU_SOURCE
/*
 * oracle.c -- CPU restatement of CNDP's parse / Toeplitz / LPM hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  The product never calls this.
 * Each function names the reference file:line it restates; byte-order
 * conventions follow a little-endian host exactly as the reference does on
 * x86 (the GPU is little-endian too, so quirks that depend on it carry over).
 */
#include "oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* byte helpers                                                              */
/* ------------------------------------------------------------------------ */
static inline uint16_t rd_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t rd_be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
/* the 16-bit value a little-endian load of p[0..1] yields ("network order
 * u16 as seen by the reference"), used where the reference compares raw
 * be16 fields against htobe16() constants */
static inline uint16_t rd_raw16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint16_t sw16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

/* Bounded packet view: bytes at or past `avail` (the end of the slab) read
 * as 0.  The reference reads whatever memory follows (undefined); the build
 * defines it as zero so the GPU path can never fault. */
struct pv {
    const uint8_t *p;
    uint64_t avail;
};
static inline uint8_t v8(struct pv v, uint64_t o) { return o < v.avail ? v.p[o] : 0; }
static inline uint16_t vbe16(struct pv v, uint64_t o) { return (uint16_t)((v8(v, o) << 8) | v8(v, o + 1)); }
static inline uint16_t vraw16(struct pv v, uint64_t o) { return (uint16_t)(v8(v, o) | (v8(v, o + 1) << 8)); }
static inline uint32_t vbe32(struct pv v, uint64_t o)
{
    return ((uint32_t)v8(v, o) << 24) | ((uint32_t)v8(v, o + 1) << 16) | ((uint32_t)v8(v, o + 2) << 8) |
           v8(v, o + 3);
}

uint64_t orc_splitmix64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* ------------------------------------------------------------------------ */
/* Toeplitz: lib/core/hash/cne_thash.h:150-163 (cne_softrss) and :178-191   */
/* (cne_softrss_be).  For every set bit i of input dword j the 32-bit key    */
/* window starting at stream bit 32*j + (31-i) is XORed in.                 */
/* ------------------------------------------------------------------------ */
static inline uint32_t key_dw_be(const uint8_t *key, uint32_t j)
{
    /* htobe32(((const uint32_t *)rss_key)[j]) on a LE host == big-endian read */
    return rd_be32(key + 4 * j);
}

uint32_t orc_softrss(const uint32_t *tuple, uint32_t len_dw, const uint8_t *key)
{
    /* visits the set bits lowest first, like the map &= map - 1 loop */
    uint32_t h = 0;
    for (uint32_t j = 0; j < len_dw; j++) {
        uint32_t hi = key_dw_be(key, j), lo = key_dw_be(key, j + 1);
        for (uint32_t map = tuple[j]; map; map &= map - 1) {
            uint32_t i = (uint32_t)__builtin_ctz(map);
            h ^= (hi << (31 - i)) | (uint32_t)((uint64_t)lo >> (i + 1));
        }
    }
    return h;
}

uint32_t orc_softrss_be(const uint32_t *tuple, uint32_t len_dw, const uint8_t *key_be)
{
    /* key already converted (cne_convert_rss_key): dwords used as stored */
    const uint32_t *k = (const uint32_t *)(const void *)key_be;
    uint32_t h = 0;
    for (uint32_t j = 0; j < len_dw; j++) {
        uint32_t hi, lo;
        memcpy(&hi, k + j, 4);
        memcpy(&lo, k + j + 1, 4);
        for (uint32_t map = tuple[j]; map; map &= map - 1) {
            uint32_t i = (uint32_t)__builtin_ctz(map);
            h ^= (hi << (31 - i)) | (uint32_t)((uint64_t)lo >> (i + 1));
        }
    }
    return h;
}

void orc_convert_rss_key(const uint8_t *orig, uint8_t *targ, int len)
{
    /* cne_thash.h:113-120: targ[i] = be32toh(orig[i]) per dword */
    for (int i = 0; i < (len >> 2); i++) {
        uint32_t v = rd_be32(orig + 4 * i);
        memcpy(targ + 4 * i, &v, 4);
    }
}

/* ------------------------------------------------------------------------ */
/* IPv4 header checksum: lib/include/net/cne_ip.h:131-214.                   */
/* Sum of native (LE) u16 words over IHL*4 bytes, folded twice, inverted.   */
/* ------------------------------------------------------------------------ */
uint16_t orc_ipv4_cksum(const uint8_t *ip)
{
    uint32_t len = (uint32_t)(ip[0] & 0x0f) * 4u;
    uint32_t sum = 0;
    uint32_t k = 0;
    for (; k + 1 < len; k += 2)
        sum += rd_raw16(ip + k);
    if (len & 1u) /* unreachable for IHL*4 but kept as in :160-165 */
        sum += ip[k];
    sum = (sum >> 16) + (sum & 0xffff);
    sum = (sum >> 16) + (sum & 0xffff);
    return (uint16_t)~(uint16_t)sum;
}

/* ------------------------------------------------------------------------ */
/* Brute-force LPM (the get_next_hop idea of lpm6_data_test.h:1100-1123):    */
/* longest covering prefix wins; for an identical (prefix, depth) the later  */
/* entry wins (cne_fib_add on an existing route replaces its next hop).      */
/* ------------------------------------------------------------------------ */
static inline uint32_t mask4(uint8_t d) { return d == 0 ? 0u : (uint32_t)(0xFFFFFFFFull << (32 - d)); }

void orc_lpm4_bruteforce(const struct orc_route4 *r, uint32_t nr, uint64_t def_nh,
                         const uint32_t *ips, uint32_t n, uint64_t *out)
{
    for (uint32_t i = 0; i < n; i++) {
        int best = -1;
        uint64_t nh = def_nh;
        for (uint32_t k = 0; k < nr; k++) {
            uint32_t m = mask4(r[k].depth);
            if (((ips[i] ^ r[k].ip) & m) != 0)
                continue;
            if ((int)r[k].depth >= best) {
                best = r[k].depth;
                nh = r[k].nh;
            }
        }
        out[i] = nh;
    }
}

static int covers6(const uint8_t *pfx, uint8_t depth, const uint8_t *ip)
{
    for (int b = 0; b < 16 && depth > 0; b++) {
        uint8_t m = depth >= 8 ? 0xff : (uint8_t)(0xff << (8 - depth));
        if ((pfx[b] ^ ip[b]) & m)
            return 0;
        depth = depth >= 8 ? (uint8_t)(depth - 8) : 0;
    }
    return 1;
}

void orc_lpm6_bruteforce(const struct orc_route6 *r, uint32_t nr, uint64_t def_nh,
                         const uint8_t (*ips)[16], uint32_t n, uint64_t *out)
{
    for (uint32_t i = 0; i < n; i++) {
        int best = -1;
        uint64_t nh = def_nh;
        for (uint32_t k = 0; k < nr; k++) {
            if (!covers6(r[k].ip, r[k].depth, ips[i]))
                continue;
            if ((int)r[k].depth >= best) {
                best = r[k].depth;
                nh = r[k].nh;
            }
        }
        out[i] = nh;
    }
}

/* ------------------------------------------------------------------------ */
/* Table painters.  Routes are painted in ascending depth (stable), so a    */
/* longer prefix always overwrites a shorter one and, at equal (prefix,      */
/* depth), the later route wins.  Layout and entry encoding follow           */
/* dir24_8.h:27-46,118-148 / trie.h:26-40,119-138: tbl24 entry = nh<<1, or  */
/* (group<<1)|1 when extended; group g covers tbl8[g*256 .. g*256+255].      */
/* ------------------------------------------------------------------------ */
static int cmp_depth4(const void *a, const void *b)
{
    const uint32_t *x = a, *y = b; /* [depth, index] pairs */
    if (x[0] != y[0])
        return x[0] < y[0] ? -1 : 1;
    return x[1] < y[1] ? -1 : (x[1] > y[1]);
}

int orc_dir24_8_build(const struct orc_route4 *r, uint32_t nr, uint64_t def_nh,
                      uint32_t num_tbl8, uint32_t *tbl24, uint32_t *tbl8)
{
    uint32_t *ord = malloc(sizeof(uint32_t) * 2 * (nr ? nr : 1));
    if (!ord)
        return -ENOMEM;
    for (uint32_t k = 0; k < nr; k++) {
        ord[2 * k] = r[k].depth;
        ord[2 * k + 1] = k;
    }
    qsort(ord, nr, 8, cmp_depth4);

    for (uint32_t i = 0; i < (1u << 24); i++)
        tbl24[i] = (uint32_t)(def_nh << 1);
    memset(tbl8, 0, (size_t)(num_tbl8 + 1) * 256 * 4);
    uint32_t groups = 0;

    for (uint32_t q = 0; q < nr; q++) {
        const struct orc_route4 *rt = &r[ord[2 * q + 1]];
        uint32_t ip = rt->ip & mask4(rt->depth);
        uint32_t v = (uint32_t)(rt->nh << 1);
        if (rt->depth <= 24) {
            uint32_t first = ip >> 8, cnt = 1u << (24 - rt->depth);
            for (uint32_t i = 0; i < cnt; i++)
                tbl24[first + i] = v;
        } else {
            uint32_t idx = ip >> 8;
            if (!(tbl24[idx] & 1u)) {
                if (groups >= num_tbl8) {
                    free(ord);
                    return -ENOSPC;
                }
                uint32_t g = groups++;
                for (uint32_t e = 0; e < 256; e++)
                    tbl8[g * 256 + e] = tbl24[idx] | 1u;
                tbl24[idx] = (g << 1) | 1u;
            }
            uint32_t g = tbl24[idx] >> 1;
            uint32_t first = ip & 0xff, cnt = 1u << (32 - rt->depth);
            for (uint32_t e = 0; e < cnt; e++)
                tbl8[g * 256 + first + e] = v | 1u;
        }
    }
    free(ord);
    return (int)groups;
}

/* dir24_8.h:131-135 (LOOKUP_FUNC 4b body) */
void orc_dir24_8_lookup(const uint32_t *tbl24, const uint32_t *tbl8, const uint32_t *ips,
                        uint32_t n, uint64_t *nh)
{
    for (uint32_t i = 0; i < n; i++) {
        uint32_t e = tbl24[ips[i] >> 8];
        if (e & 1u)
            e = tbl8[(uint8_t)ips[i] + (e >> 1) * 256u];
        nh[i] = e >> 1;
    }
}

/* dir24_8.h:118-148 LOOKUP_FUNC(4b, uint32_t, 15, 2), the lookup the
 * reference's cne_fib_lookup_bulk runs by default: prefetch the
 * tbl24 entries of the first min(15, n) keys, then look up key i while
 * prefetching key i + 15.  Same results as orc_dir24_8_lookup. */
void orc_dir24_8_lookup_bulk_pf(const uint32_t *tbl24, const uint32_t *tbl8, const uint32_t *ips, uint32_t n,
                                uint64_t *nh)
{
    const uint32_t pf = n < 15u ? n : 15u;
    uint32_t i;
    for (i = 0; i < pf; i++)
        __builtin_prefetch(&tbl24[ips[i] >> 8], 0, 3);
    for (i = 0; i < n - pf; i++) {
        __builtin_prefetch(&tbl24[ips[i + pf] >> 8], 0, 3);
        uint32_t e = tbl24[ips[i] >> 8];
        if (e & 1u)
            e = tbl8[(uint8_t)ips[i] + (e >> 1) * 256u];
        nh[i] = e >> 1;
    }
    for (; i < n; i++) {
        uint32_t e = tbl24[ips[i] >> 8];
        if (e & 1u)
            e = tbl8[(uint8_t)ips[i] + (e >> 1) * 256u];
        nh[i] = e >> 1;
    }
}

int orc_trie_build(const struct orc_route6 *r, uint32_t nr, uint64_t def_nh, uint32_t num_tbl8,
                   uint32_t *tbl24, uint32_t *tbl8)
{
    uint32_t *ord = malloc(sizeof(uint32_t) * 2 * (nr ? nr : 1));
    if (!ord)
        return -ENOMEM;
    for (uint32_t k = 0; k < nr; k++) {
        ord[2 * k] = r[k].depth;
        ord[2 * k + 1] = k;
    }
    qsort(ord, nr, 8, cmp_depth4);
    for (uint32_t i = 0; i < (1u << 24); i++)
        tbl24[i] = (uint32_t)(def_nh << 1);
    memset(tbl8, 0, (size_t)(num_tbl8 + 1) * 256 * 4);
    uint32_t groups = 0;

    for (uint32_t q = 0; q < nr; q++) {
        const struct orc_route6 *rt = &r[ord[2 * q + 1]];
        uint8_t ip[16];
        uint32_t d = rt->depth;
        for (int b = 0; b < 16; b++) {
            int bits = (int)d - 8 * b;
            uint8_t m = bits >= 8 ? 0xff : bits <= 0 ? 0 : (uint8_t)(0xff << (8 - bits));
            ip[b] = rt->ip[b] & m;
        }
        uint32_t v = (uint32_t)(rt->nh << 1);
        uint32_t idx24 = ((uint32_t)ip[0] << 16) | ((uint32_t)ip[1] << 8) | ip[2];
        if (d <= 24) {
            uint32_t cnt = 1u << (24 - d);
            for (uint32_t i = 0; i < cnt; i++)
                tbl24[idx24 + i] = v;
            continue;
        }
        uint32_t *ent = &tbl24[idx24];
        for (uint32_t k = 3; k < 16; k++) {
            if (!(*ent & 1u)) {
                if (groups >= num_tbl8) {
                    free(ord);
                    return -ENOSPC;
                }
                uint32_t g = groups++;
                for (uint32_t e = 0; e < 256; e++)
                    tbl8[g * 256 + e] = *ent;
                *ent = (g << 1) | 1u;
            }
            uint32_t g = *ent >> 1;
            int rem = (int)d - 8 * (int)k;
            if (rem <= 8) {
                uint32_t cnt = 1u << (8 - rem);
                for (uint32_t e = 0; e < cnt; e++)
                    tbl8[g * 256 + ip[k] + e] = v;
                break;
            }
            ent = &tbl8[g * 256 + ip[k]];
        }
    }
    free(ord);
    return (int)groups;
}

/* trie.h:119-138 (LOOKUP_FUNC 4b body) */
void orc_trie_lookup(const uint32_t *tbl24, const uint32_t *tbl8, const uint8_t (*ips)[16],
                     uint32_t n, uint64_t *nh)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *ip = ips[i];
        uint32_t e = tbl24[((uint32_t)ip[0] << 16) | ((uint32_t)ip[1] << 8) | ip[2]];
        uint32_t j = 3;
        while (e & 1u)
            e = tbl8[ip[j++] + (e >> 1) * 256u];
        nh[i] = e >> 1;
    }
}

/* ------------------------------------------------------------------------ */
/* cne_get_ptype: lib/core/pktmbuf/pktmbuf_ptype.c:472-744 (+ helpers       */
/* :280-468).  `proto` holds the 16-bit value a LE load of the wire field    */
/* gives, exactly like the reference, so its htobe16() comparisons (and the  */
/* quirk that IP protocol 8 / 129 alias htobe16(IPv4) / htobe16(VLAN) in the */
/* inner-header section) are reproduced.                                     */
/* ------------------------------------------------------------------------ */
#define PT_L2_ETHER 0x1u
#define PT_L2_ARP 0x3u
#define PT_L2_VLAN 0x6u
#define PT_L2_QINQ 0x7u
#define PT_L3_IPV4 0x10u
#define PT_L3_IPV4_EXT 0x30u
#define PT_L3_IPV6 0x40u
#define PT_L3_IPV6_EXT 0xc0u
#define PT_L4_TCP 0x100u
#define PT_L4_UDP 0x200u
#define PT_L4_FRAG 0x300u
#define PT_L4_SCTP 0x400u
#define PT_TUN_IP 0x1000u
#define PT_TUN_GRE 0x2000u
#define PT_TUN_NVGRE 0x4000u
#define PT_TUN_GTPC 0x7000u
#define PT_TUN_GTPU 0x8000u
#define PT_IN_L2_ETHER 0x10000u
#define PT_IN_L2_VLAN 0x20000u
#define PT_IN_L2_QINQ 0x30000u
#define PT_IN_L3_IPV4 0x100000u
#define PT_IN_L3_IPV4_EXT 0x200000u
#define PT_IN_L3_IPV6 0x300000u
#define PT_IN_L3_IPV6_EXT 0x500000u
#define PT_IN_L4_TCP 0x1000000u
#define PT_IN_L4_UDP 0x2000000u
#define PT_IN_L4_FRAG 0x3000000u
#define PT_IN_L4_SCTP 0x4000000u

#define BE(x) ((uint16_t)sw16((uint16_t)(x))) /* htobe16 on a LE host */
#define ET_IPV4 0x0800
#define ET_IPV6 0x86DD
#define ET_ARP 0x0806
#define ET_VLAN 0x8100
#define ET_QINQ 0x88A8
#define ET_MPLS 0x8847
#define ET_MPLSM 0x8848
#define ET_TEB 0x6558

static uint32_t pt_l3_ip(uint8_t vihl, int inner) /* pktmbuf_ptype.c:296-310 */
{
    if (vihl == 0x45)
        return inner ? PT_IN_L3_IPV4 : PT_L3_IPV4;
    if (vihl >= 0x46 && vihl <= 0x4f)
        return inner ? PT_IN_L3_IPV4_EXT : PT_L3_IPV4_EXT;
    return 0;
}
static int is_v6_ext(uint8_t p) /* :281-293 map entries */
{
    return p == 0 || p == 43 || p == 44 || p == 50 || p == 51 || p == 60;
}
static uint32_t pt_l4(uint8_t p, int inner) /* :312-323 */
{
    if (p == 17)
        return inner ? PT_IN_L4_UDP : PT_L4_UDP;
    if (p == 6)
        return inner ? PT_IN_L4_TCP : PT_L4_TCP;
    if (p == 132)
        return inner ? PT_IN_L4_SCTP : PT_L4_SCTP;
    return 0;
}

/* :426-468; returns -1 on "more than 5 headers", else next proto */
static int skip_v6_ext(uint16_t proto, struct pv v, uint32_t *off, int *frag)
{
    *frag = 0;
    for (int i = 0; i < 5; i++) {
        switch (proto) {
        case 0:
        case 43:
        case 60:
            proto = v8(v, *off);
            *off += ((uint32_t)v8(v, *off + 1) + 1) * 8;
            break;
        case 44:
            proto = v8(v, *off);
            *off += 8;
            *frag = 1;
            return proto;
        case 59:
            return 0;
        default:
            return proto;
        }
    }
    return -1;
}

/* :372-411 */
static uint32_t pt_tunnel(uint16_t *proto, struct pv v, uint32_t *off)
{
    switch (*proto) {
    case 47: {
        static const uint8_t opt_len[16] = {[0x0] = 4,  [0x1] = 8,  [0x2] = 8,  [0x8] = 8,
                                            [0x3] = 12, [0x9] = 12, [0xa] = 12, [0xb] = 16};
        uint16_t flags = (uint16_t)(vbe16(v, *off) >> 12);
        if (opt_len[flags] == 0)
            return 0;
        uint16_t gproto = vraw16(v, *off + 2);
        *off += opt_len[flags];
        *proto = gproto;
        return gproto == BE(ET_TEB) ? PT_TUN_NVGRE : PT_TUN_GRE;
    }
    case 4:
        *proto = BE(ET_IPV4);
        return PT_TUN_IP;
    case 41:
        *proto = BE(ET_IPV6);
        return PT_TUN_IP;
    default:
        return 0;
    }
}

uint32_t orc_get_ptype(const uint8_t *pkt, uint64_t avail, struct orc_hdr_lens *hl, uint32_t layers)
{
    struct orc_hdr_lens local;
    struct pv v = {pkt, avail};
    uint32_t pt = PT_L2_ETHER;
    uint32_t off;
    uint16_t proto;
    int ret;

    if (!hl)
        hl = &local;
    proto = vraw16(v, 12);
    off = 14;
    hl->l2_len = (uint8_t)off;
    if ((layers & 0xfu) == 0)
        return 0;
    if (proto == BE(ET_ARP))
        return PT_L2_ARP;
    if (proto == BE(ET_IPV4))
        goto l3;
    if (proto == BE(ET_VLAN)) {
        pt = PT_L2_VLAN;
        proto = vraw16(v, off + 2);
        off += 4;
        hl->l2_len = (uint8_t)(hl->l2_len + 4);
    } else if (proto == BE(ET_QINQ)) {
        pt = PT_L2_QINQ;
        proto = vraw16(v, off + 4 + 2);
        off += 8;
        hl->l2_len = (uint8_t)(hl->l2_len + 8);
    } else if (proto == BE(ET_MPLS) || proto == BE(ET_MPLSM)) {
        /* :541-556: the 5-label loop never breaks, so i == 5 always and the
         * function returns L2_ETHER without the MPLS bit or length */
        return pt;
    }
l3:
    if ((layers & 0xf0u) == 0)
        return pt;
    if (proto == BE(ET_IPV4)) {
        uint32_t ip = off;
        pt |= pt_l3_ip(v8(v, ip), 0);
        hl->l3_len = (uint16_t)((v8(v, ip) & 0xf) * 4);
        off += hl->l3_len;
        if ((layers & 0xf00u) == 0)
            return pt;
        if (vraw16(v, ip + 6) & BE(0x1fff | 0x2000)) {
            pt |= PT_L4_FRAG;
            hl->l4_len = 0;
            return pt;
        }
        proto = v8(v, ip + 9);
        pt |= pt_l4((uint8_t)proto, 0);
    } else if (proto == BE(ET_IPV6)) {
        int frag = 0;
        proto = v8(v, off + 6);
        hl->l3_len = 40;
        off += 40;
        pt |= PT_L3_IPV6 + (is_v6_ext((uint8_t)proto) ? (PT_L3_IPV6_EXT - PT_L3_IPV6) : 0);
        if ((pt & 0xf0u) == PT_L3_IPV6_EXT) {
            ret = skip_v6_ext(proto, v, &off, &frag);
            if (ret < 0)
                return pt;
            proto = (uint16_t)ret;
            hl->l3_len = (uint16_t)(off - hl->l2_len);
        }
        if (proto == 0)
            return pt;
        if ((layers & 0xf00u) == 0)
            return pt;
        if (frag) {
            pt |= PT_L4_FRAG;
            hl->l4_len = 0;
            return pt;
        }
        pt |= pt_l4((uint8_t)proto, 0);
    }

    if ((pt & 0xf00u) == PT_L4_UDP) {
        uint32_t udp = (uint32_t)hl->l2_len + hl->l3_len;
        hl->l4_len = 8;
        uint16_t dport = vraw16(v, udp + 2);
        if (dport == BE(2152))
            pt |= PT_TUN_GTPU;
        else if (dport == BE(2123))
            pt |= PT_TUN_GTPC;
        return pt;
    } else if ((pt & 0xf00u) == PT_L4_TCP) {
        uint32_t th = (uint32_t)hl->l2_len + hl->l3_len;
        hl->l4_len = (uint8_t)((v8(v, th + 12) & 0xf0) >> 2);
        return pt;
    } else if ((pt & 0xf00u) == PT_L4_SCTP) {
        hl->l4_len = 12;
        return pt;
    } else {
        uint32_t prev = off;
        hl->l4_len = 0;
        if ((layers & 0xf000u) == 0)
            return pt;
        pt |= pt_tunnel(&proto, v, &off);
        hl->tunnel_len = (uint16_t)(off - prev);
    }

    if ((layers & 0xf0000u) == 0)
        return pt;
    hl->inner_l2_len = 0;
    if (proto == BE(ET_TEB)) {
        pt |= PT_IN_L2_ETHER;
        proto = vraw16(v, off + 12);
        off += 14;
        hl->inner_l2_len = 14;
    }
    if (proto == BE(ET_VLAN)) {
        pt &= ~0xf0000u;
        pt |= PT_IN_L2_VLAN;
        proto = vraw16(v, off + 2);
        off += 4;
        hl->inner_l2_len = (uint8_t)(hl->inner_l2_len + 4);
    } else if (proto == BE(ET_QINQ)) {
        pt &= ~0xf0000u;
        pt |= PT_IN_L2_QINQ;
        proto = vraw16(v, off + 4 + 2);
        off += 8;
        hl->inner_l2_len = (uint8_t)(hl->inner_l2_len + 8);
    }
    if ((layers & 0xf00000u) == 0)
        return pt;
    if (proto == BE(ET_IPV4)) {
        uint32_t ip = off;
        pt |= pt_l3_ip(v8(v, ip), 1);
        hl->inner_l3_len = (uint16_t)((v8(v, ip) & 0xf) * 4);
        off += hl->inner_l3_len;
        if ((layers & 0xf000000u) == 0)
            return pt;
        if (vraw16(v, ip + 6) & BE(0x1fff | 0x2000)) {
            pt |= PT_IN_L4_FRAG;
            hl->inner_l4_len = 0;
            return pt;
        }
        proto = v8(v, ip + 9);
        pt |= pt_l4((uint8_t)proto, 1);
    } else if (proto == BE(ET_IPV6)) {
        int frag = 0;
        proto = v8(v, off + 6);
        hl->inner_l3_len = 40;
        off += 40;
        pt |= PT_IN_L3_IPV6 + (is_v6_ext((uint8_t)proto) ? (PT_IN_L3_IPV6_EXT - PT_IN_L3_IPV6) : 0);
        if ((pt & 0xf00000u) == PT_IN_L3_IPV6_EXT) {
            uint32_t prev = off;
            ret = skip_v6_ext(proto, v, &off, &frag);
            if (ret < 0)
                return pt;
            proto = (uint16_t)ret;
            hl->inner_l3_len = (uint16_t)(hl->inner_l3_len + off - prev);
        }
        if (proto == 0)
            return pt;
        if ((layers & 0xf000000u) == 0)
            return pt;
        if (frag) {
            pt |= PT_IN_L4_FRAG;
            hl->inner_l4_len = 0;
            return pt;
        }
        pt |= pt_l4((uint8_t)proto, 1);
    }
    if ((pt & 0xf000000u) == PT_IN_L4_UDP) {
        hl->inner_l4_len = 8;
    } else if ((pt & 0xf000000u) == PT_IN_L4_TCP) {
        hl->inner_l4_len = (uint8_t)((v8(v, off + 12) & 0xf0) >> 2);
    } else if ((pt & 0xf000000u) == PT_IN_L4_SCTP) {
        hl->inner_l4_len = 12;
    } else {
        hl->inner_l4_len = 0;
    }
    return pt;
}

/* ------------------------------------------------------------------------ */
/* Hot-path node semantics + build-defined flow hash.        */
/* ------------------------------------------------------------------------ */
#define MODE_L3FWD 0u
#define MODE_CNET 1u
#define MODE_HASH 2u
#define NH_INVALID 0xFFFFFFFFu

/* cnet ptype edges (lib/cnet/ptype/ptype_priv.h:19-29, CNET_ENABLE_IP6=1) */
#define PTN_DROP 0u
#define PTN_FRAME_PUNT 2u
#define PTN_IP4 3u
#define PTN_IP6 4u
#define PTN_GTPU 5u

/* lib/cnet/ptype/ptype.c:32-46 -- the table is indexed by ptype & 0xffff */
static uint8_t cnet_ptype_edge(uint32_t pt)
{
    switch (pt & 0xffffu) {
    case 0x0003u:
        return PTN_FRAME_PUNT;
    case 0x0211u: case 0x0111u: case 0x0231u: case 0x0291u:
        return PTN_IP4;
    case 0x8211u:
        return PTN_GTPU;
    case 0x0241u: case 0x0141u: case 0x02c1u: case 0x02e1u:
        return PTN_IP6;
    case 0x8241u:
        return PTN_GTPU;
    default:
        return PTN_DROP;
    }
}

/* exported for tests/test_oracle_golden.py (the p_nxt fixture check) */
uint32_t orc_cnet_ptype_edge(uint32_t pt) { return cnet_ptype_edge(pt); }

static inline uint32_t lookup4(const uint32_t *t24, const uint32_t *t8, uint32_t ip)
{
    uint32_t e = t24[ip >> 8];
    if (e & 1u)
        e = t8[(ip & 0xffu) + (e >> 1) * 256u];
    return e >> 1;
}
static inline uint32_t lookup6(const uint32_t *t24, const uint32_t *t8, const uint8_t *ip)
{
    uint32_t e = t24[((uint32_t)ip[0] << 16) | ((uint32_t)ip[1] << 8) | ip[2]];
    uint32_t j = 3;
    while (e & 1u)
        e = t8[ip[j++] + (e >> 1) * 256u];
    return e >> 1;
}

/* Build-defined 5-tuple: cne_ipv4_tuple / cne_ipv6_tuple (cne_thash.h:68-97)
 * filled as a NIC would: addresses host order, then dport | sport << 16.
 * L4 tuple only for TCP/UDP that is not a fragment.  ip / l4 are offsets. */
static uint32_t hash_v4(struct pv v, uint32_t ip, int l4ok, uint32_t l4, const uint8_t *key)
{
    uint32_t t[3];
    t[0] = vbe32(v, ip + 12);
    t[1] = vbe32(v, ip + 16);
    if (l4ok) {
        t[2] = (uint32_t)vbe16(v, l4 + 2) | ((uint32_t)vbe16(v, l4) << 16);
        return orc_softrss(t, 3, key);
    }
    return orc_softrss(t, 2, key);
}
static uint32_t hash_v6(struct pv v, uint32_t ip6, int l4ok, uint32_t l4, const uint8_t *key)
{
    uint32_t t[9];
    /* cne_thash_load_v6_addrs (:130-137): per-4-byte bswap into host order */
    for (int k = 0; k < 8; k++)
        t[k] = vbe32(v, ip6 + 8 + 4 * k);
    if (l4ok) {
        t[8] = (uint32_t)vbe16(v, l4 + 2) | ((uint32_t)vbe16(v, l4) << 16);
        return orc_softrss(t, 9, key);
    }
    return orc_softrss(t, 8, key);
}

/* ip4_input.c:121-140 / ip6_input.c:115-135 for a frame the ptype node
 * sends to edge pe (ip = its L3 offset); other edges: 0x80 | pe */
static void cnet_input(const struct orc_classify_args *a, struct pv v, uint32_t ip, uint8_t pe, uint32_t *nh,
                       uint8_t *edge)
{
    if (pe == PTN_IP4) {
        uint8_t hdr[60]; /* cksum over the bounded view */
        for (int k = 0; k < 60; k++)
            hdr[k] = v8(v, ip + (uint32_t)k);
        uint32_t tl = vbe16(v, ip + 2);
        uint32_t dip = 0;
        if (tl < a->buf_len && orc_ipv4_cksum(hdr) == 0)
            dip = vbe32(v, ip + 16);
        *nh = lookup4(a->tbl24, a->tbl8, dip);
        *edge = (uint8_t)(*nh >> 24);
    } else if (pe == PTN_IP6) {
        uint8_t dip[16];
        memset(dip, 0, 16);
        if ((uint32_t)vbe16(v, ip + 4) < a->buf_len)
            for (int k = 0; k < 16; k++)
                dip[k] = v8(v, ip + 24 + (uint32_t)k);
        *nh = lookup6(a->tbl24_6, a->tbl8_6, dip);
        *edge = (uint8_t)(*nh >> 24);
    } else {
        *nh = NH_INVALID;
        *edge = (uint8_t)(0x80u | pe);
    }
}

static uint32_t bin_for(const struct orc_classify_args *a, uint32_t nh, uint8_t edge, uint32_t q)
{
    const uint32_t nb = a->n_bins;
    if (a->mode == MODE_HASH)
        return q < nb ? q : nb + 1;
    if (a->mode == MODE_L3FWD) {
        if (edge == 0)
            return (nh & 0xffffu) < nb ? (nh & 0xffffu) : nb + 1;
        return (edge == 1 || edge == 0xFF) ? nb : nb + 1;
    }
    if (edge == 1)
        return (nh & 0xffffffu) < nb ? (nh & 0xffffffu) : nb + 1;
    return (edge == 0 || edge == (0x80u | PTN_DROP)) ? nb : nb + 1;
}

static void classify_one(const struct orc_classify_args *a, uint32_t i)
{
    uint64_t base = (a->offsets ? a->offsets[i] : (uint64_t)i * a->stride) + a->data_off;
    struct pv v = {a->slab + base, base < a->slab_len ? a->slab_len - base : 0};
    uint32_t nh = NH_INVALID, hash = 0, bin;
    uint8_t edge;
    uint32_t nb = a->n_bins;

    if (a->mode == MODE_L3FWD || a->mode == MODE_HASH) {
        uint16_t et = vbe16(v, 12);
        if (et == 0x0800) {
            uint32_t ihl = v8(v, 14) & 0xfu;
            uint8_t proto = v8(v, 14 + 9);
            int frag = (vbe16(v, 14 + 6) & 0x3fff) != 0;
            int l4ok = ihl >= 5 && (proto == 6 || proto == 17) && !frag;
            hash = hash_v4(v, 14, l4ok, 14 + ihl * 4, a->rss_key);
        } else if (et == 0x86DD) {
            uint8_t nx = v8(v, 14 + 6);
            int l4ok = nx == 6 || nx == 17;
            hash = hash_v6(v, 14, l4ok, 14 + 40, a->rss_key);
        }
        if (a->ptype) /* pktdev_rx.c:24-34 l3_ptype */
            a->ptype[i] = et == 0x0800 ? 0x90u : et == 0x86DD ? 0xE0u : 0u;
        if (a->mode == MODE_HASH) {
            edge = 0;
        } else if (et == 0x0800) {
            /* pktdev_rx.c:24-34 -> ptype 0x90; pkt_cls.c:19-31 -> ip4_lookup;
             * ip4_lookup.c:109-145: dip = ntohl(dst) at mtod+14, val >> 16 */
            uint32_t dip = vbe32(v, 14 + 16);
            nh = lookup4(a->tbl24, a->tbl8, dip);
            edge = (uint8_t)(nh >> 16);
        } else {
            edge = 0xFF; /* pkt_cls -> pkt_drop */
        }
    } else { /* MODE_CNET */
        struct orc_hdr_lens hl;
        memset(&hl, 0, sizeof(hl));
        uint32_t pt = orc_get_ptype(v.p, v.avail, &hl, 0x0fffffffu);
        if (a->ptype)
            a->ptype[i] = pt;
        if (a->rxmeta) {
            /* eth_rx.c:43-60: ol_flags IPv6 / BCAST / MCAST, tx_offload
             * l2_len:7 l3_len:9 l4_len:8 (pktmbuf_offload.h:396-400) */
            uint32_t m = (hl.l2_len & 0x7fu) | ((uint32_t)(hl.l3_len & 0x1ffu) << 7) |
                         ((uint32_t)hl.l4_len << 16);
            if (vraw16(v, 12) == BE(ET_IPV6))
                m |= 1u << 31;
            int bc = 1;
            for (int k = 0; k < 6; k++)
                bc &= v8(v, (uint32_t)k) == 0xFF;
            if (bc)
                m |= 1u << 30;
            else if (v8(v, 0) & 1u)
                m |= 1u << 29;
            a->rxmeta[i] = m;
        }
        uint32_t l3 = pt & 0xf0u;
        uint32_t l4t = pt & 0xf00u;
        uint32_t ip = hl.l2_len;
        int l4ok = (l4t == PT_L4_TCP || l4t == PT_L4_UDP);
        if (a->no_hash)
            ;
        else if (l3 != 0 && !(l3 & 0x40u))
            hash = hash_v4(v, ip, l4ok, ip + hl.l3_len, a->rss_key);
        else if (l3 & 0x40u)
            hash = hash_v6(v, ip, l4ok, ip + hl.l3_len, a->rss_key);
        uint8_t pe = cnet_ptype_edge(pt);
        cnet_input(a, v, ip, pe, &nh, &edge);
    }

    uint32_t q = a->reta[hash & (a->reta_size - 1)];
    /* bins: nh-id bins for the forwarding edge, n_bins for
     * drops, n_bins+1 for everything else */
    if (a->mode == MODE_HASH) {
        bin = q < nb ? q : nb + 1;
    } else if (a->mode == MODE_L3FWD) {
        if (edge == 0)
            bin = (nh & 0xffffu) < nb ? (nh & 0xffffu) : nb + 1;
        else if (edge == 1 || edge == 0xFF)
            bin = nb;
        else
            bin = nb + 1;
    } else {
        if (edge == 1)
            bin = (nh & 0xffffffu) < nb ? (nh & 0xffffffu) : nb + 1;
        else if (edge == 0 || edge == (0x80u | PTN_DROP))
            bin = nb;
        else
            bin = nb + 1;
    }
    a->nh[i] = nh;
    a->hash[i] = hash;
    a->queue[i] = (uint16_t)q;
    if (a->edge)
        a->edge[i] = edge;
    if (a->bins)
        a->bins[bin]++;
}

/* cnet with the ptype node's speculation (ptype.c:48-210), restated loop
 * for loop: per graph burst of B packets, 4-wide groups compared against
 * last_type with the uint8_t fix_spec (:109-110) -- a group whose four low
 * bytes equal last_type's goes whole to the speculated edge p_nxt[last_type]
 * -- then the per-packet tail.  last_type persists across bursts (and across
 * calls through spec_state; ctx->last_type starts at 0).  A frame sent to an
 * input node other than its own then gets that node's result. */
static int classify_cnet_spec(const struct orc_classify_args *a)
{
    const uint32_t n = a->n, B = a->spec_burst;
    uint16_t *l = malloc((size_t)(n ? n : 1) * sizeof(uint16_t));
    uint8_t *dst = malloc(n ? n : 1);
    uint32_t *pts = a->ptype ? NULL : malloc((size_t)(n ? n : 1) * 4);
    if (!l || !dst || (!a->ptype && !pts)) {
        free(l);
        free(dst);
        free(pts);
        return -ENOMEM;
    }
    struct orc_classify_args b = *a;
    if (!b.ptype)
        b.ptype = pts;
    for (uint32_t i = 0; i < n; i++) {
        classify_one(&b, i);
        l[i] = (uint16_t)(b.ptype[i] & 0xffffu);
    }
    uint16_t last_type = a->spec_state ? *a->spec_state : 0;
    for (uint32_t b0 = 0; b0 < n; b0 += B) {
        const uint32_t nb = n - b0 < B ? n - b0 : B;
        uint16_t next_index = cnet_ptype_edge(last_type);
        uint32_t k = 0;
        for (; k + 4 <= nb; k += 4) {
            const uint16_t *g = l + b0 + k;
            uint8_t fix_spec = (uint8_t)((last_type ^ g[0]) | (last_type ^ g[1]) | (last_type ^ g[2]) |
                                         (last_type ^ g[3]));
            if (fix_spec) {
                for (int j = 0; j < 4; j++)
                    dst[b0 + k + j] = cnet_ptype_edge(g[j]);
                if (last_type != g[3] && g[2] == g[3] && next_index != cnet_ptype_edge(g[3])) {
                    next_index = cnet_ptype_edge(g[3]);
                    last_type = g[3];
                } else if (next_index == cnet_ptype_edge(g[3])) {
                    last_type = g[3];
                }
            } else {
                for (int j = 0; j < 4; j++)
                    dst[b0 + k + j] = (uint8_t)next_index;
            }
        }
        for (; k < nb; k++) /* tail (:184-200): every frame to p_nxt[its type] */
            dst[b0 + k] = cnet_ptype_edge(l[b0 + k]);
    }
    if (a->spec_state)
        *a->spec_state = last_type;
    /* frames the speculation sent somewhere else than p_nxt[own type] */
    for (uint32_t i = 0; i < n; i++) {
        if (dst[i] == cnet_ptype_edge(l[i]))
            continue;
        uint64_t base = (a->offsets ? a->offsets[i] : (uint64_t)i * a->stride) + a->data_off;
        struct pv v = {a->slab + base, base < a->slab_len ? a->slab_len - base : 0};
        struct orc_hdr_lens hl;
        memset(&hl, 0, sizeof(hl));
        (void)orc_get_ptype(v.p, v.avail, &hl, 0x0fffffffu);
        const uint8_t old_edge = (uint8_t)(a->nh[i] == NH_INVALID ? 0x80u | cnet_ptype_edge(l[i])
                                                                   : (a->nh[i] >> 24));
        const uint32_t old_nh = a->nh[i];
        uint32_t nh;
        uint8_t edge;
        cnet_input(a, v, hl.l2_len, dst[i], &nh, &edge);
        a->nh[i] = nh;
        if (a->edge)
            a->edge[i] = edge;
        if (a->bins) {
            a->bins[bin_for(a, old_nh, old_edge, a->queue[i])]--;
            a->bins[bin_for(a, nh, edge, a->queue[i])]++;
        }
    }
    free(l);
    free(dst);
    free(pts);
    return 0;
}

int orc_classify(const struct orc_classify_args *a)
{
    if (!a || !a->slab || !a->rss_key || !a->reta || !a->nh || !a->hash || !a->queue)
        return -EINVAL;
    if (a->reta_size == 0 || (a->reta_size & (a->reta_size - 1)))
        return -EINVAL;
    if (a->mode != MODE_HASH && a->mode != MODE_CNET && a->mode != MODE_L3FWD)
        return -EINVAL;
    if (a->mode != MODE_HASH && (!a->tbl24 || !a->tbl8))
        return -EINVAL;
    if (a->mode == MODE_CNET && (!a->tbl24_6 || !a->tbl8_6))
        return -EINVAL;
    if (a->mode == MODE_CNET && a->spec_burst)
        return classify_cnet_spec(a);
    for (uint32_t i = 0; i < a->n; i++)
        classify_one(a, i);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline: the l3fwd node loop per 256-packet burst over pointer      */
/* arrays (pktdev_rx.c:49-103 soft parse, pkt_cls.c:60-166 classify,        */
/* ip4_lookup.c:83-204 gather + 4-wide cne_fib_lookup_bulk), plus the flow  */
/* hash / queue the build defines.                                          */
/* ------------------------------------------------------------------------ */
struct bench_shard {
    const struct orc_classify_args *a;
    uint32_t lo, hi;
    int iters;
    int cpu; /* pinned to this CPU (-1: not pinned) */
    uint64_t sink;
};

static void bench_pin(int cpu)
{
    if (cpu < 0)
        return;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

static void *bench_worker(void *arg)
{
    struct bench_shard *s = arg;
    bench_pin(s->cpu);
    const struct orc_classify_args *a = s->a;
    const uint8_t *ptrs[256];
    uint32_t ptype[256];
    uint64_t sink = 0;

    for (int it = 0; it < s->iters; it++) {
        for (uint32_t b = s->lo; b < s->hi; b += 256) {
            uint32_t cnt = s->hi - b < 256 ? s->hi - b : 256;
            /* pktdev_rx: mbuf pointer array + ethertype soft parse */
            for (uint32_t k = 0; k < cnt; k++) {
                uint32_t i = b + k;
                ptrs[k] = a->slab + (a->offsets ? a->offsets[i] : (uint64_t)i * a->stride) + a->data_off;
                uint16_t et = rd_be16(ptrs[k] + 12);
                ptype[k] = et == 0x0800 ? 0x90u : et == 0x86DD ? 0xE0u : 0u;
            }
            /* pkt_cls + ip4_lookup (4-wide gather then bulk lookup) */
            for (uint32_t k = 0; k < cnt; k += 4) {
                uint32_t dip[4];
                uint64_t dst[4];
                uint32_t m = cnt - k < 4 ? cnt - k : 4;
                for (uint32_t q = 0; q < m; q++)
                    dip[q] = ptype[k + q] == 0x90u ? rd_be32(ptrs[k + q] + 30) : 0;
                if (a->mode == MODE_HASH) /* C2: parse + hash + queue only */
                    memset(dst, 0, sizeof(dst));
                else
                    orc_dir24_8_lookup_bulk_pf(a->tbl24, a->tbl8, dip, m, dst);
                for (uint32_t q = 0; q < m; q++) {
                    const uint8_t *ip = ptrs[k + q] + 14;
                    uint32_t h = 0;
                    if (ptype[k + q] == 0x90u && !a->no_hash) {
                        struct pv v = {ptrs[k + q], 128};
                        uint32_t ihl = ip[0] & 0xfu;
                        int l4ok = ihl >= 5 && (ip[9] == 6 || ip[9] == 17) &&
                                   (rd_be16(ip + 6) & 0x3fff) == 0;
                        h = hash_v4(v, 14, l4ok, 14 + ihl * 4, a->rss_key);
                    }
                    uint32_t qn = a->reta[h & (a->reta_size - 1)];
                    sink += dst[q] + h + qn;
                }
            }
        }
    }
    s->sink = sink;
    return NULL;
}

/* cnet chain per 256-packet burst (eth_rx.c:65-109 parse into the mbuf
 * fields, ptype.c:48-210 speculation over the burst, ip4_input / ip6_input
 * length + checksum + 4-wide lookups), plus the build's flow hash: each
 * thread runs classify_one over its bursts and then walks the burst's types
 * as the ptype node does. */
static void *cnet_bench_worker(void *arg)
{
    struct bench_shard *s = arg;
    bench_pin(s->cpu);
    struct orc_classify_args b = *s->a;
    b.bins = NULL;
    uint64_t sink = 0;
    uint16_t last_type = 0;
    for (int it = 0; it < s->iters; it++) {
        for (uint32_t b0 = s->lo; b0 < s->hi; b0 += 256) {
            const uint32_t cnt = s->hi - b0 < 256 ? s->hi - b0 : 256;
            for (uint32_t k = 0; k < cnt; k++)
                classify_one(&b, b0 + k);
            uint16_t next_index = cnet_ptype_edge(last_type);
            uint32_t k = 0;
            for (; k + 4 <= cnt; k += 4) {
                const uint16_t g0 = (uint16_t)b.ptype[b0 + k], g1 = (uint16_t)b.ptype[b0 + k + 1],
                               g2 = (uint16_t)b.ptype[b0 + k + 2], g3 = (uint16_t)b.ptype[b0 + k + 3];
                const uint8_t fix = (uint8_t)((last_type ^ g0) | (last_type ^ g1) | (last_type ^ g2) |
                                              (last_type ^ g3));
                if (fix) {
                    if (last_type != g3 && g2 == g3 && next_index != cnet_ptype_edge(g3)) {
                        next_index = cnet_ptype_edge(g3);
                        last_type = g3;
                    } else if (next_index == cnet_ptype_edge(g3)) {
                        last_type = g3;
                    }
                }
                sink += next_index;
            }
            for (; k < cnt; k++)
                sink += b.nh[b0 + k] ^ b.hash[b0 + k];
        }
    }
    s->sink = sink;
    return NULL;
}

/* Per-burst CPU baseline on nthreads threads, thread t pinned to cpus[t]
 * when cpus is given: the l3fwd node loop (MODE_L3FWD / MODE_HASH) or the
 * cnet chain (MODE_CNET, needs a->ptype).  Returns seconds. */
double orc_burst_bench(const struct orc_classify_args *a, int nthreads, int iters, const int *cpus)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 512)
        nthreads = 512;
    if (a->mode == MODE_CNET && !a->ptype)
        return -1.0;
    static struct bench_shard sh[512];
    static pthread_t th[512];
    uint32_t per = (a->n + nthreads - 1) / nthreads;
    per = (per + 255) & ~255u;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        sh[t].a = a;
        sh[t].lo = (uint32_t)t * per < a->n ? (uint32_t)t * per : a->n;
        sh[t].hi = sh[t].lo + per < a->n ? sh[t].lo + per : a->n;
        sh[t].iters = iters;
        sh[t].cpu = cpus ? cpus[t] : -1;
        pthread_create(&th[t], NULL, a->mode == MODE_CNET ? cnet_bench_worker : bench_worker, &sh[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Receive-driver header writes (orc_set_driver_writes(1)): before each burst
 * reaches the node loops below, every mbuf gets its data_len (@30) and data_off
 * (@24) written, values kept, as xskdev's receive does (xskdev.c:296-297,
 * __get_mbuf_rx_aligned) -- the header line is then in this core's cache,
 * dirty, when the nodes read it: the state a real graph walk sees, and the
 * one the GPU legs get from the test harness's receive stub.  Off: the lines
 * are in whatever state the previous pass left them (the "cold" form). */
static int g_drv_writes;
void orc_set_driver_writes(int on) { g_drv_writes = on; }
static inline void drv_touch(void *const *mbufs, uint32_t cnt)
{
    if (!g_drv_writes)
        return;
    for (uint32_t k = 0; k < cnt; k++) {
        volatile uint16_t *dl = (volatile uint16_t *)((uint8_t *)mbufs[k] + 30);
        volatile uint16_t *dof = (volatile uint16_t *)((uint8_t *)mbufs[k] + 24);
        *dl = *dl;
        *dof = *dof;
    }
}

/* The ip4_lookup node's CPU work over pktmbuf_t pointer arrays, one thread
 * (ip4_lookup.c:48-256): per graph burst, mtod + 14 of every mbuf, dip /
 * ttl / checksum into node_mbuf_priv1 (udata64, @56), 4-wide
 * cne_fib_lookup_bulk with the default prefetching lookup, edge = val >> 16.
 * pktmbuf_t offsets: buf_addr @8, data_off @24 (pktmbuf.h:102-204).
 * Returns seconds for `iters` passes; writes udata64 like the node. */
static uint64_t ip4_lookup_burst(void *const *mbufs, uint32_t b, uint32_t cnt, const uint32_t *tbl24,
                                 const uint32_t *tbl8)
{
    uint64_t sink = 0;
    for (uint32_t k = 0; k < cnt; k += 4) {
        const uint32_t m = cnt - k < 4 ? cnt - k : 4;
        uint32_t dip[4];
        uint64_t dst[4];
        uint8_t *mb[4];
        const uint8_t *ip[4];
        for (uint32_t q = 0; q < m; q++) {
            mb[q] = (uint8_t *)mbufs[b + k + q];
            const uint8_t *buf = *(uint8_t *const *)(mb[q] + 8);
            ip[q] = buf + *(const uint16_t *)(mb[q] + 24) + 14;
            dip[q] = rd_be32(ip[q] + 16);
        }
        orc_dir24_8_lookup_bulk_pf(tbl24, tbl8, dip, m, dst);
        for (uint32_t q = 0; q < m; q++) {
            const uint64_t ck = (uint64_t)ip[q][10] | ((uint64_t)ip[q][11] << 8);
            *(uint64_t *)(mb[q] + 56) = (dst[q] & 0xffffu) | ((uint64_t)ip[q][8] << 16) | (ck << 32);
            sink += dst[q] >> 16;
        }
    }
    return sink;
}

double orc_ip4_lookup_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                            const uint32_t *tbl8, int iters)
{
    struct timespec t0, t1;
    uint64_t sink = 0;
    if (burst == 0)
        burst = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int it = 0; it < iters; it++) {
        for (uint32_t b = 0; b < n; b += burst) {
            const uint32_t cnt = n - b < burst ? n - b : burst;
            drv_touch(mbufs + b, cnt);
            sink += ip4_lookup_burst(mbufs, b, cnt, tbl24, tbl8);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)sink;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* The same loop with pktdev_rx's soft parse callback first (pktdev_rx.c:36-101:
 * the ethertype of every frame into m->packet_type @32, with its prefetching),
 * per burst, as l3fwd-graph's pktdev_rx -> pkt_cls -> ip4_lookup walk does
 * before ip4_lookup runs.  Returns seconds for `iters` passes. */
double orc_rx_ip4_lookup_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                               const uint32_t *tbl8, int iters)
{
    struct timespec t0, t1;
    if (burst == 0)
        burst = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int it = 0; it < iters; it++) {
        for (uint32_t b = 0; b < n; b += burst) {
            const uint32_t cnt = n - b < burst ? n - b : burst;
            drv_touch(mbufs + b, cnt);
            uint32_t k = 0;
            for (; k + 12 <= cnt; k += 4) {
                for (int j = 8; j < 12; j++)
                    __builtin_prefetch(mbufs[b + k + j]);
                for (int j = 4; j < 8; j++) {
                    const uint8_t *m = mbufs[b + k + j];
                    __builtin_prefetch(*(uint8_t *const *)(m + 8) + *(const uint16_t *)(m + 24));
                }
                for (int j = 0; j < 4; j++) {
                    uint8_t *m = mbufs[b + k + j];
                    const uint8_t *eh = *(uint8_t *const *)(m + 8) + *(const uint16_t *)(m + 24);
                    const uint16_t et = rd_be16(eh + 12);
                    *(uint32_t *)(m + 32) = et == 0x0800 ? 0x90u : et == 0x86DD ? 0xE0u : 0u;
                }
            }
            for (; k < cnt; k++) {
                uint8_t *m = mbufs[b + k];
                const uint8_t *eh = *(uint8_t *const *)(m + 8) + *(const uint16_t *)(m + 24);
                const uint16_t et = rd_be16(eh + 12);
                *(uint32_t *)(m + 32) = et == 0x0800 ? 0x90u : et == 0x86DD ? 0xE0u : 0u;
            }
            ip4_lookup_burst(mbufs, b, cnt, tbl24, tbl8);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* l3fwd-graph's receive chain per graph burst, as one core runs it:
 * pktdev_rx's soft parse (pktdev_rx.c:24-34, :37-103: packet_type =
 * l3_ptype(ether_type, 0) into m->packet_type @32), pkt_cls (pkt_cls.c:19-31:
 * p_nxt[packet_type & 0xff] -- the IPv4 types (0x10, 0x30, 0x90, with or
 * without L2_ETHER 0x01) to ip4_lookup, everything else to pkt_drop), then
 * the ip4_lookup node loop (ip4_lookup.c:108-154) over the burst's IPv4
 * mbufs, which pkt_cls hands on in order, and with rwt the ip4_rewrite node
 * (ip4_rewrite.c:40-247) over the ones ip4_lookup sent to it, in order.
 * edges (optional, n entries, in mbuf order): the FIB value >> 16 for the
 * mbufs ip4_lookup saw, 0xFFFE for those pkt_cls dropped.  Returns seconds
 * for `iters` passes. */
static inline int orc_cls_ip4(uint32_t pt)
{
    const uint32_t l = pt & 0xffu; /* pkt_cls.c:19-31 */
    return l == 0x10u || l == 0x30u || l == 0x90u || l == 0x11u || l == 0x31u || l == 0x91u;
}

/* ip4_lookup's loop over mbufs[0..n) (as orc_ip4_lookup_mbufs), each mbuf's
 * next edge (FIB value >> 16) into edge[] */
static void orc_l3_lookup_edges(void *const *mbufs, uint32_t n, const uint32_t *tbl24, const uint32_t *tbl8,
                                uint16_t *edge)
{
    for (uint32_t k = 0; k < n; k += 4) {
        const uint32_t m = n - k < 4 ? n - k : 4;
        uint32_t dip[4];
        uint64_t dst[4];
        uint8_t *mb[4];
        const uint8_t *ip[4];
        for (uint32_t q = 0; q < m; q++) {
            mb[q] = (uint8_t *)mbufs[k + q];
            const uint8_t *buf = *(uint8_t *const *)(mb[q] + 8);
            ip[q] = buf + *(const uint16_t *)(mb[q] + 24) + 14;
            dip[q] = rd_be32(ip[q] + 16);
        }
        orc_dir24_8_lookup_bulk_pf(tbl24, tbl8, dip, m, dst);
        for (uint32_t q = 0; q < m; q++) {
            const uint64_t ck = (uint64_t)ip[q][10] | ((uint64_t)ip[q][11] << 8);
            *(uint64_t *)(mb[q] + 56) = (dst[q] & 0xffffu) | ((uint64_t)ip[q][8] << 16) | (ck << 32);
            edge[k + q] = (uint16_t)(dst[q] >> 16);
        }
    }
}

double orc_l3rx_chain_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                            const uint32_t *tbl8, int iters, uint16_t *edges, const struct orc_rewrite_nh *rwt)
{
    struct timespec t0, t1;
    void *ip4[256], *rw[256];
    uint32_t at[256];
    uint16_t e4[256], tx[256];
    if (burst == 0 || burst > 256)
        burst = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int it = 0; it < iters; it++) {
        for (uint32_t b = 0; b < n; b += burst) {
            const uint32_t cnt = n - b < burst ? n - b : burst;
            drv_touch(mbufs + b, cnt);
            for (uint32_t k = 0; k < cnt; k++) {
                if (k + 8 < cnt)
                    __builtin_prefetch(mbufs[b + k + 8]);
                if (k + 4 < cnt) {
                    const uint8_t *pm = mbufs[b + k + 4];
                    __builtin_prefetch(*(uint8_t *const *)(pm + 8) + *(const uint16_t *)(pm + 24));
                }
                uint8_t *m = mbufs[b + k];
                const uint8_t *eh = *(uint8_t *const *)(m + 8) + *(const uint16_t *)(m + 24);
                const uint16_t et = rd_be16(eh + 12);
                *(uint32_t *)(m + 32) = et == 0x0800 ? 0x90u : et == 0x86DD ? 0xE0u : 0u;
            }
            uint32_t n4 = 0;
            for (uint32_t k = 0; k < cnt; k++) {
                const uint8_t *m = mbufs[b + k];
                if (orc_cls_ip4(*(const uint32_t *)(m + 32))) {
                    at[n4] = b + k;
                    ip4[n4++] = mbufs[b + k];
                } else if (edges) {
                    edges[b + k] = 0xFFFEu;
                }
            }
            orc_l3_lookup_edges(ip4, n4, tbl24, tbl8, e4);
            if (rwt) {
                uint32_t nrw = 0;
                for (uint32_t q = 0; q < n4; q++)
                    if (e4[q] == 0)
                        rw[nrw++] = ip4[q];
                orc_ip4_rewrite_node(rw, nrw, rwt, tx);
            }
            if (edges)
                for (uint32_t q = 0; q < n4; q++)
                    edges[at[q]] = e4[q];
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

double orc_l3fwd_burst_bench(const struct orc_classify_args *a, int nthreads, int iters)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    struct bench_shard sh[256];
    pthread_t th[256];
    uint32_t per = (a->n + nthreads - 1) / nthreads;
    per = (per + 255) & ~255u;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        sh[t].a = a;
        sh[t].lo = (uint32_t)t * per < a->n ? (uint32_t)t * per : a->n;
        sh[t].hi = sh[t].lo + per < a->n ? sh[t].lo + per : a->n;
        sh[t].iters = iters;
        sh[t].cpu = -1;
        pthread_create(&th[t], NULL, bench_worker, &sh[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------------------
 * ip4_rewrite (ip4_rewrite.c:40-247) and the cndpfwd MAC swap
 * ------------------------------------------------------------------------- */
static uint64_t frame_base(uint64_t stride, const uint64_t *offsets, uint32_t data_off, uint32_t i)
{
    return (offsets ? offsets[i] : (uint64_t)i * stride) + data_off;
}

static void put8(uint8_t *slab, uint64_t slab_len, uint64_t o, uint8_t v)
{
    if (o < slab_len)
        slab[o] = v;
}

void orc_ip4_rewrite(uint8_t *slab, uint64_t slab_len, uint64_t stride, const uint64_t *offsets,
                     uint32_t data_off, uint32_t n, const uint32_t *nh, uint32_t burst,
                     const struct orc_rewrite_nh *tbl, uint16_t *tx_edge)
{
    static const struct orc_rewrite_nh unset; /* calloc'ed entry (ip4_rewrite.c:258) */
    if (burst == 0)
        burst = 1;
    for (uint32_t b0 = 0; b0 < n; b0 += burst) {
        const uint32_t b1 = b0 + burst < n ? b0 + burst : n;
        uint32_t cnt = 0;
        for (uint32_t i = b0; i < b1; i++)
            cnt += nh[i] != 0xFFFFFFFFu && (nh[i] >> 16) == 0;
        const uint32_t vec = cnt & ~3u; /* packets handled by the 4-wide loop */
        uint32_t p = 0;
        for (uint32_t i = b0; i < b1; i++) {
            if (!(nh[i] != 0xFFFFFFFFu && (nh[i] >> 16) == 0)) {
                tx_edge[i] = 0xFFFF;
                continue;
            }
            const uint64_t base = frame_base(stride, offsets, data_off, i);
            /* priv1 as ip4_lookup left it: nh, ttl, cksum from the frame */
            const uint32_t nh16 = nh[i] & 0xFFFFu;
            const uint32_t ttl = base + 22 < slab_len ? slab[base + 22] : 0;
            const uint32_t ck = (base + 24 < slab_len ? slab[base + 24] : 0) |
                                ((base + 25 < slab_len ? (uint32_t)slab[base + 25] : 0) << 8);
            const struct orc_rewrite_nh *e = nh16 < 64 ? &tbl[nh16] : &unset;
            for (uint32_t k = 0; k < e->rewrite_len && k < 56; k++)
                put8(slab, slab_len, base + k, e->rewrite_data[k]);
            uint16_t nck;
            if (p < vec) { /* priv.u32[1] += htons(0x0100); cksum = u16[2] + u16[3] */
                const uint32_t c32 = ck + 0x0001u;
                nck = (uint16_t)((c32 & 0xFFFFu) + (c32 >> 16));
            } else { /* chksum = cksum + htons(0x0100); chksum += chksum >= 0xffff */
                uint16_t c16 = (uint16_t)(ck + 0x0001u);
                c16 = (uint16_t)(c16 + (c16 >= 0xffff));
                nck = c16;
            }
            put8(slab, slab_len, base + 22, (uint8_t)(ttl - 1));
            put8(slab, slab_len, base + 24, (uint8_t)(nck & 0xFF));
            put8(slab, slab_len, base + 25, (uint8_t)(nck >> 8));
            tx_edge[i] = e->tx_node;
            p++;
        }
    }
}

void orc_mac_swap(uint8_t *slab, uint64_t slab_len, uint64_t stride, const uint64_t *offsets,
                  uint32_t data_off, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t base = frame_base(stride, offsets, data_off, i);
        if (base + 12 > slab_len)
            continue; /* build-defined: frames without a whole Ethernet address pair stay */
        for (int k = 0; k < 6; k++) {
            const uint8_t t = slab[base + k];
            slab[base + k] = slab[base + 6 + k];
            slab[base + 6 + k] = t;
        }
    }
}

/* ---------------------------------------------------------------------------
 * ip4_rewrite_node_process (ip4_rewrite.c:40-247) over one burst of
 * pktmbuf_t pointers (one process() call, nb_objs = n): priv1 from udata64
 * (node_private.h:24-35), the rewrite data at mtod (:85), TTL = priv.ttl - 1,
 * the checksum from priv.cksum + htons(0x0100) -- the 4-wide loop's u32
 * end-around carry for the first n & ~3 mbufs (:97-110), the tail loop's u16
 * rule for the rest (:209-216); tx_edge = the next hop's tx_node.  Next hops
 * past the 64-entry array read an unset (zero) entry.
 * ------------------------------------------------------------------------- */
static void rw_one(uint8_t *m, const struct orc_rewrite_nh *tbl, int vec4, uint16_t *tx)
{
    static const struct orc_rewrite_nh unset;
    const uint64_t priv = *(const uint64_t *)(m + 56);
    const uint16_t nh = (uint16_t)priv, ttl = (uint16_t)(priv >> 16);
    const uint32_t ck32 = (uint32_t)(priv >> 32);
    uint8_t *d = *(uint8_t *const *)(m + 8) + *(const uint16_t *)(m + 24); /* pktmbuf_mtod */
    const struct orc_rewrite_nh *e = nh < 64 ? &tbl[nh] : &unset;
    memcpy(d, e->rewrite_data, e->rewrite_len < 56 ? e->rewrite_len : 56);
    uint16_t nck;
    if (vec4) {
        const uint32_t c32 = ck32 + 0x0001u; /* priv01.u32[1] += htons(0x0100) */
        nck = (uint16_t)((c32 & 0xFFFFu) + (c32 >> 16));
    } else {
        uint16_t c16 = (uint16_t)(ck32 + 0x0001u);
        c16 = (uint16_t)(c16 + (c16 >= 0xffff));
        nck = c16;
    }
    d[14 + 8] = (uint8_t)(ttl - 1);
    memcpy(d + 14 + 10, &nck, 2);
    *tx = e->tx_node;
}

void orc_ip4_rewrite_node(void *const *mbufs, uint32_t n, const struct orc_rewrite_nh *tbl, uint16_t *tx_edge)
{
    const uint32_t vec = n & ~3u;
    for (uint32_t i = 0; i < n; i++)
        rw_one((uint8_t *)mbufs[i], tbl, i < vec, &tx_edge[i]);
}

/* The l3fwd-graph node pair on one core: per burst ip4_lookup's loop (as
 * orc_ip4_lookup_mbufs) then ip4_rewrite_node_process over the burst's mbufs
 * the lookup sent to edge 0, in order (the rewrite node's stream).  Returns
 * seconds for `iters` passes. */
double orc_l3fwd_nodes_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                             const uint32_t *tbl8, const struct orc_rewrite_nh *tbl, int iters)
{
    struct timespec t0, t1;
    uint64_t sink = 0;
    void *rw[256];
    uint16_t tx[256];
    if (burst == 0 || burst > 256)
        burst = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int it = 0; it < iters; it++) {
        for (uint32_t b = 0; b < n; b += burst) {
            const uint32_t cnt = n - b < burst ? n - b : burst;
            uint32_t nrw = 0;
            drv_touch(mbufs + b, cnt);
            for (uint32_t k = 0; k < cnt; k += 4) {
                const uint32_t m = cnt - k < 4 ? cnt - k : 4;
                uint32_t dip[4];
                uint64_t dst[4];
                uint8_t *mb[4];
                const uint8_t *ip[4];
                for (uint32_t q = 0; q < m; q++) {
                    mb[q] = (uint8_t *)mbufs[b + k + q];
                    const uint8_t *buf = *(uint8_t *const *)(mb[q] + 8);
                    ip[q] = buf + *(const uint16_t *)(mb[q] + 24) + 14;
                    dip[q] = rd_be32(ip[q] + 16);
                }
                orc_dir24_8_lookup_bulk_pf(tbl24, tbl8, dip, m, dst);
                for (uint32_t q = 0; q < m; q++) {
                    const uint64_t ck = (uint64_t)ip[q][10] | ((uint64_t)ip[q][11] << 8);
                    *(uint64_t *)(mb[q] + 56) = (dst[q] & 0xffffu) | ((uint64_t)ip[q][8] << 16) | (ck << 32);
                    if ((dst[q] >> 16) == 0)
                        rw[nrw++] = mb[q];
                }
            }
            orc_ip4_rewrite_node(rw, nrw, tbl, tx);
            for (uint32_t q = 0; q < nrw; q++)
                sink += tx[q];
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)sink;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
