/*
 * oracle/cnet_chain.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline of the cnet
 * receive chain, never linked into the product (tests/test_abi.py checks).
 *
 * Unlike orc_classify (oracle.c, the checker: one frame at a time through a
 * bounds-checked byte view), this is the reference's cnet chain as a graph walk
 * runs it on one lcore, restated over pktmbuf_t pointer arrays with direct
 * loads and the nodes' own prefetch pattern, one 256-mbuf burst at a time:
 *
 *   eth_rx     lib/cnet/eth/eth_rx.c:35-109    mbuf_update per mbuf, 4-wide,
 *              prefetching mtod of the mbufs 4 ahead; cne_get_ptype
 *              (lib/core/pktmbuf/pktmbuf_ptype.c:472-744, restated below with
 *              the reference's header-pointer reads and lookup tables),
 *              ol_flags, tx_offload l2/l3/l4 lengths, lport,
 *              pktmbuf_adj_offset(l2_len)
 *   ptype      lib/cnet/ptype/ptype.c:48-210   4-wide speculation on
 *              last_type with the uint8_t fix_spec, the per-mbuf tail, the
 *              node context's last_type carried from burst to burst; mbufs go
 *              into per-edge streams (cne_node_enqueue)
 *   ip4_input  lib/cnet/ipv4/ip4_input.c:50-260  prefetch headers 8 ahead and
 *              data 4 ahead, data_len = total_length, length + cne_ipv4_cksum
 *              test, ipv4_save_metadata, 4-wide fib_info_lookup_index ->
 *              cne_fib_lookup_bulk (dir24_8.h:118-148's prefetching loop)
 *   ip6_input  lib/cnet/ipv6/ip6_input.c:50-260  the same with payload_len and
 *              the trie lookup (trie.h:119-138)
 *
 * Before each burst the mbufs get back the data_off / data_len pktdev_rx
 * delivers them with (eth_rx advances data_off), so every pass parses
 * received frames.  Optionally (flags & ORC_CHAIN_HASH) eth_rx also computes
 * the build's flow hash into m->hash and its RSS queue, the work the GPU line
 * does on top of the reference chain (CNDP's cnet nodes hash nothing).
 *
 * Where each mbuf went is recorded in m->udata64 = edge << 32 | nh, with the
 * checker's encoding: an input node's FIB value and its edge
 * (value >> 24), or NH_INVALID and 0x80 | ptype edge for the other ptype
 * edges; tests compare it, m->packet_type and m->hash with orc_classify.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

/* pktmbuf_t (lib/core/pktmbuf/pktmbuf.h:102-204), 64 bytes */
struct mb {
    void *pooldata;
    uint8_t *buf_addr;
    uint32_t hash;
    uint32_t meta_index;
    uint16_t data_off;
    uint16_t lport;
    uint16_t buf_len;
    uint16_t data_len;
    uint32_t packet_type;
    uint16_t refcnt;
    uint16_t rsvd16;
    uint64_t tx_offload; /* l2_len:7 l3_len:9 l4_len:8 (pktmbuf_offload.h:396-400) */
    uint64_t ol_flags;
    uint64_t udata64;
};
_Static_assert(sizeof(struct mb) == 64, "pktmbuf_t is 64 bytes");

#define MTOD(m) ((m)->buf_addr + (m)->data_off)
#define PF(p) __builtin_prefetch((const void *)(p), 0, 3)

static inline uint16_t ld16(const uint8_t *p) /* the raw (network-order) u16 */
{
    uint16_t v;
    memcpy(&v, p, 2);
    return v;
}
static inline uint32_t ld32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
#define BE16(x) ((uint16_t)__builtin_bswap16((uint16_t)(x)))

/* CNE_PTYPE_* (pktmbuf_ptype.h) */
enum {
    L2_ETHER = 0x1, L2_ARP = 0x3, L2_VLAN = 0x6, L2_QINQ = 0x7,
    L3_IPV4 = 0x10, L3_IPV4_EXT = 0x30, L3_IPV6 = 0x40, L3_IPV6_EXT = 0xc0,
    L4_TCP = 0x100, L4_UDP = 0x200, L4_FRAG = 0x300, L4_SCTP = 0x400,
    TUN_IP = 0x1000, TUN_GRE = 0x2000, TUN_NVGRE = 0x4000, TUN_GTPC = 0x7000, TUN_GTPU = 0x8000,
    IN_L2_ETHER = 0x10000, IN_L2_VLAN = 0x20000, IN_L2_QINQ = 0x30000,
    IN_L3_IPV4 = 0x100000, IN_L3_IPV4_EXT = 0x200000, IN_L3_IPV6 = 0x300000, IN_L3_IPV6_EXT = 0x500000,
    IN_L4_TCP = 0x1000000, IN_L4_UDP = 0x2000000, IN_L4_FRAG = 0x3000000, IN_L4_SCTP = 0x4000000,
};

/* pktmbuf_ptype.c:279-369: the per-byte maps */
static uint32_t map_l3_ip[256], map_in_l3_ip[256], map_l4[256], map_in_l4[256];
static uint32_t map_v6ext[256], map_in_v6ext[256];
static void maps_init(void)
{
    map_l3_ip[0x45] = L3_IPV4;
    map_in_l3_ip[0x45] = IN_L3_IPV4;
    for (int v = 0x46; v <= 0x4f; v++) {
        map_l3_ip[v] = L3_IPV4_EXT;
        map_in_l3_ip[v] = IN_L3_IPV4_EXT;
    }
    map_l4[17] = L4_UDP;
    map_l4[6] = L4_TCP;
    map_l4[132] = L4_SCTP;
    map_in_l4[17] = IN_L4_UDP;
    map_in_l4[6] = IN_L4_TCP;
    map_in_l4[132] = IN_L4_SCTP;
    static const uint8_t ext[] = {0, 43, 44, 50, 51, 60}; /* HOPOPTS ROUTING FRAGMENT ESP AH DSTOPTS */
    for (unsigned k = 0; k < sizeof(ext); k++) {
        map_v6ext[ext[k]] = L3_IPV6_EXT - L3_IPV6;
        map_in_v6ext[ext[k]] = IN_L3_IPV6_EXT - IN_L3_IPV6;
    }
}

struct hlens {
    uint8_t l2_len, inner_l2_len;
    uint16_t l3_len, inner_l3_len, tunnel_len;
    uint8_t l4_len, inner_l4_len;
};

/* pktmbuf_ptype.c:426-468 */
static int skip_ip6_ext(uint16_t proto, const uint8_t *p, uint32_t *off, int *frag)
{
    *frag = 0;
    for (int i = 0; i < 5; i++) {
        const uint8_t *xh = p + *off;
        switch (proto) {
        case 0:
        case 43:
        case 60:
            *off += ((uint32_t)xh[1] + 1) * 8;
            proto = xh[0];
            break;
        case 44:
            *off += 8;
            *frag = 1;
            return xh[0];
        case 59:
            return 0;
        default:
            return proto;
        }
    }
    return -1;
}

/* pktmbuf_ptype.c:372-411 */
static uint32_t ptype_tunnel(uint16_t *proto, const uint8_t *p, uint32_t *off)
{
    switch (*proto) {
    case 47: {
        static const uint8_t opt_len[16] = {[0x0] = 4,  [0x1] = 8,  [0x2] = 8,  [0x8] = 8,
                                            [0x3] = 12, [0x9] = 12, [0xa] = 12, [0xb] = 16};
        const uint8_t *gh = p + *off;
        const uint16_t flags = (uint16_t)(BE16(ld16(gh)) >> 12);
        if (opt_len[flags] == 0)
            return 0;
        *off += opt_len[flags];
        *proto = ld16(gh + 2);
        return *proto == BE16(0x6558) ? TUN_NVGRE : TUN_GRE;
    }
    case 4:
        *proto = BE16(0x0800);
        return TUN_IP;
    case 41:
        *proto = BE16(0x86DD);
        return TUN_IP;
    default:
        return 0;
    }
}

/* cne_get_ptype (pktmbuf_ptype.c:472-744), layers = CNE_PTYPE_ALL_MASK as
 * eth_rx.c:41 calls it, p = pktmbuf_mtod(m) */
static uint32_t get_ptype(const uint8_t *p, struct hlens *hl)
{
    uint32_t pt = L2_ETHER, off = 14;
    uint16_t proto = ld16(p + 12);
    int ret;

    hl->l2_len = 14;
    if (proto == BE16(0x0806))
        return L2_ARP;
    if (proto == BE16(0x0800))
        goto l3;
    if (proto == BE16(0x8100)) {
        pt = L2_VLAN;
        proto = ld16(p + off + 2);
        off += 4;
        hl->l2_len += 4;
    } else if (proto == BE16(0x88A8)) {
        pt = L2_QINQ;
        proto = ld16(p + off + 4 + 2);
        off += 8;
        hl->l2_len += 8;
    } else if (proto == BE16(0x8847) || proto == BE16(0x8848)) {
        return pt; /* :541-556: the label loop always runs out */
    }
l3:
    if (proto == BE16(0x0800)) {
        const uint8_t *ip4h = p + off;
        pt |= map_l3_ip[ip4h[0]];
        hl->l3_len = (uint16_t)((ip4h[0] & 0xf) * 4);
        off += hl->l3_len;
        if (ld16(ip4h + 6) & BE16(0x1fff | 0x2000)) {
            pt |= L4_FRAG;
            hl->l4_len = 0;
            return pt;
        }
        proto = ip4h[9];
        pt |= map_l4[proto];
    } else if (proto == BE16(0x86DD)) {
        const uint8_t *ip6h = p + off;
        int frag = 0;
        proto = ip6h[6];
        hl->l3_len = 40;
        off += 40;
        pt |= L3_IPV6 + map_v6ext[proto];
        if ((pt & 0xf0u) == L3_IPV6_EXT) {
            ret = skip_ip6_ext(proto, p, &off, &frag);
            if (ret < 0)
                return pt;
            proto = (uint16_t)ret;
            hl->l3_len = (uint16_t)(off - hl->l2_len);
        }
        if (proto == 0)
            return pt;
        if (frag) {
            pt |= L4_FRAG;
            hl->l4_len = 0;
            return pt;
        }
        pt |= map_l4[proto & 0xff];
    }

    if ((pt & 0xf00u) == L4_UDP) {
        const uint8_t *udp = p + hl->l2_len + hl->l3_len;
        hl->l4_len = 8;
        const uint16_t dport = ld16(udp + 2);
        if (dport == BE16(2152))
            pt |= TUN_GTPU;
        else if (dport == BE16(2123))
            pt |= TUN_GTPC;
        return pt;
    } else if ((pt & 0xf00u) == L4_TCP) {
        hl->l4_len = (uint8_t)((p[hl->l2_len + hl->l3_len + 12] & 0xf0) >> 2);
        return pt;
    } else if ((pt & 0xf00u) == L4_SCTP) {
        hl->l4_len = 12;
        return pt;
    } else {
        const uint32_t prev = off;
        hl->l4_len = 0;
        pt |= ptype_tunnel(&proto, p, &off);
        hl->tunnel_len = (uint16_t)(off - prev);
    }

    hl->inner_l2_len = 0;
    if (proto == BE16(0x6558)) {
        pt |= IN_L2_ETHER;
        proto = ld16(p + off + 12);
        off += 14;
        hl->inner_l2_len = 14;
    }
    if (proto == BE16(0x8100)) {
        pt = (pt & ~0xf0000u) | IN_L2_VLAN;
        proto = ld16(p + off + 2);
        off += 4;
        hl->inner_l2_len += 4;
    } else if (proto == BE16(0x88A8)) {
        pt = (pt & ~0xf0000u) | IN_L2_QINQ;
        proto = ld16(p + off + 4 + 2);
        off += 8;
        hl->inner_l2_len += 8;
    }
    if (proto == BE16(0x0800)) {
        const uint8_t *ip4h = p + off;
        pt |= map_in_l3_ip[ip4h[0]];
        hl->inner_l3_len = (uint16_t)((ip4h[0] & 0xf) * 4);
        off += hl->inner_l3_len;
        if (ld16(ip4h + 6) & BE16(0x1fff | 0x2000)) {
            pt |= IN_L4_FRAG;
            hl->inner_l4_len = 0;
            return pt;
        }
        proto = ip4h[9];
        pt |= map_in_l4[proto];
    } else if (proto == BE16(0x86DD)) {
        const uint8_t *ip6h = p + off;
        int frag = 0;
        proto = ip6h[6];
        hl->inner_l3_len = 40;
        off += 40;
        pt |= IN_L3_IPV6 + map_in_v6ext[proto];
        if ((pt & 0xf00000u) == IN_L3_IPV6_EXT) {
            const uint32_t prev = off;
            ret = skip_ip6_ext(proto, p, &off, &frag);
            if (ret < 0)
                return pt;
            proto = (uint16_t)ret;
            hl->inner_l3_len = (uint16_t)(hl->inner_l3_len + off - prev);
        }
        if (proto == 0)
            return pt;
        if (frag) {
            pt |= IN_L4_FRAG;
            hl->inner_l4_len = 0;
            return pt;
        }
        pt |= map_in_l4[proto & 0xff];
    }
    if ((pt & 0xf000000u) == IN_L4_UDP)
        hl->inner_l4_len = 8;
    else if ((pt & 0xf000000u) == IN_L4_TCP)
        hl->inner_l4_len = (uint8_t)((p[off + 12] & 0xf0) >> 2);
    else if ((pt & 0xf000000u) == IN_L4_SCTP)
        hl->inner_l4_len = 12;
    else
        hl->inner_l4_len = 0;
    return pt;
}

/* ptype node edges (lib/cnet/ptype/ptype_priv.h:19-29) and p_nxt
 * (ptype.c:32-46), indexed by the 16-bit masked type */
#define PTN_DROP 0u
#define PTN_PUNT 2u
#define PTN_IP4 3u
#define PTN_IP6 4u
#define PTN_GTPU 5u
#define PTN_MAX 6u
static uint8_t p_nxt[65536];
static void pnxt_init(void)
{
    p_nxt[0x0003] = PTN_PUNT;
    p_nxt[0x0211] = p_nxt[0x0111] = p_nxt[0x0231] = p_nxt[0x0291] = PTN_IP4;
    p_nxt[0x8211] = PTN_GTPU;
    p_nxt[0x0241] = p_nxt[0x0141] = p_nxt[0x02c1] = p_nxt[0x02e1] = PTN_IP6;
    p_nxt[0x8241] = PTN_GTPU;
}
static void tables_init(void)
{
    maps_init();
    pnxt_init();
}

#define NH_INVALID 0xFFFFFFFFu
#define OL_IPV6 (1ull << 63) /* CNE_MBUF_TYPE_IPv6 / BCAST / MCAST (pktmbuf_offload.h:365-412) */
#define OL_BCAST (1ull << 62)
#define OL_MCAST (1ull << 61)

struct chain_ctx {
    const struct orc_cnet_chain_args *a;
    uint16_t last_type;          /* the ptype node context (ptype.c:70) */
    uint64_t sink;
};

/* the build-defined flow hash over the parsed tuple */
static uint32_t flow_hash(const uint8_t *p, uint32_t pt, const struct hlens *hl, const uint8_t *key)
{
    const uint32_t l3 = pt & 0xf0u, l4t = pt & 0xf00u;
    const int l4ok = l4t == L4_TCP || l4t == L4_UDP;
    const uint8_t *ip = p + hl->l2_len, *l4 = ip + hl->l3_len;
    uint32_t t[9];
    if (l3 != 0 && !(l3 & 0x40u)) {
        t[0] = __builtin_bswap32(ld32(ip + 12));
        t[1] = __builtin_bswap32(ld32(ip + 16));
        if (l4ok) {
            t[2] = (uint32_t)BE16(ld16(l4 + 2)) | ((uint32_t)BE16(ld16(l4)) << 16);
            return orc_softrss(t, 3, key);
        }
        return orc_softrss(t, 2, key);
    }
    if (l3 & 0x40u) {
        for (int k = 0; k < 8; k++)
            t[k] = __builtin_bswap32(ld32(ip + 8 + 4 * k));
        if (l4ok) {
            t[8] = (uint32_t)BE16(ld16(l4 + 2)) | ((uint32_t)BE16(ld16(l4)) << 16);
            return orc_softrss(t, 9, key);
        }
        return orc_softrss(t, 8, key);
    }
    return 0;
}

/* eth_rx.c:35-63 mbuf_update (+ the optional build hash) */
static inline void mbuf_update(struct chain_ctx *c, struct mb *m, uint16_t lpid)
{
    struct hlens hl;
    memset(&hl, 0, sizeof(hl));
    const uint8_t *eh = MTOD(m);
    m->packet_type = get_ptype(eh, &hl);
    m->ol_flags = 0;
    if (ld16(eh + 12) == BE16(0x86DD))
        m->ol_flags |= OL_IPV6;
    const uint32_t d0 = ld32(eh);
    const uint16_t d1 = ld16(eh + 4);
    if (d0 == 0xFFFFFFFFu && d1 == 0xFFFFu)
        m->ol_flags |= OL_BCAST;
    else if (eh[0] & 1u)
        m->ol_flags |= OL_MCAST;
    m->tx_offload = (uint64_t)(hl.l2_len & 0x7fu) | ((uint64_t)(hl.l3_len & 0x1ffu) << 7) |
                    ((uint64_t)hl.l4_len << 16);
    m->lport = lpid;
    if (c->a->flags & ORC_CHAIN_HASH) {
        const uint32_t h = flow_hash(eh, m->packet_type, &hl, c->a->rss_key);
        m->hash = h;
        c->sink += c->a->reta[h & (c->a->reta_size - 1)];
    }
    /* pktmbuf_adj_offset(m, l2_len) (pktmbuf.h:1054-1070) */
    if (hl.l2_len <= m->data_len) {
        m->data_off = (uint16_t)(m->data_off + hl.l2_len);
        m->data_len = (uint16_t)(m->data_len - hl.l2_len);
    }
}

/* eth_rx.c:65-109 eth_pkt_parse */
static void eth_rx_burst(struct chain_ctx *c, struct mb **pkts, uint16_t n_left)
{
    const uint16_t lpid = c->a->lport;
    if (n_left >= 4)
        for (int i = 0; i < 4; i++)
            PF(MTOD(pkts[i]));
    while (n_left >= 4) {
        if (n_left >= 8)
            for (int i = 4; i < 8; i++)
                PF(MTOD(pkts[i]));
        mbuf_update(c, pkts[0], lpid);
        mbuf_update(c, pkts[1], lpid);
        mbuf_update(c, pkts[2], lpid);
        mbuf_update(c, pkts[3], lpid);
        pkts += 4;
        n_left -= 4;
    }
    while (n_left > 0) {
        mbuf_update(c, pkts[0], lpid);
        pkts++;
        n_left--;
    }
}

/* ptype.c:48-210: every mbuf of the burst into the stream of its edge */
static void ptype_burst(struct chain_ctx *c, struct mb **pkts, uint16_t nb, struct mb **st[PTN_MAX],
                        uint16_t cnt[PTN_MAX])
{
    uint16_t left = nb, last_type = c->last_type;
    uint16_t next_index = p_nxt[last_type];
    if (left >= 4)
        for (int i = 0; i < 4; i++)
            PF(MTOD(pkts[i]));
    while (left >= 4) {
        if (left > 11)
            for (int i = 8; i < 12; i++)
                PF(pkts[i]);
        if (left > 7)
            for (int i = 4; i < 8; i++)
                PF(MTOD(pkts[i]));
        const uint16_t l0 = (uint16_t)pkts[0]->packet_type, l1 = (uint16_t)pkts[1]->packet_type,
                       l2 = (uint16_t)pkts[2]->packet_type, l3 = (uint16_t)pkts[3]->packet_type;
        const uint8_t fix_spec = (uint8_t)((last_type ^ l0) | (last_type ^ l1) | (last_type ^ l2) |
                                           (last_type ^ l3));
        if (__builtin_expect(fix_spec != 0, 0)) {
            const uint16_t l[4] = {l0, l1, l2, l3};
            for (int j = 0; j < 4; j++) {
                const uint8_t e = p_nxt[l[j]];
                st[e][cnt[e]++] = pkts[j];
            }
            if (last_type != l3 && l2 == l3 && next_index != p_nxt[l3]) {
                next_index = p_nxt[l3];
                last_type = l3;
            } else if (next_index == p_nxt[l3]) {
                last_type = l3;
            }
        } else {
            for (int j = 0; j < 4; j++)
                st[next_index][cnt[next_index]++] = pkts[j];
        }
        pkts += 4;
        left -= 4;
    }
    while (left > 0) { /* :171-187 */
        const uint16_t l0 = (uint16_t)pkts[0]->packet_type;
        const uint8_t e = (l0 != last_type && p_nxt[l0] != next_index) ? p_nxt[l0] : (uint8_t)next_index;
        st[e][cnt[e]++] = pkts[0];
        pkts++;
        left--;
    }
    c->last_type = last_type;
}

static inline void record(struct mb *m, uint32_t nh, uint32_t edge)
{
    m->udata64 = (uint64_t)edge << 32 | nh;
}

/* ip4_input.c:33-48 ipv4_save_metadata into pktmbuf_metadata(m) = m + 1 */
static inline void ipv4_save_metadata(struct mb *m, const uint8_t *ip)
{
    uint8_t *md = (uint8_t *)(m + 1); /* struct cnet_metadata {faddr, laddr} */
    md[0] = 2; /* AF_INET */
    md[1] = 4;
    memcpy(md + 4, ip + 12, 4);
    md[20] = 2;
    md[21] = 4;
    memcpy(md + 24, ip + 16, 4);
}
static inline void ipv6_save_metadata(struct mb *m, const uint8_t *ip6)
{
    uint8_t *md = (uint8_t *)(m + 1);
    md[0] = 10; /* AF_INET6 */
    md[1] = 16;
    memcpy(md + 4, ip6 + 8, 16);
    md[20] = 10;
    md[21] = 16;
    memcpy(md + 24, ip6 + 24, 16);
}

/* ip4_input.c:50-260 over the ptype node's ip4_input stream */
static void ip4_input_burst(struct chain_ctx *c, struct mb **pkts, uint16_t left)
{
    const struct orc_cnet_chain_args *a = c->a;
    if (left >= 4)
        for (int i = 0; i < 4; i++)
            PF(MTOD(pkts[i]));
    while (left > 0) {
        const uint16_t k = left >= 4 ? 4 : 1; /* 4-wide, then one at a time (:205-240) */
        if (k == 4) {
            if (left > 11)
                for (int i = 8; i < 12; i++)
                    PF(pkts[i]);
            if (left > 7)
                for (int i = 4; i < 8; i++)
                    PF(MTOD(pkts[i]));
        }
        uint32_t dip[4] = {0, 0, 0, 0};
        uint64_t dst[4];
        for (int j = 0; j < k; j++) {
            struct mb *m = pkts[j];
            const uint8_t *ip4 = MTOD(m);
            m->data_len = BE16(ld16(ip4 + 2));
            if (m->data_len < m->buf_len && orc_ipv4_cksum(ip4) == 0)
                dip[j] = __builtin_bswap32(ld32(ip4 + 16));
            ipv4_save_metadata(m, ip4);
        }
        orc_dir24_8_lookup_bulk_pf(a->tbl24, a->tbl8, dip, k, dst);
        for (int j = 0; j < k; j++)
            record(pkts[j], (uint32_t)dst[j], (uint32_t)(dst[j] >> 24));
        pkts += k;
        left = (uint16_t)(left - k);
    }
}

/* trie.h:119-138 LOOKUP_FUNC(4b) */
static void trie_lookup(const uint32_t *t24, const uint32_t *t8, uint8_t ips[][16], uint64_t *nh, int n)
{
    for (int i = 0; i < n; i++) {
        uint32_t e = t24[(uint32_t)ips[i][0] << 16 | (uint32_t)ips[i][1] << 8 | ips[i][2]];
        uint32_t j = 3;
        while (e & 1u)
            e = t8[ips[i][j++] + (e >> 1) * 256u];
        nh[i] = e >> 1;
    }
}

/* ip6_input.c:50-260 over the ptype node's ip6_input stream */
static void ip6_input_burst(struct chain_ctx *c, struct mb **pkts, uint16_t left)
{
    const struct orc_cnet_chain_args *a = c->a;
    if (left >= 4)
        for (int i = 0; i < 4; i++)
            PF(MTOD(pkts[i]));
    while (left > 0) {
        const uint16_t k = left >= 4 ? 4 : 1;
        if (k == 4) {
            if (left > 11)
                for (int i = 8; i < 12; i++)
                    PF(pkts[i]);
            if (left > 7)
                for (int i = 4; i < 8; i++)
                    PF(MTOD(pkts[i]));
        }
        uint8_t dip[4][16];
        uint64_t dst[4];
        memset(dip, 0, sizeof(dip));
        for (int j = 0; j < k; j++) {
            struct mb *m = pkts[j];
            const uint8_t *ip6 = MTOD(m);
            m->data_len = BE16(ld16(ip6 + 4));
            if (m->data_len < m->buf_len)
                memcpy(dip[j], ip6 + 24, 16);
            ipv6_save_metadata(m, ip6);
        }
        trie_lookup(a->tbl24_6, a->tbl8_6, dip, dst, k);
        for (int j = 0; j < k; j++)
            record(pkts[j], (uint32_t)dst[j], (uint32_t)(dst[j] >> 24));
        pkts += k;
        left = (uint16_t)(left - k);
    }
}

/* one graph walk: pktdev_rx's burst -> eth_rx -> ptype -> ip4_input / ip6_input */
static void walk(struct chain_ctx *c, struct mb **pkts, uint32_t i0, uint16_t nb)
{
    const struct orc_cnet_chain_args *a = c->a;
    struct mb *sbuf[PTN_MAX][256];
    struct mb **st[PTN_MAX];
    uint16_t cnt[PTN_MAX] = {0};
    for (uint32_t e = 0; e < PTN_MAX; e++)
        st[e] = sbuf[e];
    for (uint16_t j = 0; j < nb; j++) { /* the fields pktdev_rx delivers */
        pkts[j]->data_off = a->rx_data_off;
        pkts[j]->data_len = a->rx_len[i0 + j];
    }
    eth_rx_burst(c, pkts, nb);
    ptype_burst(c, pkts, nb, st, cnt);
    ip4_input_burst(c, st[PTN_IP4], cnt[PTN_IP4]);
    ip6_input_burst(c, st[PTN_IP6], cnt[PTN_IP6]);
    for (uint32_t e = 0; e < PTN_MAX; e++) /* punt / gtpu_input / drop streams */
        if (e != PTN_IP4 && e != PTN_IP6)
            for (uint16_t j = 0; j < cnt[e]; j++)
                record(st[e][j], NH_INVALID, 0x80u | e);
}

struct chain_shard {
    const struct orc_cnet_chain_args *a;
    uint32_t lo, hi;
    int iters, cpu;
    uint64_t sink;
};

static void *chain_worker(void *arg)
{
    struct chain_shard *s = arg;
    if (s->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(s->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    struct chain_ctx c = {s->a, s->a->state ? *s->a->state : 0, 0};
    const uint32_t B = s->a->burst ? s->a->burst : 256;
    struct mb **mbufs = (struct mb **)(uintptr_t)s->a->mbufs;
    for (int it = 0; it < s->iters; it++)
        for (uint32_t b = s->lo; b < s->hi; b += B)
            walk(&c, mbufs + b, b, (uint16_t)(s->hi - b < B ? s->hi - b : B));
    s->sink = c.sink + c.last_type;
    if (s->a->state && s->lo == 0)
        *s->a->state = c.last_type;
    return NULL;
}

double orc_cnet_chain(const struct orc_cnet_chain_args *a, int nthreads, int iters, const int *cpus)
{
    static pthread_once_t once = PTHREAD_ONCE_INIT;
    pthread_once(&once, tables_init);
    if (!a || !a->mbufs || !a->rx_len || !a->tbl24 || !a->tbl8 || !a->tbl24_6 || !a->tbl8_6)
        return -1.0;
    if ((a->flags & ORC_CHAIN_HASH) && (!a->rss_key || !a->reta || !a->reta_size))
        return -1.0;
    if (a->burst > 256)
        return -1.0;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 512)
        nthreads = 512;
    const uint32_t B = a->burst ? a->burst : 256;
    uint32_t per = (a->n + nthreads - 1) / nthreads;
    per = (per + B - 1) / B * B;
    struct chain_shard *sh = calloc((size_t)nthreads, sizeof(*sh));
    pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
    if (!sh || !th) {
        free(sh);
        free(th);
        return -1.0;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        sh[t].a = a;
        sh[t].lo = (uint64_t)t * per < a->n ? (uint32_t)t * per : a->n;
        sh[t].hi = (uint64_t)sh[t].lo + per < a->n ? sh[t].lo + per : a->n;
        sh[t].iters = iters;
        sh[t].cpu = cpus ? cpus[t] : -1;
        pthread_create(&th[t], NULL, chain_worker, &sh[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(sh);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
