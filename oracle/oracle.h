/*
 * oracle.h -- CPU restatement of CNDP's parse / Toeplitz / LPM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / the timed CPU baseline.  The
 * product (cndp_amd/, libcndp_gpu.so) never links, loads or calls it.
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the CNDP v25.08.0 tree).  Pinning:
 *   - Toeplitz: Microsoft RSS verification vectors (public KAT) + equality
 *     with the reference's own cne_softrss compiled from its header
 *     (oracle/_ref, tests/golden/thash_ref.bin).
 *   - DIR-24-8 / trie lookup arithmetic: equality with the reference's
 *     dir24_8_lookup_bulk_4b / cne_trie_lookup_bulk_4b macros compiled from
 *     their headers (tests/golden/lookup_ref.bin); route-set semantics pinned by
 *     the reference's fib_test.c / fib6_test.c ladders and the 1000-rule
 *     lpm6_data_test.h table with its brute-force get_next_hop oracle.
 *   - IPv4 checksum: equality with the reference's cne_ipv4_cksum.
 *   - cne_get_ptype restatement: PARITY UNPINNED (the reference file
 *     pktmbuf_ptype.c needs libbsd headers absent here and has no tests).
 */
#ifndef CNDP_ORACLE_H
#define CNDP_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Toeplitz (lib/core/hash/cne_thash.h:150-191) ---------------------- */
uint32_t orc_softrss(const uint32_t *tuple, uint32_t len_dw, const uint8_t *key);
uint32_t orc_softrss_be(const uint32_t *tuple, uint32_t len_dw, const uint8_t *key_be);
void orc_convert_rss_key(const uint8_t *orig, uint8_t *targ, int len);

/* ---- IPv4 header checksum (lib/include/net/cne_ip.h:131-214) ----------- */
uint16_t orc_ipv4_cksum(const uint8_t *ip_hdr);

/* ---- LPM brute force (test/testcne/lpm6_data_test.h:1100-1123 idea) ---- */
struct orc_route4 {
    uint32_t ip;    /* host order */
    uint8_t depth;
    uint64_t nh;
};
struct orc_route6 {
    uint8_t ip[16];
    uint8_t depth;
    uint64_t nh;
};
void orc_lpm4_bruteforce(const struct orc_route4 *r, uint32_t nr, uint64_t def_nh,
                         const uint32_t *ips, uint32_t n, uint64_t *out);
void orc_lpm6_bruteforce(const struct orc_route6 *r, uint32_t nr, uint64_t def_nh,
                         const uint8_t (*ips)[16], uint32_t n, uint64_t *out);

/* ---- DIR-24-8, 4-byte entries (lib/usr/clib/fib/dir24_8.h:118-148) ------
 * Independent table painter (routes sorted by depth, ranges painted) so the
 * product's incremental RIB-driven builder is checked against a different
 * construction.  tbl24 has 1<<24 entries; tbl8 has (num_tbl8+1)*256. */
int orc_dir24_8_build(const struct orc_route4 *r, uint32_t nr, uint64_t def_nh,
                      uint32_t num_tbl8, uint32_t *tbl24, uint32_t *tbl8);
void orc_dir24_8_lookup(const uint32_t *tbl24, const uint32_t *tbl8, const uint32_t *ips,
                        uint32_t n, uint64_t *nh);

/* ---- IPv6 trie, 4-byte entries (lib/usr/clib/fib/trie.h:119-138) ------- */
int orc_trie_build(const struct orc_route6 *r, uint32_t nr, uint64_t def_nh,
                   uint32_t num_tbl8, uint32_t *tbl24, uint32_t *tbl8);
void orc_trie_lookup(const uint32_t *tbl24, const uint32_t *tbl8, const uint8_t (*ips)[16],
                     uint32_t n, uint64_t *nh);

/* ---- cne_get_ptype (lib/core/pktmbuf/pktmbuf_ptype.c:472-744) ---------- */
struct orc_hdr_lens {
    uint8_t l2_len;
    uint8_t inner_l2_len;
    uint16_t l3_len;
    uint16_t inner_l3_len;
    uint16_t tunnel_len;
    uint8_t l4_len;
    uint8_t inner_l4_len;
};
/* bytes at pkt[avail..] read as 0 (bounded view) */
uint32_t orc_get_ptype(const uint8_t *pkt, uint64_t avail, struct orc_hdr_lens *hl, uint32_t layers);

/* ---- hot path: build-defined flow hash / queue / bins + node semantics --
 * Layout of one packet: slab + (offsets ? offsets[i] : i*stride) + data_off.
 * mode CNDP_MODE_L3FWD: pktdev_rx soft parse (pktdev_rx.c:24-34) -> pkt_cls
 * (pkt_cls.c:19-31) -> ip4_lookup (ip4_lookup.c:108-154).
 * mode CNDP_MODE_CNET: eth_rx (eth_rx.c:35-63) -> ptype (ptype.c:32-46) ->
 * ip4_input (ip4_input.c:108-154) / ip6_input (ip6_input.c:108-150).
 * mode CNDP_MODE_HASH: parse + Toeplitz + queue only (config 2).
 * Outputs: nh[i] (u32 FIB value or 0xFFFFFFFF), hash[i], queue[i],
 * bins[n_bins + 2] (+= counts), edge[i] (final graph edge, optional). */
struct orc_classify_args {
    uint32_t mode;
    const uint8_t *slab;
    uint64_t slab_len;          /* bytes past the slab end read as 0 */
    uint64_t stride;
    const uint64_t *offsets;
    uint32_t data_off;
    uint32_t n;
    uint32_t buf_len;           /* pktmbuf buf_len for cnet length checks */
    const uint32_t *tbl24;      /* v4 DIR-24-8 */
    const uint32_t *tbl8;
    const uint32_t *tbl24_6;    /* v6 trie */
    const uint32_t *tbl8_6;
    const uint8_t *rss_key;     /* 40 bytes, NIC byte order */
    const uint16_t *reta;
    uint32_t reta_size;         /* power of two */
    uint32_t n_bins;
    uint32_t *nh;
    uint32_t *hash;
    uint16_t *queue;
    uint8_t *edge;              /* may be NULL */
    uint64_t *bins;             /* may be NULL */
    uint32_t *ptype;            /* may be NULL: m->packet_type (eth_rx.c:41 / pktdev_rx.c:24-34) */
    uint32_t *rxmeta;           /* may be NULL (cnet): eth_rx.c:43-60 lengths + ol_flags, packed
                                 * as in cndp_gpu.h */
    uint32_t spec_burst;        /* cnet: 0 = route by p_nxt[ptype] per packet; B > 0 = the
                                 * ptype node's speculative 4-wide loop (ptype.c:48-210) over
                                 * graph bursts of B packets, uint8_t fix_spec quirk included */
    uint16_t *spec_state;       /* in/out: the node's ctx->last_type (NULL = start at 0) */
    uint32_t no_hash;           /* 1: skip the build's flow hash (hash 0, queue reta[0]) -- the
                                 * reference's own chain runs no Toeplitz */
};
int orc_classify(const struct orc_classify_args *a);

/* Per-burst restatement of the l3fwd node loop over pktmbuf-style pointer
 * arrays (256-pkt bursts, ip4_lookup.c:83-241), used as the CPU baseline.
 * Multi-threaded over nthreads contiguous shards; returns elapsed seconds. */
double orc_l3fwd_burst_bench(const struct orc_classify_args *a, int nthreads, int iters);
double orc_burst_bench(const struct orc_classify_args *a, int nthreads, int iters, const int *cpus);
/* receive-driver header writes before each burst of the mbuf node loops (oracle.c) */
void orc_set_driver_writes(int on);
double orc_ip4_lookup_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                            const uint32_t *tbl8, int iters);
double orc_rx_ip4_lookup_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                               const uint32_t *tbl8, int iters);

/* ---- the cnet chain as a graph walk runs it (oracle/cnet_chain.c) --------
 * eth_rx -> ptype -> ip4_input / ip6_input per burst over pktmbuf_t pointer
 * arrays, direct loads and the nodes' prefetching; the CPU baseline of C4/C5
 * and of the cnet node boundary.  Each mbuf needs 64 B of cnet_metadata
 * after its header (pktmbuf_metadata's default).  mbufs[i] gets data_off =
 * rx_data_off and data_len = rx_len[i] before each pass (pktdev_rx).  Results:
 * m->packet_type, ol_flags, tx_offload, lport, data_off/data_len, metadata,
 * m->hash (ORC_CHAIN_HASH) and m->udata64 = edge << 32 | nh.  Shards over
 * nthreads (pinned to cpus[t] when given); returns seconds for iters passes. */
#define ORC_CHAIN_HASH 1u
struct orc_cnet_chain_args {
    void *const *mbufs;
    uint32_t n;
    uint32_t burst;             /* graph burst, <= 256 (0 = 256) */
    const uint16_t *rx_len;     /* frame length of mbufs[i] */
    uint16_t rx_data_off;
    uint16_t lport;
    uint32_t flags;             /* ORC_CHAIN_* */
    const uint32_t *tbl24, *tbl8;     /* rt4 DIR-24-8 4 B */
    const uint32_t *tbl24_6, *tbl8_6; /* rt6 trie 4 B */
    const uint8_t *rss_key;
    const uint16_t *reta;
    uint32_t reta_size;
    uint16_t *state;            /* in/out ptype ctx->last_type (thread 0's), or NULL */
};
double orc_cnet_chain(const struct orc_cnet_chain_args *a, int nthreads, int iters, const int *cpus);
void orc_dir24_8_lookup_bulk_pf(const uint32_t *tbl24, const uint32_t *tbl8, const uint32_t *ips, uint32_t n,
                                uint64_t *nh);

/* ip4_rewrite node (ip4_rewrite.c:40-247) over a batch cut into graph
 * bursts of `burst` packets.  nh[i] is the l3fwd classify output (edge << 16
 * | nh, CNDP_NH_INVALID for non-IPv4); packets with edge 0 form the
 * rewrite stream of their burst, in order.  For each: memcpy of the next
 * hop's rewrite data to the frame start, TTL - 1, checksum + 0x0100 with
 * the 4-wide loop's end-around carry (:97-100,104) for the first
 * (cnt & ~3) packets of the stream and the tail loop's rule (:214-216) for
 * the rest; tx_edge[i] = the next hop's tx node (0xFFFF when the packet is
 * not in a rewrite stream).  Next hops >= 64 behave as unset entries. */
struct orc_rewrite_nh {
    uint16_t rewrite_len;
    uint16_t tx_node;
    uint16_t enabled;
    uint16_t rsvd;
    uint8_t rewrite_data[56];
};
double orc_l3rx_chain_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                            const uint32_t *tbl8, int iters, uint16_t *edges, const struct orc_rewrite_nh *rwt);
void orc_ip4_rewrite(uint8_t *slab, uint64_t slab_len, uint64_t stride, const uint64_t *offsets,
                     uint32_t data_off, uint32_t n, const uint32_t *nh, uint32_t burst,
                     const struct orc_rewrite_nh *tbl, uint16_t *tx_edge);

/* ip4_rewrite_node_process over one burst of pktmbuf_t pointers (nb_objs = n) */
void orc_ip4_rewrite_node(void *const *mbufs, uint32_t n, const struct orc_rewrite_nh *tbl, uint16_t *tx_edge);
/* ip4_lookup then ip4_rewrite per burst on one core (seconds for iters passes) */
double orc_l3fwd_nodes_mbufs(void *const *mbufs, uint32_t n, uint32_t burst, const uint32_t *tbl24,
                             const uint32_t *tbl8, const struct orc_rewrite_nh *tbl, int iters);

/* cndpfwd loopback: swap_mac_addresses (examples/cndpfwd/main.h:303-315)
 * on every frame of the batch. */
void orc_mac_swap(uint8_t *slab, uint64_t slab_len, uint64_t stride, const uint64_t *offsets,
                  uint32_t data_off, uint32_t n);

/* splitmix64 packet generator shared by tests and bench (seed 0x43444E50). */
uint64_t orc_splitmix64(uint64_t *state);

#ifdef __cplusplus
}
#endif
#endif
