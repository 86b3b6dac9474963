/*
 * cndp_gpu.h -- batch parse + flow-hash + LPM classify on MI355X (libcndp_gpu.so).
 *
 * This is the data-plane half of the drop-in boundary.  It replaces, for a
 * batch of many bursts at once, the per-burst arithmetic of these reference
 * graph nodes (CNDP v25.08.0):
 *
 *   mode CNDP_MODE_L3FWD  (examples/l3fwd-graph chain)
 *     pktdev_rx soft parse   lib/usr/clib/nodes/pktdev_rx.c:24-34,37-103
 *     pkt_cls  classify      lib/usr/clib/nodes/pkt_cls.c:19-31,34-182
 *     ip4_lookup             lib/usr/clib/nodes/ip4_lookup.c:48-256
 *       -> cne_fib_lookup_bulk (DIR-24-8 4B) lib/usr/clib/fib/dir24_8.h:118-148
 *   mode CNDP_MODE_CNET   (examples/cnet-graph chain)
 *     eth_rx  (cne_get_ptype) lib/cnet/eth/eth_rx.c:35-63,
 *                             lib/core/pktmbuf/pktmbuf_ptype.c:472-744
 *     ptype                   lib/cnet/ptype/ptype.c:32-46,48-210
 *     ip4_input (len+cksum)   lib/cnet/ipv4/ip4_input.c:50-260
 *     ip6_input               lib/cnet/ipv6/ip6_input.c:52-260
 *       -> cne_fib6_lookup_bulk (trie 4B) lib/usr/clib/fib/trie.h:119-138
 *   mode CNDP_MODE_HASH   parse + Toeplitz + RSS queue only (config 2)
 *   flow hash in every mode: cne_softrss (lib/core/hash/cne_thash.h:150-163)
 *   over the NIC-style 5-tuple (cne_ipv4_tuple / cne_ipv6_tuple, :68-97).
 *
 * Packet i lives at slab + (offsets ? offsets[i] : i * stride) + data_off,
 * i.e. a frame slab indexed like an AF_XDP UMEM (2 KiB frames, data at
 * +256) or a packed slab (64-B slots).  Bytes at or past slab + slab_len
 * read as zero.  All batch pointers are DEVICE pointers (hipMalloc / torch);
 * work is enqueued on `stream` (a hipStream_t, NULL = null stream) and the
 * call returns without waiting.  Errors are negative errno values.  Calls on
 * one context that share its scratch (cnet mode, the bin partition) are
 * ordered across streams: a call on another stream than the previous one's
 * first waits for that stream, so a stream given to such a call must stay
 * alive until the next such call on another stream (or cndp_gpu_fini), or be
 * handed back with cndp_gpu_stream_release before it is destroyed.
 *
 * Per-packet outputs (SoA, any may be NULL except as noted):
 *   nh[i]    u32 FIB value (l3fwd: edge<<16 | nh id; cnet: edge<<24 | idx),
 *            CNDP_NH_INVALID when the packet never reached a lookup
 *   hash[i]  u32 Toeplitz flow hash (0 for non-IP)
 *   queue[i] u16 RSS queue = reta[hash & (reta_size - 1)]
 *   edge[i]  u8  final graph edge
 *   bins[n_bins + 2] u64 counters, accumulated (+=): next-hop bins
 *            [0, n_bins), drops at n_bins, everything else at n_bins + 1.
 */
#ifndef CNDP_GPU_H
#define CNDP_GPU_H

#include <stdint.h>

#include "cndp_fib.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CNDP_MODE_L3FWD 0u
#define CNDP_MODE_CNET 1u
#define CNDP_MODE_HASH 2u

#define CNDP_NH_INVALID 0xFFFFFFFFu
#define CNDP_EDGE_CLS_DROP 0xFFu /* l3fwd: pkt_cls sent the packet to pkt_drop */
#define CNDP_RSS_KEY_LEN 40u
#define CNDP_RETA_MAX 512u
#define CNDP_BINS_MAX 1024u

typedef struct cndp_gpu_ctx cndp_gpu_ctx_t;

struct cndp_batch {
    uint32_t mode;          /* CNDP_MODE_* */
    uint32_t n;             /* packets */
    const void *slab;       /* device */
    uint64_t slab_len;      /* bytes readable from slab */
    uint64_t stride;        /* used when offsets == NULL */
    const uint64_t *offsets; /* device, optional: byte offset of frame i */
    uint32_t data_off;      /* added to every frame offset (pktmbuf data_off) */
    uint32_t buf_len;       /* pktmbuf buf_len (cnet length checks), e.g. 1984 */
    uint32_t *nh;           /* device outputs, see above */
    uint32_t *hash;
    uint16_t *queue;
    uint8_t *edge;
    uint64_t *bins;
    uint32_t n_bins;        /* <= CNDP_BINS_MAX */
    uint32_t *ptype;        /* optional out: m->packet_type -- cnet: cne_get_ptype
                             * (eth_rx.c:41); l3fwd / hash: pktdev_rx's l3_ptype */
    uint32_t *rxmeta;       /* optional out (cnet): the rest of eth_rx's mbuf_update
                             * (eth_rx.c:43-60): bits 0-23 = tx_offload's l2_len:7 |
                             * l3_len:9 | l4_len:8, bits 29-31 = ol_flags >> 32
                             * (MCAST, BCAST, IPv6); lengths the reference leaves
                             * unset are 0 */
};
#define CNDP_RXMETA_L2(m) ((m) & 0x7fu)
#define CNDP_RXMETA_L3(m) (((m) >> 7) & 0x1ffu)
#define CNDP_RXMETA_L4(m) (((m) >> 16) & 0xffu)

/* Create / destroy a context bound to HIP device `device` (-1 = current). */
int cndp_gpu_init(int device, cndp_gpu_ctx_t **out);
void cndp_gpu_fini(cndp_gpu_ctx_t *ctx);
int cndp_gpu_device(const cndp_gpu_ctx_t *ctx);

/* RSS configuration: 40-byte Toeplitz key in NIC byte order (NULL keeps the
 * Microsoft default key) and a redirection table (NULL = reta[i] = i % nb_q
 * with reta_size 128).  reta_size must be a power of two <= CNDP_RETA_MAX. */
int cndp_gpu_set_rss(cndp_gpu_ctx_t *ctx, const uint8_t *key, uint32_t key_len,
                     const uint16_t *reta, uint32_t reta_size, uint32_t nb_queues);

/* Bind the FIBs used by classify (fib6 may be NULL unless mode CNET).
 * The tables must be DIR-24-8 4B / trie 4B (the l3fwd and cnet layouts). */
int cndp_gpu_set_fib(cndp_gpu_ctx_t *ctx, struct cne_fib *fib4, struct cne_fib6 *fib6);

/* Enqueue one classify pass over a device-resident batch. */
int cndp_gpu_classify(cndp_gpu_ctx_t *ctx, const struct cndp_batch *b, void *stream);

/* Hand back a stream before destroying it: if the context's last
 * scratch-sharing call ran on `stream`, the ordering point is recorded on it
 * now, so the next call (on any stream) waits for that work without touching
 * `stream` again.  A no-op for any other stream. */
int cndp_gpu_stream_release(cndp_gpu_ctx_t *ctx, void *stream);

/* Same over HOST buffers (an AF_XDP UMEM, socket buffers): the slab is
 * streamed into a device mirror in 64 MiB segments while earlier packet
 * chunks are classified and their results copied back (three streams), and
 * the call waits.  Results equal cndp_gpu_classify on a device copy.  Pinned
 * memory (cndp_gpu_host_register, hipHostMalloc) gives full PCIe rate;
 * pageable memory works at the driver's staging rate. */
int cndp_gpu_classify_host(cndp_gpu_ctx_t *ctx, const struct cndp_batch *host_batch);

/* pktmbuf shim for l3fwd-graph: one call per graph burst (or batch of
 * bursts) of pktmbuf_t pointers in host memory.  Runs pktdev_rx's ptype
 * parse (pktdev_rx.c:24-34), pkt_cls (pkt_cls.c:19-31) and ip4_lookup
 * (ip4_lookup.c:48-256) on the GPU and writes back what those nodes write:
 * m->packet_type, m->udata64 = node_mbuf_priv1 {nh, ttl, cksum}
 * (node_private.h:24-35), plus m->hash (the flow hash, build-defined) when
 * CNDP_TUNE_MBUF_HASH is set.
 * edges[i] = the ip4_lookup next edge (val >> 16: 0 rewrite, 1 drop), or
 * CNDP_MBUF_EDGE_CLS_DROP when pkt_cls sends the frame to pkt_drop.  Header
 * windows are gathered into pinned staging, classified, and the call waits
 * on `stream`.  mbufs: pktmbuf_t layout of pktmbuf.h:102-204. */
#define CNDP_MBUF_EDGE_CLS_DROP 0xFFFFu
int cndp_gpu_l3fwd_mbufs(cndp_gpu_ctx_t *ctx, void *const *mbufs, uint32_t n, uint16_t *edges,
                         void *stream);

/* ---- asynchronous node path over pktmbuf_t bursts (cndp_gpu_mq_*) -------
 * The graph-node boundary without a PCIe round trip per burst: a node's
 * process() callback hands each burst of pktmbuf_t pointers to
 * cndp_gpu_mq_submit, which never waits; bursts collect into a batch, whole
 * batches run on the GPU on the queue's own stream (up to `depth` in flight,
 * double-buffered pinned staging), and cndp_gpu_mq_poll returns finished
 * mbufs -- with every field the replaced nodes write already written back --
 * plus the next edge of each, in submission order.  A graph's source node
 * (node/ip4_lookup_gpu.c) polls once per walk, which also launches a partly
 * filled batch when it is older than max_delay_us, or when the GPU has
 * nothing in flight and the batch holds batch / 2 mbufs or is older than
 * max_delay_us / 2.
 *
 * Frame bytes: when conf.umem names a region registered with
 * cndp_gpu_host_register (the AF_XDP UMEM / pktmbuf pool, cne_lport.h:91),
 * the queue works in place (zero-copy) over every region the context holds:
 * the host reads each mbuf's header line -- the node handing the burst over
 * has just touched it -- and passes the frame address (buf_addr + data_off),
 * and the kernels read the frame bytes where they lie and write the results
 * straight into the mbuf.  An mbuf or frame outside every registered region
 * comes back untouched with edge CNDP_MQ_EDGE_NONE (cnet: the frames of one
 * batch must share a region -- one pool per port -- others come back the
 * same way).  With conf.umem NULL,
 * the host copies each frame into pinned staging (ip4_lookup: 64 B, enough for
 * every byte the node reads; cnet: 128 B for a frame whose header walk stays
 * there -- Ethernet with at most one tag, then IPv4 or IPv6 without extension
 * headers carrying TCP / UDP / SCTP, an IPv4 fragment, ARP or MPLS -- else the
 * buffer from data_off to buf_len, at most conf.stage_max bytes) and poll
 * writes the results back.  Bytes past a frame's buffer, which the reference
 * parse reads only for malformed extension-header lengths, are the next
 * staged frame's here (undefined in the reference either way).
 * Completion is a flag the batch's last kernel raises in pinned memory, so
 * poll costs a load, not a HIP call.  A batch whose launch fails comes back
 * from poll with every edge CNDP_MQ_EDGE_NONE, so each accepted mbuf has one
 * owner; the error is returned by the next submit.
 *
 * Modes and what is written back (pktmbuf_t layout, pktmbuf.h:102-204):
 *   CNDP_MQ_IP4_LOOKUP  the ip4_lookup node (ip4_lookup.c:48-256): udata64 =
 *                       node_mbuf_priv1 {nh, ttl, cksum} (node_private.h:24-35);
 *                       edge = FIB value >> 16 (0 ip4_rewrite, 1 pkt_drop).
 *                       The FIB is the context's fib4 (normally
 *                       cndp_node_ip4_lookup_fib()).
 *   CNDP_MQ_CNET        eth_rx (eth_rx.c:35-63) + ptype (ptype.c:48-210, its
 *                       4-wide speculation with the uint8_t fix_spec quirk over
 *                       the submitted bursts, node state kept in the context)
 *                       + ip4_input / ip6_input (length + checksum, FIB):
 *                       packet_type, ol_flags, tx_offload l2/l3/l4_len, lport,
 *                       data_off/data_len as pktmbuf_adj_offset(l2_len), then
 *                       data_len = total_length / payload_len for frames an
 *                       input node took.  edge = CNDP_MQ_EDGE(node, e): node
 *                       CNDP_MQ_NODE_PTYPE with e = the ptype edge (pkt_drop 0,
 *                       punt 2, gtpu 5), or CNDP_MQ_NODE_IP4 / _IP6 with e =
 *                       the input node's edge (drop 0, forward 1, proto 2).
 *                       Frames an input node takes also get its cnet_metadata
 *                       (ipv4/ipv6_save_metadata, ip4_input.c:33-48,
 *                       ip6_input.c:32-48): faddr / laddr {family, len, addr}
 *                       at pktmbuf_metadata(m) -- conf.metadata(m) when set
 *                       (the node passes pktmbuf_metadata), else m + 64, its
 *                       default -- unless CNDP_MQ_F_NO_METADATA.
 *                       Each submit call is one graph burst (<= 256 mbufs;
 *                       larger calls are cut into 256s).
 *   CNDP_MQ_MAC_SWAP    cndpfwd's loopback mode (examples/cndpfwd/main.c:317-339):
 *                       destination and source MAC swapped in the frame
 *                       (swap_mac_addresses, main.h:303-315); edge 0 (tx).
 *                       Needs no FIB.
 *   CNDP_MQ_IP4_REWRITE the ip4_rewrite node (ip4_rewrite.c:40-247) per submitted
 *                       burst: the next hop's rewrite data at mtod, TTL - 1 and
 *                       the checksum + htons(0x0100) from node_mbuf_priv1 in
 *                       udata64 (the 4-wide loop's end-around carry for the
 *                       first nb & ~3 mbufs of the burst, the tail loop's rule
 *                       for the rest); edge = the next hop's tx_node
 *                       (cne_node_ip4_rewrite_add / ip4_rewrite_set_next, the
 *                       process-global table unless the context has its own).
 *   flag CNDP_MQ_F_HASH also store the Toeplitz flow hash in m->hash (no
 *                       reference node writes it, so it is off by default).
 */
typedef struct cndp_gpu_mq cndp_gpu_mq_t;

#define CNDP_MQ_IP4_LOOKUP 0u
#define CNDP_MQ_CNET 1u
#define CNDP_MQ_MAC_SWAP 2u
#define CNDP_MQ_IP4_REWRITE 3u
#define CNDP_MQ_F_HASH (1u << 0)
#define CNDP_MQ_F_NO_METADATA (1u << 1) /* cnet: leave cnet_metadata unwritten */
/* Zero-copy ip4_lookup and cnet: the host hands over mbuf pointers only and
 * the kernels read each header (buf_addr, data_off, the lengths) in place --
 * no host touch per mbuf, dependent PCIe reads per mbuf instead of one.
 * ip4_lookup: frames in any region the context registered.  cnet: a batch's
 * region is its first mbuf's (frames elsewhere come back with
 * CNDP_MQ_EDGE_NONE), and cnet_metadata is written by the device for the
 * mbufs of pools whose conf.metadata(m) is m + 64 -- learnt per pool
 * (pooldata, header word 0) from the first mbuf of a burst, so the hook must
 * depend on the mbuf's pool only, as pktmbuf_metadata does -- and by poll
 * through the hook for the others.  The default of the GPU ip4_lookup and
 * ip4_rewrite nodes, whose host thread, not the device, bounds the node rate;
 * not of eth_rx, whose batch the extra header pass over PCIe slows more than
 * the host saves. */
#define CNDP_MQ_F_DEVICE_HEADERS (1u << 2)
/* ip4_lookup: the l3fwd-graph receive chain in front of it too -- pktdev_rx's
 * soft parse (eth_pkt_parse_cb, pktdev_rx.c:24-34, :37-103: packet_type =
 * l3_ptype(ether_type, 0), written into the mbuf) and pkt_cls (pkt_cls.c:19-31:
 * only IPv4 goes on to ip4_lookup); an mbuf pkt_cls sends to pkt_drop comes
 * back with edge CNDP_MQ_EDGE_CLS_DROP and its udata64 untouched.  For a source
 * node that replaces pktdev_rx -> pkt_cls -> ip4_lookup (pktdev_rx_gpu.c). */
#define CNDP_MQ_F_RX_PARSE (1u << 3)
#define CNDP_MQ_EDGE_CLS_DROP 0xFFFEu
/* ip4_lookup, zero-copy only: ip4_rewrite too (ip4_rewrite.c:40-247) over
 * the mbufs ip4_lookup sends to it, per submitted burst -- the burst's first
 * (its count & ~3) of them take the 4-wide loop's checksum rule, the rest the
 * tail's, as when ip4_rewrite gets that burst's stream in one call -- with
 * the rewrite data, TTL and checksum written into the frame; edge = the next
 * hop's tx_node (ip4_rewrite's edge index, 0 pkt_drop); an mbuf ip4_lookup
 * sent elsewhere (pkt_drop) comes back with CNDP_MQ_EDGE_LOOKUP_DROP. */
#define CNDP_MQ_F_REWRITE (1u << 4)
/* cnet and ip4_lookup, zero-copy with host headers: the kernels still read
 * each frame in place, but the results -- cnet: the fields eth_rx and the
 * input nodes write and the cnet_metadata addresses; ip4_lookup: udata64 and,
 * with CNDP_MQ_F_RX_PARSE, packet_type -- come back as coalesced records that
 * poll writes into the mbufs on the calling lcore, instead of small posted
 * stores a mbuf from the device (cnet three to five, ip4_lookup one or two).
 * The device's PCIe transaction rate, which bounds the zero-copy forms summed
 * over lcores, then carries one read a frame (plus, with CNDP_MQ_F_REWRITE,
 * the frame's rewrite); the lcores' writes scale with the lcores (DESIGN.md
 * §6).  Same fields, same values.  cnet: -EINVAL with CNDP_MQ_F_DEVICE_HEADERS
 * (poll reads the header fields it adjusts); ip4_lookup takes both (the device
 * reads header and frame, poll only stores). */
#define CNDP_MQ_F_HOST_WRITEBACK (1u << 5)
#define CNDP_MQ_EDGE_LOOKUP_DROP 0xFFFDu
#define CNDP_MQ_NODE_PTYPE 0u
#define CNDP_MQ_NODE_IP4 1u
#define CNDP_MQ_NODE_IP6 2u
#define CNDP_MQ_EDGE(node, e) ((uint16_t)(((node) << 8) | (e)))
#define CNDP_MQ_EDGE_NONE 0xFFFFu
#define CNDP_MQ_DEPTH_MAX 16u

struct cndp_mq_conf {
    uint32_t mode;         /* CNDP_MQ_* */
    uint32_t flags;        /* CNDP_MQ_F_* */
    uint32_t batch;        /* mbufs per GPU launch, >= 256 (0 = 8192) */
    uint32_t depth;        /* batches in flight, 2..16 (0 = 4) */
    uint32_t max_delay_us; /* a partly filled batch launches at this age (0 = 50 us) */
    uint32_t stage_max;    /* cnet staged mode: most bytes copied per frame (0 = 2048) */
    void *umem;            /* registered region the mbufs live in, or NULL */
    uint16_t lport;        /* cnet: m->lport (eth_rx.c:59) */
    uint16_t rsvd[3];
    /* cnet: pktmbuf_metadata(m) (pktmbuf.h:1209-1220), or NULL for its
     * default m + sizeof(pktmbuf_t) */
    void *(*metadata)(const void *m);
};

int cndp_gpu_mq_create(cndp_gpu_ctx_t *ctx, const struct cndp_mq_conf *conf, cndp_gpu_mq_t **out);
/* Waits for batches in flight; mbufs not yet polled are simply forgotten. */
void cndp_gpu_mq_free(cndp_gpu_mq_t *q);
/* Accepts up to n mbufs (a graph burst), returns how many (0 when every
 * batch slot is in flight or waiting to be polled), or a negative errno
 * (-EINVAL: bad arguments; a failed launch: its HIP error as -EIO / -ENOMEM,
 * returned by the call after the one that accepted the batch's mbufs). */
int cndp_gpu_mq_submit(cndp_gpu_mq_t *q, void *const *mbufs, uint32_t n);
/* Launch the partly filled batch now (no-op when empty). */
int cndp_gpu_mq_flush(cndp_gpu_mq_t *q);
/* Never waits: up to max finished mbufs and their edges, oldest first. */
int cndp_gpu_mq_poll(cndp_gpu_mq_t *q, void **mbufs, uint16_t *edges, uint32_t max);
/* Block until the oldest batch in flight has finished (0 if none). */
int cndp_gpu_mq_wait(cndp_gpu_mq_t *q);
/* mbufs accepted and not yet returned by poll. */
uint32_t cndp_gpu_mq_pending(const cndp_gpu_mq_t *q);
/* Counters since create: batches launched (CNDP_MQ_STAT_BATCHES) and the
 * mbufs in them (CNDP_MQ_STAT_MBUFS); -EINVAL for an unknown key. */
#define CNDP_MQ_STAT_BATCHES 1
#define CNDP_MQ_STAT_MBUFS 2
int64_t cndp_gpu_mq_stat(const cndp_gpu_mq_t *q, int key);

/* ip4_rewrite node on the device (ip4_rewrite.c).  Control plane mirrors
 * ip4_rewrite_set_next (:252-263) and cne_node_ip4_rewrite_add (:265-295):
 * next_hop < 64, rewrite_len <= 56, the dst_port must have a next index,
 * else -EINVAL.  cndp_gpu_ip4_rewrite rewrites the device slab of `b` IN
 * PLACE for the packets whose l3fwd classify value b->nh[i] has edge 0:
 * rewrite data at the frame start, TTL - 1, checksum + 0x0100 with the
 * reference's 4-wide / tail loop rules inside each graph burst of `burst`
 * packets; tx_edge[i] (device, may be NULL) = the next hop's tx node, or
 * 0xFFFF for packets that do not go through ip4_rewrite. */
int cndp_gpu_ip4_rewrite_set_next(cndp_gpu_ctx_t *ctx, uint16_t port_id, uint16_t next_index);
int cndp_gpu_ip4_rewrite_add(cndp_gpu_ctx_t *ctx, uint16_t next_hop, const uint8_t *rewrite_data,
                             uint8_t rewrite_len, uint16_t dst_port);
int cndp_gpu_ip4_rewrite(cndp_gpu_ctx_t *ctx, const struct cndp_batch *b, uint32_t burst,
                         uint16_t *tx_edge, void *stream);

/* The whole l3fwd-graph data path in one call: classify (CNDP_MODE_L3FWD,
 * b->nh required) then ip4_rewrite as above.  Packed 64-B slots in
 * 256-packet bursts run as ONE fused kernel (the rewrite is applied to the
 * frame tile already staged in LDS); other layouts run the two kernels. */
int cndp_gpu_classify_rewrite(cndp_gpu_ctx_t *ctx, const struct cndp_batch *b, uint32_t burst,
                              uint16_t *tx_edge, void *stream);

/* cndpfwd loopback (examples/cndpfwd/main.c:317-339): swap the Ethernet
 * destination and source addresses of every frame of the device slab. */
int cndp_gpu_mac_swap(cndp_gpu_ctx_t *ctx, const struct cndp_batch *b, void *stream);

/* Pin and map host memory for the device (zero-copy ingest: pass *dev_ptr
 * as cndp_batch.slab to cndp_gpu_classify and the kernel reads the frames
 * over PCIe in place).  Registration is process-wide and reference counted:
 * registering a region another context (or the application) registered
 * takes a reference and returns 0; each unregister (and cndp_gpu_fini) drops
 * one, the last one registered here unregisters.  -EEXIST for a larger range
 * at an address already registered. */
int cndp_gpu_host_register(cndp_gpu_ctx_t *ctx, void *ptr, uint64_t len, void **dev_ptr);
int cndp_gpu_host_unregister(cndp_gpu_ctx_t *ctx, void *ptr);

/* Device frame memory for device-resident batches (the receive ring a NIC's
 * peer DMA or a host copy fills; cndp_batch.slab points into it): HBM of
 * device `device` (-1 = current), uncached on the GPU by default, so a peer's
 * writes need no GPU cache maintenance and the classify kernels' 64-B window
 * reads allocate no L2 lines (faster for IMIX / jumbo strides).
 * CNDP_FRAMES_CACHED: plain device memory.  The calling thread's current device is
 * unchanged.  -EINVAL, -ENODEV, -ENOMEM, -EIO. */
#define CNDP_FRAMES_CACHED 1u
int cndp_gpu_frames_alloc(int device, uint64_t bytes, uint32_t flags, void **dptr);
int cndp_gpu_frames_free(void *dptr);

/* Stable partition of packet indices by bin (the per-edge streams a graph
 * walk would build): bin_of[i] in [0, n_bins+2) (device), outputs
 * bin_start[n_bins+3] (exclusive prefix, device) and order[n] (device).
 * The result equals a stable counting sort of i by bin_of[i]. */
int cndp_gpu_bin_partition(cndp_gpu_ctx_t *ctx, const uint16_t *bin_of, uint32_t n,
                           uint32_t n_bins, uint32_t *bin_start, uint32_t *order, void *stream);

/* Bin id per packet as counted in cndp_batch.bins, from classify outputs. */
int cndp_gpu_bin_ids(cndp_gpu_ctx_t *ctx, uint32_t mode, const uint32_t *nh, const uint8_t *edge,
                     const uint16_t *queue, uint32_t n, uint32_t n_bins, uint16_t *bin_of,
                     void *stream);

/* Kernel variant knobs (performance only; results never change):
 *   CNDP_TUNE_NT            1 = non-temporal hint on the once-touched streams: frame loads
 *                           and output stores (per-lane kernel), output stores only
 *                           (wave-tile kernels) (default 1)
 *   CNDP_TUNE_UNROLL        packets per lane per loop trip: 1 (the only value kept)
 *   CNDP_TUNE_BLOCKS_PER_CU grid = CUs x this, grid-stride beyond (default 0 = auto:
 *                           1 512-thread block for the balanced streamed wave-tile kernel,
 *                           2 for the static one, 4 for the others)
 *   CNDP_TUNE_TILE          l3fwd/hash kernel for packed 64-B slots: 1 = streamed wave tile
 *                           (frames two tiles ahead, each FIB gather level one loop trip
 *                           apart; default), 0 = the per-lane kernel every other layout
 *                           (strided UMEM frames, IMIX offsets) uses
 *   CNDP_TUNE_DIR16         1 = resolve IPv4 lookups through the L2-resident /16 directory
 *                           kept in front of tbl24 (default 1)
 *   CNDP_TUNE_CNET_TILE     cnet kernel: 1 = deferred-chain wave tile (fast path, the FIB
 *                           chain of each tile finished one loop trip later, two window
 *                           tiles in flight) + the general per-lane parse of the frames it
 *                           leaves (default), 0 = the general per-lane parse for every frame
 *   CNDP_TUNE_HOST_CHUNK    packets per pipelined chunk of cndp_gpu_classify_host
 *                           (>= 1024, default 1M)
 *   CNDP_TUNE_CNET_SPEC     cnet: graph burst size B of the ptype node's speculative
 *                           4-wide loop (ptype.c:48-210, uint8_t fix_spec quirk
 *                           included); the node state (last_type) persists across calls
 *                           and restarts at 0 on the next call after this key is set.
 *                           0 = route every frame by p_nxt[its type] instead (default 256)
 *   CNDP_TUNE_RW_WB         fused classify+rewrite write-back: 0 = the 16-B parts the
 *                           rewrite touches of rewritten frames, 1 = whole rewritten
 *                           frames, 2 = whole tiles holding a rewrite (default: full
 *                           coalesced lines beat partial-line writes on HBM)
 *   CNDP_TUNE_LOAD_NT       wave-tile kernels: 1 = frame tiles loaded with the
 *                           non-temporal hint, so the once-read stream neither allocates
 *                           in L2 / the Infinity Cache nor evicts the FIB directory from
 *                           them (default 1)
 *   CNDP_TUNE_MBUF_HASH     1 = cndp_gpu_l3fwd_mbufs also stores the flow hash in m->hash
 *                           (no reference node writes it; default 0)
 *   CNDP_TUNE_SPEC_SCAN     cnet speculation: how burst maps are composed. 0 = auto (none
 *                           when no low byte of the batch's ptypes carries two p_nxt
 *                           edges -- only the final node state is walked -- else maps of
 *                           8 entries when <= 8 ptype signatures occur, 64 up to 64, a
 *                           sequential walk beyond), 1 = always 64-entry maps, 2 = always
 *                           the sequential walk (default 0; 1 and 2 exist for tests)
 *   CNDP_TUNE_CNET_FOLD     cnet: where the frames the fast kernel leaves and the
 *                           speculation classes pass run -- 0 = auto (in the fast
 *                           kernel's last block when the previous call left no such
 *                           frames, else a second launch), 1 = always the last block,
 *                           2 = always the second launch (tests force both)
 *   CNDP_TUNE_SPEC_GRID     cnet speculation local pass grid: 0 = auto (a small grid
 *                           after a uniform batch), 1 = 2 blocks, 2 = one wave per
 *                           4 chunks (tests force both)
 *   CNDP_TUNE_SPEC_LISTS    cnet speculation, bursts of a multiple of 4 <= 256:
 *                           1 = the fast kernel lists the chunks with a frame off its
 *                           low byte's common edge and, when no group of the batch can
 *                           move the node state off a common edge, the local pass
 *                           replays only those (default); 0 = the local pass looks at
 *                           every chunk (tests force both)
 *   CNDP_TUNE_SPEC_TYPES    cnet speculation: how the fast kernel keeps the packet types
 *                           of a tile whose every frame is on its low byte's common edge
 *                           (IPv4 / IPv6 x TCP / UDP) -- 0 = auto (as 2-bit codes, 16 B a
 *                           tile, when the previous call was a uniform batch, whose
 *                           passes read no such type; a batch that needs them after all
 *                           gets them written out by one more launch), 1 = always the
 *                           types, 2 = always codes (tests force all three)
 *   CNDP_TUNE_STREAM_BAL    wave-tile kernels' schedule: 1 = static (wave w takes tiles w,
 *                           w + W, ...), 2 = balanced (one block a CU -- 512 threads for the
 *                           streamed l3fwd / hash kernel, 1024 for the cnet kernel -- whose
 *                           waves share its tiles through an LDS counter), 0 = auto:
 *                           balanced for the l3fwd / hash kernel (C3 2-3 % faster, C2 1-2 %)
 *                           and for cnet frames at a stride (C5 2.5-3.6 %), static for cnet
 *                           frames at offsets (IMIX C4: balanced 0.8-3 % slower)
 *   CNDP_TUNE_SPEC_WAIT     cnet speculation: bound, in microseconds, on each wait of the
 *                           general resolution pass for an earlier phase's work items
 *                           (default 1000000; the waits end by construction -- work is
 *                           handed out in ticket order, so no co-residency is assumed --
 *                           the bound only turns a fault into an error).  -1 = fault
 *                           injection for tests: every such wait expires.  An expired
 *                           wait is reported, never silent: the context's next
 *                           cndp_gpu_classify of a cnet batch returns -EIO (and restarts
 *                           the node state), a node queue's poll returns that batch with
 *                           every edge CNDP_MQ_EDGE_NONE and its next submit -EIO, and
 *                           CNDP_STAT_SPEC_ERR reads 1 until then
 *   CNDP_TUNE_HOST_WINDOW   cndp_gpu_classify_host, l3fwd / hash modes, frames at a stride
 *                           wider than 64 B (the AF_XDP UMEM layout): 1 = only each frame's
 *                           first 64 bytes from data_off cross PCIe, one strided 2-D copy per
 *                           chunk into packed 64-B slots (the parse reads no byte past them;
 *                           default), 0 = the whole slab is mirrored */
#define CNDP_TUNE_NT 1
#define CNDP_TUNE_UNROLL 2
#define CNDP_TUNE_BLOCKS_PER_CU 3
#define CNDP_TUNE_TILE 4
#define CNDP_TUNE_DIR16 5
#define CNDP_TUNE_CNET_TILE 6
#define CNDP_TUNE_HOST_CHUNK 7
#define CNDP_TUNE_RW_WB 8
#define CNDP_TUNE_CNET_SPEC 9
#define CNDP_TUNE_LOAD_NT 10
#define CNDP_TUNE_SPEC_SCAN 11
#define CNDP_TUNE_MBUF_HASH 12
#define CNDP_TUNE_CNET_FOLD 13
#define CNDP_TUNE_SPEC_GRID 14
#define CNDP_TUNE_SPEC_LISTS 15
#define CNDP_TUNE_SPEC_TYPES 16
#define CNDP_TUNE_STREAM_BAL 17
#define CNDP_TUNE_SPEC_WAIT 18
#define CNDP_TUNE_HOST_WINDOW 19
int cndp_gpu_set_tuning(cndp_gpu_ctx_t *ctx, int key, int value);

/* Observability: the last cnet classify's shape, read from pinned host words
 * the kernels update (no HIP call) -- with the ptype-node speculation model on
 * (CNDP_TUNE_CNET_SPEC, the default); with it off they are not updated.
 * Returns -EINVAL for an unknown key or a NULL context.
 *   CNDP_STAT_CNET_WORKLIST  bit length of the number of frames the last call
 *                            left to the general parse (0: every frame took
 *                            the fast path)
 *   CNDP_STAT_CNET_UNIFORM   1 when the last call's ptypes all had the entering
 *                            node state's low byte (the uniform speculation pass)
 *   CNDP_STAT_SPEC_ERR       1 when a speculation pass wait expired and has not been
 *                            reported yet (CNDP_TUNE_SPEC_WAIT) */
#define CNDP_STAT_CNET_WORKLIST 1
#define CNDP_STAT_CNET_UNIFORM 2
#define CNDP_STAT_SPEC_ERR 3
int64_t cndp_gpu_get_stat(cndp_gpu_ctx_t *ctx, int key);

/* Version / build info string. */
const char *cndp_gpu_version(void);

#ifdef __cplusplus
}
#endif
#endif
