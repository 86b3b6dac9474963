/*
 * eth_rx_gpu.c -- the cnet receive path (eth_rx -> ptype -> ip4_input /
 * ip6_input) as one graph source node with its arithmetic on the MI355X
 * (libcndp_gpu.so).
 *
 * Built in a CNDP tree in place of lib/cnet/eth/eth_rx.c.
 * It keeps that file's interface to the rest of cnet:
 *   - the node "eth_rx", a source node (CNE_NODE_SOURCE_F, eth_rx.c:171-190)
 *     that pkt_ctrl.c:55-72 clones per port ("eth_rx-<port>") through
 *     eth_rx_node_get() and registers in eth_rx_get_node_data_get()'s list
 *     ({port_id, nid} elements, eth_rx_priv.h), which node init looks up;
 *   - per call, one pktdev_rx_burst of up to CNE_GRAPH_BURST_SIZE mbufs from
 *     the node's port (eth_rx.c:112-130).
 * What the next nodes receive is what the reference chain hands them: the
 * mbuf fields eth_rx's mbuf_update writes (packet_type, l2/l3/l4 lengths,
 * ol_flags, lport, data_off / data_len after pktmbuf_adj_offset,
 * eth_rx.c:35-63), ptype's 4-wide speculative routing with its node state
 * (ptype.c:48-210), ip4_input / ip6_input's data_len, checksum / length test
 * and FIB lookup in this_cnet->rt4_finfo / rt6_finfo (ip4_input.c:50-260,
 * ip6_input.c:50-260).  So the mbufs leave this node on the edges the
 * reference's ptype and input nodes would have used:
 *   ptype's pkt_drop / punt_kernel / punt_l2_kernel / gtpu_input,
 *   ip4_input's ip4_forward / ip4_proto, ip6_input's ip6_forward / ip6_proto.
 * The node also keeps an edge to "ptype" (never used), so the graph still
 * reaches ptype, ip4_input and ip6_input, which stay registered and idle.
 *
 * Each burst is handed to an asynchronous queue (cndp_gpu_mq_submit, mode
 * CNDP_MQ_CNET) that batches bursts and runs whole batches on the device;
 * finished mbufs come back in receive order from cndp_gpu_mq_poll, which is
 * called on every graph walk (this is a source node, so that is also the flush
 * of a partly filled batch on an idle port).  When every batch slot is in
 * flight the node drains and then waits for the oldest batch.
 *
 * Tuning from the environment: CNDP_GPU_DEVICE (0), CNDP_GPU_BATCH (8192),
 * CNDP_GPU_DEPTH (4), CNDP_GPU_DELAY_US (50), CNDP_GPU_MQ_FLAGS (the queue's
 * header / result form; default host headers, results written back by the
 * lcores with more than four receive nodes -- see init).  Frames are read in place when
 * the application registered its UMEMs with cndp_node_gpu_umem_add(), else
 * staged.  One GPU context and queue per cloned node (per port and graph).
 *
 * Graph stats: ptype, ip4_input and ip6_input get the calls and objects they
 * would have processed added to their node stats (cne_graph_worker.h:156-160)
 * at each poll, so cne_graph_stats / the cluster stats show the traffic they
 * stand for (see node_stat below).
 *
 * The input nodes' cnet_metadata (ipv4/ipv6_save_metadata, ip4_input.c:33-48,
 * ip6_input.c:32-48), which tcp_input / udp_input read, is written at
 * pktmbuf_metadata(m) for every frame this node sends on an ip4_input /
 * ip6_input edge.
 */
#include <errno.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <cne_graph.h>
#include <cne_graph_worker.h>
#include <pktdev.h>
#include <pktmbuf.h>
#include <cnet.h>
#include <cnet_fib_info.h>

#include "eth_rx_priv.h"

#include "cndp_gpu.h"
#include "cndp_node.h"
#include "gpu_node_enqueue.h"

#define RX_BURST 256 /* CNE_GRAPH_BURST_SIZE (cne_graph.h:30) */
#define ETH_RX_HOST_WB_MIN 4

/* ETH_RX_GPU_PROF (diagnostic builds only): where the node's host thread
 * spends its time -- [0] pktdev_rx_burst, [1] cndp_gpu_mq_submit, [2] poll,
 * [3] edge mapping + stats, [4] the per-edge enqueue, [5] waits -- in seconds,
 * read and cleared by eth_rx_gpu_prof() */
#ifdef ETH_RX_GPU_PROF
#include <time.h>
static double prof_t[6];
static inline double prof_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
#define PROF_T0() double prof_a = prof_now(), prof_b
#define PROF_LAP(k) (prof_b = prof_now(), prof_t[k] += prof_b - prof_a, prof_a = prof_b)
void eth_rx_gpu_prof(double *out)
{
    for (int k = 0; k < 6; k++) {
        out[k] = prof_t[k];
        prof_t[k] = 0.0;
    }
}
#else
#define PROF_T0() (void)0
#define PROF_LAP(k) (void)0
#endif

/* this node's edges: the next nodes of ptype, ip4_input and ip6_input */
enum eth_rx_gpu_next {
    ETH_RX_GPU_NEXT_PKT_DROP,    /* ptype / ip4_input / ip6_input ..._PKT_DROP */
    ETH_RX_GPU_NEXT_PKT_PUNT,    /* PTYPE_NEXT_PKT_PUNT */
    ETH_RX_GPU_NEXT_FRAME_PUNT,  /* PTYPE_NEXT_FRAME_PUNT */
    ETH_RX_GPU_NEXT_GTPU_INPUT,  /* PTYPE_NEXT_GTPU_INPUT */
    ETH_RX_GPU_NEXT_IP4_FORWARD, /* CNE_NODE_IP4_INPUT_NEXT_FORWARD */
    ETH_RX_GPU_NEXT_IP4_PROTO,   /* CNE_NODE_IP4_INPUT_NEXT_PROTO */
    ETH_RX_GPU_NEXT_IP6_FORWARD, /* CNE_NODE_IP6_INPUT_NEXT_FORWARD */
    ETH_RX_GPU_NEXT_IP6_PROTO,   /* CNE_NODE_IP6_INPUT_NEXT_PROTO */
    ETH_RX_GPU_NEXT_PTYPE,       /* keeps ptype (and behind it the input nodes) in the graph */
    ETH_RX_GPU_NEXT_MAX,
};

/* ptype_priv.h:19-29 with CNET_ENABLE_IP6: the ptype edge ids the queue returns */
#define PT_NEXT_PKT_PUNT 1
#define PT_NEXT_FRAME_PUNT 2
#define PT_NEXT_GTPU_INPUT 5

static struct eth_rx_node_main eth_rx_main;

struct gpu_rx_state {
    cndp_gpu_ctx_t *gpu;
    cndp_gpu_mq_t *q;
    /* the replaced nodes in this graph (NULL when absent): their walk stats
     * are credited with the objects they would have processed */
    struct cne_node *st_ptype, *st_ip4, *st_ip6;
    void *rx[RX_BURST];
    void *done[RX_BURST];
    uint16_t edge[RX_BURST];
    void *grp[RX_BURST]; /* a poll's mbufs grouped by edge */
};

struct gpu_rx_ctx { /* node->ctx is CNE_NODE_CTX_SZ (16) bytes */
    uint16_t port_id; /* eth_rx_node_ctx_t's one field, where the reference keeps it */
    struct gpu_rx_state *st;
};
_Static_assert(sizeof(struct gpu_rx_ctx) <= CNE_NODE_CTX_SZ, "node context");
#define GPU_RX_CTX(node) ((struct gpu_rx_ctx *)(node)->ctx)

/* the queue's metadata hook: where ip4/ip6_input would write cnet_metadata */
static void *rx_metadata(const void *m)
{
    return pktmbuf_metadata((const pktmbuf_t *)m);
}

static uint32_t env_u32(const char *name, uint32_t dflt)
{
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, NULL, 0) : dflt;
}

/* the queue's (node << 8 | node edge) as one of this node's edges; a FIB value
 * whose next index names no input edge, and an mbuf the zero-copy queue could
 * not read (outside the registered UMEM), leave by pkt_drop */
static inline cne_edge_t rx_edge(uint16_t e)
{
    const unsigned node = e >> 8, x = e & 0xffu;
    if (e == CNDP_MQ_EDGE_NONE)
        return ETH_RX_GPU_NEXT_PKT_DROP;
    if (node == CNDP_MQ_NODE_IP4)
        return x == CNDP_INPUT_NEXT_FORWARD ? ETH_RX_GPU_NEXT_IP4_FORWARD
             : x == CNDP_INPUT_NEXT_PROTO   ? ETH_RX_GPU_NEXT_IP4_PROTO
                                            : ETH_RX_GPU_NEXT_PKT_DROP;
    if (node == CNDP_MQ_NODE_IP6)
        return x == CNDP_INPUT_NEXT_FORWARD ? ETH_RX_GPU_NEXT_IP6_FORWARD
             : x == CNDP_INPUT_NEXT_PROTO   ? ETH_RX_GPU_NEXT_IP6_PROTO
                                            : ETH_RX_GPU_NEXT_PKT_DROP;
    return x == PT_NEXT_PKT_PUNT     ? ETH_RX_GPU_NEXT_PKT_PUNT
         : x == PT_NEXT_FRAME_PUNT   ? ETH_RX_GPU_NEXT_FRAME_PUNT
         : x == PT_NEXT_GTPU_INPUT   ? ETH_RX_GPU_NEXT_GTPU_INPUT
                                     : ETH_RX_GPU_NEXT_PKT_DROP;
}

/* rx_edge as a table over the queue's three nodes (the per-mbuf branches
 * mispredicted on IMIX, where IPv4 and IPv6 frames alternate): filled once */
static uint8_t rx_edge_tab[3][256];

static void rx_edge_tab_fill(void)
{
    for (unsigned n = 0; n < 3; n++)
        for (unsigned x = 0; x < 256; x++)
            rx_edge_tab[n][x] = (uint8_t)rx_edge((uint16_t)(n << 8 | x));
}

static inline uint16_t rx_edge_fast(uint16_t e)
{
    const unsigned node = e >> 8;
    return node < 3 ? rx_edge_tab[node][e & 0xffu] : ETH_RX_GPU_NEXT_PKT_DROP;
}

/* cne_graph_walk counts, per node, the calls made to it and the objects they
 * returned (cne_graph_worker.h:156-160), which cne_graph_stats and the cnet
 * cluster stats print.  ptype, ip4_input and ip6_input never run under this
 * node, so it counts for them: per poll, one call of ptype with every mbuf,
 * and one call of each input node with the mbufs the ptype node routed to it
 * (its speculation included).  Their total_cycles stay 0: no CPU time is
 * spent in them. */
static inline void node_stat(struct cne_node *n, uint16_t objs)
{
    if (n && objs) {
        n->total_calls++;
        n->total_objs += objs;
    }
}

/* hand every finished mbuf on to its edge, one enqueue per edge */
static uint16_t rx_drain(struct cne_graph *graph, struct cne_node *node, struct gpu_rx_state *st)
{
    uint16_t total = 0;
    for (;;) {
        PROF_T0();
        const int k = cndp_gpu_mq_poll(st->q, st->done, st->edge, RX_BURST);
        PROF_LAP(2);
        if (k <= 0)
            break;
        uint16_t n4 = 0, n6 = 0;
        for (int i = 0; i < k; i++) { /* EDGE_NONE's node is 0xff: counted by neither */
            const uint16_t e = st->edge[i];
            n4 = (uint16_t)(n4 + (e >> 8 == CNDP_MQ_NODE_IP4));
            n6 = (uint16_t)(n6 + (e >> 8 == CNDP_MQ_NODE_IP6));
            st->edge[i] = rx_edge_fast(e);
        }
        if (cne_graph_has_stats_feature()) {
            node_stat(st->st_ptype, (uint16_t)k);
            node_stat(st->st_ip4, n4);
            node_stat(st->st_ip6, n6);
        }
        PROF_LAP(3);
        gpu_enqueue_by_edge(graph, node, st->done, st->edge, (uint16_t)k, ETH_RX_GPU_NEXT_MAX, st->grp);
        PROF_LAP(4);
        total = (uint16_t)(total + k);
        if (k < RX_BURST)
            break;
    }
    return total;
}

static uint16_t eth_rx_gpu_process(struct cne_graph *graph, struct cne_node *node, void **objs, uint16_t cnt)
{
    (void)objs;
    (void)cnt;
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    struct gpu_rx_state *st = ctx->st;
    rx_drain(graph, node, st); /* free slots first */
    PROF_T0();
    const uint16_t count = pktdev_rx_burst(ctx->port_id, (pktmbuf_t **)st->rx, RX_BURST);
    PROF_LAP(0);
    if (count == PKTDEV_ADMIN_STATE_DOWN)
        return count;
    uint16_t done = 0;
    while (done < count) {
        const int k = cndp_gpu_mq_submit(st->q, st->rx + done, (uint32_t)(count - done));
        PROF_LAP(1);
        if (k < 0) { /* the device failed: the mbufs still have to go somewhere */
            cne_node_enqueue(graph, node, ETH_RX_GPU_NEXT_PKT_DROP, st->rx + done, (uint16_t)(count - done));
            break;
        }
        done = (uint16_t)(done + k);
        if (done < count && rx_drain(graph, node, st) == 0) {
            PROF_T0();
            const int w = cndp_gpu_mq_wait(st->q);
            PROF_LAP(5);
            if (w < 0) {
                cne_node_enqueue(graph, node, ETH_RX_GPU_NEXT_PKT_DROP, st->rx + done, (uint16_t)(count - done));
                break;
            }
        }
    }
    rx_drain(graph, node, st);
    return count;
}

static void rx_state_free(struct gpu_rx_state *st)
{
    if (!st)
        return;
    cndp_gpu_mq_free(st->q);
    cndp_gpu_fini(st->gpu);
    free(st);
}

static int eth_rx_gpu_init(const struct cne_graph *graph, struct cne_node *node)
{
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    memset(ctx, 0, sizeof(*ctx));
    for (eth_rx_node_elem_t *elem = eth_rx_main.head; elem; elem = elem->next)
        if (elem->nid == node->id) { /* eth_rx.c:146-158 */
            ctx->port_id = elem->ctx.port_id;
            break;
        }
    struct cnet *cnet = this_cnet;
    if (!cnet || !cnet->rt4_finfo || !cnet->rt6_finfo)
        return -EINVAL;
    struct gpu_rx_state *st = calloc(1, sizeof(*st));
    if (!st)
        return -ENOMEM;
    rx_edge_tab_fill();
    int r = cndp_gpu_init((int)env_u32("CNDP_GPU_DEVICE", 0), &st->gpu);
    if (r < 0) {
        free(st);
        return -ENODEV; /* no CPU path behind this node: fail loudly at graph create */
    }
    if ((r = cndp_gpu_set_fib(st->gpu, cnet->rt4_finfo->fib, cnet->rt6_finfo->fib6)) < 0)
        goto fail;
    struct cndp_mq_conf conf;
    memset(&conf, 0, sizeof(conf));
    conf.mode = CNDP_MQ_CNET;
    conf.lport = ctx->port_id;
    conf.batch = env_u32("CNDP_GPU_BATCH", 8192);
    conf.depth = env_u32("CNDP_GPU_DEPTH", 4);
    conf.max_delay_us = env_u32("CNDP_GPU_DELAY_US", 50);
    conf.metadata = rx_metadata;
    /* the host resolves each frame from the mbuf header (measured faster here
     * than the device reading the headers over PCIe: 70-75 against 61 Mpps,
     * DESIGN.md §6); with more than ETH_RX_HOST_WB_MIN receive nodes on the GPU
     * the results come back as records the lcores write into the mbufs
     * (CNDP_MQ_F_HOST_WRITEBACK): the device's small PCIe stores bound the
     * in-place form near 100 Mpps summed over lcores, the records scale with
     * them (bench node_lcores: 100 against 150 Mpps at 8 lcores, 47 against
     * 27 at one).  The clones pkt_ctrl.c registered, one per port, are the
     * receive nodes the application runs.  CNDP_GPU_MQ_FLAGS overrides
     * (4: CNDP_MQ_F_DEVICE_HEADERS). */
    uint32_t n_rx = 0;
    for (eth_rx_node_elem_t *e = eth_rx_main.head; e; e = e->next)
        n_rx++;
    conf.flags = env_u32("CNDP_GPU_MQ_FLAGS", n_rx > ETH_RX_HOST_WB_MIN ? CNDP_MQ_F_HOST_WRITEBACK : 0u);
    /* zero-copy: the kernels read the frames in the UMEMs (registration is
     * shared and counted across the per-port contexts) */
    void *umem = NULL;
    uint64_t ulen = 0;
    for (uint32_t i = 0; cndp_node_gpu_umem_get(i, &umem, &ulen) == 0; i++)
        if (cndp_gpu_host_register(st->gpu, umem, ulen, NULL) == 0 && !conf.umem)
            conf.umem = umem;
    if ((r = cndp_gpu_mq_create(st->gpu, &conf, &st->q)) < 0)
        goto fail;
    /* graph.c:291-295 lays the graph's nodes out before their init runs */
    st->st_ptype = cne_graph_get_node_by_name(graph, "ptype");
    st->st_ip4 = cne_graph_get_node_by_name(graph, "ip4_input");
    st->st_ip6 = cne_graph_get_node_by_name(graph, "ip6_input");
    ctx->st = st;
    return 0;
fail:
    rx_state_free(st);
    return r;
}

static void eth_rx_gpu_fini(const struct cne_graph *graph, struct cne_node *node)
{
    (void)graph;
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    rx_state_free(ctx->st);
    ctx->st = NULL;
}

static struct cne_node_register eth_rx_node_base = {
    .process = eth_rx_gpu_process,
    .flags = CNE_NODE_SOURCE_F,
    .name = "eth_rx",
    .init = eth_rx_gpu_init,
    .fini = eth_rx_gpu_fini,
    .nb_edges = ETH_RX_GPU_NEXT_MAX,
    .next_nodes =
        {
            [ETH_RX_GPU_NEXT_PKT_DROP] = "pkt_drop",
            [ETH_RX_GPU_NEXT_PKT_PUNT] = "punt_kernel",
            [ETH_RX_GPU_NEXT_FRAME_PUNT] = "punt_l2_kernel",
            [ETH_RX_GPU_NEXT_GTPU_INPUT] = "gtpu_input",
            [ETH_RX_GPU_NEXT_IP4_FORWARD] = "ip4_forward",
            [ETH_RX_GPU_NEXT_IP4_PROTO] = "ip4_proto",
            [ETH_RX_GPU_NEXT_IP6_FORWARD] = "ip6_forward",
            [ETH_RX_GPU_NEXT_IP6_PROTO] = "ip6_proto",
            [ETH_RX_GPU_NEXT_PTYPE] = "ptype",
        },
};
CNE_NODE_REGISTER(eth_rx_node_base);

/* eth_rx_priv.h: what pkt_ctrl.c uses to clone the node per port */
struct eth_rx_node_main *eth_rx_get_node_data_get(void)
{
    return &eth_rx_main;
}

struct cne_node_register *eth_rx_node_get(void)
{
    return &eth_rx_node_base;
}
