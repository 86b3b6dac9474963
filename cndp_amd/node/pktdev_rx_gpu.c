/*
 * pktdev_rx_gpu.c -- the l3fwd-graph receive chain (pktdev_rx -> pkt_cls ->
 * ip4_lookup) as one graph source node with its arithmetic on the MI355X
 * (libcndp_gpu.so).
 *
 * Built in a CNDP tree in place of lib/usr/clib/nodes/pktdev_rx.c
 * (INTEGRATION.md §2b), together with ip4_lookup_gpu.c (which owns the node
 * FIB, cne_node_ip4_route_add).  It keeps pktdev_rx.c's interface to the rest
 * of the build:
 *   - the node "pktdev_rx", a source node (CNE_NODE_SOURCE_F,
 *     pktdev_rx.c:186-199) that pktdev_ctrl.c:40-64 clones per port
 *     ("pktdev_rx-<port>") through pktdev_rx_node_get() and records in
 *     pktdev_rx_get_node_data_get()'s list ({port_id, nid} elements,
 *     pktdev_rx_priv.h), which node init looks up; its two reference edges,
 *     "ip4_lookup" and "pkt_cls", stay (never used: they keep both nodes in
 *     the graph l3fwd-graph's patterns build, fwd.c:128-139);
 *   - per call, one pktdev_rx_burst of up to CNE_GRAPH_BURST_SIZE mbufs from
 *     the node's port (pktdev_rx.c:107-125).
 * What the next nodes receive is what the reference chain hands them: the
 * soft parse's packet_type (eth_pkt_parse_cb, pktdev_rx.c:24-34, :37-103),
 * pkt_cls's routing (only IPv4 goes on, pkt_cls.c:19-31) and ip4_lookup's
 * node_mbuf_priv1 {nh, ttl, cksum} in udata64 with its next edge = FIB value
 * >> 16 (ip4_lookup.c:108-154).  So the mbufs leave this node on the edges
 * the reference's pkt_cls and ip4_lookup would have used: ip4_rewrite, or
 * pkt_drop (non-IPv4 from pkt_cls; a route to the drop edge from ip4_lookup).
 *
 * With the frames in registered UMEM (zero-copy) the queue also runs
 * ip4_rewrite (CNDP_MQ_F_REWRITE): the rewrite data, TTL and checksum go into
 * each frame the lookup sends to ip4_rewrite, with the 4-wide / tail checksum
 * rule of ip4_rewrite getting the burst's stream in one call, and the mbuf
 * leaves directly on its next hop's pktdev_tx edge.  For that this node
 * carries, after its own four edges, a copy of ip4_rewrite's edge list
 * (pkt_drop, pktdev_tx-<port>...), kept by a hook on ip4_rewrite_set_next
 * (pktdev_ctrl.c:81-86) on the node and its per-port clones.  ip4_rewrite
 * stays registered and idle and gets the stats of the mbufs it stands for.
 * CNDP_GPU_RX_REWRITE=0 keeps ip4_rewrite as the next node (staged frames
 * always do).
 *
 * Why: the host thread never touches a frame.  In the reference chain the
 * soft parse reads each frame's Ethernet header and writes packet_type on the
 * core, which leaves the lines the GPU ip4_lookup node then reads over PCIe
 * dirty in the core's cache (43-52 Mpps for the GPU node
 * behind it against 62-67 for one core).  Here the queue (mode
 * CNDP_MQ_IP4_LOOKUP with CNDP_MQ_F_RX_PARSE, and by default
 * CNDP_MQ_F_DEVICE_HEADERS) does the parse, the classification and the
 * lookup in one kernel over the mbufs where they lie.
 *
 * Each burst is handed to that asynchronous queue (cndp_gpu_mq_submit);
 * finished mbufs come back in receive order from cndp_gpu_mq_poll, called on
 * every graph walk (this is a source node, so that is also the flush of a
 * partly filled batch on an idle port).  When every batch slot is in flight
 * the node drains and then waits for the oldest batch.
 *
 * Tuning from the environment: CNDP_GPU_DEVICE (0), CNDP_GPU_BATCH (8192),
 * CNDP_GPU_DEPTH (4), CNDP_GPU_DELAY_US (50), CNDP_GPU_MQ_FLAGS (the
 * queue's flags besides CNDP_MQ_F_RX_PARSE; default CNDP_MQ_F_DEVICE_HEADERS
 * for up to two receive nodes, host headers for three or four, host
 * writeback beyond -- see init).  Frames are read in place when the application
 * registered its UMEMs with cndp_node_gpu_umem_add(), else staged.  One GPU
 * context and queue per cloned node (per port and graph).
 *
 * Graph stats: pkt_cls and ip4_lookup (and ip4_rewrite, fused) get the calls
 * and objects they would have processed added to their node stats
 * (cne_graph_worker.h:156-160) at each poll -- every mbuf for pkt_cls, the
 * IPv4 ones for ip4_lookup, the ones sent on to it for ip4_rewrite.
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

#include "pktdev_rx_priv.h"

#include "cndp_gpu.h"
#include "cndp_node.h"
#include "gpu_node_enqueue.h"

#define RX_BURST 256 /* CNE_GRAPH_BURST_SIZE (cne_graph.h:30) */

/* the reference's two edges (pktdev_rx_priv.h), then the two this node uses,
 * then (with the rewrite on the device) ip4_rewrite's edges */
enum {
    PKTDEV_RX_GPU_NEXT_REWRITE = PKTDEV_RX_NEXT_MAX, /* ip4_lookup's CNE_NODE_IP4_LOOKUP_NEXT_REWRITE */
    PKTDEV_RX_GPU_NEXT_PKT_DROP,                     /* pkt_cls's and ip4_lookup's pkt_drop */
    PKTDEV_RX_GPU_NEXT_MAX,
    PKTDEV_RX_GPU_NEXT_TX0 = PKTDEV_RX_GPU_NEXT_MAX, /* ip4_rewrite's edge 0 (pkt_drop), 1, ... */
};
#define RX_EDGES_MAX 64 /* GPU_NODE_EDGES_MAX */
#define RX_DEVICE_HEADERS_MAX 2
#define RX_HOST_WB_MIN 4

static struct pktdev_rx_node_main pktdev_rx_main;

/* ip4_lookup_gpu.c links only with this file (see there) */
const int cndp_pktdev_rx_gpu_linked = 1;

struct gpu_rx_state {
    cndp_gpu_ctx_t *gpu;
    cndp_gpu_mq_t *q;
    /* the replaced nodes in this graph (NULL when absent): their walk stats
     * are credited with the objects they would have processed */
    struct cne_node *st_cls, *st_lookup, *st_rewrite;
    int fused;          /* CNDP_MQ_F_REWRITE: the queue's edges are ip4_rewrite's */
    int tx0_drop;       /* fused and ip4_rewrite's edge 0 is pkt_drop */
    uint16_t nb_edges;  /* this node's edges at graph create */
    void *rx[RX_BURST];
    void *done[RX_BURST];
    uint16_t edge[RX_BURST];
    void *grp[RX_BURST]; /* a poll's mbufs grouped by edge */
};

struct gpu_rx_ctx { /* node->ctx is CNE_NODE_CTX_SZ (16) bytes */
    pktdev_rx_node_ctx_t rctx; /* the reference's context, where it keeps it */
    struct gpu_rx_state *st;
};
_Static_assert(sizeof(struct gpu_rx_ctx) <= CNE_NODE_CTX_SZ, "node context");
#define GPU_RX_CTX(node) ((struct gpu_rx_ctx *)(node)->ctx)

static uint32_t env_u32(const char *name, uint32_t dflt)
{
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, NULL, 0) : dflt;
}

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
        const int k = cndp_gpu_mq_poll(st->q, st->done, st->edge, RX_BURST);
        if (k <= 0)
            break;
        uint16_t n4 = 0, nrw = 0;
        if (st->fused) {
            for (int i = 0; i < k; i++) {
                /* ip4_rewrite's tx_node: that edge of the copied list (past
                 * it: pkt_drop); pkt_cls's and ip4_lookup's drops and an
                 * unreachable mbuf: pkt_drop */
                const uint16_t e = st->edge[i];
                n4 = (uint16_t)(n4 + (e < CNDP_MQ_EDGE_CLS_DROP));
                nrw = (uint16_t)(nrw + (e < CNDP_MQ_EDGE_LOOKUP_DROP));
                st->edge[i] = e < CNDP_MQ_EDGE_LOOKUP_DROP && PKTDEV_RX_GPU_NEXT_TX0 + e < st->nb_edges &&
                                      !(e == 0 && st->tx0_drop)
                                  ? (uint16_t)(PKTDEV_RX_GPU_NEXT_TX0 + e)
                                  : PKTDEV_RX_GPU_NEXT_PKT_DROP;
            }
        } else {
            for (int i = 0; i < k; i++) {
                const uint16_t e = st->edge[i];
                /* IPv4 (ip4_lookup ran): its value >> 16, 0 = rewrite; pkt_cls's
                 * drop, an unreachable mbuf and a value naming no edge: pkt_drop */
                n4 = (uint16_t)(n4 + (e < CNDP_MQ_EDGE_CLS_DROP));
                st->edge[i] = e == CNE_NODE_IP4_LOOKUP_NEXT_REWRITE ? PKTDEV_RX_GPU_NEXT_REWRITE
                                                                    : PKTDEV_RX_GPU_NEXT_PKT_DROP;
            }
        }
        if (cne_graph_has_stats_feature()) {
            node_stat(st->st_cls, (uint16_t)k);
            node_stat(st->st_lookup, n4);
            node_stat(st->st_rewrite, nrw);
        }
        gpu_enqueue_by_edge(graph, node, st->done, st->edge, (uint16_t)k, st->nb_edges, st->grp);
        total = (uint16_t)(total + k);
        if (k < RX_BURST)
            break;
    }
    return total;
}

static uint16_t pktdev_rx_gpu_process(struct cne_graph *graph, struct cne_node *node, void **objs, uint16_t cnt)
{
    (void)objs;
    (void)cnt;
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    struct gpu_rx_state *st = ctx->st;
    rx_drain(graph, node, st); /* free slots first */
    const uint16_t count = pktdev_rx_burst(ctx->rctx.port_id, (pktmbuf_t **)st->rx, RX_BURST);
    if (count == PKTDEV_ADMIN_STATE_DOWN)
        return count;
    uint16_t done = 0;
    while (done < count) {
        const int k = cndp_gpu_mq_submit(st->q, st->rx + done, (uint32_t)(count - done));
        if (k < 0) { /* the device failed: the mbufs still have to go somewhere */
            cne_node_enqueue(graph, node, PKTDEV_RX_GPU_NEXT_PKT_DROP, st->rx + done, (uint16_t)(count - done));
            break;
        }
        done = (uint16_t)(done + k);
        if (done < count && rx_drain(graph, node, st) == 0 && cndp_gpu_mq_wait(st->q) < 0) {
            cne_node_enqueue(graph, node, PKTDEV_RX_GPU_NEXT_PKT_DROP, st->rx + done, (uint16_t)(count - done));
            break;
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

static int pktdev_rx_gpu_init(const struct cne_graph *graph, struct cne_node *node)
{
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    memset(ctx, 0, sizeof(*ctx));
    for (pktdev_rx_node_elem_t *elem = pktdev_rx_main.head; elem; elem = elem->next)
        if (elem->nid == node->id) { /* pktdev_rx.c:151-165 */
            memcpy(&ctx->rctx, &elem->ctx, sizeof(ctx->rctx));
            break;
        }
    ctx->rctx.cls_next = PKTDEV_RX_NEXT_PKT_CLS;
    struct gpu_rx_state *st = calloc(1, sizeof(*st));
    if (!st)
        return -ENOMEM;
    int r = cndp_node_ip4_lookup_init();
    if (r < 0 || cndp_gpu_init((int)env_u32("CNDP_GPU_DEVICE", 0), &st->gpu) < 0) {
        free(st);
        return -ENODEV; /* no CPU path behind this node: fail loudly at graph create */
    }
    if ((r = cndp_gpu_set_fib(st->gpu, cndp_node_ip4_lookup_fib(), NULL)) < 0)
        goto fail;
    struct cndp_mq_conf conf;
    memset(&conf, 0, sizeof(conf));
    conf.mode = CNDP_MQ_IP4_LOOKUP;
    conf.batch = env_u32("CNDP_GPU_BATCH", 8192);
    conf.depth = env_u32("CNDP_GPU_DEPTH", 4);
    conf.max_delay_us = env_u32("CNDP_GPU_DELAY_US", 50);
    /* the headers on the device while at most RX_DEVICE_HEADERS_MAX receive
     * nodes share the GPU, on the host beyond: with device headers every mbuf
     * costs the GPU ~5 small PCIe transactions, which bound the sum over the
     * lcores near 110 Mpps however many there are, while host headers add a
     * header read on each lcore and leave one frame read for the device
     * (bench node_lcores: 60 / 103 / 108 / 110 Mpps at 1 / 2 / 4 / 8 lcores
     * against 54 / 102 / 150 / 163).  Beyond RX_HOST_WB_MIN the results come
     * back as records the lcores' polls write (CNDP_MQ_F_HOST_WRITEBACK): the
     * device's reads of the frames are then its only small transactions
     * (205-209 against 168-169 Mpps at 8 lcores, even at 4).  The clones
     * pktdev_ctrl.c registered, one per port, are the receive nodes the
     * application runs. */
    uint32_t n_rx = 0;
    for (pktdev_rx_node_elem_t *e = pktdev_rx_main.head; e; e = e->next)
        n_rx++;
    conf.flags = CNDP_MQ_F_RX_PARSE | env_u32("CNDP_GPU_MQ_FLAGS", n_rx > RX_HOST_WB_MIN          ? CNDP_MQ_F_HOST_WRITEBACK
                                                                   : n_rx > RX_DEVICE_HEADERS_MAX ? 0u
                                                                                                  : CNDP_MQ_F_DEVICE_HEADERS);
    /* zero-copy: the kernels read the frames in the UMEMs (registration is
     * shared and counted across the per-port contexts) */
    void *umem = NULL;
    uint64_t ulen = 0;
    for (uint32_t i = 0; cndp_node_gpu_umem_get(i, &umem, &ulen) == 0; i++)
        if (cndp_gpu_host_register(st->gpu, umem, ulen, NULL) == 0 && !conf.umem)
            conf.umem = umem;
    st->nb_edges = (uint16_t)cne_node_edge_count(node->id);
    if (st->nb_edges > RX_EDGES_MAX)
        st->nb_edges = RX_EDGES_MAX;
    /* ip4_rewrite on the device when the frames are in place and this node
     * carries ip4_rewrite's edges (ip4_rewrite_set_next ran, rx_mirror_edges) */
    st->fused = conf.umem && st->nb_edges > PKTDEV_RX_GPU_NEXT_TX0 && env_u32("CNDP_GPU_RX_REWRITE", 1);
    if (st->fused) {
        conf.flags |= CNDP_MQ_F_REWRITE;
        /* ip4_rewrite's edge 0 is pkt_drop (ip4_rewrite.c's next_nodes): its
         * drops then take this node's own pkt_drop edge, so pkt_drop gets one
         * enqueue per poll in receive order */
        char *names[RX_EDGES_MAX];
        st->tx0_drop = cne_node_edge_count(node->id) <= RX_EDGES_MAX &&
                       cne_node_edge_get(node->id, names) == st->nb_edges &&
                       strcmp(names[PKTDEV_RX_GPU_NEXT_TX0], "pkt_drop") == 0;
    }
    if ((r = cndp_gpu_mq_create(st->gpu, &conf, &st->q)) < 0)
        goto fail;
    /* graph.c:291-295 lays the graph's nodes out before their init runs */
    st->st_cls = cne_graph_get_node_by_name(graph, "pkt_cls");
    st->st_lookup = cne_graph_get_node_by_name(graph, "ip4_lookup");
    st->st_rewrite = st->fused ? cne_graph_get_node_by_name(graph, "ip4_rewrite") : NULL;
    ctx->st = st;
    return 0;
fail:
    rx_state_free(st);
    return r;
}

static void pktdev_rx_gpu_fini(const struct cne_graph *graph, struct cne_node *node)
{
    (void)graph;
    struct gpu_rx_ctx *ctx = GPU_RX_CTX(node);
    rx_state_free(ctx->st);
    ctx->st = NULL;
}

static struct cne_node_register pktdev_rx_node_base = {
    .process = pktdev_rx_gpu_process,
    .flags = CNE_NODE_SOURCE_F,
    .name = "pktdev_rx",
    .init = pktdev_rx_gpu_init,
    .fini = pktdev_rx_gpu_fini,
    .nb_edges = PKTDEV_RX_GPU_NEXT_MAX,
    .next_nodes =
        {
            [PKTDEV_RX_NEXT_PKT_CLS] = "pkt_cls",
            [PKTDEV_RX_NEXT_IP4_LOOKUP] = "ip4_lookup",
            [PKTDEV_RX_GPU_NEXT_REWRITE] = "ip4_rewrite",
            [PKTDEV_RX_GPU_NEXT_PKT_DROP] = "pkt_drop",
        },
};
CNE_NODE_REGISTER(pktdev_rx_node_base);

/* ip4_rewrite_set_next's hook (pktdev_ctrl.c:81-86 calls it right after it
 * added a port's pktdev_tx edge to ip4_rewrite): this node and every clone of
 * it take ip4_rewrite's edge list after their own four, so the tx_node the
 * queue returns names the same next node here */
static int rx_mirror_edges(uint16_t port_id, uint16_t next_index)
{
    (void)port_id;
    (void)next_index;
    const cne_node_t rw = cne_node_from_name("ip4_rewrite");
    if (rw == CNE_NODE_ID_INVALID)
        return 0; /* no ip4_rewrite node in this build: nothing to mirror */
    char *names[RX_EDGES_MAX]; /* cne_node_edge_get hands out the node's own name pointers */
    const cne_edge_t n = cne_node_edge_count(rw);
    if (n == CNE_EDGE_ID_INVALID || n > RX_EDGES_MAX - PKTDEV_RX_GPU_NEXT_TX0)
        return -EINVAL;
    if (cne_node_edge_get(rw, names) != n)
        return -EINVAL;
    if (cne_node_edge_update(pktdev_rx_node_base.id, PKTDEV_RX_GPU_NEXT_TX0, (const char **)names, n) ==
        CNE_EDGE_ID_INVALID)
        return -EINVAL;
    for (pktdev_rx_node_elem_t *e = pktdev_rx_main.head; e; e = e->next)
        if (cne_node_edge_update(e->nid, PKTDEV_RX_GPU_NEXT_TX0, (const char **)names, n) == CNE_EDGE_ID_INVALID)
            return -EINVAL;
    return 0;
}

__attribute__((constructor)) static void rx_gpu_hook(void)
{
    cndp_node_ip4_rewrite_next_hook(rx_mirror_edges);
}

/* unloaded (dlclose): ip4_rewrite_set_next must not call into this module */
__attribute__((destructor)) static void rx_gpu_hook_off(void)
{
    cndp_node_ip4_rewrite_next_unhook(rx_mirror_edges);
}

/* pktdev_rx_priv.h: what pktdev_ctrl.c uses to clone the node per port */
struct pktdev_rx_node_main *pktdev_rx_get_node_data_get(void)
{
    return &pktdev_rx_main;
}

struct cne_node_register *pktdev_rx_node_get(void)
{
    return &pktdev_rx_node_base;
}
