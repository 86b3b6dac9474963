/*
 * ip4_rewrite_gpu.c -- the l3fwd-graph "ip4_rewrite" node with its per-packet
 * work on the MI355X (libcndp_gpu.so).
 *
 * Built in a CNDP tree in place of lib/usr/clib/nodes/ip4_rewrite.c
 * (INTEGRATION.md §2).  It keeps that file's interface to the rest of the
 * nodes library:
 *   - the node "ip4_rewrite" with its one static edge, pkt_drop
 *     (ip4_rewrite.c:314-326), returned by ip4_rewrite_node_get(), to which
 *     cne_node_eth_config adds one "pktdev_tx-<port>" edge per port and then
 *     calls ip4_rewrite_set_next(port, edge) (pktdev_ctrl.c:75-86);
 *   - the next-hop table behind cne_node_ip4_rewrite_add / ip4_rewrite_set_next,
 *     which libcndp_gpu exports (process-global, as ip4_rewrite_nm is);
 *   - per mbuf what ip4_rewrite_node_process does (:40-247): the next hop's
 *     rewrite data at mtod, TTL - 1, the checksum + htons(0x0100) from
 *     node_mbuf_priv1 (udata64) -- the 4-wide loop's rule for the first
 *     nb_objs & ~3 mbufs of each burst, the tail loop's for the rest -- and
 *     the next hop's tx_node as the next edge.
 * Each process() burst goes whole to an asynchronous queue (cndp_gpu_mq_*,
 * mode CNDP_MQ_IP4_REWRITE), so the burst boundaries the checksum rule
 * depends on are the node's own.  Finished mbufs come back in order and are
 * enqueued to their tx edges by process() and by "ip4_rewrite_gpu_drain", a
 * source node every cne_graph_walk calls (also the flush of a partly filled
 * batch).  Its edges mirror ip4_rewrite's: the library calls back here from
 * ip4_rewrite_set_next, right after pktdev_ctrl.c added the tx edge, and the
 * drain node gets the same edge list.
 *
 * Tuning from the environment (the application stays unchanged):
 *   CNDP_GPU_DEVICE (0), CNDP_GPU_BATCH (8192), CNDP_GPU_DEPTH (4),
 *   CNDP_GPU_DELAY_US (50).  Frames are written in place when the application
 *   registered its UMEMs with cndp_node_gpu_umem_add(), else staged.
 */
#include <errno.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include <cne_graph.h>
#include <cne_graph_worker.h>
#include <pktmbuf.h>

#include "cndp_gpu.h"
#include "cndp_node.h"
#include "gpu_node_enqueue.h"

#define RW_POLL_MAX 256
#define RW_GRAPHS_MAX 256
#define RW_EDGES_MAX 64 /* pkt_drop + one tx edge per port (CNE_MAX_ETHPORTS = 32) */
#define DRAIN_NODE_NAME "ip4_rewrite_gpu_drain"

/* ip4_lookup.c:38 (defined by the ip4_lookup node, ip4_lookup_gpu.c here) */
extern int node_mbuf_priv1_dynfield_offset;

struct rw_graph_state {
    int refs; /* the two nodes of one graph */
    cndp_gpu_ctx_t *gpu;
    cndp_gpu_mq_t *q;
    uint16_t nb_edges; /* ip4_rewrite's edge count at graph create */
    void *done[RW_POLL_MAX];
    uint16_t edge[RW_POLL_MAX];
    void *grp[RW_POLL_MAX]; /* a poll's mbufs grouped by edge */
};

static pthread_mutex_t rw_lock = PTHREAD_MUTEX_INITIALIZER;
static struct rw_graph_state *rw_by_graph[RW_GRAPHS_MAX];

struct rw_node_ctx { /* node->ctx is CNE_NODE_CTX_SZ (16) bytes */
    struct rw_graph_state *st;
};
_Static_assert(sizeof(struct rw_node_ctx) <= CNE_NODE_CTX_SZ, "node context");
#define RW_NODE_STATE(node) (((struct rw_node_ctx *)(node)->ctx)->st)

static uint32_t env_u32(const char *name, uint32_t dflt)
{
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, NULL, 0) : dflt;
}

static void rw_state_put(struct rw_graph_state *st)
{
    if (st && --st->refs == 0) {
        cndp_gpu_mq_free(st->q);
        cndp_gpu_fini(st->gpu);
        free(st);
    }
}

static struct cne_node_register ip4_rewrite_node;
static struct cne_node_register ip4_rewrite_gpu_drain_node;

/* the state of this graph, created by whichever of the two nodes starts first */
static struct rw_graph_state *rw_state_get(const struct cne_graph *graph)
{
    const unsigned gid = graph->id;
    if (gid >= RW_GRAPHS_MAX)
        return NULL;
    pthread_mutex_lock(&rw_lock);
    struct rw_graph_state *st = rw_by_graph[gid];
    if (st) {
        st->refs++;
        pthread_mutex_unlock(&rw_lock);
        return st;
    }
    st = calloc(1, sizeof(*st));
    if (!st)
        goto fail;
    st->refs = 1;
    if (cndp_gpu_init((int)env_u32("CNDP_GPU_DEVICE", 0), &st->gpu) < 0)
        goto fail;
    struct cndp_mq_conf conf = {0};
    conf.mode = CNDP_MQ_IP4_REWRITE;
    conf.batch = env_u32("CNDP_GPU_BATCH", 8192);
    conf.depth = env_u32("CNDP_GPU_DEPTH", 4);
    conf.max_delay_us = env_u32("CNDP_GPU_DELAY_US", 50);
    /* the kernel reads each mbuf header (buf_addr, data_off, node_mbuf_priv1)
     * itself; CNDP_GPU_RW_MQ_FLAGS (else CNDP_GPU_MQ_FLAGS) = 0 for the
     * host-header path; the receive nodes' result form
     * (CNDP_MQ_F_HOST_WRITEBACK) is not one of this queue's */
    conf.flags = env_u32("CNDP_GPU_RW_MQ_FLAGS", env_u32("CNDP_GPU_MQ_FLAGS", CNDP_MQ_F_DEVICE_HEADERS)) &
                 ~CNDP_MQ_F_HOST_WRITEBACK;
    void *umem = NULL;
    uint64_t ulen = 0;
    for (uint32_t i = 0; cndp_node_gpu_umem_get(i, &umem, &ulen) == 0; i++)
        if (cndp_gpu_host_register(st->gpu, umem, ulen, NULL) == 0 && !conf.umem)
            conf.umem = umem;
    if (cndp_gpu_mq_create(st->gpu, &conf, &st->q) < 0)
        goto fail;
    st->nb_edges = cne_node_edge_count(ip4_rewrite_node.id);
    rw_by_graph[gid] = st;
    pthread_mutex_unlock(&rw_lock);
    return st;
fail:
    if (st) {
        if (st->gpu)
            cndp_gpu_fini(st->gpu);
        free(st);
    }
    pthread_mutex_unlock(&rw_lock);
    return NULL;
}

static void rw_state_release(const struct cne_graph *graph, struct rw_graph_state *st)
{
    pthread_mutex_lock(&rw_lock);
    if (st && st->refs == 1 && graph->id < RW_GRAPHS_MAX && rw_by_graph[graph->id] == st)
        rw_by_graph[graph->id] = NULL;
    rw_state_put(st);
    pthread_mutex_unlock(&rw_lock);
}

/* objs to their tx edges, one enqueue per edge (gpu_node_enqueue.h); an mbuf
 * the queue could not reach and an edge the node does not have (a next hop
 * never configured) leave by pkt_drop (edge 0, the unset entry's tx_node).
 * edge[] is rewritten in place. */
static void rw_enqueue(struct cne_graph *graph, struct cne_node *node, struct rw_graph_state *st, void **objs,
                       uint16_t *edge, uint16_t n)
{
    const uint16_t ne = st->nb_edges <= GPU_NODE_EDGES_MAX ? st->nb_edges : GPU_NODE_EDGES_MAX;
    for (uint16_t i = 0; i < n; i++)
        edge[i] = edge[i] < ne ? edge[i] : 0;
    gpu_enqueue_by_edge(graph, node, objs, edge, n, ne, st->grp);
}

/* hand every finished mbuf on to its tx edge */
static uint16_t rw_drain(struct cne_graph *graph, struct cne_node *node, struct rw_graph_state *st)
{
    uint16_t total = 0;
    for (;;) {
        const int k = cndp_gpu_mq_poll(st->q, st->done, st->edge, RW_POLL_MAX);
        if (k <= 0)
            break;
        rw_enqueue(graph, node, st, st->done, st->edge, (uint16_t)k);
        total = (uint16_t)(total + k);
        if (k < RW_POLL_MAX)
            break;
    }
    return total;
}

static uint16_t ip4_rewrite_gpu_process(struct cne_graph *graph, struct cne_node *node, void **objs,
                                        uint16_t nb_objs)
{
    struct rw_graph_state *st = RW_NODE_STATE(node);
    /* the queue takes the burst in 256s (a multiple of 4, so its nb_objs & ~3
     * split, the checksum rule, is the node's own); when every batch slot is
     * busy, drain and then wait for the oldest batch */
    uint16_t done = 0;
    while (done < nb_objs) {
        const int k = cndp_gpu_mq_submit(st->q, objs + done, (uint32_t)(nb_objs - done));
        if (k < 0) { /* the device failed: the mbufs still have to go somewhere */
            cne_node_enqueue(graph, node, 0, objs + done, (uint16_t)(nb_objs - done));
            break;
        }
        done = (uint16_t)(done + k);
        if (done < nb_objs && rw_drain(graph, node, st) == 0 && cndp_gpu_mq_wait(st->q) < 0) {
            cne_node_enqueue(graph, node, 0, objs + done, (uint16_t)(nb_objs - done));
            break;
        }
    }
    rw_drain(graph, node, st);
    return nb_objs;
}

static int ip4_rewrite_gpu_init(const struct cne_graph *graph, struct cne_node *node)
{
    node_mbuf_priv1_dynfield_offset = offsetof(pktmbuf_t, udata64); /* ip4_rewrite.c:257 */
    struct rw_graph_state *st = rw_state_get(graph);
    if (!st)
        return -ENODEV; /* no CPU path behind this node: fail loudly at graph create */
    RW_NODE_STATE(node) = st;
    return 0;
}

static void ip4_rewrite_gpu_fini(const struct cne_graph *graph, struct cne_node *node)
{
    rw_state_release(graph, RW_NODE_STATE(node));
    RW_NODE_STATE(node) = NULL;
}

static struct cne_node_register ip4_rewrite_node = {
    .process = ip4_rewrite_gpu_process,
    .name = "ip4_rewrite",
    .init = ip4_rewrite_gpu_init,
    .fini = ip4_rewrite_gpu_fini,
    /* Default edge i.e '0' is pkt drop (ip4_rewrite.c:318) */
    .nb_edges = 1,
    .next_nodes =
        {
            [0] = "pkt_drop",
        },
};
CNE_NODE_REGISTER(ip4_rewrite_node);

/* ip4_rewrite_priv.h: what pktdev_ctrl.c uses to add the tx edges */
struct cne_node_register *ip4_rewrite_node_get(void)
{
    return &ip4_rewrite_node;
}

/* the source node: called once per cne_graph_walk, polls (and so flushes) */
static uint16_t ip4_rewrite_gpu_drain_process(struct cne_graph *graph, struct cne_node *node, void **objs,
                                              uint16_t nb_objs)
{
    (void)objs;
    (void)nb_objs;
    struct rw_graph_state *st = RW_NODE_STATE(node);
    return st ? rw_drain(graph, node, st) : 0;
}

static int ip4_rewrite_gpu_drain_init(const struct cne_graph *graph, struct cne_node *node)
{
    struct rw_graph_state *st = rw_state_get(graph);
    if (!st)
        return -ENODEV;
    RW_NODE_STATE(node) = st;
    return 0;
}

static struct cne_node_register ip4_rewrite_gpu_drain_node = {
    .process = ip4_rewrite_gpu_drain_process,
    .flags = CNE_NODE_SOURCE_F,
    .name = DRAIN_NODE_NAME,
    .init = ip4_rewrite_gpu_drain_init,
    .fini = ip4_rewrite_gpu_fini,
    .nb_edges = 1,
    .next_nodes =
        {
            [0] = "pkt_drop",
        },
};
CNE_NODE_REGISTER(ip4_rewrite_gpu_drain_node);

/* ip4_rewrite_set_next's hook: the drain node takes ip4_rewrite's edge list,
 * so the tx edge indices the queue returns mean the same on both */
static int rw_mirror_edges(uint16_t port_id, uint16_t next_index)
{
    (void)port_id;
    (void)next_index;
    char *names[RW_EDGES_MAX]; /* cne_node_edge_get hands out the node's own name pointers */
    const cne_edge_t n = cne_node_edge_count(ip4_rewrite_node.id);
    if (n == CNE_EDGE_ID_INVALID || n > RW_EDGES_MAX)
        return -EINVAL;
    if (cne_node_edge_get(ip4_rewrite_node.id, names) != n)
        return -EINVAL;
    const cne_edge_t r = cne_node_edge_update(ip4_rewrite_gpu_drain_node.id, 0, (const char **)names, n);
    return r == CNE_EDGE_ID_INVALID || r == 0 ? -EINVAL : 0;
}

__attribute__((constructor)) static void rw_gpu_hook(void)
{
    cndp_node_ip4_rewrite_next_hook(rw_mirror_edges);
}

/* unloaded (dlclose): ip4_rewrite_set_next must not call into this module */
__attribute__((destructor)) static void rw_gpu_hook_off(void)
{
    cndp_node_ip4_rewrite_next_unhook(rw_mirror_edges);
}
