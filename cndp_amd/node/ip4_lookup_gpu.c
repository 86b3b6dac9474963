/*
 * ip4_lookup_gpu.c -- the l3fwd-graph "ip4_lookup" node with its arithmetic on
 * the MI355X (libcndp_gpu.so).
 *
 * Built in a CNDP tree in place of lib/usr/clib/nodes/ip4_lookup.c (see
 * INTEGRATION.md): it registers a node under the same name and edges
 * (ip4_lookup.c:345-359), owns the lookup FIB the same way (ip4_lookup_nm,
 * :31-42; here libcndp_gpu holds it and exports cne_node_ip4_route_add), and
 * writes the same per-mbuf result: node_mbuf_priv1 {nh, ttl, cksum} in
 * udata64 and the next edge = FIB value >> 16 (:108-154).  So
 * examples/l3fwd-graph links and runs unchanged: its "ip4*" graph pattern
 * (fwd.c:128) picks up both nodes below.
 *
 * What differs is time, not results: process() never waits for the GPU.
 * Each burst is handed to an asynchronous queue (cndp_gpu_mq_submit) that
 * batches bursts and runs whole batches on the device; finished mbufs come
 * back from cndp_gpu_mq_poll in arrival order and are enqueued to
 * ip4_rewrite / pkt_drop.  Completions are collected
 *   - by process() itself after each submit, and
 *   - by "ip4_lookup_gpu_drain", a source node (CNE_NODE_SOURCE_F) with the
 *     same two edges that every cne_graph_walk calls; its poll also launches
 *     a partly filled batch when the GPU is idle or the batch is older than
 *     CNDP_GPU_DELAY_US, which is the flush timer an idle port needs.
 * When every batch slot is in flight, process() drains and then waits for the
 * oldest batch (back-pressure instead of dropping).
 *
 * Tuning from the environment (the application stays unchanged):
 *   CNDP_GPU_DEVICE (0), CNDP_GPU_BATCH (8192), CNDP_GPU_DEPTH (4),
 *   CNDP_GPU_DELAY_US (50).  Frames are read in place when the application
 *   registered its UMEMs with cndp_node_gpu_umem_add() (every one of them:
 *   the graph's ports may use different pools), else staged.  An mbuf the
 *   queue cannot reach (outside every registered UMEM) leaves by pkt_drop.
 *
 * With the frames in registered UMEM (zero-copy) the queue also runs
 * ip4_rewrite (CNDP_MQ_F_REWRITE), as pktdev_rx_gpu.c does for the receive
 * chain: the rewrite data, TTL and checksum go into each frame the lookup
 * sends to ip4_rewrite, and the mbuf leaves directly on its next hop's
 * pktdev_tx edge.  For that both nodes here carry, after ip4_lookup's two
 * edges, a copy of ip4_rewrite's edge list (pkt_drop, pktdev_tx-<port>...),
 * kept by a hook on ip4_rewrite_set_next (pktdev_ctrl.c:81-86).  ip4_rewrite
 * stays registered and idle and gets the stats of the mbufs it stands for.
 * Its checksum rule (4-wide loop for the first count & ~3 mbufs it gets, the
 * tail loop's for the rest, ip4_rewrite.c:97-110, :209-216) is applied per
 * process() call of this node, as when ip4_rewrite gets the stream this call
 * sends it -- per 256-mbuf piece (CNE_GRAPH_BURST_SIZE) of a call larger than
 * that.  CNDP_GPU_LOOKUP_REWRITE=0 keeps ip4_rewrite as the next node (staged
 * frames always do).
 *
 * One GPU context and queue per graph (graphs are per lcore, cne_graph_worker.h
 * notes a graph is not shared between threads); contexts share the node FIB,
 * whose device mirror libcndp_gpu keeps on one device per process.
 *
 * Linked only together with pktdev_rx_gpu.c: behind
 * CNDP's own pktdev_rx the core has already parsed every frame and left its
 * header line dirty, and one core then runs parse + lookup faster than parse
 * + this node (0.73-0.9 x), so a build that would put this node
 * there does not link -- the reference to cndp_pktdev_rx_gpu_linked below
 * makes the GPU receive node come with it, and an unchanged l3fwd-graph gets
 * the whole receive chain on the device (this node then stays idle, its
 * drain node polling an empty queue).  IP4_LOOKUP_GPU_STANDALONE builds the
 * node alone, for the tests and the bench's measurement of that case.
 */
#include <errno.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <cne_graph.h>
#include <cne_graph_worker.h>
#include <pktmbuf.h>

#include "cndp_gpu.h"
#include "cndp_node.h"
#include "gpu_node_enqueue.h"

#define GPU_POLL_MAX 256
#define GPU_GRAPHS_MAX 256 /* graph ids this module tracks */
#define DRAIN_NODE_NAME "ip4_lookup_gpu_drain"
/* ip4_lookup's two edges, then (with the rewrite on the device) ip4_rewrite's */
#define LOOKUP_GPU_NEXT_TX0 CNE_NODE_IP4_LOOKUP_NEXT_MAX
#define LOOKUP_EDGES_MAX GPU_NODE_EDGES_MAX

/* ip4_lookup.c:38: the rewrite node reads priv1 at this offset */
int node_mbuf_priv1_dynfield_offset = -1;

struct gpu_graph_state {
    int refs; /* the two nodes of one graph */
    cndp_gpu_ctx_t *gpu;
    cndp_gpu_mq_t *q;
    struct cne_node *st_rewrite; /* fused: the idle ip4_rewrite, credited in its stats */
    int fused;                   /* CNDP_MQ_F_REWRITE: the queue's edges are ip4_rewrite's */
    int tx0_drop;                /* fused and ip4_rewrite's edge 0 is pkt_drop */
    uint16_t nb_edges;           /* the nodes' edges at graph create */
    void *done[GPU_POLL_MAX];
    uint16_t edge[GPU_POLL_MAX];
    void *grp[GPU_POLL_MAX]; /* a poll's mbufs grouped by edge */
};

static pthread_mutex_t gs_lock = PTHREAD_MUTEX_INITIALIZER;
static struct gpu_graph_state *gs_by_graph[GPU_GRAPHS_MAX];

struct gpu_node_ctx { /* node->ctx is CNE_NODE_CTX_SZ (16) bytes */
    struct gpu_graph_state *st;
};
_Static_assert(sizeof(struct gpu_node_ctx) <= CNE_NODE_CTX_SZ, "node context");
#define GPU_NODE_STATE(node) (((struct gpu_node_ctx *)(node)->ctx)->st)

static uint32_t env_u32(const char *name, uint32_t dflt)
{
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, NULL, 0) : dflt;
}

static void state_put(struct gpu_graph_state *st)
{
    if (st && --st->refs == 0) {
        cndp_gpu_mq_free(st->q);
        cndp_gpu_fini(st->gpu);
        free(st);
    }
}

/* the state of this graph, created by whichever of the two nodes starts first
 * (both carry the same edges) */
static struct gpu_graph_state *state_get(const struct cne_graph *graph, const struct cne_node *node)
{
    const unsigned gid = graph->id;
    if (gid >= GPU_GRAPHS_MAX)
        return NULL;
    pthread_mutex_lock(&gs_lock);
    struct gpu_graph_state *st = gs_by_graph[gid];
    if (st) {
        st->refs++;
        pthread_mutex_unlock(&gs_lock);
        return st;
    }
    st = calloc(1, sizeof(*st));
    if (!st)
        goto fail;
    st->refs = 1;
    if (cndp_node_ip4_lookup_init() < 0 || cndp_gpu_init((int)env_u32("CNDP_GPU_DEVICE", 0), &st->gpu) < 0)
        goto fail;
    if (cndp_gpu_set_fib(st->gpu, cndp_node_ip4_lookup_fib(), NULL) < 0)
        goto fail;
    struct cndp_mq_conf conf = {0};
    conf.mode = CNDP_MQ_IP4_LOOKUP;
    conf.batch = env_u32("CNDP_GPU_BATCH", 8192);
    conf.depth = env_u32("CNDP_GPU_DEPTH", 4);
    conf.max_delay_us = env_u32("CNDP_GPU_DELAY_US", 50);
    /* the kernel reads each mbuf header itself: the host thread hands over
     * pointers only (121 against 79 Mpps per thread with the
     * host resolving addresses from the headers); CNDP_GPU_MQ_FLAGS=0 for that */
    conf.flags = env_u32("CNDP_GPU_MQ_FLAGS", CNDP_MQ_F_DEVICE_HEADERS);
    /* zero-copy: the kernels read the frames in the UMEMs (registration is
     * shared and counted across the graphs' contexts) */
    void *umem = NULL;
    uint64_t ulen = 0;
    for (uint32_t i = 0; cndp_node_gpu_umem_get(i, &umem, &ulen) == 0; i++)
        if (cndp_gpu_host_register(st->gpu, umem, ulen, NULL) == 0 && !conf.umem)
            conf.umem = umem;
    const cne_edge_t ne = cne_node_edge_count(node->id);
    st->nb_edges = ne == CNE_EDGE_ID_INVALID ? CNE_NODE_IP4_LOOKUP_NEXT_MAX
                   : ne > LOOKUP_EDGES_MAX   ? LOOKUP_EDGES_MAX
                                             : (uint16_t)ne;
    /* ip4_rewrite on the device when the frames are in place and the nodes
     * carry ip4_rewrite's edges (ip4_rewrite_set_next ran, lk_mirror_edges) */
    st->fused = conf.umem && st->nb_edges > LOOKUP_GPU_NEXT_TX0 && env_u32("CNDP_GPU_LOOKUP_REWRITE", 1);
    if (st->fused) {
        conf.flags |= CNDP_MQ_F_REWRITE;
        /* ip4_rewrite's edge 0 is pkt_drop (ip4_rewrite.c's next_nodes): its
         * drops take ip4_lookup's own pkt_drop edge, one enqueue per poll */
        char *names[LOOKUP_EDGES_MAX];
        st->tx0_drop = ne <= LOOKUP_EDGES_MAX && cne_node_edge_get(node->id, names) == ne &&
                       strcmp(names[LOOKUP_GPU_NEXT_TX0], "pkt_drop") == 0;
        /* graph.c:291-295 lays the graph's nodes out before their init runs */
        st->st_rewrite = cne_graph_get_node_by_name(graph, "ip4_rewrite");
    }
    if (cndp_gpu_mq_create(st->gpu, &conf, &st->q) < 0)
        goto fail;
    gs_by_graph[gid] = st;
    pthread_mutex_unlock(&gs_lock);
    return st;
fail:
    if (st) {
        if (st->gpu)
            cndp_gpu_fini(st->gpu);
        free(st);
    }
    pthread_mutex_unlock(&gs_lock);
    return NULL;
}

static void state_release(const struct cne_graph *graph, struct gpu_graph_state *st)
{
    pthread_mutex_lock(&gs_lock);
    if (st && st->refs == 1 && graph->id < GPU_GRAPHS_MAX && gs_by_graph[graph->id] == st)
        gs_by_graph[graph->id] = NULL;
    state_put(st);
    pthread_mutex_unlock(&gs_lock);
}

/* hand every finished mbuf on to its edge, one enqueue per edge */
static uint16_t gpu_drain(struct cne_graph *graph, struct cne_node *node, struct gpu_graph_state *st)
{
    uint16_t total = 0;
    for (;;) {
        const int k = cndp_gpu_mq_poll(st->q, st->done, st->edge, GPU_POLL_MAX);
        if (k <= 0)
            break;
        if (st->fused) {
            /* ip4_rewrite's tx_node: that edge of the copied list (past it:
             * pkt_drop); ip4_lookup's drops and an unreachable mbuf: pkt_drop */
            uint16_t nrw = 0;
            for (int i = 0; i < k; i++) {
                const uint16_t e = st->edge[i];
                nrw = (uint16_t)(nrw + (e < CNDP_MQ_EDGE_LOOKUP_DROP));
                st->edge[i] = e < CNDP_MQ_EDGE_LOOKUP_DROP && LOOKUP_GPU_NEXT_TX0 + e < st->nb_edges &&
                                      !(e == 0 && st->tx0_drop)
                                  ? (uint16_t)(LOOKUP_GPU_NEXT_TX0 + e)
                                  : CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP;
            }
            if (st->st_rewrite && nrw && cne_graph_has_stats_feature()) {
                st->st_rewrite->total_calls++;
                st->st_rewrite->total_objs += nrw;
            }
        } else {
            /* a FIB value naming no edge of this node (ip4_lookup.c:150 takes
             * val >> 16 as is) and an mbuf the queue could not reach
             * (CNDP_MQ_EDGE_NONE) leave by pkt_drop */
            for (int i = 0; i < k; i++)
                if (st->edge[i] >= CNE_NODE_IP4_LOOKUP_NEXT_MAX)
                    st->edge[i] = CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP;
        }
        gpu_enqueue_by_edge(graph, node, st->done, st->edge, (uint16_t)k,
                            st->fused ? st->nb_edges : CNE_NODE_IP4_LOOKUP_NEXT_MAX, st->grp);
        total = (uint16_t)(total + k);
        if (k < GPU_POLL_MAX)
            break;
    }
    return total;
}

static uint16_t ip4_lookup_gpu_process(struct cne_graph *graph, struct cne_node *node, void **objs,
                                       uint16_t nb_objs)
{
    struct gpu_graph_state *st = GPU_NODE_STATE(node);
    uint16_t done = 0;
    while (done < nb_objs) {
        const int k = cndp_gpu_mq_submit(st->q, objs + done, (uint32_t)(nb_objs - done));
        if (k < 0) { /* the device failed: the objects still have to go somewhere */
            cne_node_enqueue(graph, node, CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP, objs + done,
                             (uint16_t)(nb_objs - done));
            break;
        }
        done = (uint16_t)(done + k);
        if (done < nb_objs && gpu_drain(graph, node, st) == 0 && cndp_gpu_mq_wait(st->q) < 0) {
            cne_node_enqueue(graph, node, CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP, objs + done,
                             (uint16_t)(nb_objs - done));
            break;
        }
    }
    gpu_drain(graph, node, st);
    return nb_objs;
}

#ifndef IP4_LOOKUP_GPU_STANDALONE
extern const int cndp_pktdev_rx_gpu_linked; /* pktdev_rx_gpu.c: the receive chain comes with this node */
#endif

static int ip4_lookup_gpu_init(const struct cne_graph *graph, struct cne_node *node)
{
#ifndef IP4_LOOKUP_GPU_STANDALONE
    if (!cndp_pktdev_rx_gpu_linked)
        return -ENOENT;
#endif
    node_mbuf_priv1_dynfield_offset = offsetof(pktmbuf_t, udata64); /* ip4_lookup.c:322 */
    struct gpu_graph_state *st = state_get(graph, node);
    if (!st)
        return -ENODEV; /* no CPU path behind this node: fail loudly at graph create */
    GPU_NODE_STATE(node) = st;
    return 0;
}

static void ip4_lookup_gpu_fini(const struct cne_graph *graph, struct cne_node *node)
{
    state_release(graph, GPU_NODE_STATE(node));
    GPU_NODE_STATE(node) = NULL;
}

static struct cne_node_register ip4_lookup_node = {
    .process = ip4_lookup_gpu_process,
    .name = "ip4_lookup",
    .init = ip4_lookup_gpu_init,
    .fini = ip4_lookup_gpu_fini,
    .nb_edges = CNE_NODE_IP4_LOOKUP_NEXT_MAX,
    .next_nodes =
        {
            [CNE_NODE_IP4_LOOKUP_NEXT_REWRITE] = "ip4_rewrite",
            [CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP] = "pkt_drop",
        },
};
CNE_NODE_REGISTER(ip4_lookup_node);

/* the source node: called once per cne_graph_walk, polls (and so flushes) */
static uint16_t ip4_lookup_gpu_drain_process(struct cne_graph *graph, struct cne_node *node, void **objs,
                                             uint16_t nb_objs)
{
    (void)objs;
    (void)nb_objs;
    struct gpu_graph_state *st = GPU_NODE_STATE(node);
    return st ? gpu_drain(graph, node, st) : 0;
}

static int ip4_lookup_gpu_drain_init(const struct cne_graph *graph, struct cne_node *node)
{
    struct gpu_graph_state *st = state_get(graph, node);
    if (!st)
        return -ENODEV;
    GPU_NODE_STATE(node) = st;
    return 0;
}

static struct cne_node_register ip4_lookup_gpu_drain_node = {
    .process = ip4_lookup_gpu_drain_process,
    .flags = CNE_NODE_SOURCE_F,
    .name = DRAIN_NODE_NAME,
    .init = ip4_lookup_gpu_drain_init,
    .fini = ip4_lookup_gpu_fini,
    .nb_edges = CNE_NODE_IP4_LOOKUP_NEXT_MAX,
    .next_nodes =
        {
            [CNE_NODE_IP4_LOOKUP_NEXT_REWRITE] = "ip4_rewrite",
            [CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP] = "pkt_drop",
        },
};
CNE_NODE_REGISTER(ip4_lookup_gpu_drain_node);

/* ip4_rewrite_set_next's hook (pktdev_ctrl.c:81-86 calls it right after it
 * added a port's pktdev_tx edge to ip4_rewrite): both nodes take ip4_rewrite's
 * edge list after ip4_lookup's two, so the tx_node the queue returns names the
 * same next node here */
static int lk_mirror_edges(uint16_t port_id, uint16_t next_index)
{
    (void)port_id;
    (void)next_index;
    const cne_node_t rw = cne_node_from_name("ip4_rewrite");
    if (rw == CNE_NODE_ID_INVALID)
        return 0; /* no ip4_rewrite node in this build: nothing to mirror */
    char *names[LOOKUP_EDGES_MAX]; /* cne_node_edge_get hands out the node's own name pointers */
    const cne_edge_t n = cne_node_edge_count(rw);
    if (n == CNE_EDGE_ID_INVALID || n > LOOKUP_EDGES_MAX - LOOKUP_GPU_NEXT_TX0)
        return -EINVAL;
    if (cne_node_edge_get(rw, names) != n)
        return -EINVAL;
    if (cne_node_edge_update(ip4_lookup_node.id, LOOKUP_GPU_NEXT_TX0, (const char **)names, n) ==
            CNE_EDGE_ID_INVALID ||
        cne_node_edge_update(ip4_lookup_gpu_drain_node.id, LOOKUP_GPU_NEXT_TX0, (const char **)names, n) ==
            CNE_EDGE_ID_INVALID)
        return -EINVAL;
    return 0;
}

__attribute__((constructor)) static void lk_gpu_hook(void)
{
    cndp_node_ip4_rewrite_next_hook(lk_mirror_edges);
}

/* unloaded (dlclose): ip4_rewrite_set_next must not call into this module */
__attribute__((destructor)) static void lk_gpu_hook_off(void)
{
    cndp_node_ip4_rewrite_next_unhook(lk_mirror_edges);
}
