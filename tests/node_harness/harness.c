/*
 * Test-only driver for the GPU graph node sources (cndp_amd/node/ip4_lookup_gpu.c,
 * and eth_rx_gpu.c with cnet_stubs.c): collects the nodes the
 * source registers (CNE_NODE_REGISTER), instantiates them for one graph, calls
 * their process callbacks as cne_graph_walk would (the source node once per
 * walk, ip4_lookup once per burst it is given) and records, per edge name,
 * the objects each node enqueues -- the way graph_test.c (test/testcne) drives
 * fake nodes without a NIC.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cne_graph_worker.h"

#define MAX_REG 8
#define MAX_OUT (1u << 22)

static const struct cne_node_register *regs[MAX_REG];
static int n_regs;

cne_node_t __cne_node_register(const struct cne_node_register *node)
{
    if (n_regs == MAX_REG)
        return CNE_NODE_ID_INVALID;
    regs[n_regs] = node;
    return (cne_node_t)n_regs++;
}

static struct cne_graph g;
static struct cne_node nodes[MAX_REG];
static int inited[MAX_REG];
/* objects enqueued per edge name: 0 = "ip4_rewrite", 1 = "pkt_drop", 2 = other */
static void **out[3];
static uint32_t n_out[3];
static uint64_t enqueue_calls;
/* and per edge name (any node's edges) */
#define MAX_NAMES 16
static char e_name[MAX_NAMES][CNE_NODE_NAMESIZE];
static void **e_out[MAX_NAMES];
static uint32_t e_n[MAX_NAMES], n_names;
static uint64_t n_total;

static int name_slot(const char *to)
{
    for (uint32_t k = 0; k < n_names; k++)
        if (strcmp(e_name[k], to) == 0)
            return (int)k;
    if (n_names == MAX_NAMES || !(e_out[n_names] = malloc(sizeof(void *) * MAX_OUT)))
        return -1;
    strncpy(e_name[n_names], to, CNE_NODE_NAMESIZE - 1);
    e_n[n_names] = 0;
    return (int)n_names++;
}

static int find(const char *name)
{
    for (int i = 0; i < n_regs; i++)
        if (strcmp(regs[i]->name, name) == 0)
            return i;
    return -1;
}

/* the buckets of (registration, edge), looked up once: the per-call cost
 * stays a copy, as cne_node_enqueue's is (it counts in the node rates) */
#define MAX_EDGES 16
static const struct cne_node_register *slot_reg[MAX_REG];
static int8_t slot_k[MAX_REG][MAX_EDGES], slot_s[MAX_REG][MAX_EDGES];

static void slots_of(int r, const struct cne_node_register *reg)
{
    slot_reg[r] = reg;
    for (int e = 0; e < MAX_EDGES; e++) {
        const char *to = e < reg->nb_edges ? reg->next_nodes[e] : "";
        slot_k[r][e] = (int8_t)(strcmp(to, "ip4_rewrite") == 0 ? 0 : strcmp(to, "pkt_drop") == 0 ? 1 : 2);
        slot_s[r][e] = (int8_t)name_slot(to);
    }
}

static void put(void **dst, uint32_t *n, void **objs, uint16_t nb)
{
    const uint32_t k = *n + nb <= MAX_OUT ? nb : MAX_OUT - *n;
    memcpy(dst + *n, objs, k * sizeof(void *));
    *n += k;
}

void harness_enqueue(struct cne_node *node, cne_edge_t next, void **objs, uint16_t nb_objs)
{
    int r = 0;
    while (r < n_regs && slot_reg[r] != node->reg)
        r++;
    if (r == n_regs) { // first enqueue from this registration
        for (r = 0; r < n_regs && regs[r] != node->reg; r++)
            ;
        if (r == n_regs)
            return;
        slots_of(r, node->reg);
    }
    const int e = next < MAX_EDGES ? next : MAX_EDGES - 1;
    put(out[slot_k[r][e]], &n_out[slot_k[r][e]], objs, nb_objs);
    if (slot_s[r][e] >= 0)
        put(e_out[slot_s[r][e]], &e_n[slot_s[r][e]], objs, nb_objs);
    n_total += nb_objs;
    enqueue_calls++;
}

/* node names and flags as registered, for the test to check */
int harness_node_info(int i, char *name, uint64_t *flags, int *nb_edges, const char **e0, const char **e1)
{
    if (i < 0 || i >= n_regs)
        return -1;
    strcpy(name, regs[i]->name);
    *flags = regs[i]->flags;
    *nb_edges = regs[i]->nb_edges;
    *e0 = regs[i]->nb_edges > 0 ? regs[i]->next_nodes[0] : NULL;
    *e1 = regs[i]->nb_edges > 1 ? regs[i]->next_nodes[1] : NULL;
    return n_regs;
}

/* cne_node_clone (cne_graph.h): a node "<name>-<suffix>" with the parent's
 * callbacks and edges and a context of its own, as pkt_ctrl.c:61 makes one
 * eth_rx per port; returns its id */
cne_node_t harness_clone(const char *name, const char *suffix)
{
    const int i = find(name);
    if (i < 0 || n_regs == MAX_REG)
        return CNE_NODE_ID_INVALID;
    const size_t sz = sizeof(struct cne_node_register) + regs[i]->nb_edges * sizeof(const char *);
    struct cne_node_register *r = malloc(sz);
    if (!r)
        return CNE_NODE_ID_INVALID;
    memcpy(r, regs[i], sz);
    char nm[2 * CNE_NODE_NAMESIZE + 2];
    snprintf(nm, sizeof(nm), "%s-%s", regs[i]->name, suffix);
    memcpy(r->name, nm, CNE_NODE_NAMESIZE - 1);
    r->name[CNE_NODE_NAMESIZE - 1] = 0;
    r->parent_id = regs[i]->id;
    r->id = (cne_node_t)n_regs;
    regs[n_regs] = r;
    return (cne_node_t)n_regs++;
}

/* forget the clones (back to the registered nodes) */
void harness_drop_clones(void)
{
    memset(slot_reg, 0, sizeof(slot_reg));
    while (n_regs > 0 && regs[n_regs - 1]->parent_id != CNE_NODE_ID_INVALID) {
        free((void *)regs[n_regs - 1]);
        n_regs--;
    }
}

/* graph create: init every registered node (graph id gid) */
int harness_graph_create(int gid)
{
    g.id = (cne_graph_t)gid;
    for (int k = 0; k < 3; k++) {
        if (!out[k] && !(out[k] = malloc(sizeof(void *) * MAX_OUT)))
            return -12;
        n_out[k] = 0;
    }
    for (uint32_t k = 0; k < n_names; k++)
        e_n[k] = 0;
    n_total = 0;
    for (int i = 0; i < n_regs; i++) {
        memset(&nodes[i], 0, sizeof(nodes[i]));
        nodes[i].id = regs[i]->id;
        nodes[i].reg = regs[i];
        int r = regs[i]->init ? regs[i]->init(&g, &nodes[i]) : 0;
        if (r)
            return r;
        inited[i] = 1;
    }
    return 0;
}

void harness_graph_destroy(void)
{
    for (int i = 0; i < n_regs; i++)
        if (inited[i] && regs[i]->fini)
            regs[i]->fini(&g, &nodes[i]);
    memset(inited, 0, sizeof(inited));
}

/* one burst into the named node's process() */
int harness_process(const char *name, void **objs, uint16_t n)
{
    const int i = find(name);
    if (i < 0)
        return -1;
    return regs[i]->process(&g, &nodes[i], objs, n);
}

/* the source nodes' turn of one cne_graph_walk */
int harness_walk_sources(void)
{
    int total = 0;
    for (int i = 0; i < n_regs; i++)
        if (regs[i]->flags & CNE_NODE_SOURCE_F)
            total += regs[i]->process(&g, &nodes[i], NULL, 0);
    return total;
}

uint32_t harness_take(int k, void **dst, uint32_t max)
{
    const uint32_t n = n_out[k] < max ? n_out[k] : max;
    memcpy(dst, out[k], n * sizeof(void *));
    return n;
}

uint32_t harness_count(int k) { return n_out[k]; }
uint64_t harness_enqueue_calls(void) { return enqueue_calls; }
uint64_t harness_total(void) { return n_total; }
#ifndef HARNESS_CNET
extern int node_mbuf_priv1_dynfield_offset;
int harness_priv1_offset(void) { return node_mbuf_priv1_dynfield_offset; }
#endif

/* the objects enqueued to the edge named `to`, in enqueue order */
uint32_t harness_take_edge(const char *to, void **dst, uint32_t max)
{
    for (uint32_t k = 0; k < n_names; k++)
        if (strcmp(e_name[k], to) == 0) {
            const uint32_t n = e_n[k] < max ? e_n[k] : max;
            memcpy(dst, e_out[k], n * sizeof(void *));
            return n;
        }
    return 0;
}

/* the edge names of registered node i (up to max), for registry checks */
int harness_node_edges(int i, const char **names, int max)
{
    if (i < 0 || i >= n_regs)
        return -1;
    int k = 0;
    for (; k < regs[i]->nb_edges && k < max; k++)
        names[k] = regs[i]->next_nodes[k];
    return k;
}

/* ---- measurement drivers (bench.py's node-boundary leg) ------------------
 * harness_drive: graph walks over the named node, as cne_graph_walk would
 * run them on one lcore: per walk, the source nodes, then one burst of
 * `burst` mbufs into `name`'s process(); after the last burst, walks until
 * every mbuf has been enqueued.  `passes` times over objs[0..n).  Returns
 * seconds (CLOCK_MONOTONIC), or -1 if mbufs went missing. */
#include <time.h>
static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

double harness_drive(const char *name, void **objs, uint32_t n, uint16_t burst, int passes)
{
    const int i = find(name);
    if (i < 0 || burst == 0)
        return -1.0;
    const double t0 = now_s();
    for (int p = 0; p < passes; p++) {
        for (int k = 0; k < 3; k++)
            n_out[k] = 0;
        for (uint32_t b = 0; b < n; b += burst) {
            harness_walk_sources();
            const uint16_t c = (uint16_t)(n - b < burst ? n - b : burst);
            regs[i]->process(&g, &nodes[i], objs + b, c);
        }
        for (long spin = 0; n_out[0] + n_out[1] + n_out[2] < n; spin++) {
            if (spin > 100000000L)
                return -1.0;
            harness_walk_sources();
        }
    }
    return now_s() - t0;
}

/* Graph walks (source nodes only) until `want` objects have been enqueued in
 * all since graph create / the last reset: the cnet receive node pulls its
 * bursts from the harness receive queue itself.  Returns seconds, -1 on a
 * stall (the spin bound). */
double harness_walk_until(uint64_t want)
{
    const double t0 = now_s();
    for (long spin = 0; n_total < want; spin++) {
        if (spin > 100000000L)
            return -1.0;
        harness_walk_sources();
    }
    return now_s() - t0;
}

void harness_reset_counts(void)
{
    for (int k = 0; k < 3; k++)
        n_out[k] = 0;
    for (uint32_t k = 0; k < n_names; k++)
        e_n[k] = 0;
    n_total = 0;
}

/* The asynchronous queue alone, driven by one thread the way a node does:
 * submit a burst, poll what finished, wait when every slot is busy. */
#include "cndp_gpu.h"
double harness_mq_drive(cndp_gpu_mq_t *q, void **objs, uint32_t n, uint16_t burst, int passes)
{
    void *done[1024];
    uint16_t edges[1024];
    const double t0 = now_s();
    for (int p = 0; p < passes; p++) {
        uint32_t got = 0;
        for (uint32_t b = 0; b < n;) {
            const uint32_t c = n - b < burst ? n - b : burst;
            const int k = cndp_gpu_mq_submit(q, objs + b, c);
            if (k < 0)
                return -1.0;
            b += (uint32_t)k;
            int r = cndp_gpu_mq_poll(q, done, edges, 1024);
            if (r < 0)
                return -1.0;
            got += (uint32_t)r;
            if (k == 0 && r == 0 && cndp_gpu_mq_wait(q) < 0)
                return -1.0;
        }
        for (long spin = 0; got < n; spin++) {
            if (spin > 100000000L)
                return -1.0;
            const int r = cndp_gpu_mq_poll(q, done, edges, 1024);
            if (r < 0)
                return -1.0;
            got += (uint32_t)r;
        }
    }
    return now_s() - t0;
}

/* Latency of one request of n mbufs through the queue, as cndpfwd's
 * loopback takes it: bursts of `burst` submitted back to back, then polled
 * until all n are back; us[r] = microseconds of repetition r. */
int harness_mq_latency(cndp_gpu_mq_t *q, void **objs, uint32_t n, uint16_t burst, int reps, double *us)
{
    void *done[1024];
    uint16_t edges[1024];
    for (int r = 0; r < reps; r++) {
        const double t0 = now_s();
        uint32_t got = 0;
        for (uint32_t b = 0; b < n;) {
            const uint32_t c = n - b < burst ? n - b : burst;
            const int k = cndp_gpu_mq_submit(q, objs + b, c);
            if (k < 0)
                return -1;
            b += (uint32_t)k;
            if (k == 0) {
                const int p = cndp_gpu_mq_poll(q, done, edges, 1024);
                if (p < 0)
                    return -1;
                got += (uint32_t)p;
            }
        }
        if (cndp_gpu_mq_flush(q) < 0)
            return -1;
        for (long spin = 0; got < n; spin++) {
            if (spin > 100000000L)
                return -1;
            const int p = cndp_gpu_mq_poll(q, done, edges, 1024);
            if (p < 0)
                return -1;
            got += (uint32_t)p;
        }
        us[r] = (now_s() - t0) * 1e6;
    }
    return 0;
}
