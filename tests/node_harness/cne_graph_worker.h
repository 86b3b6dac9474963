/*
 * Test-only stand-in for cne_graph_worker.h (see cne_graph.h here): the graph
 * and node objects a node's callbacks see (the reference's field names), and cne_node_enqueue (same
 * signature as cne_graph_worker.h:310-311), which the harness records per edge.
 */
#ifndef NODE_HARNESS_CNE_GRAPH_WORKER_H
#define NODE_HARNESS_CNE_GRAPH_WORKER_H
#include "cne_graph.h"

struct cne_graph {
    cne_graph_t id;
    char name[CNE_GRAPH_NAMESIZE];
};

struct cne_node {
    uint8_t ctx[CNE_NODE_CTX_SZ];
    cne_node_t id;
    char name[CNE_NODE_NAMESIZE];
    uint64_t total_cycles; /* the per-node stats cne_graph_walk keeps (cne_graph_worker.h:156-160) */
    uint64_t total_calls;
    uint64_t total_objs;
    const struct cne_node_register *reg;
};

void harness_enqueue(struct cne_node *node, cne_edge_t next, void **objs, uint16_t nb_objs);

static inline void cne_node_enqueue(struct cne_graph *graph, struct cne_node *node, cne_edge_t next,
                                    void **objs, uint16_t nb_objs)
{
    (void)graph;
    harness_enqueue(node, next, objs, nb_objs);
}
#endif
