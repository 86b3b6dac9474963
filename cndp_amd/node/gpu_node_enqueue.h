/*
 * gpu_node_enqueue.h -- shared by the GPU graph node sources in this directory
 * (ip4_lookup_gpu.c, ip4_rewrite_gpu.c, eth_rx_gpu.c).
 *
 * A finished batch comes back from the queue with each mbuf's next edge, in
 * submission order.  The edges of consecutive mbufs change every packet or
 * two when traffic spreads over several next nodes (IPv4 / IPv6 input, tx
 * ports), and one cne_node_enqueue per run then costs more than the node's
 * own work.  gpu_enqueue_by_edge hands the mbufs over with one
 * cne_node_enqueue per edge instead: a stable counting sort, so every edge's
 * stream keeps the order the mbufs arrived in -- which is all a graph walk
 * can observe (the reference nodes' speculative stream plus enqueue_x1 keep
 * the same per-edge order, e.g. ip4_rewrite.c:138-199).
 */
#ifndef CNDP_GPU_NODE_ENQUEUE_H
#define CNDP_GPU_NODE_ENQUEUE_H
#include <stdint.h>

#include <cne_graph.h>
#include <cne_graph_worker.h>

#define GPU_NODE_EDGES_MAX 64

/* objs[0..n): edge[i] (already one of the node's edges, < nb_edges <= 64);
 * tmp: room for n pointers */
static inline void gpu_enqueue_by_edge(struct cne_graph *graph, struct cne_node *node, void **objs,
                                       const uint16_t *edge, uint16_t n, uint16_t nb_edges, void **tmp)
{
    uint16_t start[GPU_NODE_EDGES_MAX + 1] = {0};
    uint16_t distinct = 0;
    for (uint16_t i = 0; i < n; i++)
        distinct = (uint16_t)(distinct + (start[edge[i] + 1]++ == 0));
    if (distinct <= 1) {
        if (n)
            cne_node_enqueue(graph, node, edge[0], objs, n);
        return;
    }
    for (uint16_t e = 1; e <= nb_edges; e++) /* start[e] = first slot of edge e */
        start[e] = (uint16_t)(start[e] + start[e - 1]);
    for (uint16_t i = 0; i < n; i++) /* start[e] moves to the end of edge e */
        tmp[start[edge[i]]++] = objs[i];
    for (uint16_t e = 0, lo = 0; e < nb_edges; e++) {
        if (start[e] > lo)
            cne_node_enqueue(graph, node, e, &tmp[lo], (uint16_t)(start[e] - lo));
        lo = start[e];
    }
}
#endif
