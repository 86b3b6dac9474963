/*
 * Test-only stand-in for the subset of CNDP's graph API (lib/usr/clib/graph/
 * cne_graph.h) that the GPU node sources (cndp_amd/node) use, so they can
 * be compiled and driven here and on the GPU box, where no CNDP tree exists.
 * Same type names, field names and signatures as the reference declares them
 * (cne_graph.h:32-42, :94-128, :427-472); the behaviour behind them is the
 * harness's own (harness.c).  Never used by the product library.
 */
#ifndef NODE_HARNESS_CNE_GRAPH_H
#define NODE_HARNESS_CNE_GRAPH_H
#include <stdint.h>

#define CNE_NODE_NAMESIZE 64
#define CNE_GRAPH_NAMESIZE 64
#define CNE_NODE_ID_INVALID UINT32_MAX
#define CNE_NODE_SOURCE_F (1ULL << 0)
#define CNE_NODE_CTX_SZ 16

typedef uint32_t cne_node_t;
typedef uint16_t cne_edge_t;
typedef uint16_t cne_graph_t;

struct cne_graph;
struct cne_node;
typedef uint16_t (*cne_node_process_t)(struct cne_graph *graph, struct cne_node *node, void **objs,
                                       uint16_t nb_objs);
typedef int (*cne_node_init_t)(const struct cne_graph *graph, struct cne_node *node);
typedef void (*cne_node_fini_t)(const struct cne_graph *graph, struct cne_node *node);

struct cne_node_register {
    char name[CNE_NODE_NAMESIZE];
    uint64_t flags;
    cne_node_process_t process;
    cne_node_init_t init;
    cne_node_fini_t fini;
    cne_node_t id;
    cne_node_t parent_id;
    cne_edge_t nb_edges;
    const char *next_nodes[];
};

cne_node_t __cne_node_register(const struct cne_node_register *node);

/* cne_graph.h:522-569 (edges of a registered node; the harness keeps them) */
#define CNE_EDGE_ID_INVALID UINT16_MAX
cne_edge_t cne_node_edge_count(cne_node_t id);
cne_edge_t cne_node_edge_update(cne_node_t id, cne_edge_t from, const char **next_nodes, uint16_t nb_edges);
cne_node_t cne_node_edge_get(cne_node_t id, char *next_nodes[]);
cne_node_t cne_node_from_name(const char *name); /* cne_graph.h:500 */

/* cne_graph.h:370 (the node of this name in this graph) and :649 */
struct cne_node *cne_graph_get_node_by_name(const struct cne_graph *graph, const char *node_name);
static inline int cne_graph_has_stats_feature(void) { return 1; }

#define CNE_NODE_REGISTER(node)                                                      \
    __attribute__((constructor)) static void cne_node_register_##node(void)         \
    {                                                                                \
        node.parent_id = CNE_NODE_ID_INVALID;                                        \
        node.id = __cne_node_register(&node);                                        \
    }
#endif
