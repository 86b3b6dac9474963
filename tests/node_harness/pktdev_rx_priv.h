/*
 * Test-only stand-in for pktdev_rx_priv.h (lib/usr/clib/nodes/pktdev_rx_priv.h):
 * the per-port clone list pktdev_ctrl.c:40-64 fills and pktdev_rx's init
 * reads, and the node's two reference edges.  Same type, field and
 * enumerator names as the reference declares them.
 */
#ifndef NODE_HARNESS_PKTDEV_RX_PRIV_H
#define NODE_HARNESS_PKTDEV_RX_PRIV_H
#include "cne_graph.h"
typedef struct pktdev_rx_node_ctx {
    uint16_t port_id;
    uint16_t cls_next;
} pktdev_rx_node_ctx_t;
typedef struct pktdev_rx_node_elem {
    struct pktdev_rx_node_elem *next;
    struct pktdev_rx_node_ctx ctx;
    cne_node_t nid;
} pktdev_rx_node_elem_t;
enum pktdev_rx_next_nodes {
    PKTDEV_RX_NEXT_IP4_LOOKUP,
    PKTDEV_RX_NEXT_PKT_CLS,
    PKTDEV_RX_NEXT_MAX,
};
struct pktdev_rx_node_main {
    pktdev_rx_node_elem_t *head;
};
struct pktdev_rx_node_main *pktdev_rx_get_node_data_get(void);
struct cne_node_register *pktdev_rx_node_get(void);
#endif
