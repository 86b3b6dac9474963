/*
 * Test-only stand-in for eth_rx_priv.h (lib/cnet/eth/eth_rx_priv.h): the
 * per-port clone list pkt_ctrl.c:55-72 fills and eth_rx's init reads.  Same
 * type and field names as the reference declares them.
 */
#ifndef NODE_HARNESS_ETH_RX_PRIV_H
#define NODE_HARNESS_ETH_RX_PRIV_H
#include "cne_graph.h"
typedef struct eth_rx_node_ctx {
    uint16_t port_id;
} eth_rx_node_ctx_t;
typedef struct eth_rx_node_elem {
    struct eth_rx_node_elem *next;
    struct eth_rx_node_ctx ctx;
    cne_node_t nid;
} eth_rx_node_elem_t;
struct eth_rx_node_main {
    eth_rx_node_elem_t *head;
};
struct eth_rx_node_main *eth_rx_get_node_data_get(void);
struct cne_node_register *eth_rx_node_get(void);
#endif
