/*
 * Test-only: what the GPU eth_rx node source (cndp_amd/node/eth_rx_gpu.c)
 * needs from the rest of CNDP, for tests/test_node_graph.py: the cnet
 * instance with its two route FIBs (this_cnet) and pkt_ctrl.c's per-port
 * registration of the node (the receive queues are rx_stubs.c's).
 */
#include <stdlib.h>
#include <string.h>

#include "cne_graph.h"
#include "cnet.h"
#include "cnet_fib_info.h"
#include "eth_rx_priv.h"

static fib_info_t fi4, fi6;
static struct cnet cn;
static int have_cnet;

struct cnet *cnet_get(void) { return have_cnet ? &cn : NULL; }

/* this_cnet's route FIBs (the handles cnet_route4.c / cnet_route6.c add to) */
void harness_cnet_set(struct cne_fib *fib4, struct cne_fib6 *fib6)
{
    fi4.fib = fib4;
    fi6.fib6 = fib6;
    cn.rt4_finfo = &fi4;
    cn.rt6_finfo = &fi6;
    have_cnet = 1;
}

/* pkt_ctrl.c:55-72: node nid receives from port port_id */
int harness_eth_rx_port(cne_node_t nid, uint16_t port_id)
{
    for (eth_rx_node_elem_t *e = eth_rx_get_node_data_get()->head; e; e = e->next)
        if (e->nid == nid) { /* re-registration (a later test): update */
            e->ctx.port_id = port_id;
            return 0;
        }
    struct eth_rx_node_main *m = eth_rx_get_node_data_get();
    eth_rx_node_elem_t *e = calloc(1, sizeof(*e));
    if (!e)
        return -12;
    e->ctx.port_id = port_id;
    e->nid = nid;
    e->next = m->head;
    m->head = e;
    return 0;
}

/* cnet's other synchronous FIB callers, running on their own thread while the
 * graph walks: ip4_forward.c:134-178 looks up 4 destinations per call in the
 * ARP and route FIBs, ip4_output.c:87-118 / cnet_arp.c:77 / cnet_route4.c:77
 * one key per call.  `rounds` passes over keys[0..n) in calls of per_call keys;
 * the answers of the last pass land in out.  Returns 0 or the first error. */
#include "cndp_fib.h"
int harness_fib_caller(struct cne_fib *fib, const uint32_t *keys, uint64_t *out, uint32_t n,
                       uint32_t per_call, uint32_t rounds)
{
    for (uint32_t r = 0; r < rounds; r++)
        for (uint32_t o = 0; o < n; o += per_call) {
            const uint32_t k = n - o < per_call ? n - o : per_call;
            const int rc = cne_fib_lookup_bulk(fib, (uint32_t *)(uintptr_t)(keys + o), out + o, (int)k);
            if (rc < 0)
                return rc;
        }
    return 0;
}

/* The nodes eth_rx_gpu.c stands in for, as cnet registers them (ptype.c:213,
 * ip4_input.c:274, ip6_input.c:275), so they are in the graph with stats of
 * their own; eth_rx_gpu never enqueues to them.  Registered on request (after
 * eth_rx, which keeps node id 0). */
static uint16_t idle_process(struct cne_graph *graph, struct cne_node *node, void **objs, uint16_t nb)
{
    (void)graph;
    (void)node;
    (void)objs;
    return nb;
}
static struct cne_node_register stub_ptype = {.name = "ptype", .process = idle_process};
static struct cne_node_register stub_ip4 = {.name = "ip4_input", .process = idle_process};
static struct cne_node_register stub_ip6 = {.name = "ip6_input", .process = idle_process};
void harness_register_input_nodes(void)
{
    static int done;
    if (done)
        return;
    done = 1;
    struct cne_node_register *r[3] = {&stub_ptype, &stub_ip4, &stub_ip6};
    for (int i = 0; i < 3; i++) {
        r[i]->parent_id = CNE_NODE_ID_INVALID;
        r[i]->id = __cne_node_register(r[i]);
    }
}

/* forget every port registration (pkt_ctrl.c's list back to empty) */
void harness_eth_rx_ports_reset(void)
{
    struct eth_rx_node_main *m = eth_rx_get_node_data_get();
    while (m->head) {
        eth_rx_node_elem_t *e = m->head;
        m->head = e->next;
        free(e);
    }
}
