/*
 * Test-only: a receive queue per port standing in for pktdev_rx_burst
 * (pktdev.h:184-204), for the GPU source nodes that receive (eth_rx_gpu.c,
 * pktdev_rx_gpu.c): harness_rx_load hands a port the mbuf pointers its next
 * bursts return.
 */
#include <stdlib.h>

#include "pktdev.h"

#define PORTS 8

static void **rxq[PORTS];
static uint32_t rx_n[PORTS], rx_pos[PORTS];
static int rx_down[PORTS];
static int rx_writes; /* harness_rx_driver_writes */

/* as xskdev's receive (xskdev.c:296-297, __get_mbuf_rx_aligned) each
 * returned mbuf gets data_len and data_off written, so its header line is in
 * the receiving core's cache, dirty, when the node sees it (values kept) */
void harness_rx_driver_writes(int on) { rx_writes = on; }

/* the next mbufs of port lport_id, at most nb_pkts of them */
uint16_t pktdev_rx_burst(uint16_t lport_id, pktmbuf_t **rx_pkts, const uint16_t nb_pkts)
{
    if (lport_id >= PORTS)
        return 0;
    if (rx_down[lport_id])
        return PKTDEV_ADMIN_STATE_DOWN;
    uint32_t k = rx_n[lport_id] - rx_pos[lport_id];
    k = k < nb_pkts ? k : nb_pkts;
    for (uint32_t i = 0; i < k; i++) {
        pktmbuf_t *m = (pktmbuf_t *)rxq[lport_id][rx_pos[lport_id] + i];
        if (rx_writes) {
            volatile uint16_t *dl = &m->data_len, *dof = &m->data_off;
            *dl = *dl;
            *dof = *dof;
        }
        rx_pkts[i] = m;
    }
    rx_pos[lport_id] += k;
    return (uint16_t)k;
}

/* load port p's receive queue with n mbuf pointers (copied) */
int harness_rx_load(uint16_t p, void **objs, uint32_t n)
{
    if (p >= PORTS)
        return -1;
    free(rxq[p]);
    rxq[p] = malloc(sizeof(void *) * (n ? n : 1));
    if (!rxq[p])
        return -12;
    for (uint32_t i = 0; i < n; i++)
        rxq[p][i] = objs[i];
    rx_n[p] = n;
    rx_pos[p] = 0;
    return 0;
}

void harness_rx_down(uint16_t p, int down)
{
    if (p < PORTS)
        rx_down[p] = down;
}

uint32_t harness_rx_left(uint16_t p) { return p < PORTS ? rx_n[p] - rx_pos[p] : 0; }

