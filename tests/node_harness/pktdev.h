/*
 * Test-only stand-in for pktdev.h (lib/core/pktdev/pktdev.h:39, :184-204): the
 * receive call the GPU eth_rx node source makes.  The reference's is a static
 * inline over pktdev_devices[]; here the harness (cnet_stubs.c) hands out
 * mbuf pointers it was loaded with.
 */
#ifndef NODE_HARNESS_PKTDEV_H
#define NODE_HARNESS_PKTDEV_H
#include <stdint.h>
#include "pktmbuf.h"
#define PKTDEV_ADMIN_STATE_DOWN 0xFFFF
uint16_t pktdev_rx_burst(uint16_t lport_id, pktmbuf_t **rx_pkts, const uint16_t nb_pkts);
#endif
