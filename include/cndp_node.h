/*
 * cndp_node.h -- graph-node control API of libcndp_gpu.so.
 *
 * These are the control functions CNDP's graph applications and the cnet
 * route code call on the nodes this library replaces.  Names, signatures,
 * argument meaning and return codes are the reference's (CNDP v25.08.0), so
 * examples/l3fwd-graph (fwd.c:187-196) and lib/cnet/route (cnet_route4.c:55,
 * cnet_route6.c:55) link against this library unchanged:
 *
 *   reference declaration                 implementation it replaces
 *   node_ip4_api.h:52-53  cne_node_ip4_route_add    ip4_lookup.c:259-289
 *   node_ip4_api.h:70-71  cne_node_ip4_rewrite_add  ip4_rewrite.c:282-312
 *   ip4_rewrite_priv.h    ip4_rewrite_set_next      ip4_rewrite.c:266-277
 *   ip4_node_api.h:36     cne_node_ip4_add_input    lib/cnet/ipv4/ip4_input.c:263-272
 *   ip6_node_api.h:36     cne_node_ip6_add_input    lib/cnet/ipv6/ip6_input.c:263-274
 *
 * Like the reference node library, libcndp_gpu owns the l3fwd lookup FIB
 * (ip4_lookup_nm, ip4_lookup.c:31-42): it is created once by the ip4_lookup
 * node's init (cndp_node_ip4_lookup_init here, ip4_lookup_node_init there),
 * and cne_node_ip4_route_add adds to it -- and, exactly as the reference,
 * does nothing (returns 0) before that init.  The rewrite table
 * (ip4_rewrite_nm, ip4_rewrite_priv.h:45-50) is process-global too; every
 * GPU context that has not been given a table of its own
 * (cndp_gpu_ip4_rewrite_add) rewrites with it.
 *
 * The enum below is token-compatible with node_ip4_api.h:28-34 and sits
 * behind its include guard, so a file that includes both headers compiles and
 * the compiler checks each prototype here against the reference's
 * (tests/test_abi.py::test_prototypes_match_reference).
 */
#ifndef CNDP_NODE_H
#define CNDP_NODE_H

#include <stdint.h>

#include "cndp_fib.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef __INCLUDE_CNE_NODE_IP4_API_H__
#define __INCLUDE_CNE_NODE_IP4_API_H__
/* node_ip4_api.h:28-34 */
enum cne_node_ip4_lookup_next {
    CNE_NODE_IP4_LOOKUP_NEXT_REWRITE,
    CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP,
    CNE_NODE_IP4_LOOKUP_NEXT_MAX,
};
#endif

/* ip4_input_priv.h:26-31 / ip6_input_priv.h:25-30 edge ids, and the shift of
 * the edge inside a cnet FIB value (cnet_route4.h:28 RT4_NEXT_INDEX_SHIFT) */
#define CNDP_INPUT_NEXT_PKT_DROP 0
#define CNDP_INPUT_NEXT_FORWARD 1
#define CNDP_INPUT_NEXT_PROTO 2
#define CNDP_RT_NEXT_INDEX_SHIFT 24

/* ip4_rewrite_priv.h:15-16 */
#define CNDP_IP4_REWRITE_MAX_NH 64
#define CNDP_IP4_REWRITE_MAX_LEN 56
#define CNDP_IP4_REWRITE_MAX_PORTS 32 /* CNE_MAX_ETHPORTS, cne_common.h:44 */

/* ---- reference API ------------------------------------------------------ */
/* val = (next_node << 16 | next_hop) & 0xFFFFFF added to the node FIB;
 * 0 when the FIB does not exist yet; else cne_fib_add's code. */
int cne_node_ip4_route_add(uint32_t ip, uint8_t depth, uint16_t next_hop,
                           enum cne_node_ip4_lookup_next next_node);
/* -EINVAL: next_hop >= 64, rewrite_len > 56, or dst_port without a next index
 * (this library also rejects dst_port >= 32, which the reference reads out of
 * bounds); -ENOMEM when the table cannot be allocated. */
int cne_node_ip4_rewrite_add(uint16_t next_hop, uint8_t *rewrite_data, uint8_t rewrite_len,
                             uint16_t dst_port);
/* pktdev_ctrl.c:81-86 calls this for each port's pktdev_tx edge;
 * -EINVAL for port_id >= 32 (the reference writes out of bounds). */
int ip4_rewrite_set_next(uint16_t port_id, uint16_t next_index);
/* Adds fn to the calls ip4_rewrite_set_next makes after it stored the next
 * index: 0 (also when fn is already there), -EINVAL for NULL, -ENOSPC when
 * CNDP_NODE_RW_HOOKS_MAX distinct hooks are registered.  The GPU ip4_rewrite
 * node (cndp_amd/node/ip4_rewrite_gpu.c) uses it to give its drain source
 * node the tx edges pktdev_ctrl.c:81 adds, the GPU pktdev_rx and ip4_lookup
 * nodes to give them to themselves; each registers from its constructor and
 * removes the hook from its destructor (cndp_node_ip4_rewrite_next_unhook:
 * 0, or -ENOENT when fn is not registered). */
#define CNDP_NODE_RW_HOOKS_MAX 16
int cndp_node_ip4_rewrite_next_hook(int (*fn)(uint16_t port_id, uint16_t next_index));
int cndp_node_ip4_rewrite_next_unhook(int (*fn)(uint16_t port_id, uint16_t next_index));
/* nh = idx | (depth == 32 ? PROTO : FORWARD) << 24, then cne_fib_add /
 * cne_fib6_add.  cne_node_ip6_add_input keeps the reference's depth == 32
 * test (ip6_input.c:268) for IPv6 as well. */
int cne_node_ip4_add_input(struct cne_fib *fib, uint32_t ip, uint8_t depth, uint32_t idx);
int cne_node_ip6_add_input(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth,
                           uint32_t idx);

/* ---- build extensions ---------------------------------------------------
 * cndp_node_ip4_lookup_init: create the node FIB once, as setup_fib does
 * (ip4_lookup.c:292-311: DIR-24-8, 4-B next hops, 1024 routes, 256 tbl8
 * groups, default nh = PKT_DROP << 16); 0, or a negative errno.
 * cndp_node_ip4_lookup_fib: that FIB (NULL before init) -- the table the
 * GPU ip4_lookup node classifies with (node/ip4_lookup_gpu.c).
 * cndp_node_ip4_lookup_fini: free it (process teardown, tests).
 * cndp_node_ip4_rewrite_get: one entry of the rewrite table (tests, tools);
 * -EINVAL for next_hop >= 64, -ENOENT when the table was never allocated. */
int cndp_node_ip4_lookup_init(void);
struct cne_fib *cndp_node_ip4_lookup_fib(void);
void cndp_node_ip4_lookup_fini(void);
int cndp_node_ip4_rewrite_get(uint16_t next_hop, uint8_t *rewrite_data, uint16_t *rewrite_len,
                              uint16_t *tx_node, uint16_t *enabled);
void cndp_node_ip4_rewrite_reset(void);

/* Host regions (AF_XDP UMEMs, the pktmbuf pool: lport_cfg_t.umem_addr /
 * umem_size, cne_lport.h:91) the GPU nodes may read frames from in place.
 * An application that calls this once per UMEM gets zero-copy nodes; without
 * it the nodes stage frame bytes through pinned memory.  Up to 16 regions;
 * -ENOSPC beyond, -EINVAL for a NULL / empty region.
 * cndp_node_gpu_umem_get: region i (-ENOENT past the last). */
int cndp_node_gpu_umem_add(void *addr, uint64_t len);
int cndp_node_gpu_umem_get(uint32_t i, void **addr, uint64_t *len);
void cndp_node_gpu_umem_reset(void);

#ifdef __cplusplus
}
#endif
#endif
