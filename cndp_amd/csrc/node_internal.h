/*
 * node_internal.h -- node state shared by the host control plane (node.c)
 * and the device runtime (cndp_gpu.hip).  Not part of the exported ABI.
 */
#ifndef CNDP_NODE_INTERNAL_H
#define CNDP_NODE_INTERNAL_H

#include <stdint.h>

#include "../../include/cndp_node.h"

#ifdef __cplusplus
extern "C" {
#endif

/* struct ip4_rewrite_nh_header (ip4_rewrite_priv.h:24-38), same layout */
struct cndp_rw_nh {
    uint16_t rewrite_len;
    uint16_t tx_node;
    uint16_t enabled;
    uint16_t rsvd;
    uint8_t rewrite_data[CNDP_IP4_REWRITE_MAX_LEN];
};

/* Copy the process-global rewrite table (64 entries) into tbl and return its
 * generation (bumped by every change; 0 = never written). */
uint64_t cndp_node_rw_snapshot(struct cndp_rw_nh *tbl);
uint64_t cndp_node_rw_gen(void);

#ifdef __cplusplus
}
#endif
#endif
