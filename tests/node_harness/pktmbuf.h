/*
 * Test-only stand-in for pktmbuf.h: the pktmbuf_t layout of pktmbuf.h:102-204
 * as the node source needs it (offsetof(pktmbuf_t, udata64)).
 */
#ifndef NODE_HARNESS_PKTMBUF_H
#define NODE_HARNESS_PKTMBUF_H
#include <stdint.h>
typedef struct pktmbuf_s {
    void *pooldata;
    void *buf_addr;
    uint32_t hash;
    uint32_t meta_index;
    uint16_t data_off;
    uint16_t lport;
    uint16_t buf_len;
    uint16_t data_len;
    uint32_t packet_type;
    uint16_t refcnt;
    uint16_t rsvd16;
    uint64_t tx_offload;
    uint64_t ol_flags;
    uint64_t udata64;
} pktmbuf_t;
_Static_assert(sizeof(pktmbuf_t) == 64, "pktmbuf_t is one cache line");
#endif
