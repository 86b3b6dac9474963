/*
 * Test-only stand-in for pktmbuf.h: the pktmbuf_t layout of pktmbuf.h:102-204
 * as the node sources need it (offsetof(pktmbuf_t, udata64), pktmbuf_metadata).
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

/* the two fields of pktmbuf_info_t (pktmbuf.h:77-88) pktmbuf_metadata reads
 * (test-only layout: the harness builds these itself) */
typedef struct pktmbuf_info_s {
    uint32_t metadata_bufsz;
    char *metadata;
} pktmbuf_info_t;

/* pktmbuf.h:1209-1220 */
static inline void *pktmbuf_metadata(const pktmbuf_t *m)
{
    const pktmbuf_info_t *p;
    if (!m)
        return (void *)0;
    if ((p = (const pktmbuf_info_t *)m->pooldata) != (void *)0 && p->metadata)
        return p->metadata + (uint64_t)m->meta_index * p->metadata_bufsz;
    return (char *)m + sizeof(pktmbuf_t);
}
#endif
