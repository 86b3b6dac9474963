/*
 * rib.h -- control-plane route store for the GPU FIBs.
 *
 * A path-compressed binary trie over 128-bit keys (IPv4 routes live in the
 * top 32 bits).  It provides the RIB queries the FIB builders need, with the
 * observable behaviour of the reference RIB (lib/usr/clib/rib/cne_rib.c,
 * cne_rib6.c): node budget = max_nodes (route nodes + branch nodes, so
 * insert fails exactly when the reference's node mempool would run dry),
 * exact / longest-prefix lookups, nearest valid ancestor, and "is there a
 * more specific route inside ip/depth" (cne_rib_get_nxt(..., COVER) != NULL).
 * Host-only; never touched by a kernel.
 */
#ifndef CNDP_RIB_H
#define CNDP_RIB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t hi, lo;
} cndp_key128;

struct cndp_rnode {
    cndp_key128 key;
    uint8_t depth;
    uint8_t valid;
    uint64_t nh;
    struct cndp_rnode *kid[2];
    struct cndp_rnode *up;
};

struct cndp_rib {
    struct cndp_rnode *root;
    uint32_t nodes;
    uint32_t max_nodes;
    uint32_t routes;
    uint8_t max_depth; /* 32 or 128 */
};

static inline cndp_key128 cndp_key_from_v4(uint32_t ip)
{
    cndp_key128 k = {(uint64_t)ip << 32, 0};
    return k;
}
cndp_key128 cndp_key_from_v6(const uint8_t ip[16]);
void cndp_key_to_v6(cndp_key128 k, uint8_t ip[16]);
cndp_key128 cndp_key_mask(cndp_key128 k, uint32_t depth);
int cndp_key_bit(cndp_key128 k, uint32_t pos); /* pos 0 = most significant */
int cndp_key_covered(cndp_key128 k, cndp_key128 pfx, uint32_t depth);

int cndp_rib_init(struct cndp_rib *rib, uint32_t max_nodes, uint8_t max_depth);
void cndp_rib_fini(struct cndp_rib *rib);

/* returns the (valid) node, or NULL if it already exists or no node left */
struct cndp_rnode *cndp_rib_insert(struct cndp_rib *rib, cndp_key128 key, uint32_t depth);
void cndp_rib_remove(struct cndp_rib *rib, cndp_key128 key, uint32_t depth);
struct cndp_rnode *cndp_rib_lookup(const struct cndp_rib *rib, cndp_key128 key);
struct cndp_rnode *cndp_rib_lookup_exact(const struct cndp_rib *rib, cndp_key128 key,
                                         uint32_t depth);
struct cndp_rnode *cndp_rib_parent(const struct cndp_rnode *n);
/* any valid route with depth > `depth` inside key/depth? */
int cndp_rib_has_more_specific(const struct cndp_rib *rib, cndp_key128 key, uint32_t depth);

/* Calls fn for each outermost valid route strictly inside key/depth, in
 * ascending address order (the routes that punch holes into key/depth). */
typedef int (*cndp_rib_visit_fn)(const struct cndp_rnode *n, void *arg);
int cndp_rib_for_each_hole(const struct cndp_rib *rib, cndp_key128 key, uint32_t depth,
                           cndp_rib_visit_fn fn, void *arg);
/* every valid route, pre-order */
int cndp_rib_for_each(const struct cndp_rib *rib, cndp_rib_visit_fn fn, void *arg);

#ifdef __cplusplus
}
#endif
#endif
