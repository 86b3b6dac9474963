/*
 * cndp_fib.h -- drop-in FIB API of libcndp_gpu.so (IPv4 DIR-24-8 + IPv6 trie).
 *
 * Each entry point keeps the exact name, signature, argument meaning and
 * error behaviour of the reference call it replaces, so code written against
 * CNDP's lib/usr/clib/fib/cne_fib.h and cne_fib6.h builds and links against
 * this library unchanged.  The control plane (RIB + table build) runs on the
 * host and paints one table image in the reference's entry encoding; the
 * image is mirrored to HBM and kept in sync incrementally, and every batch
 * kernel (cndp_gpu.h, the graph nodes) reads the mirror.
 *
 * cne_fib_lookup_bulk / cne_fib6_lookup_bulk answer as the selected lookup
 * says, as in the reference (cne_fib.c:86, cne_fib_select_lookup):
 *   CNE_FIB_LOOKUP_DEFAULT and every scalar / vector selector -- synchronously
 *     on the calling thread from the host image (the prefetching loop of
 *     dir24_8.h:118-148 / trie.h:119-138).  This is what a FIB is created
 *     with, so cnet's per-packet callers (ip4_forward, ip4_output, ARP, ND,
 *     route) keep their CPU rate when this library replaces CNDP's FIB;
 *   CNE_FIB_LOOKUP_GPU (extension, also accepted by DUMMY FIBs) -- a launch
 *     on the device mirror per call; without a usable GPU it returns -ENODEV
 *     and fills every next hop with the FIB default.
 *
 *   reference (CNDP v25.08.0)                    this library
 *   cne_fib.h:103   cne_fib_create               same
 *   cne_fib.h:113   cne_fib_free                 same
 *   cne_fib.h:129   cne_fib_add                  same
 *   cne_fib.h:143   cne_fib_delete               same
 *   cne_fib.h:162   cne_fib_lookup_bulk          same (host image, or GPU when selected)
 *   cne_fib.h:173   cne_fib_get_dp               same (host table image)
 *   cne_fib.h:183   cne_fib_get_rib              returns the build's RIB
 *   cne_fib.h:197   cne_fib_select_lookup        same (+ CNE_FIB_LOOKUP_GPU)
 *   cne_fib6.h:41-138  cne_fib6_*                same set for IPv6, including
 *                                                cne_fib6_get_rib (cne_fib6.h:124)
 *
 * The type definitions below (enums, struct cne_fib_conf, the function
 * typedefs) are token-compatible with the reference's and sit behind the
 * reference's own include guards (_CNE_FIB_H_ / _CNE_FIB6_H_): a translation
 * unit that already included CNDP's cne_fib.h / cne_fib6.h skips them, and the
 * prototypes that follow are then checked by the compiler against the
 * reference declarations (tests/test_abi.py::test_prototypes_match_reference).
 * Extensions (device-resident batches, no reference counterpart):
 *   cndp_fib_lookup_dev / cndp_fib6_lookup_dev, cndp_fib_sync / cndp_fib6_sync,
 *   cndp_fib_sync_stats / cndp_fib6_sync_stats.
 */
#ifndef CNDP_FIB_H
#define CNDP_FIB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct cne_fib;
struct cne_fib6;
struct cne_rib;
struct cne_rib6;

#ifndef CNE_FIB6_MAXDEPTH
#define CNE_FIB6_MAXDEPTH 128 /* private_fib6.h:28 */
#endif

#ifndef _CNE_FIB_H_
#define _CNE_FIB_H_
#define CNE_FIB_MAXDEPTH 32 /* cne_fib.h:31 */
#define IPV6_ADDR_LEN 16    /* cne_inet.h:33 (an enum constant there) */

/* cne_fib.h:34-38 */
enum cne_fib_type {
    CNE_FIB_DUMMY,
    CNE_FIB_DIR24_8,
    CNE_FIB_TRIE
};

/* cne_fib.h:41-45 */
typedef int (*cne_fib_modify_fn_t)(struct cne_fib *fib, uint32_t ip, uint8_t depth,
                                   uint64_t next_hop, int op);
typedef void (*cne_fib_lookup_fn_t)(void *fib, const uint32_t *ips, uint64_t *next_hops,
                                    const unsigned int n);

/* cne_fib.h:47-50 */
enum cne_fib_op {
    CNE_FIB_ADD,
    CNE_FIB_DEL,
};

/* cne_fib.h:53-58: entry width is (1 << nh_sz) bytes */
enum cne_fib_dir24_8_nh_sz {
    CNE_FIB_DIR24_8_1B,
    CNE_FIB_DIR24_8_2B,
    CNE_FIB_DIR24_8_4B,
    CNE_FIB_DIR24_8_8B,
};

/* cne_fib.h:60 */
enum cne_fib_trie_nh_sz { CNE_FIB_TRIE_2B = 1, CNE_FIB_TRIE_4B, CNE_FIB_TRIE_8B };

/* cne_fib.h:63-73, plus CNE_FIB_LOOKUP_GPU appended (every reference selector
 * binds the host loop; CNE_FIB_LOOKUP_GPU the device mirror) */
enum cne_fib_lookup_type {
    CNE_FIB_LOOKUP_DEFAULT,
    CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO,
    CNE_FIB_LOOKUP_DIR24_8_SCALAR_INLINE,
    CNE_FIB_LOOKUP_DIR24_8_SCALAR_UNI,
    CNE_FIB_LOOKUP_DIR24_8_VECTOR_AVX512,
    CNE_FIB_LOOKUP_TRIE_SCALAR,
    CNE_FIB_LOOKUP_TRIE_VECTOR_AVX512,
    CNE_FIB_LOOKUP_GPU
};

/* cne_fib.h:76-91 (same layout) */
struct cne_fib_conf {
    enum cne_fib_type type;
    uint64_t default_nh;
    int max_routes;
    union {
        struct {
            enum cne_fib_dir24_8_nh_sz nh_sz;
            uint32_t num_tbl8;
        } dir24_8;
        struct {
            enum cne_fib_trie_nh_sz nh_sz;
            uint32_t num_tbl8;
        } trie;
    };
};
#endif /* _CNE_FIB_H_ */
#ifndef _CNE_FIB6_H_
#define _CNE_FIB6_H_
#endif
/* the GPU selector's value, also when CNDP's own cne_fib.h defined the enum */
#define CNDP_FIB_LOOKUP_GPU 7

/* ---- IPv4 (lib/usr/clib/fib/cne_fib.h) ---------------------------------- */
struct cne_fib *cne_fib_create(const char *name, struct cne_fib_conf *conf);
void cne_fib_free(struct cne_fib *fib);
int cne_fib_add(struct cne_fib *fib, uint32_t ip, uint8_t depth, uint64_t next_hop);
int cne_fib_delete(struct cne_fib *fib, uint32_t ip, uint8_t depth);
int cne_fib_lookup_bulk(struct cne_fib *fib, uint32_t *ips, uint64_t *next_hops, int n);
void *cne_fib_get_dp(struct cne_fib *fib);
struct cne_rib *cne_fib_get_rib(struct cne_fib *fib);
int cne_fib_select_lookup(struct cne_fib *fib, enum cne_fib_lookup_type type);

/* ---- IPv6 (lib/usr/clib/fib/cne_fib6.h) --------------------------------- */
struct cne_fib6 *cne_fib6_create(const char *name, struct cne_fib_conf *conf);
void cne_fib6_free(struct cne_fib6 *fib);
int cne_fib6_add(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth,
                 uint64_t next_hop);
int cne_fib6_delete(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth);
int cne_fib6_lookup_bulk(struct cne_fib6 *fib, uint8_t ips[][IPV6_ADDR_LEN], uint64_t *next_hops,
                         int n);
void *cne_fib6_get_dp(struct cne_fib6 *fib);
struct cne_rib6 *cne_fib6_get_rib(struct cne_fib6 *fib);
int cne_fib6_select_lookup(struct cne_fib6 *fib, enum cne_fib_lookup_type type);

/* ---- build extensions ---------------------------------------------------
 * Host table image as mirrored to HBM (entry width 1 << nh_sz bytes).
 * tbl24: 1<<24 entries; tbl8: (tbl8_groups) * 256 entries. */
struct cndp_fib_image {
    uint32_t nh_sz;
    uint32_t tbl8_groups;
    const void *tbl24;
    const void *tbl8;
    uint64_t def_nh;
};
int cndp_fib_image(struct cne_fib *fib, struct cndp_fib_image *out);
int cndp_fib6_image(struct cne_fib6 *fib, struct cndp_fib_image *out);

/* Upload pending table changes to the current HIP device (stream may be
 * NULL for the null stream).  Lookups and classify call this themselves. */
int cndp_fib_sync(struct cne_fib *fib, void *stream);
int cndp_fib6_sync(struct cne_fib6 *fib, void *stream);

/* Device-resident bulk lookups: ips / next_hops are device pointers;
 * asynchronous on `stream`. */
int cndp_fib_lookup_dev(struct cne_fib *fib, const uint32_t *ips, uint64_t *next_hops, uint32_t n,
                        void *stream);
int cndp_fib6_lookup_dev(struct cne_fib6 *fib, const uint8_t *ips16, uint64_t *next_hops,
                         uint32_t n, void *stream);

/* counters: tbl8 groups in use / reserved (cne_fib internal state) */
int cndp_fib_stats(struct cne_fib *fib, uint32_t *routes, uint32_t *tbl8_used, uint32_t *rsvd);
int cndp_fib6_stats(struct cne_fib6 *fib, uint32_t *routes, uint32_t *tbl8_used, uint32_t *rsvd);

/* device mirror traffic: host -> device bytes and device painter commands of
 * every sync so far.  A sync paints only the entry ranges changed since the
 * previous one on the device (fills of uniform runs, copies of the rest, the
 * way dir24_8.c:249-453 writes them), or copies the bounding ranges of the
 * changes when there were more than 1024 separate ranges or the mirror is new. */
int cndp_fib_sync_stats(struct cne_fib *fib, uint64_t *bytes, uint64_t *cmds);
int cndp_fib6_sync_stats(struct cne_fib6 *fib, uint64_t *bytes, uint64_t *cmds);

#ifdef __cplusplus
}
#endif
#endif
