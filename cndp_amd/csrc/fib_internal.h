/*
 * fib_internal.h -- table images shared by the host control plane (fib.c)
 * and the device runtime (cndp_gpu.hip).
 *
 * One struct cndp_tbl holds a DIR-24-8 (IPv4) or trie (IPv6) image in the
 * reference's entry encoding (dir24_8.h:27-46 / trie.h:26-40):
 *   tbl24[1<<24]        entry = nh << 1, or (group << 1) | 1 when extended
 *   tbl8[groups*256]    DIR-24-8: (nh << 1) | 1 ; trie: like tbl24 (chains)
 * Entry width is 1 << nh_sz bytes.  The device mirror is a byte-for-byte copy
 * in HBM, refreshed from the dirty entry ranges on sync.
 */
#ifndef CNDP_FIB_INTERNAL_H
#define CNDP_FIB_INTERNAL_H

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include "rib.h"
#include "../../include/cndp_fib.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CNDP_TBL24_ENT (1u << 24)
#define CNDP_TBL8_GRP 256u
#define CNDP_LK_SLOTS 16u   /* concurrent host-array lookups per table */
#define CNDP_TBL_LOG 1024u  /* changed entry ranges kept per table between syncs */

struct cndp_range {
    uint64_t lo, hi;
};

struct cndp_tbl {
    uint32_t nh_sz;     /* log2(entry bytes) */
    uint32_t is_trie;   /* 0 = DIR-24-8, 1 = IPv6 trie */
    uint8_t *tbl24;
    uint8_t *tbl8;      /* (cap_groups + 1) groups */
    uint64_t *used;     /* bitmap over cap_groups */
    uint32_t num_tbl8;  /* allocatable groups (0 = unlimited, growable) */
    uint32_t cap_groups;
    uint32_t cur_tbl8s;
    /* dirty entry ranges [lo, hi) pending upload */
    uint64_t d24_lo, d24_hi, d8_lo, d8_hi;
    /* the same changes as a list of ranges (the device painter of
     * cndp_tbl_dev_sync: fills / copies of just these entries); more than
     * CNDP_TBL_LOG ranges since the last sync falls back to copying the
     * bounding ranges above */
    struct cndp_range log24[CNDP_TBL_LOG], log8[CNDP_TBL_LOG];
    uint32_t n_log24, n_log8;  /* > CNDP_TBL_LOG: overflowed */
    uint64_t sync_bytes;       /* host -> device bytes of all syncs (stat) */
    uint64_t sync_cmds;        /* device painter commands of all syncs (stat) */
    void *paint_host;          /* pinned + mapped painter staging: commands, then payload */
    uint64_t paint_cap;
    /* device mirror */
    int dev_id;
    void *dev_tbl24;
    void *dev_tbl8;
    uint32_t dev_groups; /* groups allocated on the device */
    /* /16 directory in front of tbl24 (DIR-24-8 4-B images, device side):
     * dir16[k] = tbl24 value shared by all 256 entries of /16 block k (bit0
     * clear), or (page << 1) | 1 with pages[page*256 + b] = tbl24[k*256 + b].
     * Built on the host at sync time from the dirty tbl24 range. */
    uint32_t *dir16;     /* 65536 entries */
    int32_t *page_of;    /* page id per /16 block, -1 = uniform */
    uint32_t *pages;     /* cap_pages * 256 entries */
    uint32_t cap_pages;
    uint32_t *page_free;
    uint32_t n_free, n_pages_used, page_hwm;
    uint64_t dd_lo, dd_hi; /* dirty dir16 entries */
    uint64_t dp_lo, dp_hi; /* dirty page entries */
    void *dev_dir16;
    void *dev_pages;
    uint32_t dev_cap_pages;
    /* host-array lookups (cne_fib_lookup_bulk): callers are many forwarding
     * threads on one FIB (examples/cndpfwd/l3-fwd.c:85).  dev_lock guards the
     * host image, its dirty ranges and the device mirror; each small call
     * takes one of the staging slots below for itself, so calls from
     * different threads run concurrently (own stream, staging and flag) */
    uint64_t def_nh;        /* written to every next hop of a lookup that cannot run */
    pthread_mutex_t dev_lock;
    struct cndp_lk_slot {
        int busy;           /* taken by one call (atomic exchange) */
        void *stream;       /* hipStream_t (non-blocking) */
        uint8_t *host;      /* pinned + mapped staging: keys, next hops, completion flag */
        uint8_t *hdev;      /* device address of host */
        uint32_t *ticket;   /* device arrival counter of the call's blocks */
        uint32_t seq;       /* the value the flag takes next */
    } lk[CNDP_LK_SLOTS];
    void *lk_stream;        /* hipStream_t of large lookups (DMA path, under dev_lock) */
    uint8_t *lk_dbuf;       /* device scratch for large lookups */
    /* device buffers replaced while launches on other threads may still hold
     * their address: freed once no launch holds a view of the table (views,
     * taken and counted under dev_lock, dropped after the launch) */
    void **dev_old;
    uint32_t n_old, cap_old;
    uint32_t views;
};

struct cne_fib {
    char name[64];
    enum cne_fib_type type;
    uint64_t def_nh;
    int lookup_type;
    uint32_t rsvd_tbl8s;
    struct cndp_rib rib;
    struct cndp_tbl t;
};

struct cne_fib6 {
    char name[64];
    enum cne_fib_type type;
    uint64_t def_nh;
    int lookup_type;
    uint32_t rsvd_tbl8s;
    struct cndp_rib rib;
    struct cndp_tbl t;
};

/* implemented in cndp_gpu.hip (device side of the mirror) */
int cndp_tbl_dev_sync(struct cndp_tbl *t, void *stream);
void cndp_tbl_dev_free(struct cndp_tbl *t);
int cndp_tbl_lookup4_host(struct cndp_tbl *t, const uint32_t *ips, uint64_t *nh, uint32_t n);
int cndp_tbl_lookup6_host(struct cndp_tbl *t, const uint8_t *ips16, uint64_t *nh, uint32_t n);
int cndp_tbl_lookup4_dev(struct cndp_tbl *t, const uint32_t *ips, uint64_t *nh, uint32_t n,
                         void *stream);
int cndp_tbl_lookup6_dev(struct cndp_tbl *t, const uint8_t *ips16, uint64_t *nh, uint32_t n,
                         void *stream);

#ifdef __cplusplus
}
#endif
#endif
