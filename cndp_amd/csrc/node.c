/*
 * node.c -- control plane of the graph nodes libcndp_gpu replaces
 * (include/cndp_node.h).  Restates, with the reference's semantics:
 *   ip4_lookup_nm + setup_fib + cne_node_ip4_route_add
 *                           lib/usr/clib/nodes/ip4_lookup.c:31-42,259-311
 *   ip4_rewrite_nm + ip4_rewrite_set_next + cne_node_ip4_rewrite_add
 *                           lib/usr/clib/nodes/ip4_rewrite.c:266-312
 *   cne_node_ip4_add_input  lib/cnet/ipv4/ip4_input.c:263-272
 *   cne_node_ip6_add_input  lib/cnet/ipv6/ip6_input.c:263-274
 * Both global tables are guarded by one mutex: the reference leaves them
 * unlocked (routes are added from the main thread before the graphs walk),
 * the lock only makes concurrent use by GPU contexts on other threads safe.
 */
#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "node_internal.h"

static pthread_mutex_t node_lock = PTHREAD_MUTEX_INITIALIZER;

/* ---- ip4_lookup (ip4_lookup.c:31-42): one FIB, the socket-0 entry ------- */
static struct cne_fib *ip4_lookup_fib_tbl;

int cndp_node_ip4_lookup_init(void)
{
    int r = 0;
    pthread_mutex_lock(&node_lock);
    if (!ip4_lookup_fib_tbl) {
        /* setup_fib, ip4_lookup.c:292-311 */
        struct cne_fib_conf conf;
        memset(&conf, 0, sizeof(conf));
        conf.type = CNE_FIB_DIR24_8;
        conf.default_nh = ((uint32_t)CNE_NODE_IP4_LOOKUP_NEXT_PKT_DROP) << 16;
        conf.max_routes = 1024;                /* IPV4_L3FWD_FIB_MAX_RULES */
        conf.dir24_8.nh_sz = CNE_FIB_DIR24_8_4B;
        conf.dir24_8.num_tbl8 = 1u << 8;       /* IPV4_L3FWD_FIB_NUMBER_TBL8S */
        ip4_lookup_fib_tbl = cne_fib_create("fib", &conf);
        if (!ip4_lookup_fib_tbl)
            r = errno ? -errno : -ENOMEM;
    }
    pthread_mutex_unlock(&node_lock);
    return r;
}

struct cne_fib *cndp_node_ip4_lookup_fib(void)
{
    pthread_mutex_lock(&node_lock);
    struct cne_fib *f = ip4_lookup_fib_tbl;
    pthread_mutex_unlock(&node_lock);
    return f;
}

void cndp_node_ip4_lookup_fini(void)
{
    pthread_mutex_lock(&node_lock);
    struct cne_fib *f = ip4_lookup_fib_tbl;
    ip4_lookup_fib_tbl = NULL;
    pthread_mutex_unlock(&node_lock);
    cne_fib_free(f);
}

int cne_node_ip4_route_add(uint32_t ip, uint8_t depth, uint16_t next_hop,
                           enum cne_node_ip4_lookup_next next_node)
{
    /* Embedded next node id into 24 bit next hop (ip4_lookup.c:273) */
    const uint32_t val = (uint32_t)((((uint64_t)next_node << 16) | next_hop) & ((1ull << 24) - 1));
    int r = 0;
    pthread_mutex_lock(&node_lock);
    if (ip4_lookup_fib_tbl) /* the reference skips sockets without a FIB */
        r = cne_fib_add(ip4_lookup_fib_tbl, ip, depth, val);
    pthread_mutex_unlock(&node_lock);
    return r < 0 ? r : 0;
}

/* ---- ip4_rewrite (ip4_rewrite_priv.h:45-50) ----------------------------- */
struct rw_main {
    struct cndp_rw_nh nh[CNDP_IP4_REWRITE_MAX_NH];
    uint16_t next_index[CNDP_IP4_REWRITE_MAX_PORTS];
};
static struct rw_main *ip4_rewrite_nm;
static uint64_t rw_gen;

static int rw_alloc(void)
{
    if (!ip4_rewrite_nm) {
        ip4_rewrite_nm = calloc(1, sizeof(*ip4_rewrite_nm));
        if (!ip4_rewrite_nm)
            return -ENOMEM;
    }
    return 0;
}

/* one per GPU node module loaded in a process (each registers from its
 * constructor and removes itself from its destructor, so a module unloaded by
 * dlclose leaves no pointer behind).  hook_lock: ip4_rewrite_set_next calls
 * the hooks under its read side, and unhook takes the write side, so a
 * destructor returns only once no call into its module is in flight. */
#define RW_HOOKS_MAX CNDP_NODE_RW_HOOKS_MAX
static int (*rw_next_hook[RW_HOOKS_MAX])(uint16_t port_id, uint16_t next_index);
static pthread_rwlock_t hook_lock = PTHREAD_RWLOCK_INITIALIZER;

int cndp_node_ip4_rewrite_next_hook(int (*fn)(uint16_t port_id, uint16_t next_index))
{
    if (!fn)
        return -EINVAL;
    int r = -ENOSPC, free_k = -1;
    pthread_rwlock_wrlock(&hook_lock);
    for (int k = 0; k < RW_HOOKS_MAX; k++) {
        if (rw_next_hook[k] == fn) {
            r = 0;
            break;
        }
        if (!rw_next_hook[k] && free_k < 0)
            free_k = k;
    }
    if (r && free_k >= 0) {
        rw_next_hook[free_k] = fn;
        r = 0;
    }
    pthread_rwlock_unlock(&hook_lock);
    return r;
}

int cndp_node_ip4_rewrite_next_unhook(int (*fn)(uint16_t port_id, uint16_t next_index))
{
    int r = -ENOENT;
    pthread_rwlock_wrlock(&hook_lock); /* waits for hook calls in flight */
    for (int k = 0; k < RW_HOOKS_MAX && fn; k++)
        if (rw_next_hook[k] == fn) {
            rw_next_hook[k] = NULL;
            r = 0;
        }
    pthread_rwlock_unlock(&hook_lock);
    return r;
}

int ip4_rewrite_set_next(uint16_t port_id, uint16_t next_index)
{
    if (port_id >= CNDP_IP4_REWRITE_MAX_PORTS)
        return -EINVAL;
    pthread_mutex_lock(&node_lock);
    int r = rw_alloc();
    if (!r)
        ip4_rewrite_nm->next_index[port_id] = next_index;
    pthread_mutex_unlock(&node_lock);
    /* pktdev_ctrl.c:81-84 calls this right after adding the port's tx edge to
     * ip4_rewrite: the GPU rewrite node mirrors that edge on its drain node,
     * the GPU receive node on its own (and its clones'); the hooks run under
     * the read side of hook_lock (a hook must not hook or unhook) */
    pthread_rwlock_rdlock(&hook_lock);
    for (int k = 0; k < RW_HOOKS_MAX && !r; k++)
        if (rw_next_hook[k])
            r = rw_next_hook[k](port_id, next_index);
    pthread_rwlock_unlock(&hook_lock);
    return r;
}

int cne_node_ip4_rewrite_add(uint16_t next_hop, uint8_t *rewrite_data, uint8_t rewrite_len,
                             uint16_t dst_port)
{
    /* same checks in the same order as ip4_rewrite.c:286-302 */
    if (next_hop >= CNDP_IP4_REWRITE_MAX_NH)
        return -EINVAL;
    if (rewrite_len > CNDP_IP4_REWRITE_MAX_LEN)
        return -EINVAL;
    pthread_mutex_lock(&node_lock);
    int r = rw_alloc();
    if (!r && (dst_port >= CNDP_IP4_REWRITE_MAX_PORTS || !ip4_rewrite_nm->next_index[dst_port]))
        r = -EINVAL;
    if (!r && rewrite_len && !rewrite_data)
        r = -EINVAL;
    if (!r) {
        struct cndp_rw_nh *nh = &ip4_rewrite_nm->nh[next_hop];
        if (rewrite_len)
            memcpy(nh->rewrite_data, rewrite_data, rewrite_len);
        nh->tx_node = ip4_rewrite_nm->next_index[dst_port];
        nh->rewrite_len = rewrite_len;
        nh->enabled = 1;
        rw_gen++;
    }
    pthread_mutex_unlock(&node_lock);
    return r;
}

int cndp_node_ip4_rewrite_get(uint16_t next_hop, uint8_t *rewrite_data, uint16_t *rewrite_len,
                              uint16_t *tx_node, uint16_t *enabled)
{
    if (next_hop >= CNDP_IP4_REWRITE_MAX_NH)
        return -EINVAL;
    int r = 0;
    pthread_mutex_lock(&node_lock);
    if (!ip4_rewrite_nm) {
        r = -ENOENT;
    } else {
        const struct cndp_rw_nh *nh = &ip4_rewrite_nm->nh[next_hop];
        if (rewrite_data)
            memcpy(rewrite_data, nh->rewrite_data, CNDP_IP4_REWRITE_MAX_LEN);
        if (rewrite_len)
            *rewrite_len = nh->rewrite_len;
        if (tx_node)
            *tx_node = nh->tx_node;
        if (enabled)
            *enabled = nh->enabled;
    }
    pthread_mutex_unlock(&node_lock);
    return r;
}

void cndp_node_ip4_rewrite_reset(void)
{
    pthread_mutex_lock(&node_lock);
    free(ip4_rewrite_nm);
    ip4_rewrite_nm = NULL;
    rw_gen++;
    pthread_mutex_unlock(&node_lock);
}

uint64_t cndp_node_rw_snapshot(struct cndp_rw_nh *tbl)
{
    pthread_mutex_lock(&node_lock);
    if (ip4_rewrite_nm)
        memcpy(tbl, ip4_rewrite_nm->nh, sizeof(ip4_rewrite_nm->nh));
    else
        memset(tbl, 0, sizeof(struct cndp_rw_nh) * CNDP_IP4_REWRITE_MAX_NH);
    const uint64_t g = rw_gen;
    pthread_mutex_unlock(&node_lock);
    return g;
}

uint64_t cndp_node_rw_gen(void)
{
    pthread_mutex_lock(&node_lock);
    const uint64_t g = rw_gen;
    pthread_mutex_unlock(&node_lock);
    return g;
}

/* ---- cnet input nodes ---------------------------------------------------- */
int cne_node_ip4_add_input(struct cne_fib *fib, uint32_t ip, uint8_t depth, uint32_t idx)
{
    uint64_t nh = idx;
    nh |= (uint64_t)((depth == 32) ? CNDP_INPUT_NEXT_PROTO : CNDP_INPUT_NEXT_FORWARD)
          << CNDP_RT_NEXT_INDEX_SHIFT;
    return cne_fib_add(fib, ip, depth, nh);
}

int cne_node_ip6_add_input(struct cne_fib6 *fib, const uint8_t ip[IPV6_ADDR_LEN], uint8_t depth,
                           uint32_t idx)
{
    uint64_t nh = idx;
    /* ip6_input.c:268 tests depth == 32, not 128: kept */
    nh |= (uint64_t)((depth == 32) ? CNDP_INPUT_NEXT_PROTO : CNDP_INPUT_NEXT_FORWARD)
          << CNDP_RT_NEXT_INDEX_SHIFT;
    return cne_fib6_add(fib, ip, depth, nh);
}

/* ---- regions the GPU nodes may read in place ----------------------------- */
#define UMEM_MAX 16
static struct {
    void *addr;
    uint64_t len;
} umems[UMEM_MAX];
static uint32_t n_umems;

int cndp_node_gpu_umem_add(void *addr, uint64_t len)
{
    if (!addr || !len)
        return -EINVAL;
    int r = 0;
    pthread_mutex_lock(&node_lock);
    if (n_umems == UMEM_MAX) {
        r = -ENOSPC;
    } else {
        umems[n_umems].addr = addr;
        umems[n_umems].len = len;
        n_umems++;
    }
    pthread_mutex_unlock(&node_lock);
    return r;
}

int cndp_node_gpu_umem_get(uint32_t i, void **addr, uint64_t *len)
{
    int r = 0;
    pthread_mutex_lock(&node_lock);
    if (i >= n_umems) {
        r = -ENOENT;
    } else {
        if (addr)
            *addr = umems[i].addr;
        if (len)
            *len = umems[i].len;
    }
    pthread_mutex_unlock(&node_lock);
    return r;
}

void cndp_node_gpu_umem_reset(void)
{
    pthread_mutex_lock(&node_lock);
    n_umems = 0;
    pthread_mutex_unlock(&node_lock);
}
