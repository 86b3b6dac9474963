/*
 * rib.c -- path-compressed binary trie used as the FIBs' control plane.
 * See rib.h.  Node-set semantics match lib/usr/clib/rib/cne_rib.c:219-300
 * (insert creates at most one branch node) and :185-212 (remove splices out
 * invalid nodes that have fewer than two children, walking upwards).
 */
#include "rib.h"

#include <stdlib.h>
#include <string.h>

cndp_key128 cndp_key_from_v6(const uint8_t ip[16])
{
    cndp_key128 k = {0, 0};
    for (int i = 0; i < 8; i++) {
        k.hi = (k.hi << 8) | ip[i];
        k.lo = (k.lo << 8) | ip[8 + i];
    }
    return k;
}

void cndp_key_to_v6(cndp_key128 k, uint8_t ip[16])
{
    for (int i = 7; i >= 0; i--) {
        ip[i] = (uint8_t)(k.hi & 0xff);
        ip[8 + i] = (uint8_t)(k.lo & 0xff);
        k.hi >>= 8;
        k.lo >>= 8;
    }
}

cndp_key128 cndp_key_mask(cndp_key128 k, uint32_t depth)
{
    cndp_key128 r;
    if (depth == 0) {
        r.hi = r.lo = 0;
    } else if (depth <= 64) {
        r.hi = k.hi & (~0ULL << (64 - depth));
        r.lo = 0;
    } else if (depth < 128) {
        r.hi = k.hi;
        r.lo = k.lo & (~0ULL << (128 - depth));
    } else {
        r = k;
    }
    return r;
}

int cndp_key_bit(cndp_key128 k, uint32_t pos)
{
    if (pos < 64)
        return (int)((k.hi >> (63 - pos)) & 1u);
    return (int)((k.lo >> (127 - pos)) & 1u);
}

static inline int key_eq(cndp_key128 a, cndp_key128 b) { return a.hi == b.hi && a.lo == b.lo; }

int cndp_key_covered(cndp_key128 k, cndp_key128 pfx, uint32_t depth)
{
    cndp_key128 x = {k.hi ^ pfx.hi, k.lo ^ pfx.lo};
    x = cndp_key_mask(x, depth);
    return x.hi == 0 && x.lo == 0;
}

static uint32_t common_len(cndp_key128 a, cndp_key128 b)
{
    uint64_t h = a.hi ^ b.hi, l = a.lo ^ b.lo;
    if (h)
        return (uint32_t)__builtin_clzll(h);
    if (l)
        return 64u + (uint32_t)__builtin_clzll(l);
    return 128u;
}

int cndp_rib_init(struct cndp_rib *rib, uint32_t max_nodes, uint8_t max_depth)
{
    if (!rib || max_nodes == 0)
        return -1;
    memset(rib, 0, sizeof(*rib));
    rib->max_nodes = max_nodes;
    rib->max_depth = max_depth;
    return 0;
}

static void free_subtree(struct cndp_rnode *n)
{
    /* iterative post-order free using the up pointers */
    while (n) {
        if (n->kid[0]) {
            n = n->kid[0];
            continue;
        }
        if (n->kid[1]) {
            n = n->kid[1];
            continue;
        }
        struct cndp_rnode *up = n->up;
        if (up) {
            if (up->kid[0] == n)
                up->kid[0] = NULL;
            else
                up->kid[1] = NULL;
        }
        free(n);
        n = up;
    }
}

void cndp_rib_fini(struct cndp_rib *rib)
{
    if (!rib)
        return;
    free_subtree(rib->root);
    rib->root = NULL;
    rib->nodes = rib->routes = 0;
}

static struct cndp_rnode *node_new(struct cndp_rib *rib, cndp_key128 key, uint32_t depth, int valid)
{
    struct cndp_rnode *n = calloc(1, sizeof(*n));
    if (!n)
        return NULL;
    n->key = key;
    n->depth = (uint8_t)depth;
    n->valid = (uint8_t)valid;
    rib->nodes++;
    return n;
}

struct cndp_rnode *cndp_rib_insert(struct cndp_rib *rib, cndp_key128 key, uint32_t depth)
{
    if (!rib || depth > rib->max_depth)
        return NULL;
    key = cndp_key_mask(key, depth);

    struct cndp_rnode **link = &rib->root, *above = NULL;
    while (*link) {
        struct cndp_rnode *n = *link;
        if (n->depth == depth && key_eq(n->key, key)) {
            if (n->valid)
                return NULL; /* route exists */
            n->valid = 1;    /* promote a branch node */
            rib->routes++;
            return n;
        }
        if (n->depth >= depth || !cndp_key_covered(key, n->key, n->depth))
            break;
        above = n;
        link = &n->kid[cndp_key_bit(key, n->depth)];
    }

    if (*link == NULL) {
        if (rib->nodes >= rib->max_nodes)
            return NULL;
        struct cndp_rnode *leaf = node_new(rib, key, depth, 1);
        if (!leaf)
            return NULL;
        leaf->up = above;
        *link = leaf;
        rib->routes++;
        return leaf;
    }

    struct cndp_rnode *old = *link;
    uint32_t split = common_len(key, old->key);
    if (split > depth)
        split = depth;
    if (split > old->depth)
        split = old->depth;

    if (split == depth) {
        /* the new route is an ancestor of `old` */
        if (rib->nodes >= rib->max_nodes)
            return NULL;
        struct cndp_rnode *n = node_new(rib, key, depth, 1);
        if (!n)
            return NULL;
        n->kid[cndp_key_bit(old->key, depth)] = old;
        n->up = old->up;
        old->up = n;
        *link = n;
        rib->routes++;
        return n;
    }

    /* diverge below `split`: a branch node plus the new leaf */
    if (rib->nodes + 2 > rib->max_nodes)
        return NULL;
    struct cndp_rnode *leaf = node_new(rib, key, depth, 1);
    if (!leaf)
        return NULL;
    struct cndp_rnode *br = node_new(rib, cndp_key_mask(key, split), split, 0);
    if (!br) {
        free(leaf);
        rib->nodes--;
        return NULL;
    }
    int side = cndp_key_bit(key, split);
    br->kid[side] = leaf;
    br->kid[!side] = old;
    br->up = old->up;
    old->up = br;
    leaf->up = br;
    *link = br;
    rib->routes++;
    return leaf;
}

struct cndp_rnode *cndp_rib_lookup_exact(const struct cndp_rib *rib, cndp_key128 key,
                                         uint32_t depth)
{
    if (!rib || depth > rib->max_depth)
        return NULL;
    key = cndp_key_mask(key, depth);
    struct cndp_rnode *n = rib->root;
    while (n) {
        if (n->depth == depth && key_eq(n->key, key))
            return n->valid ? n : NULL;
        if (n->depth >= depth || !cndp_key_covered(key, n->key, n->depth))
            return NULL;
        n = n->kid[cndp_key_bit(key, n->depth)];
    }
    return NULL;
}

struct cndp_rnode *cndp_rib_lookup(const struct cndp_rib *rib, cndp_key128 key)
{
    struct cndp_rnode *best = NULL, *n = rib ? rib->root : NULL;
    while (n && cndp_key_covered(key, n->key, n->depth)) {
        if (n->valid)
            best = n;
        if (n->depth >= rib->max_depth)
            break;
        n = n->kid[cndp_key_bit(key, n->depth)];
    }
    return best;
}

struct cndp_rnode *cndp_rib_parent(const struct cndp_rnode *n)
{
    struct cndp_rnode *p = n ? n->up : NULL;
    while (p && !p->valid)
        p = p->up;
    return p;
}

void cndp_rib_remove(struct cndp_rib *rib, cndp_key128 key, uint32_t depth)
{
    struct cndp_rnode *n = cndp_rib_lookup_exact(rib, key, depth);
    if (!n)
        return;
    n->valid = 0;
    rib->routes--;
    while (n && !n->valid) {
        if (n->kid[0] && n->kid[1])
            return; /* still a branch point */
        struct cndp_rnode *child = n->kid[0] ? n->kid[0] : n->kid[1];
        struct cndp_rnode *up = n->up;
        if (child)
            child->up = up;
        if (!up)
            rib->root = child;
        else if (up->kid[0] == n)
            up->kid[0] = child;
        else
            up->kid[1] = child;
        free(n);
        rib->nodes--;
        n = up;
    }
}

/* root of the sub-trie holding every node inside key/depth, or NULL */
static struct cndp_rnode *subtree_of(const struct cndp_rib *rib, cndp_key128 key, uint32_t depth)
{
    key = cndp_key_mask(key, depth);
    struct cndp_rnode *n = rib->root;
    while (n && n->depth < depth) {
        if (!cndp_key_covered(key, n->key, n->depth))
            return NULL;
        n = n->kid[cndp_key_bit(key, n->depth)];
    }
    if (n && !cndp_key_covered(n->key, key, depth))
        return NULL;
    return n;
}

int cndp_rib_for_each_hole(const struct cndp_rib *rib, cndp_key128 key, uint32_t depth,
                           cndp_rib_visit_fn fn, void *arg)
{
    struct cndp_rnode *stack[136];
    int sp = 0;
    struct cndp_rnode *top = subtree_of(rib, key, depth);
    if (top)
        stack[sp++] = top;
    while (sp) {
        struct cndp_rnode *n = stack[--sp];
        if (n->valid && n->depth > depth) {
            int r = fn(n, arg);
            if (r)
                return r;
            continue;
        }
        /* push right first so the left (lower addresses) pops first */
        if (n->kid[1])
            stack[sp++] = n->kid[1];
        if (n->kid[0])
            stack[sp++] = n->kid[0];
    }
    return 0;
}

static int stop_at_first(const struct cndp_rnode *n, void *arg)
{
    (void)n;
    (void)arg;
    return 1;
}

int cndp_rib_has_more_specific(const struct cndp_rib *rib, cndp_key128 key, uint32_t depth)
{
    return cndp_rib_for_each_hole(rib, key, depth, stop_at_first, NULL) != 0;
}

int cndp_rib_for_each(const struct cndp_rib *rib, cndp_rib_visit_fn fn, void *arg)
{
    struct cndp_rnode *stack[136];
    int sp = 0;
    if (rib && rib->root)
        stack[sp++] = rib->root;
    while (sp) {
        struct cndp_rnode *n = stack[--sp];
        if (n->valid) {
            int r = fn(n, arg);
            if (r)
                return r;
        }
        if (n->kid[1])
            stack[sp++] = n->kid[1];
        if (n->kid[0])
            stack[sp++] = n->kid[0];
    }
    return 0;
}
