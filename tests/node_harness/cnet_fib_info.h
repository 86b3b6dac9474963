/*
 * Test-only stand-in for cnet_fib_info.h (lib/cnet/incs/cnet_fib_info.h:29-40):
 * the FIB handles the cnet input nodes look up in.  Only the fields the GPU
 * eth_rx node source reads; the harness fills them (cnet_stubs.c).
 */
#ifndef NODE_HARNESS_CNET_FIB_INFO_H
#define NODE_HARNESS_CNET_FIB_INFO_H
#include <stdint.h>
struct cne_fib;
struct cne_fib6;
typedef struct fib_info {
    union {
        struct cne_fib *fib;
        struct cne_fib6 *fib6;
    };
    void **idx2obj;
} fib_info_t;
#endif
