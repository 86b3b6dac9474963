/*
 * Test-only stand-in for cnet.h (lib/cnet/cnet/cnet.h:52-53, :72): the cnet
 * instance whose route FIBs the input nodes use, reached through this_cnet.
 */
#ifndef NODE_HARNESS_CNET_H
#define NODE_HARNESS_CNET_H
struct fib_info;
struct cnet {
    struct fib_info *rt4_finfo;
    struct fib_info *rt6_finfo;
};
struct cnet *cnet_get(void);
#define this_cnet cnet_get()
#endif
