"""Where the GPU eth_rx node's host thread spends its time (diagnostic).

Drives cndp_amd/node/eth_rx_gpu.c built with ETH_RX_GPU_PROF
(tests/node_harness/libcnet_harness_prof.so) through graph walks over the
bench's cnet pool -- 262,144 IMIX mbufs in 2-KiB frames, zero-copy, 256-mbuf
bursts, every pass from the received mbufs -- and prints ns per mbuf for each
phase of the node's process(): pktdev_rx_burst, cndp_gpu_mq_submit, poll,
edge mapping + stats, the per-edge enqueue, waits; the rest of the walk (the
harness's own enqueue bookkeeping) is the difference to the walk time.  The
queue alone (no node: submit / poll from a loop) is timed beside it.
CNDP_GPU_MQ_FLAGS selects the queue's flags for both (default 0, host headers;
4 device headers).
usage: python tools/node_probe_cnet.py [--passes 4] [--json out]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--json")
    args = ap.parse_args()
    import torch
    from cndp_amd import native as N
    from cndp_amd import pktgen
    from cndp_amd.classify import Classifier
    from cndp_amd.fib import Fib, Fib6, node_ip4_add_input, node_ip6_add_input
    from cndp_amd.mbuf import MbufPool, MbufQueue
    assert torch.cuda.is_available()
    L = N.lib()
    H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libcnet_harness_prof.so"))
    H.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_cnet_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    H.harness_eth_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
    H.harness_walk_until.argtypes = [ctypes.c_uint64]
    H.harness_walk_until.restype = ctypes.c_double
    H.harness_mq_drive.restype = ctypes.c_double
    H.harness_mq_drive.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
    H.eth_rx_gpu_prof.argtypes = [ctypes.c_void_p]
    routes, v6 = pktgen.l3fwd_routes(), pktgen.v6_routes()
    f4 = Fib("np4", N.CNE_FIB_DIR24_8, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
    for i, (ip, d, _) in enumerate(routes):
        node_ip4_add_input(f4, ip, d, i)
    f6 = Fib6("np6", N.CNE_FIB_TRIE, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
    for ip, d, i in v6:
        node_ip6_add_input(f6, ip, d, i)
    n = args.n
    pool = MbufPool(n)
    pool.fill(pktgen.imix(n, v4routes=routes, v6routes=v6, seed=98))
    ptrs = pool.ptrs(np.arange(n))
    hdr0 = pool.hdr.copy()
    res = {"mbufs": n, "passes": args.passes}
    # the node, graph walks
    L.cndp_node_gpu_umem_reset()
    L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
    H.harness_cnet_set(f4.h, f6.h)
    H.harness_eth_rx_port(0, 0)
    assert H.harness_graph_create(40) == 0
    phases = np.zeros(6)
    t = 0.0
    buf = np.zeros(6)
    for p in range(args.passes + 1):
        pool.hdr[:] = hdr0
        H.harness_rx_load(0, ptrs, n)
        H.harness_reset_counts()
        H.eth_rx_gpu_prof(buf.ctypes.data)
        dt = H.harness_walk_until(n)
        H.eth_rx_gpu_prof(buf.ctypes.data)
        if p:
            t += dt
            phases += buf
    H.harness_graph_destroy()
    L.cndp_node_gpu_umem_reset()
    tot = n * args.passes
    names = ["pktdev_rx_burst", "mq_submit", "mq_poll", "edge_map_stats", "enqueue_by_edge", "wait"]
    res["node_Mpps"] = round(tot / t / 1e6, 2)
    res["node_ns_per_mbuf"] = round(t / tot * 1e9, 2)
    res["phases_ns_per_mbuf"] = {k: round(v / tot * 1e9, 2) for k, v in zip(names, phases)}
    res["phases_ns_per_mbuf"]["rest_of_walk"] = round((t - phases.sum()) / tot * 1e9, 2)
    # the queue alone
    cl = Classifier(0)
    cl.set_fib(f4, f6)
    cl.host_register(pool.mem)
    flags = int(os.environ.get("CNDP_GPU_MQ_FLAGS", 0))  # as the node takes it
    res["queue_flags"] = flags
    q = MbufQueue(cl, N.CNDP_MQ_CNET, flags=flags, batch=8192, depth=4, umem=pool.base)
    t = 0.0
    for p in range(args.passes + 1):
        pool.hdr[:] = hdr0
        dt = H.harness_mq_drive(q.h, ptrs, n, 256, 1)
        t += dt if p else 0.0
    q.close()
    cl.host_unregister(pool.mem)
    cl.close()
    res["queue_alone_Mpps"] = round(tot / t / 1e6, 2)
    print(json.dumps(res))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
