"""Time the ip4_lookup node queue alone per frame path and batch size, beside
the reference node loop on one core, all in one process on one box (for A/B
and rocprofv3 runs): python3 tools/node_probe_l3.py [zc,zcdev,staged]

  zc      zero-copy, the host resolves each frame address from the mbuf header
  zcdev   zero-copy, CNDP_MQ_F_DEVICE_HEADERS: the kernel reads the headers
  staged  the host copies the 16-B window (bytes 20..35) into pinned staging"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.classify import Classifier  # noqa: E402
from cndp_amd.fib import NodeFib, cne_node_ip4_route_add  # noqa: E402
from cndp_amd.mbuf import MbufPool, MbufQueue  # noqa: E402
from oracle import oracle as O  # noqa: E402

modes = (sys.argv[1] if len(sys.argv) > 1 else "zc,zcdev,staged").split(",")
H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so"))
H.harness_mq_drive.restype = ctypes.c_double
H.harness_mq_drive.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
n = 1 << 20
routes = pktgen.l3fwd_routes()
L = N.lib()
NodeFib.fini()
L.cndp_node_ip4_lookup_init()
for ip, d, nh in routes:
    cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
cl = Classifier(0)
cl.set_fib(NodeFib())
pool = MbufPool(n)
pool.fill(pktgen.packed_ipv4(n, routes=routes, seed=99))
ptrs = pool.ptrs(np.arange(n))
t24, t8 = (x.copy() for x in NodeFib().image())
cl.host_register(pool.mem)
for mode in modes:
    for batch in (8192, 32768):
        flags = N.CNDP_MQ_F_DEVICE_HEADERS if mode == "zcdev" else 0
        q = MbufQueue(cl, N.CNDP_MQ_IP4_LOOKUP, flags=flags, batch=batch, depth=4,
                      umem=pool.base if mode.startswith("zc") else None)
        H.harness_mq_drive(q.h, ptrs, n, 256, 1)
        t = H.harness_mq_drive(q.h, ptrs, n, 256, 3)
        print(f"{mode} ip4_lookup batch {batch}: {n * 3 / t / 1e6:.2f} Mpps", flush=True)
        q.close()
    O.ip4_lookup_mbufs(ptrs, n, (t24, t8), 256, 1)
    t = O.ip4_lookup_mbufs(ptrs, n, (t24, t8), 256, 3)
    print(f"cpu ip4_lookup node loop, 1 core: {n * 3 / t / 1e6:.2f} Mpps", flush=True)
cl.host_unregister(pool.mem)
