"""Time the ip4_lookup node queue alone (zero-copy or staged) per batch size,
for rocprofv3 runs: python3 tools/node_probe_l3.py [zc|staged]"""
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

mode = sys.argv[1] if len(sys.argv) > 1 else "zc"
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
pool = MbufPool(n, hugepages=mode.endswith("hp"))
pool.fill(pktgen.packed_ipv4(n, routes=routes, seed=99))
ptrs = pool.ptrs(np.arange(n))
umem = None
if mode.startswith("zc"):
    cl.host_register(pool.mem)
    umem = pool.base
for batch in (8192, 32768):
    q = MbufQueue(cl, N.CNDP_MQ_IP4_LOOKUP, batch=batch, depth=4, umem=umem)
    H.harness_mq_drive(q.h, ptrs, n, 256, 1)
    t = H.harness_mq_drive(q.h, ptrs, n, 256, 3)
    print(f"{mode} ip4_lookup batch {batch}: {n * 3 / t / 1e6:.2f} Mpps", flush=True)
    q.close()
