"""The GPU ip4_lookup graph node (harness graph walks, as bench.py's
node_boundary drives it) beside the queue alone and the CPU node loop, with
the host time split between the source-node turns and process() calls; for
rocprofv3 kernel traces.  python3 tools/node_probe_graph.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.fib import NodeFib, cne_node_ip4_route_add  # noqa: E402
from cndp_amd.mbuf import MbufPool  # noqa: E402
from oracle import oracle as O  # noqa: E402

H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so"))
H.harness_drive.restype = ctypes.c_double
H.harness_drive.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
H.harness_prof.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
n = 1 << 20
routes = pktgen.l3fwd_routes()
L = N.lib()
pool = MbufPool(n)
pool.fill(pktgen.packed_ipv4(n, routes=routes, seed=99))
ptrs = pool.ptrs(np.arange(n))
for zc in (True, False, True):
    NodeFib.fini()
    L.cndp_node_gpu_umem_reset()
    if zc:
        L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
    assert H.harness_graph_create(40) == 0
    for ip, d, nh in routes:
        cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
    H.harness_drive(b"ip4_lookup", ptrs, n, 256, 1)
    src, proc = ctypes.c_double(), ctypes.c_double()
    H.harness_prof(ctypes.byref(src), ctypes.byref(proc))
    t = H.harness_drive(b"ip4_lookup", ptrs, n, 256, 3)
    H.harness_prof(ctypes.byref(src), ctypes.byref(proc))
    H.harness_graph_destroy()
    print(f"graph node {'zc' if zc else 'staged'}: {n * 3 / t / 1e6:.2f} Mpps; per mbuf: source turns "
          f"{src.value / n / 3 * 1e9:.2f} ns, process {proc.value / n / 3 * 1e9:.2f} ns", flush=True)
fib = NodeFib()
t24, t8 = (x.copy() for x in fib.image())
O.ip4_lookup_mbufs(ptrs, n, (t24, t8), 256, 1)
t = O.ip4_lookup_mbufs(ptrs, n, (t24, t8), 256, 3)
print(f"cpu ip4_lookup node loop, 1 core: {n * 3 / t / 1e6:.2f} Mpps", flush=True)
NodeFib.fini()
L.cndp_node_gpu_umem_reset()
