"""The l3fwd-graph node pair on the GPU (ip4_lookup -> ip4_rewrite, harness
chained walks as bench.py's node_boundary drives them) beside the lookup node
alone; host time split between the source-node turns and process() calls
(which include the chained ip4_rewrite).  Diagnostic:
python3 tools/node_probe_chain.py"""
import ctypes
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.fib import NodeFib, cne_node_ip4_route_add  # noqa: E402
from cndp_amd.mbuf import MbufPool  # noqa: E402

H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so"))
H.harness_drive.restype = ctypes.c_double
H.harness_drive.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
H.harness_prof.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
H.cne_node_edge_update.restype = ctypes.c_uint16
H.cne_node_edge_update.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16]
H.cne_node_edge_count.restype = ctypes.c_uint16
H.cne_node_edge_count.argtypes = [ctypes.c_uint32]
H.harness_chain.argtypes = [ctypes.c_int]
n, passes = 1 << 20, 3
routes = pktgen.l3fwd_routes()
L = N.lib()
pool = MbufPool(n)
pool.fill(pktgen.packed_ipv4(n, routes=routes, seed=99))
ptrs = pool.ptrs(np.arange(n))
name = ctypes.create_string_buffer(64)
fl, ne, e0, e1 = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_char_p(), ctypes.c_char_p()
k = H.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
rw_id = [i for i in range(k) if H.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0),
                                                    ctypes.byref(e1)) >= 0 and name.value == b"ip4_rewrite"][0]
L.cndp_node_ip4_rewrite_reset()
rnd = random.Random(7)
for p in range(4):
    nm = ctypes.c_char_p(f"pktdev_tx-{p}".encode())
    H.cne_node_edge_update(rw_id, 0xFFFF, ctypes.byref(nm), 1)
    assert L.ip4_rewrite_set_next(p, H.cne_node_edge_count(rw_id) - 1) == 0
for nh in range(64):
    data = bytes(rnd.randrange(256) for _ in range(12))
    assert L.cne_node_ip4_rewrite_add(nh, ctypes.create_string_buffer(data, 12), 12, nh % 4) == 0
L.cndp_node_gpu_umem_reset()
L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
gid = 50
for rep in range(2):
    for label, chain in (("lookup alone", 0), ("lookup + rewrite", 1)):
        NodeFib.fini()
        H.harness_chain(chain)
        assert H.harness_graph_create(gid) == 0
        gid += 1
        for ip, d, nh in routes:
            cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
        H.harness_drive(b"ip4_lookup", ptrs, n, 256, 1)
        src, proc = ctypes.c_double(), ctypes.c_double()
        H.harness_prof(ctypes.byref(src), ctypes.byref(proc))
        t = H.harness_drive(b"ip4_lookup", ptrs, n, 256, passes)
        H.harness_prof(ctypes.byref(src), ctypes.byref(proc))
        H.harness_graph_destroy()
        print(f"{label} zc: {n * passes / t / 1e6:.2f} Mpps; per mbuf: source turns "
              f"{src.value / n / passes * 1e9:.2f} ns, process {proc.value / n / passes * 1e9:.2f} ns", flush=True)
H.harness_chain(0)
H.harness_edges_reset()
L.cndp_node_gpu_umem_reset()
L.cndp_node_ip4_rewrite_reset()
NodeFib.fini()
