"""Time the cnet node queue alone (zero-copy or staged), for rocprofv3 runs:
python3 tools/node_probe.py [zc|staged] [passes]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.classify import Classifier  # noqa: E402
from cndp_amd.fib import Fib, Fib6, node_ip4_add_input, node_ip6_add_input  # noqa: E402
from cndp_amd.mbuf import MbufPool, MbufQueue  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "staged"
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so"))
H.harness_mq_drive.restype = ctypes.c_double
H.harness_mq_drive.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
nc = 1 << 18
routes = pktgen.l3fwd_routes()
v6 = pktgen.v6_routes()
cl = Classifier(0)
f4 = Fib("np4", N.CNE_FIB_DIR24_8, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
for i, (ip, d, _) in enumerate(routes):
    node_ip4_add_input(f4, ip, d, i)
f6 = Fib6("np6", N.CNE_FIB_TRIE, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
for ip, d, i in v6:
    node_ip6_add_input(f6, ip, d, i)
cl.set_fib(f4, f6)
pool = MbufPool(nc, hugepages=mode.endswith("hp"))
pool.fill(pktgen.imix(nc, v4routes=routes, v6routes=v6, seed=98))
ptrs = pool.ptrs(np.arange(nc))
hdr0 = pool.hdr.copy()
umem = None
if mode.startswith("zc"):
    cl.host_register(pool.mem)
    umem = pool.base
for batch in (8192, 32768):
    q = MbufQueue(cl, N.CNDP_MQ_CNET, batch=batch, depth=4, umem=umem)
    t = 0.0
    for p in range(passes + 1):  # headers restored: eth_rx advanced data_off
        pool.hdr[:] = hdr0
        dt = H.harness_mq_drive(q.h, ptrs, nc, 256, 1)
        t += dt if p else 0.0
    print(f"{mode} batch {batch}: {nc * passes / t / 1e6:.2f} Mpps ({t * 1e3:.1f} ms)", flush=True)
    q.close()
print("worklist size class after the last call:", N.lib().cndp_gpu_get_stat(cl.h, N.CNDP_STAT_CNET_WORKLIST))
