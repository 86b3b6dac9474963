"""C1 request latency (cndpfwd loopback, 512 packets as two 256-bursts) through
the MAC-swap node queue at several batch / depth settings (diagnostic).
python tools/c1_lat.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.classify import Classifier  # noqa: E402
from cndp_amd.mbuf import MbufPool, MbufQueue  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so"))
H.harness_mq_latency.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int,
                                 ctypes.c_void_p]
cl = Classifier(0)
pool = MbufPool(512)
pool.fill(pktgen.cndpfwd_udp(512))
ptrs = pool.ptrs(np.arange(512))
reps = 400
for zc in (True, False):
    if zc:
        cl.host_register(pool.mem)
    for batch, depth in ((256, 2), (512, 2), (512, 1), (256, 4)):
        os.environ.pop("CNDP_GPU_DELAY_US", None)
        q = MbufQueue(cl, N.CNDP_MQ_MAC_SWAP, batch=batch, depth=depth, umem=pool.base if zc else None)
        us = np.zeros(reps)
        rc = H.harness_mq_latency(q.h, ptrs, 512, 256, reps, us.ctypes.data)
        q.close()
        print(f"{'zc' if zc else 'staged':6s} batch {batch:3d} depth {depth}: rc {rc} median {np.median(us[20:]):6.1f} us"
              f" p99 {np.percentile(us[20:], 99):6.1f}", flush=True)
    if zc:
        cl.host_unregister(pool.mem)
