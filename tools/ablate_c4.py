"""C4 cnet ablation (diagnostic): kernel time vs IPv6 share and speculation.
python tools/ablate_c4.py [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd import native as N  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
st = bench.build_state("c4", dev, 0, n, ring=1)
cl = st["cl"]
stream = torch.cuda.current_stream(dev)
for v6 in (0.0, 0.5, 1.0):
    fr = pktgen.imix(n, v4routes=st["routes"], v6routes=st["v6routes"], device=dev, v6_frac=v6)
    out = cl.alloc_outputs(n, 64, device=dev, edge=True)
    for spec in (256, 0):
        cl.set_tuning(cnet_spec=spec)
        for _ in range(3):
            cl.classify(fr, N.CNDP_MODE_CNET, out=out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(10):
            cl.classify(fr, N.CNDP_MODE_CNET, out=out)
        b.record(stream)
        torch.cuda.synchronize()
        print(f"v6_frac {v6:.1f} spec {spec:3d}: {a.elapsed_time(b) / 10:.4f} ms", flush=True)
    del fr, out
