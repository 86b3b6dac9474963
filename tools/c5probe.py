# diagnostic: how many C5 frames does the ptype-node speculation re-route, and from which state?
import sys, os
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench
from cndp_amd import native as N
dev = torch.device("cuda:0")
st = bench.build_state("c5", dev, 0, 1 << 21)
cl = st["cl"] if "cl" in st else st["classifier"]
fr, out = st["frames"], st["out"]
own = None
for k in range(4):
    o = cl.alloc_outputs(fr.n, 64, device=dev, meta=True)
    cl.classify(fr, N.CNDP_MODE_CNET, out=o)
    torch.cuda.synchronize()
    pt = o["ptype"].cpu().numpy() & 0xFFFF
    e = o["edge"].cpu().numpy()
    vals, cnt = np.unique(pt, return_counts=True)
    ev, ec = np.unique(e, return_counts=True)
    print("call", k, "types", dict(zip([hex(v) for v in vals], cnt.tolist())), "edges", dict(zip(ev.tolist(), ec.tolist())))
