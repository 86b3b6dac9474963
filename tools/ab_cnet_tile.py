"""C4 / C5 main kernel A/B: CNDP_TUNE_CNET_TILE 1 (register-staged deferred
chain) vs 2 (LDS-DMA staged, six waves a SIMD), interleaved on the bench's
frames, outputs compared (diagnostic).  python tools/ab_cnet_tile.py [cfg...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
bpcs = [int(x) for x in os.environ.get("AB_BPC", "6").split(",")]


def timed(cl, fr, mode, out, reps=20):
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        cl.classify(fr, mode, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        cl.classify(fr, mode, out=out)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for cfg in sys.argv[1:] or ["c4", "c5"]:
    st = bench.build_state(cfg, dev, 0, None, ring=1)
    cl, fr, mode, out = st["cl"], st["frames"], st["mode"], st["out"]
    variants = [("tile1", dict(cnet_tile=1, blocks_per_cu=0))] + \
        [(f"dma_bpc{b}", dict(cnet_tile=2, blocks_per_cu=b)) for b in bpcs]
    ref = None
    for r in range(3):
        for name, tun in variants:
            cl.set_tuning(**tun)
            cl.set_tuning(cnet_spec=256)  # the same node state at every variant's start
            ms = timed(cl, fr, mode, out)
            cl.set_tuning(cnet_spec=256)
            cl.classify(fr, mode, out=out)
            torch.cuda.synchronize()
            got = {k: out[k].clone() for k in ("nh", "hash", "queue", "edge")}
            if ref is None:
                ref = got
            diff = {k: int((got[k] != ref[k]).sum()) for k in got}
            print(f"{cfg} {name:10s} round {r}: {ms:.4f} ms per call  diffs {diff}", flush=True)
    cl.set_tuning(cnet_tile=1, blocks_per_cu=0)
    del st, fr, out
    torch.cuda.empty_cache()
