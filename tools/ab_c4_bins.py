"""C4 main kernel with and without the bin counters (diagnostic): the same
frames classified with out["bins"] set and with it None, interleaved.
python tools/ab_c4_bins.py [cfg...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")


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
    nob = dict(out)
    nob["bins"] = None
    for r in range(3):
        for name, o in (("bins", out), ("no_bins", nob)):
            print(f"{cfg} {name:8s} round {r}: {timed(cl, fr, mode, o):.4f} ms", flush=True)
    del st, fr, out, nob
    torch.cuda.empty_cache()
