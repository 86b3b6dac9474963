"""Interleaved A/B of classify tuning knobs on the bench's frames (diagnostic).
AB='{"a": {"dir16": 1}, "b": {"dir16": 0}}' python tools/ab_tune.py c4 c5
Outputs of every variant are compared with the first one's."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
variants = json.loads(os.environ.get("AB", '{"dir16_1": {"dir16": 1}, "dir16_0": {"dir16": 0}}'))


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
    ref = None
    for r in range(3):
        for name, tun in variants.items():
            cl.set_tuning(**tun)
            if mode == 1:
                cl.set_tuning(cnet_spec=256)
            ms = timed(cl, fr, mode, out)
            if mode == 1:
                cl.set_tuning(cnet_spec=256)
            cl.classify(fr, mode, out=out)
            torch.cuda.synchronize()
            got = {k: out[k].clone() for k in ("nh", "hash", "queue") if out.get(k) is not None}
            if ref is None:
                ref = got
            diff = {k: int((got[k] != ref[k]).sum()) for k in got}
            print(f"{cfg} {name:10s} round {r}: {ms:.4f} ms per call  diffs {diff}", flush=True)
    del st, fr, out
    torch.cuda.empty_cache()
