#!/usr/bin/env python3
"""Where does the C3 classify kernel spend its time?  (diagnostic, not product)

Runs the product kernel through the C-ABI with outputs / stages removed
(NULL output pointers, HASH mode = no LPM) on the C3 batch, so the cost of
each stage shows up as a time difference on the same box:

    python tools/ablate.py [--tile 1] [--in-route-frac 0.9]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import native as N  # noqa: E402


def timeit(cl, fr, mode, out, stream, reps=30):
    for _ in range(3):
        cl.classify(fr, mode, out=out, stream=stream.cuda_stream)
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        cl.classify(fr, mode, out=out, stream=stream.cuda_stream)
        b.record(stream)
        evs.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--in-route-frac", type=float, default=0.9)
    ap.add_argument("--tiles", default="1,4")
    ap.add_argument("--bpcs", default="2,4")
    ap.add_argument("--nts", default="0,1")
    ap.add_argument("--dir16s", default="1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = bench.build_state("c3", dev, 0, None, args.in_route_frac)
    cl, fr, full = st["cl"], st["frames"], st["out"]
    n = st["n"]
    stream = torch.cuda.Stream(dev)
    L3, HS = N.CNDP_MODE_L3FWD, N.CNDP_MODE_HASH
    cases = [
        ("full (nh,hash,queue,bins)", L3, dict(full)),
        ("no bins", L3, dict(full, bins=None)),
        ("no hash out", L3, dict(full, hash=None)),
        ("nh+queue", L3, dict(full, hash=None, bins=None)),
        ("nh only", L3, dict(full, hash=None, queue=None, bins=None)),
        ("hash mode (no LPM), all outs", HS, dict(full, nh=None)),
        ("hash mode, queue only", HS, dict(full, nh=None, hash=None, bins=None)),
    ]
    ints = lambda v: [int(x) for x in v.split(",")]  # noqa: E731
    for tile in ints(args.tiles):
        for bpc in ints(args.bpcs):
            for nt in ints(args.nts):
                for d16 in ints(args.dir16s):
                    cl.set_tuning(tile=tile, dir16=d16, nt=nt, unroll=1, blocks_per_cu=bpc)
                    for name, mode, out in cases:
                        if d16 == 0 and mode == HS:
                            continue
                        ms = timeit(cl, fr, mode, out, stream)
                        print(f"[ablate tile={tile} bpc={bpc} nt={nt} dir16={d16}] {name:30s} {ms:.4f} ms "
                              f"{n / ms / 1e3:9.1f} Mpps", flush=True)


if __name__ == "__main__":
    main()
