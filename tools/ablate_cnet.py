#!/usr/bin/env python3
"""Where does the cnet classify kernel spend its time?  (diagnostic, not product)

Times CNDP_MODE_CNET through the C-ABI on variants of the C4 input (IPv6
share 0 / 0.5 / 1, IMIX vs packed 64-B slots) with outputs removed, for both
cnet kernels, on one box:

    python tools/ablate_cnet.py
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from tools.ablate import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = bench.build_state("c4", dev, 0, 1 << 20)   # FIBs + classifier (small batch, replaced below)
    cl, routes, v6 = st["cl"], st["routes"], st["v6routes"]
    n = 1 << 22
    stream = torch.cuda.Stream(dev)
    inputs = [
        ("imix v6=0.5", lambda: pktgen.imix(n, v4routes=routes, v6routes=v6, device=dev, v6_frac=0.5)),
        ("imix v6=0", lambda: pktgen.imix(n, v4routes=routes, v6routes=v6, device=dev, v6_frac=0.0)),
        ("imix v6=1", lambda: pktgen.imix(n, v4routes=routes, v6routes=v6, device=dev, v6_frac=1.0)),
        ("packed64 v4", lambda: pktgen.packed_ipv4(n, routes=routes, device=dev)),
    ]
    made = [(name, make()) for name, make in inputs]   # all generated up front
    torch.cuda.synchronize()
    full = cl.alloc_outputs(n, 64, device=dev, edge=True)
    for name, fr in made:
        cases = [("full", dict(full)), ("nh+edge", dict(full, hash=None, queue=None, bins=None))]
        for ct in (1, 0):
            cl.set_tuning(cnet_tile=ct)
            for cname, out in cases:
                ms = timeit(cl, fr, N.CNDP_MODE_CNET, out, stream)
                print(f"[ablate-cnet {name:12s} cnet_tile={ct}] {cname:8s} {ms:.4f} ms {n / ms / 1e3:9.1f} Mpps",
                      flush=True)


if __name__ == "__main__":
    main()
