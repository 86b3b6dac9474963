"""A/B: the receive nodes (GPU pktdev_rx, GPU eth_rx) with the harness's
pktdev_rx_burst writing each mbuf's data_len / data_off as xskdev's receive
does (xskdev.c:296-297), so the header lines are dirty in the host core's
cache when the node sees them -- against the plain stub (headers as the pool
left them).  Host-read and device-read header forms both.  Interleaved, two
rounds.  usage: python3 tools/ab_rx_writes.py > out.json"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
libs = [ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", f)) for f in ("librx_harness.so", "libcnet_harness.so")]
out = {"rounds": []}
ROUNDS = int(os.environ.get("AB_ROUNDS", "2"))
for rnd in range(ROUNDS):
    for mode in (0, 1):
        for H in libs:
            H.harness_rx_driver_writes(mode)
        nb = bench.node_boundary(dev)
        rc, cn = nb["l3fwd_rx_chain"], nb["cnet"]
        row = {"driver_writes": mode, "round": rnd,
               "rx_chain": {k: v for k, v in rc.items() if k.endswith("_Mpps")},
               "cnet": {k: v for k, v in cn.items() if k.endswith("_Mpps") and "node" in k or k == "cpu_1core_Mpps"},
               "rx_chain_results_equal": rc.get("results_equal_cpu_chain"),
               "rx_chain_mismatches": rc.get("results_mismatches"),
               "cnet_results_equal": cn.get("results_equal_cpu_chain")}
        print(json.dumps(row), file=sys.stderr, flush=True)
        out["rounds"].append(row)
print(json.dumps(out))
