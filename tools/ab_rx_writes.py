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
MODE = [0]
_rx_chain = bench.l3fwd_rx_chain


def rx_chain(*a, **k):
    """the receive-chain leg with the stub's writes set; loaded here, after
    node_boundary's ip4_rewrite_set_next calls, as in bench.py"""
    ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "librx_harness.so")).harness_rx_driver_writes(MODE[0])
    return _rx_chain(*a, **k)


bench.l3fwd_rx_chain = rx_chain
out = {"rounds": []}
ROUNDS = int(os.environ.get("AB_ROUNDS", "2"))
for rnd in range(ROUNDS):
    for mode in (0, 1):
        MODE[0] = mode
        ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libcnet_harness.so")).harness_rx_driver_writes(mode)
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
