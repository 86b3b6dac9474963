"""Rates of the host-array FIB lookups (cne_fib_lookup_bulk /
cne_fib6_lookup_bulk) in both selections of cne_fib_select_lookup.

* "c_rate": tests/c_link/fib_rate (plain C, no ctypes call in the timed loop):
  per-thread Mlookups/s of the default selection (the host image, what a FIB is
  created with, cne_fib.c:86) and of CNE_FIB_LOOKUP_GPU, for cnet's call shapes
  -- 1 key (ip4_output.c:87,118, cnet_arp.c:77), 4 keys (ip4_forward.c:134-178,
  ip4_lookup.c:141), 256 keys (a burst, examples/cndpfwd/l3-fwd.c:85) -- on
  the rt4 / arp / nd6 FIBs cnet creates, and the default path on 1-8 threads.
* the rest: per-call latency of the GPU selection from Python, n = 4, 256, 64K
  (median / p99 over many calls) and 256-key calls from 1-16 threads.
usage: python tools/fib_latency.py [--json out.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.fib import Fib, Fib6, node_ip4_route_add  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--calls", type=int, default=2000)
    args = ap.parse_args()
    res = {}
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "c_link", "fib_rate")
    import subprocess
    import torch
    r = subprocess.run([exe] + (["--gpu"] if torch.cuda.is_available() else []), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    res["c_rate"] = json.loads(r.stdout)
    f = Fib("lat", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=256, lookup=N.CNE_FIB_LOOKUP_GPU)
    for ip, d, nh in pktgen.l3fwd_routes():
        node_ip4_route_add(f, ip, d, nh, 0)
    f6 = Fib6("lat6", N.CNE_FIB_TRIE, default_nh=0, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15,
              lookup=N.CNE_FIB_LOOKUP_GPU)
    for ip, d, i in pktgen.v6_routes():
        f6.add(ip, d, i)
    rng = np.random.default_rng(0)
    L = N.lib()
    for n in (4, 256, 65536):
        ips = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        ips[::2] = (10 << 24) | (ips[::2] & 0x0003FFFF)
        out = np.zeros(n, np.uint64)
        ips6 = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        ips6[:, :4] = [0x20, 0x01, 0x0d, 0xb8]
        calls = args.calls if n <= 256 else max(50, args.calls // 20)
        for tag, fn, arg in (("v4", L.cne_fib_lookup_bulk, (f.h, ips.ctypes.data, out.ctypes.data, n)),
                             ("v6", L.cne_fib6_lookup_bulk, (f6.h, ips6.ctypes.data, out.ctypes.data, n))):
            for _ in range(20):
                assert fn(*arg) == 0
            t = np.empty(calls)
            for k in range(calls):
                t0 = time.perf_counter_ns()
                fn(*arg)
                t[k] = time.perf_counter_ns() - t0
            res[f"{tag}_n{n}"] = {"median_us": round(float(np.median(t)) / 1e3, 2),
                                 "p99_us": round(float(np.percentile(t, 99)) / 1e3, 2),
                                 "Mlookups_per_s": round(n / (float(np.median(t)) / 1e3), 2)}
    # per-burst callers on several threads (one FIB, 256-key calls): the
    # aggregate rate, as cndpfwd's forwarding threads would see it
    import threading
    for T in (1, 2, 4, 8, 16):
        stop = threading.Event()
        counts = [0] * T

        def worker(w):
            ips = rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)
            out = np.zeros(256, np.uint64)
            a = (f.h, ips.ctypes.data, out.ctypes.data, 256)
            c = 0
            while not stop.is_set():
                L.cne_fib_lookup_bulk(*a)
                c += 1
            counts[w] = c

        th = [threading.Thread(target=worker, args=(w,)) for w in range(T)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        time.sleep(1.0)
        stop.set()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        res[f"v4_n256_threads{T}"] = {"calls_per_s": round(sum(counts) / dt),
                                      "Mlookups_per_s": round(sum(counts) * 256 / dt / 1e6, 2)}
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
