"""Route churn cost on the device mirror (diagnostic): K route adds at
scattered prefixes, then the first GPU-selection lookup (which syncs the
mirror); its time and the sync bytes / painter commands (cndp_fib_sync_stats).
Run once with the painter (default) and once with CNDP_FIB_PAINT=0.
python tools/fib_churn.py"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from cndp_amd import native as N  # noqa: E402
from cndp_amd.fib import Fib  # noqa: E402


def stats(f):
    b, c = ctypes.c_uint64(), ctypes.c_uint64()
    N.lib().cndp_fib_sync_stats(f.h, ctypes.byref(b), ctypes.byref(c))
    return b.value, c.value


res = {"painter": os.environ.get("CNDP_FIB_PAINT", "1") != "0"}
rng = np.random.default_rng(3)
f = Fib("churn", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=1 << 16, nh_sz=N.CNE_FIB_DIR24_8_4B,
        num_tbl8=4096, lookup=N.CNE_FIB_LOOKUP_GPU)
keys = rng.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.uint32)
f.lookup_bulk(keys)
for k in (1, 2, 8, 32, 64, 256):
    rows = []
    for rep in range(20):
        for _ in range(k):
            d = int(rng.choice([16, 24, 24, 24, 28, 32]))
            ip = int(rng.integers(0, 2**32)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF)
            f.add(ip, d, int(rng.integers(0, 1 << 15)))
        b0, c0 = stats(f)
        t = time.perf_counter()
        f.lookup_bulk(keys)
        dt = time.perf_counter() - t
        b1, c1 = stats(f)
        rows.append((dt * 1e6, b1 - b0, c1 - c0))
    a = np.array(rows)
    res[f"changes_{k}"] = {"median_us": round(float(np.median(a[:, 0])), 1),
                           "median_bytes": int(np.median(a[:, 1])), "median_cmds": int(np.median(a[:, 2]))}
    print(k, res[f"changes_{k}"], flush=True)
print(json.dumps(res))
