"""Where a k_cnet_defer loop trip spends its time (diagnostic): the CD_STAMP=1
build (tools/abbuild.sh stamp -DCD_STAMP=1) sums s_memtime deltas per wave
over four stages of cd_trip -- B's FIB chain, A's tile / parse / hash, the
first gather + offsets + window loads issued, B's result stores -- and this
prints their mean cycles per trip over the waves of the last launch, for the
bench's C4 and C5 batches.  usage: python3 tools/cnet_stamps.py [c4 c5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CNDP_GPU_LIB", os.path.join(ROOT, "cndp_amd", "lib", "libcndp_gpu_stamp.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import native as N  # noqa: E402

dev = torch.device("cuda:0")
for arg in sys.argv[1:] or ["c4", "c5"]:
    cfg, _, opt = arg.partition(":")  # c4:nobins -- no bin counters
    st = bench.build_state(cfg, dev, 0, None)
    if opt == "nobins":
        for _, o in st["ring"]:
            o["bins"] = None
    for k in range(6):
        bench.run_step(st, None, k)
    torch.cuda.synchronize()
    buf = np.zeros(8192 * 8, np.uint64)
    assert N.lib().cndp_gpu_debug_stamps(buf.ctypes.data_as(__import__("ctypes").c_void_p), buf.size) == 0
    w = buf.reshape(-1, 8).astype(np.float64)
    w = w[w[:, 5] > 0]
    per = w[:, [0, 1, 2, 6, 3, 4]] / w[:, 5:6]
    m = per.mean(axis=0)
    print(f"{arg}: {len(w)} waves, {w[:, 5].mean():.1f} trips a wave; cycles a trip: chain {m[0]:.0f}, "
          f"tile+parse+hash {m[1]:.0f}, issue {m[2]:.0f}, speculation words {m[3]:.0f}, result stores "
          f"{m[4]:.0f}; loop {m[5]:.0f} (sum {m[:5].sum():.0f})", flush=True)
    del st
    torch.cuda.empty_cache()
