"""Which path each k_spec_local_t block took on the bench's C4 / C5 batches
(diagnostic): the CD_STAMP=1 build (tools/abbuild.sh stamp -DCD_STAMP=1)
records per block its start / inputs-in / end times (s_memrealtime, 100 MHz)
and a path code (1 uniform pass, 2 nothing to do: SPEC_SKIP or one low byte,
3 lists mode, a block past the listed chunks, 4 lists mode with a chunk,
5 every chunk looked at); this prints the histogram and the time spans of the
last call.  usage: python3 tools/spec_paths.py [c4 c5]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CNDP_GPU_LIB", os.path.join(ROOT, "cndp_amd", "lib", "libcndp_gpu_stamp.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import native as N  # noqa: E402

BLK = 4096
dev = torch.device("cuda:0")
for cfg in sys.argv[1:] or ["c4", "c5"]:
    st = bench.build_state(cfg, dev, 0, None)
    for k in range(6):
        bench.run_step(st, None, k)
    torch.cuda.synchronize()
    buf = np.zeros(BLK * 16 + 8, np.uint64)
    assert N.lib().cndp_gpu_debug_spec_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size) == 0
    rows = buf[:BLK * 16].reshape(BLK, 16)
    live = rows[rows[:, 0] > 0]
    t0 = live[:, 0].min()
    codes, counts = np.unique(live[:, 4], return_counts=True)
    print(f"{cfg}: {len(live)} local blocks; path codes {dict(zip(codes.tolist(), counts.tolist()))}; "
          f"nl {int(live[:, 5].max())}", flush=True)
    for name, col in (("start", 0), ("inputs in", 1), ("LUT in LDS", 2), ("end", 3)):
        v = live[:, col]
        v = v[v > 0]
        if v.size:
            d = (v.astype(np.int64) - int(t0)) / 100.0
            print(f"  {name:10s} p50 {np.median(d):6.2f} us  max {d.max():6.2f} us", flush=True)
    fb = buf[BLK * 16:BLK * 16 + 3]
    if fb[0]:
        print(f"  fallback block 0: start {(int(fb[0]) - int(t0)) / 100:.2f} us, decided "
              f"{(int(fb[1]) - int(t0)) / 100:.2f} us, full {int(fb[2]) >> 32}", flush=True)
