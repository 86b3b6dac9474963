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
    buf = np.zeros(8192 * 16, np.uint64)
    assert N.lib().cndp_gpu_debug_stamps(buf.ctypes.data_as(__import__("ctypes").c_void_p), buf.size) == 0
    raw = buf.reshape(-1, 16)
    if os.environ.get("CNET_STAMPS_SAVE"):  # the per-wave rows (wave = block * CT_WAVES + wave in block)
        np.save(os.path.join(os.environ["CNET_STAMPS_SAVE"], f"stamps_{arg.replace(':', '_')}.npy"), raw)
    raw = raw[raw[:, 5] > 0]
    w = raw[:, :8].astype(np.float64)
    per = w[:, [0, 1, 2, 6, 3, 4]] / w[:, 5:6]
    m = per.mean(axis=0)
    print(f"{arg}: {len(w)} waves, {w[:, 5].mean():.1f} trips a wave; cycles a trip: chain {m[0]:.0f}, "
          f"tile+parse+hash {m[1]:.0f}, issue {m[2]:.0f}, speculation words {m[3]:.0f}, result stores "
          f"{m[4]:.0f}; loop {m[5]:.0f} (sum {m[:5].sum():.0f})", flush=True)
    if raw[:, 8].any():  # s_memrealtime timeline (100 MHz), microseconds from the first wave's prologue
        t = (raw[:, 8:12].astype(np.int64) - int(raw[:, 8].min())) / 100.0
        q = lambda c: " / ".join(f"{x:.1f}" for x in np.percentile(t[:, c], [0, 50, 99, 100]))
        lw = t[:, 2] - t[:, 1]
        print(f"  us (min / p50 / p99 / max): prologue issued {q(0)}; loop start {q(1)}; loop end {q(2)}; "
              f"wave end {q(3)}; loop length {lw.min():.1f} / {np.median(lw):.1f} / {lw.max():.1f}; "
              f"clock {np.median(w[:, 4] / np.maximum(lw, 1e-3)) / 1e3:.2f} GHz", flush=True)
        if raw[:, 12].any():
            z = int(raw[:, 8].min())
            tk = raw[:, 14].astype(np.uint64)
            last = (tk >> np.uint64(63)) != 0
            tkt = ((tk & np.uint64((1 << 63) - 1)).astype(np.int64) - z) / 100.0
            q2 = lambda v: " / ".join(f"{x:.1f}" for x in np.percentile(v, [0, 50, 99, 100]))
            print(f"  tail us (min / p50 / p99 / max): odd tiles done {q2((raw[:, 12].astype(np.int64) - z) / 100.0)}; "
                  f"flushes issued {q2((raw[:, 13].astype(np.int64) - z) / 100.0)}; ticket {q2(tkt[raw[:, 14] > 0])}; "
                  f"last block's ticket {tkt[last].max() if last.any() else 0:.1f}, its end "
                  f"{((raw[last, 11].astype(np.int64) - z) / 100.0).max() if last.any() else 0:.1f}", flush=True)
        sp = np.zeros(4096 * 16 + 8, np.uint64)
        if hasattr(N.lib(), "cndp_gpu_debug_spec_stamps") and \
                N.lib().cndp_gpu_debug_spec_stamps(sp.ctypes.data_as(__import__("ctypes").c_void_p), sp.size) == 0:
            kend = int(raw[:, 11].max())
            b = sp[:4096 * 16].reshape(-1, 16).astype(np.int64)
            b = b[b[:, 0] >= kend - 200]  # this launch's blocks (from the last cnet wave's end, 2 us slack)
            if len(b):
                rel = lambda v: (v - kend) / 100.0
                paths = {int(k): int(v) for k, v in zip(*np.unique(b[:, 4], return_counts=True))}
                fill = b[b[:, 2] > 0]
                endv = np.where(b[:, 3] > 0, b[:, 3], b[:, 1])
                print(f"  spec (us after the last cnet wave ended): local_t {len(b)} blocks, paths {paths} "
                      f"(1 unif 2 stop 3 lists-idle 4 lists 5 chunks), list {int(b[:, 5].max())}; first start "
                      f"{rel(b[:, 0].min()):.1f}, last start {rel(b[:, 0].max()):.1f}, inputs in (p50) "
                      f"{np.median(rel(b[:, 1])):.1f}, tables filled (p50 / max) "
                      f"{np.median(rel(fill[:, 2])) if len(fill) else 0:.1f} / {rel(fill[:, 2].max()) if len(fill) else 0:.1f}, "
                      f"last end {rel(endv.max()):.1f}", flush=True)
                v15 = b[b[:, 15] > 0][:, 15]
                if len(v15):
                    print(f"    first burst: longest walk (groups) p50 {np.median(v15 & 0xffffffff):.0f} max "
                          f"{(v15 & 0xffffffff).max()}, walking lanes p50 {np.median(v15 >> 32):.0f}", flush=True)
                for k, nm in ((6, "lookback"), (7, "types staged"), (14, "burst 0 walk set up"), (10, "walk burst 0"), (11, "walk burst 1"),
                              (12, "walk burst 2"), (13, "walk burst 3"), (8, "replay walk"), (9, "replay fixed")):
                    v = b[b[:, k] > 0][:, k]
                    if len(v):
                        print(f"    {nm}: {len(v)} blocks, p50 {np.median(rel(v)):.1f} max {rel(v.max()):.1f}", flush=True)
                f0, f1, fx = (int(v) for v in sp[4096 * 16:4096 * 16 + 3])
                if f0 >= kend:
                    print(f"  fallback block 0: start {rel(f0):.1f}, decided {rel(f1):.1f} (replays {fx & 0xffffffff},"
                          f" full {fx >> 32})", flush=True)
    del st
    torch.cuda.empty_cache()
