"""The C3 shape's drain (diagnostic): tools/probe_drain.hip's balanced probe
with per-wave end stamps, against run-time tile hand-out across CUs (per-XCD
counters, chunks of 4-32 tiles), interleaved on one box.
usage: python3 tools/probe_drain.py   (libprobe_drain.so built beside it:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/probe_drain.hip -o tools/libprobe_drain.so)"""
import ctypes
import os
import statistics

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
P = ctypes.CDLL(os.path.join(HERE, "libprobe_drain.so"))
vp = ctypes.c_void_p
P.pd_bal.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, vp]
P.pd_dyn.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int, vp, vp]
P.pd_hyb.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int, ctypes.c_uint32, vp, vp]
P.pd_sched.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int, ctypes.c_uint32, vp, vp]

dev = torch.device("cuda:0")
n = 1 << 24
slab = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device=dev)
a = torch.zeros(n, dtype=torch.int32, device=dev)
b = torch.zeros(n, dtype=torch.int32, device=dev)
q = torch.zeros(n, dtype=torch.int16, device=dev)
ctr = torch.zeros(9 * 64, dtype=torch.int32, device=dev)
st = torch.zeros(256 * 8 * 2, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream()
sid = s.cuda_stream


def launch(v, stamps=False):
    sp = st.data_ptr() if stamps else None
    if v == "bal":
        return P.pd_bal(slab.data_ptr(), n, a.data_ptr(), b.data_ptr(), q.data_ptr(), sp, sid)
    if v.startswith("sch"):  # sch<C>_<percent of the rounds static>
        c, pct = v[3:].split("_")
        ks = int((n // 64) // 256 * int(pct) / 100)
        return P.pd_sched(slab.data_ptr(), n, a.data_ptr(), b.data_ptr(), q.data_ptr(), ctr.data_ptr(), int(c), ks,
                          sp, sid)
    if v.startswith("hyb"):  # hyb<C>_<percent of the rounds static>
        c, pct = v[3:].split("_")
        ks = int((n // 64) // 256 * int(pct) / 100)
        return P.pd_hyb(slab.data_ptr(), n, a.data_ptr(), b.data_ptr(), q.data_ptr(), ctr.data_ptr(), int(c), ks,
                        sp, sid)
    return P.pd_dyn(slab.data_ptr(), n, a.data_ptr(), b.data_ptr(), q.data_ptr(), ctr.data_ptr(), int(v[3:]), sp,
                    sid)


variants = ["bal", "sch4_70", "sch4_50", "sch4_60", "sch8_50", "sch8_70", "sch2_70", "sch4_80", "sch8_0", "bal"]
variants = list(dict.fromkeys(variants))
# correctness: every tile's outputs written (each variant from zeroed outputs)
ref = None
for v in variants:
    a.zero_()
    assert launch(v) == 0
    torch.cuda.synchronize()
    got = a.cpu().numpy()
    if ref is None:
        ref = got
    print(f"{v}: outputs equal to bal's: {np.array_equal(got, ref)}", flush=True)

times = {v: [] for v in variants}
for rnd in range(7):
    for v in variants:
        for _ in range(3):
            launch(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(50):
            launch(v)
        e1.record(s)
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 50)
for v in variants:
    print(f"{v}: ms per launch min {min(times[v]):.4f} median {statistics.median(times[v]):.4f} "
          f"({' '.join(f'{x:.4f}' for x in times[v])})", flush=True)

# drain: per-wave end times (100 MHz) of one launch each
for v in ("bal", "sch4_70", "sch4_50"):
    st.zero_()
    launch(v, stamps=True)
    torch.cuda.synchronize()
    w = st.cpu().numpy().reshape(-1, 2)
    end = (w[:, 0] - w[:, 0].min()) / 100.0
    xcc = w[:, 1]
    per = {int(x): round(float(np.median(end[xcc == x])), 2) for x in np.unique(xcc)}
    print(f"{v}: wave ends after the first: p50 {np.median(end):.2f} us, p90 {np.percentile(end, 90):.2f}, "
          f"max {end.max():.2f}; per-XCD p50 {per}", flush=True)
