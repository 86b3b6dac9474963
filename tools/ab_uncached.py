"""C4 / C5 main kernels on the bench's frames in a hipMalloc'd (torch) slab vs
the same bytes copied into hipExtMallocWithFlags(hipDeviceMallocUncached /
Finegrained) slabs, interleaved (diagnostic).  python tools/ab_uncached.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda:0")
torch.cuda.init()


class Buf:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 2,
                                         "strides": None}


def hip_slab(n, flag):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(flag))
    assert rc == 0, rc
    return p, torch.as_tensor(Buf(p.value, n), device=dev)


def timed(cl, fr, mode, out, reps=20):
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        cl.classify(fr, mode, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        cl.classify(fr, mode, out=out)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for cfg in sys.argv[1:] or ["c4", "c5"]:
    st = bench.build_state(cfg, dev, 0, None, ring=1)
    cl, fr, mode, out = st["cl"], st["frames"], st["mode"], st["out"]
    variants = {"hipMalloc": fr}
    keep = []
    for name, flag in (("uncached", 3), ("finegrained", 1)):
        p, t = hip_slab(fr.slab.numel(), flag)
        t.copy_(fr.slab)
        keep.append(p)
        variants[name] = pktgen.Frames(t, fr.n, stride=fr.stride, offsets=fr.offsets, data_off=fr.data_off,
                                       lengths=fr.lengths)
    ref = None
    for r in range(2):
        for name, f in variants.items():
            ms = timed(cl, f, mode, out)
            got = {k: out[k].clone() for k in ("hash", "queue", "nh")}
            if ref is None:
                ref = got
            same = all(torch.equal(got[k], ref[k]) for k in ("hash", "queue"))
            dnh = int((got["nh"] != ref["nh"]).sum())
            print(f"{cfg} {name:12s} round {r}: {ms:.4f} ms per call  hash/queue {'same' if same else 'DIFFER'}"
                  f"  nh diffs {dnh}", flush=True)
    del variants, st, fr, out
    for p in keep:
        hip.hipFree(p)
    torch.cuda.empty_cache()
