"""Many-seed parity sweep (diagnostic): random frames through every classify
mode, the kernel each layout selects, the CNDP_TUNE_* schedule and
speculation knobs, and chained cnet calls (the ptype node state carried
across two calls) against the oracle, on one GPU.  Seeds, slot sizes,
data offsets and batch lengths vary per round; IMIX and strided C4 / C5
shapes with random destinations are mixed in.  Prints one line per case and
a summary; exit status 1 on any mismatch.

    python3 tools/fuzz_sweep.py [rounds]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from cndp_amd import native as N  # noqa: E402
from cndp_amd import pktgen  # noqa: E402
from cndp_amd.classify import Classifier  # noqa: E402
from oracle import oracle as O  # noqa: E402
from helpers import (CNET_DEF, assert_same, cnet_fibs, l3fwd_fib, l3fwd_oracle_tables,  # noqa: E402
                     oracle_classify)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda:0")
    fib, vals = l3fwd_fib()
    l3 = Classifier(0)
    l3.set_fib(fib)
    t43 = l3fwd_oracle_tables(vals)
    f4, f6, routes, v6, v4vals, v6vals = cnet_fibs()
    cn = Classifier(0)
    cn.set_fib(f4, f6)
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    rng = np.random.default_rng(20261018)
    cases = bad = 0
    t0 = time.time()
    for r in range(rounds):
        seed = int(rng.integers(1, 1 << 30))
        slot = int(rng.choice([64, 80, 97, 128, 192, 256]))
        n = int(rng.integers(1, 120000))
        doff = int(rng.choice([0, 0, 2, 16]))
        fr = pktgen.fuzz_frames(n, seed=seed, slot=slot, device=dev)
        fr.data_off = doff
        shapes = [("fuzz", fr)]
        if r % 3 == 0:
            shapes.append(("imix", pktgen.imix(int(rng.integers(1000, 200000)), v4routes=routes, v6routes=v6,
                                               device=dev, seed=seed, v6_frac=float(rng.random()))))
        if r % 4 == 1:
            shapes.append(("c5", pktgen.packed_ipv4(int(rng.integers(1000, 100000)), slot=1536, frame_len=1500,
                                                    routes=routes, device=dev, seed=seed)))
        for name, f in shapes:
            for mode, cl, kw, variants in (
                    (O.MODE_CNET, cn, dict(tables4=t4, tables6=t6),
                     [dict(cnet_tile=0), dict(cnet_tile=1), dict(cnet_tile=1, stream_bal=2),
                      dict(cnet_tile=1, stream_bal=1), dict(spec_scan=1), dict(spec_scan=2),
                      dict(spec_types=1), dict(spec_types=2), dict(spec_lists=0), dict(spec_grid=1),
                      dict(cnet_fold=1), dict(cnet_fold=2)]),
                    (O.MODE_L3FWD, l3, dict(tables4=t43), [dict(tile=0), dict(tile=1), dict(tile=1, stream_bal=1),
                                                          dict(tile=1, stream_bal=2)]),
                    (O.MODE_HASH, l3, {}, [dict(tile=1), dict(tile=1, stream_bal=1)])):
                if name != "fuzz" and mode != O.MODE_CNET:
                    continue
                ref = oracle_classify(mode, f, **kw)
                nmode = {O.MODE_CNET: N.CNDP_MODE_CNET, O.MODE_L3FWD: N.CNDP_MODE_L3FWD,
                         O.MODE_HASH: N.CNDP_MODE_HASH}[mode]
                for v in variants:
                    cl.set_tuning(**v)
                    if nmode == N.CNDP_MODE_CNET:
                        cl.set_tuning(cnet_spec=256)
                    out = cl.classify(f, nmode, n_bins=64)
                    torch.cuda.synchronize()
                    got = {k: v2 for k, v2 in out.items() if k != "n_bins"}
                    cases += 1
                    try:
                        assert_same(got, ref)
                        status = "ok"
                    except AssertionError as ex:
                        bad += 1
                        status = f"MISMATCH {ex}"
                    print(f"round {r} {name} n={f.n} mode={mode} {v}: {status}", flush=True)
                    cl.set_tuning(stream_bal=0, tile=1, cnet_tile=1, spec_scan=0, spec_types=0, spec_lists=1,
                                  spec_grid=0, cnet_fold=0)
                if nmode == N.CNDP_MODE_CNET and f.n > 512:
                    # chained calls: the ptype node state carried from a first
                    # call over a burst-aligned head into a second one
                    cut = (f.n // 2) // 256 * 256
                    st = np.zeros(1, np.uint16)
                    cl.set_tuning(cnet_spec=256)
                    for lo, hi in ((0, cut), (cut, f.n)):
                        if f.offsets is not None:
                            part = pktgen.Frames(f.slab, hi - lo, offsets=f.offsets[lo:hi].contiguous(),
                                                 data_off=f.data_off)
                        else:
                            part = pktgen.Frames(f.slab[lo * f.stride:], hi - lo, stride=f.stride,
                                                 data_off=f.data_off)
                        r_ = oracle_classify(mode, part, spec_burst=256, spec_state=st, **kw)
                        out = cl.classify(part, nmode, n_bins=64)
                        torch.cuda.synchronize()
                        cases += 1
                        try:
                            assert_same({k: v2 for k, v2 in out.items() if k != "n_bins"}, r_)
                            status = "ok"
                        except AssertionError as ex:
                            bad += 1
                            status = f"MISMATCH {ex}"
                        print(f"round {r} {name} n={part.n} chained [{lo},{hi}): {status}", flush=True)
    print(f"{cases} cases, {bad} mismatches, {time.time() - t0:.0f} s", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
