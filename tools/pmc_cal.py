#!/usr/bin/env python3
"""Summarise tools/pmc_cal.sh: per kernel (median over its dispatches) the
counters of every pass, and the bytes each reading implies, against the known
read bytes of the probe7 calibration kernels.

    python tools/pmc_cal.py gpurun_out/cal [--json profiles/r04_pmc_cal.json]

Per kernel:
  fetch_B      FETCH_SIZE x 1024 (rocprofv3's derived counter, as reported)
  req          TCC_EA0_RDREQ and its 32 / 64 / 128-B parts
  req_B        32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (bytes the request sizes say)
  dram_B       32 x TCC_EA0_RDREQ_DRAM_32B (read bytes to DRAM, size-independent)
  write_B      WRITE_SIZE x 1024
"""
import csv
import glob
import json
import os
import statistics
import sys

KNOWN = {  # probe7 kernels: bytes read per dispatch
    "k_cal_stream": 4 << 30,
    "k_cal_c5<64u>": 64 * (1 << 25),
    "k_cal_c5<128u>": 128 * (1 << 25),
    "k_cal_c5<32u>": 32 * (1 << 25),
    "k_cal_c5<256u>": 256 * (1 << 25),
    "k_cal_c4win": 64 * (1 << 24) + 8 * (1 << 24),
}


def short(name):
    n = name.replace("void ", "")
    n = n.split("(")[0]
    return n


def load(d):
    vals = {}  # "<program>:<kernel>" -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        prog = os.path.relpath(f, d).split(os.sep)[0].split("_")[0]  # probe / c4 / c5 (pass dirs <prog>_<pass>)
        for r in csv.DictReader(open(f)):
            k = prog + ":" + short(r["Kernel_Name"])
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cal"
    out = None
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
    vals = load(d)
    res = {}
    for k, cs in sorted(vals.items()):
        m = {c: statistics.median(v) for c, v in cs.items()}
        r = {"dispatches": max(len(v) for v in cs.values())}
        if "FETCH_SIZE" in m:
            r["fetch_B"] = m["FETCH_SIZE"] * 1024
        if "TCC_EA0_RDREQ_sum" in m:
            r["req"] = {s: m.get(c) for s, c in (("all", "TCC_EA0_RDREQ_sum"), ("32B", "TCC_EA0_RDREQ_32B_sum"),
                                                 ("64B", "TCC_EA0_RDREQ_64B_sum"),
                                                 ("128B", "TCC_EA0_RDREQ_128B_sum"))}
            r["req_B"] = sum(b * (m.get(c) or 0.0) for b, c in ((32, "TCC_EA0_RDREQ_32B_sum"),
                                                               (64, "TCC_EA0_RDREQ_64B_sum"),
                                                               (128, "TCC_EA0_RDREQ_128B_sum")))
        if "TCC_EA0_RDREQ_DRAM_32B_sum" in m:
            r["dram_B"] = 32 * m["TCC_EA0_RDREQ_DRAM_32B_sum"]
            r["dram_req"] = m.get("TCC_EA0_RDREQ_DRAM_sum")
            r["bubble"] = m.get("TCC_BUBBLE_sum")
        if "WRITE_SIZE" in m:
            r["write_B"] = m["WRITE_SIZE"] * 1024
        for kk, known in KNOWN.items():
            kn = k.split(":", 1)[1]
            if kn == kk or kn.startswith(kk):
                r["known_read_B"] = known
                for f in ("fetch_B", "req_B", "dram_B"):
                    if f in r:
                        r[f + "_over_known"] = round(r[f] / known, 4)
        res[k] = r
    for k, r in res.items():
        print(k, json.dumps(r))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
