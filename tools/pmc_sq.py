#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh: per program and kernel, the median over its
dispatches of each SQ counter, and per-wave figures (counter / SQ_WAVES).
    python tools/pmc_sq.py gpurun_out/sq_<tag> [--json out]"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    vals = {}
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        prog = os.path.relpath(f, d).split(os.sep)[0].rsplit("_p", 1)[0]
        for r in csv.DictReader(open(f)):
            k = prog + ":" + r["Kernel_Name"].replace("void ", "").split("(")[0]
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res = {}
    for k, cs in sorted(vals.items()):
        m = {c: statistics.median(v) for c, v in cs.items()}
        w = m.get("SQ_WAVES")
        r = {"counters": m}
        if w:
            r["per_wave"] = {c: round(v / w, 1) for c, v in m.items() if c != "SQ_WAVES"}
        res[k] = r
        print(k, json.dumps(r.get("per_wave", m)))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
