#!/usr/bin/env python3
"""Summarise a gpurun rocprofv3 session into profiles/ (committed evidence).

    python tools/pmc_summary.py --cfg c3 --round r01 [--out gpurun_out]

Reads <out>/prof_stats/run_kernel_stats.csv (+ kernel trace) and the
separate --pmc passes <out>/prof_fetch, <out>/prof_write, and writes
  profiles/<round>_<cfg>_kernel_stats.csv   (rocprofv3 --stats, verbatim)
  profiles/<round>_<cfg>_pmc.csv            (per-dispatch counters of our kernels)
  profiles/pmc_<cfg>.json                   (what bench.py reports as roofline.traffic)
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) counts 64 B per
L2->fabric read request and reads ½ of a wide coalesced stream, so it is
doubled; WRITE_SIZE (KB) is taken as is; both x 1024.
"""
import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c3")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--kernel", default="k_classify")
    ap.add_argument("--algo-bytes", type=float, default=None)
    ap.add_argument("--packets", type=int, default=1 << 24)
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(args.out, "prof_stats", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{args.round}_{args.cfg}_kernel_stats.csv"))
    rows, fetch, write, dur = [], [], [], []
    for sub, name in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
        p = os.path.join(args.out, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            if args.kernel not in r["Kernel_Name"]:
                continue
            rows.append({k: r[k] for k in ("Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size",
                                            "LDS_Block_Size", "VGPR_Count", "SGPR_Count", "Counter_Name",
                                            "Counter_Value", "Start_Timestamp", "End_Timestamp")})
            v = float(r["Counter_Value"])
            (fetch if name == "FETCH_SIZE" else write).append(v)
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if rows:
        with open(os.path.join(prof, f"{args.round}_{args.cfg}_pmc.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)
    kstats = None
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            if args.kernel in r["Name"]:
                kstats = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                          "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    if fetch and write:
        fkb = statistics.median(fetch)
        wkb = statistics.median(write)
        hbm = 2 * fkb * 1024 + wkb * 1024
        res = {"cfg": args.cfg, "round": args.round, "kernel": args.kernel,
               "fetch_size_kb_median": fkb, "write_size_kb_median": wkb,
               "hbm_read_bytes_corrected": 2 * fkb * 1024, "hbm_write_bytes": wkb * 1024,
               "hbm_bytes_per_launch": hbm,
               "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md HBM section; WRITE_SIZE as is",
               "kernel_stats": kstats}
        if args.algo_bytes:
            res["algorithmic_bytes_per_launch"] = args.algo_bytes * args.packets
            res["traffic_over_algorithmic"] = hbm / (args.algo_bytes * args.packets)
        if kstats:
            res["hbm_gbs_at_avg_duration"] = hbm / kstats["avg_ns"]
        with open(os.path.join(prof, f"pmc_{args.cfg}.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
