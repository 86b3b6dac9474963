#!/usr/bin/env python3
"""profiles/pmc_<cfg>.json (the bench line's roofline.traffic) from a
tools/pmc_cal.py summary: per config, the product kernel's calibrated DRAM
read bytes (32 x TCC_EA0_RDREQ_DRAM_32B, which reads known streams at 1.000x,
DESIGN.md §6 method) plus WRITE_SIZE x 1024, per launch (median of the
profiled dispatches).

    python tools/pmc_json.py <cal.json> <round> [cfg ...]   (default c2 c3 c4 c5)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"c2": "k_classify_stream_bal<2, true, true>", "c3": "k_classify_stream_bal<0, true, true>",
          "c4": "k_cnet_defer<", "c5": "k_cnet_defer<"}
PKTS = {"c2": 1 << 24, "c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25}
ALGO = {"c2": 70, "c3": 74, "c4": 74, "c5": 68}


def main():
    cal = json.load(open(sys.argv[1]))
    rnd = sys.argv[2]
    for cfg in sys.argv[3:] or ["c2", "c3", "c4", "c5"]:
        rows = [(k, v) for k, v in cal.items() if k.startswith(cfg + ":" + KERNEL[cfg])]
        if not rows:
            print(f"{cfg}: no dispatches of {KERNEL[cfg]}")
            continue
        name, r = max(rows, key=lambda kv: kv[1]["dispatches"])
        algo = ALGO[cfg] * PKTS[cfg]
        out = {"cfg": cfg, "round": rnd, "kernel": name.split(":", 1)[1],
               "hbm_read_bytes_dram": r["dram_B"], "hbm_read_bytes_req": r.get("req_B"),
               "fetch_size_bytes_reported": r.get("fetch_B"), "hbm_write_bytes": r["write_B"],
               "hbm_bytes_per_launch": r["dram_B"] + r["write_B"], "dispatches": r["dispatches"],
               "algorithmic_bytes_per_launch": algo,
               "traffic_over_algorithmic": round((r["dram_B"] + r["write_B"]) / algo, 4),
               "note": ("tools/pmc_cal.sh passes over bench.py --config " + cfg + " --steps 3 --warmup 1; read bytes "
                        "= 32 x TCC_EA0_RDREQ_DRAM_32B (1.000x on known streams, profiles/r04_pmc_cal.json), "
                        "writes = WRITE_SIZE x 1024, medians over the dispatches")}
        path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(cfg, out["hbm_bytes_per_launch"], out["traffic_over_algorithmic"])


if __name__ == "__main__":
    main()
