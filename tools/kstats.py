"""Print our kernels' rocprofv3 --stats rows (diagnostic): python tools/kstats.py <run_kernel_stats.csv>"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if n.startswith("k_") or n.startswith("void k_"):
        print(f"{n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.2f} us")
