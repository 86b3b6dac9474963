"""Print this library's kernels from rocprofv3 --stats csv files (avg / min / max µs)."""
import csv
import sys

for p in sys.argv[1:]:
    print("==", p)
    for r in csv.DictReader(open(p)):
        if " k_" in " " + r["Name"].replace("void ", " "):
            print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>4s} avg={float(r['AverageNs']) / 1e3:8.2f} "
                  f"min={float(r['MinNs']) / 1e3:8.2f} max={float(r['MaxNs']) / 1e3:8.2f}")
