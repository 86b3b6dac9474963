"""Keep only this library's kernels (k_*) in rocprofv3 counter CSVs, in place
(gpurun copies back at most 64 MiB).  python tools/pmc_filter.py <csv>..."""
import csv
import sys

for f in sys.argv[1:]:
    with open(f) as fh:
        rows = list(csv.DictReader(fh))
    if not rows:
        continue
    keep = [r for r in rows if r["Kernel_Name"].startswith(("k_", "void k_"))]
    with open(f, "w", newline="") as o:
        w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(keep)
