"""Counter values per dispatch, in dispatch order, runs of the same kernel
collapsed to their mean (diagnostic).  python tools/pmc_seq.py <csv>..."""
import collections
import csv
import sys

disp = collections.OrderedDict()
for f in sys.argv[1:]:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            d = disp.setdefault(int(r["Dispatch_Id"]), {"k": r["Kernel_Name"]})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
runs = []
for _, d in sorted(disp.items()):
    if runs and runs[-1][0] == d["k"]:
        runs[-1][1].append(d)
    else:
        runs.append((d["k"], [d]))
for k, ds in runs:
    keys = sorted(x for x in ds[0] if x != "k")
    vals = " ".join(f"{c}={sum(d.get(c, 0) for d in ds) / len(ds):.4g}" for c in keys)
    print(f"{k[:40]:40s} x{len(ds):<3d} {vals}")
