#!/bin/bash
# One C4 bench run under rocprofv3 --kernel-trace: the start / end of the
# cnet kernels of the last timed steps (main kernel, speculation passes) and
# the gaps between them.  Diagnostic: tools/c4_timeline.sh [config]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
cfg=${1:-c4}
out=gpurun_out/tl_$cfg
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out -o run \
    -- python3 bench.py --config $cfg --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-imix --no-parity --no-node \
    > $out/bench.log 2>&1 || { echo "prof failed"; tail -5 $out/bench.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if any(k in n for k in ("k_cnet", "k_spec", "k_classify")):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0][5:40]))
rows.sort()
prev = None
for s, e, n in rows[-24:]:
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{n:36s} dur {(e - s) / 1e3:8.2f} us  gap-before {gap:7.2f} us")
    prev = e
PY
find $out -name '*kernel_trace.csv' -size +20M -delete
