#!/bin/bash
# Round-4 session V: C4 / C5 kernel statistics from the bench command under
# rocprofv3, with the window-read probe re-run on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04v}
for cfg in c4 c5; do
    d=$OUT/${TAG}_$cfg
    mkdir -p $d
    echo "[$(date +%T)] $cfg"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/prof -o run \
        -- python3 bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-node --extra "" \
        > $d/bench.json 2> $d/bench.log || { echo "$cfg failed rc=$?"; exit 1; }
    find $d/prof -name '*kernel_trace.csv' -size +20M -delete
    python3 tools/kstats.py $(find $d/prof -name '*kernel_stats.csv') | head -12
done
echo "[$(date +%T)] probe8"
timeout -k 10 200 ./tools/probe8 24 8 1 > $OUT/${TAG}_probe8.log 2>&1 && cat $OUT/${TAG}_probe8.log
echo done
