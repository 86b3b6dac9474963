#!/bin/bash
# rocprofv3 evidence for every bench config: kernel stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: one TCC pass each),
# filtered to this library's kernels, summarised into profiles/ by
# tools/pmc_summary.py (run it on the CPU side after gpurun merges gpurun_out/).
# usage: CFGS="c2 c3 c4 c5" tools/prof_configs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
CFGS=${CFGS:-"c2 c3 c4 c5"}
for cfg in $CFGS; do
    out=gpurun_out/p_$cfg
    mkdir -p $out
    args="bench.py --config $cfg --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-node --extra ''"
    echo "[$(date +%T)] $cfg stats"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_stats -o run \
        -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
        > $out/stats.log 2>&1 || { echo "stats failed rc=$?"; exit 1; }
    echo "[$(date +%T)] $cfg fetch"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/prof_fetch -o run \
        -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
        > $out/fetch.log 2>&1 || { echo "fetch failed rc=$?"; exit 1; }
    echo "[$(date +%T)] $cfg write"
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/prof_write -o run \
        -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
        > $out/write.log 2>&1 || { echo "write failed rc=$?"; exit 1; }
    python3 tools/pmc_filter.py $(find $out/prof_fetch $out/prof_write -name '*counter_collection.csv')
    # keep the merged output small: drop the big per-dispatch trace files
    find $out/prof_stats -name '*kernel_trace.csv' -size +20M -delete
done
echo done
