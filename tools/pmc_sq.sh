#!/bin/bash
# SQ counters (wave lifetime / stall split / instruction mix) for one bench
# config, one --pmc pass: MI355X_MICROARCH.md allows 8 SQ counters per pass.
# usage: CFGS="c4 c5" tools/pmc_sq.sh   (summarise with tools/pmc_sq.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
CFGS=${CFGS:-"c4 c5"}
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"}
for cfg in $CFGS; do
    out=gpurun_out/sq_$cfg
    mkdir -p $out
    echo "[$(date +%T)] $cfg sq"
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $out/prof -o run \
        -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
        > $out/sq.log 2>&1 || { echo "sq $cfg failed rc=$?"; exit 1; }
    python3 tools/pmc_sq.py $(find $out/prof -name '*counter_collection.csv') > $out/summary.txt
    find $out/prof -name '*counter_collection.csv' -size +20M -delete
    cat $out/summary.txt
done
echo done
