#!/bin/bash
# HBM read-counter calibration (diagnostic).  tools/probe7 "once" launches
# kernels whose read bytes are known exactly (a dense 4 GiB stream; 64/128/
# 32/256 B per 1536-B frame; the C4 IMIX windows); the same counter passes then
# run over the product's C4 / C5 bench kernels.  One rocprofv3 --pmc pass per
# counter group (at most 4 TCC counters a pass, MI355X_MICROARCH.md):
#   fetch : FETCH_SIZE
#   req   : TCC_EA0_RDREQ / _32B / _64B / _128B (request counts by size)
#   dram  : TCC_EA0_RDREQ_DRAM_32B (DRAM read traffic in 32-B units), _DRAM, TCC_BUBBLE
#   write : WRITE_SIZE
# usage: tools/pmc_cal.sh [probe|c4|c5]...   (default: probe c4 c5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/cal
mkdir -p $OUT
WHAT=${*:-probe c4 c5}
declare -A PASS=(
  [fetch]="FETCH_SIZE"
  [req]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  [dram]="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum"
  [write]="WRITE_SIZE"
)
for w in $WHAT; do
    if [ "$w" = probe ]; then
        cmd=(./tools/probe7 once)
    else
        cmd=(python3 bench.py --config $w --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "")
    fi
    for p in fetch req dram write; do
        echo "[$(date +%T)] $w $p"
        timeout -s KILL 240 rocprofv3 --pmc ${PASS[$p]} --output-format csv -d $OUT/${w}_$p -o run -- "${cmd[@]}" \
            > $OUT/${w}_$p.log 2>&1
        rc=$?
        echo "  rc=$rc"
        if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
    done
    python3 tools/pmc_filter.py $(find $OUT/${w}_* -name '*counter_collection.csv') 2>/dev/null
done
python3 tools/pmc_cal.py $OUT
