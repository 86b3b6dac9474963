#!/bin/bash
# SQ (wave-state / instruction-mix / LDS) counters over the bench kernels
# (diagnostic).  One rocprofv3 --pmc pass per group of <= 8 SQ counters; the
# counters the box does not list (rocprofv3 -L) are dropped from a pass.
# usage: tools/pmc_sq.sh <tag> [c4|c5|c3]...   -> gpurun_out/sq_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1 || { echo "counter list failed"; exit 1; }
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
  "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
)
for w in ${*:-c4}; do
    for i in "${!PASSES[@]}"; do
        cs=""
        for c in ${PASSES[$i]}; do
            grep -qw "$c" $OUT/list.txt && cs="$cs $c"
        done
        [ -z "$cs" ] && continue
        echo "[$(date +%T)] $w pass $i:$cs"
        timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $OUT/${w}_p$i -o run -- \
            python3 bench.py --config $w --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-node \
            > $OUT/${w}_p$i.log 2>&1
        rc=$?
        echo "  rc=$rc"
        if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
    done
    python3 tools/pmc_filter.py $(find $OUT/${w}_p* -name '*counter_collection.csv') 2>/dev/null
done
python3 tools/pmc_sq.py $OUT
