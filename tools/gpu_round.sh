#!/bin/bash
# One GPU-box session: smoke -> pytest -m gpu -> bench -> rocprofv3 stats -> PMC passes.
# Every GPU step has its own time limit; a crash / fault / timeout (rc >= 124)
# stops the script.  Plain test failures (rc 1) still let the bench run.
# usage: tools/gpu_round.sh [all|tests|bench|prof]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
WHAT=${1:-all}
CFG=${CFG:-c3}

step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}

rocm-smi --showproductname > $OUT/smi.log 2>&1 || true

if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
    step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 1200 python3 -m pytest tests -m gpu -q -p no:cacheprovider -x
fi
if [ "$WHAT" = all ] || [ "$WHAT" = sweep ]; then
    step sweep_$CFG 600 python3 bench.py --config $CFG --sweep --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-e2e --no-imix
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
    step bench 600 python3 bench.py --config $CFG --steps 50 --warmup 5
    grep '^{' $OUT/bench.log > $OUT/bench_$CFG.json || true
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
    step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stats -o run \
        -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-imix
    step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run \
        -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-imix
    step prof_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run \
        -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-e2e --no-imix
    # keep only this library's kernels (gpurun returns at most 64 MiB)
    python3 tools/pmc_filter.py $(find $OUT/prof_fetch $OUT/prof_write -name '*counter_collection.csv')
fi
echo done
