#!/bin/bash
# GPU check of the cnet speculation passes: parity tests, then per-kernel
# stats and SQ counters for C4 / C5 (tools/pmc_sq.sh).
# usage: KEXPR="speculation or mq" tools/gpu_spec_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu ${KEXPR:+-k "$KEXPR"} \
    > gpurun_out/t_spec.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/t_spec.log; exit 1; }
tail -3 gpurun_out/t_spec.log
for c in ${CFGS:-c4 c5}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$c -o run \
        -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
        > gpurun_out/st_$c.log 2>&1 || { echo "stats $c failed"; exit 1; }
    find gpurun_out/st_$c -name '*kernel_trace.csv' -delete
done
[ -n "$NO_SQ" ] || CFGS="${CFGS:-c4 c5}" bash tools/pmc_sq.sh
