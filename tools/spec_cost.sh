#!/bin/bash
# C4 main-kernel cost of the ptype-node speculation bookkeeping: kernel stats
# with the model on (default) and off (--cnet-spec 0), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
    for sp in default 0; do
        out=gpurun_out/spec_${sp}_$r
        extra=""
        [ "$sp" = default ] || extra="--cnet-spec 0"
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
            -- python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" $extra \
            > $out.log 2>&1 || { echo "run $sp failed"; exit 1; }
        find $out -name '*kernel_trace.csv' -delete
        echo "spec=$sp"; python3 tools/kstats.py $out/run_kernel_stats.csv
    done
done
