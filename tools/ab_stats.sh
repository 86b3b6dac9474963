#!/bin/bash
# A/B kernel stats: for each library variant (cndp_amd/lib/libcndp_gpu_<v>.so,
# "base" = the default build) and config, one rocprofv3 --stats run.
# usage: VARIANTS="base wpb16" CFGS="c4 c5" tools/ab_stats.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
    lib=""
    [ "$v" = base ] || lib=$PWD/cndp_amd/lib/libcndp_gpu_$v.so
    for c in ${CFGS:-c4 c5}; do
        out=gpurun_out/ab_${v}_$c
        CNDP_GPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
            -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" \
            > $out.log 2>&1 || { echo "ab $v $c failed"; exit 1; }
        find $out -name '*kernel_trace.csv' -delete
        python3 tools/kstats.py $out/run_kernel_stats.csv
    done
done
