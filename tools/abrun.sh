#!/bin/bash
# A/B timing (diagnostic): tools/abrun.sh "<bench args>" base name1 name2 ...
# runs bench.py with each library build (base = the default libcndp_gpu.so),
# twice, interleaved; prints kernel_ms per build.  Each run has its own limit.
cd "$(dirname "$0")/.."
args=$1
shift
mkdir -p gpurun_out
for r in 1 2; do
    for v in "$@"; do
        if [ "$v" = base ]; then unset CNDP_GPU_LIB; else export CNDP_GPU_LIB=$PWD/cndp_amd/lib/libcndp_gpu_$v.so; fi
        timeout -k 10 300 python3 bench.py $args --no-e2e --no-cpu-baseline --no-imix --no-parity --no-node \
            > gpurun_out/ab_${v}_$r.log 2>&1 || { echo "run $v failed"; exit 1; }
        echo "$v $r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$r.log | head -1)"
    done
done
