#!/bin/bash
# A/B timing with a bench argument set per build (diagnostic):
#   tools/abpairs.sh ROUNDS "name|lib|bench args" ...
# lib = base (the default libcndp_gpu.so) or a tools/abbuild.sh name; every
# entry runs once per round, interleaved; prints kernel_ms and ms_per_step.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rounds=$1
shift
for r in $(seq 1 "$rounds"); do
    for e in "$@"; do
        IFS='|' read -r name lib args <<< "$e"
        if [ "$lib" = base ]; then unset CNDP_GPU_LIB; else export CNDP_GPU_LIB=$PWD/cndp_amd/lib/libcndp_gpu_$lib.so; fi
        timeout -k 10 300 python3 bench.py $args --no-e2e --no-cpu-baseline --no-imix --no-parity --no-node \
            > gpurun_out/abp_${name}_$r.log 2>&1 || { echo "run $name failed"; tail -5 gpurun_out/abp_${name}_$r.log; exit 1; }
        echo "$name $r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abp_${name}_$r.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_${name}_$r.log | head -1) $(grep -o '"probe_ms": [0-9.]*' gpurun_out/abp_${name}_$r.log | head -1)"
    done
done
