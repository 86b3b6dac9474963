#!/bin/bash
# C4 kernel statistics of the default build and the inline-replay build
# ("inl", tools/abbuild.sh inl -DCNDP_SPEC_INLINE=1), one rocprofv3 run each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base inl; do
    if [ $v = base ]; then unset CNDP_GPU_LIB; else export CNDP_GPU_LIB=$PWD/cndp_amd/lib/libcndp_gpu_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_$v -o run \
        -- python3 bench.py --config c4 --steps 30 --warmup 3 --no-e2e --no-cpu-baseline --no-imix --no-parity --no-node \
        > gpurun_out/sp_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
    find gpurun_out/sp_$v -name '*kernel_trace.csv' -size +20M -delete
    python3 - gpurun_out/sp_$v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("k_cnet", "k_spec", "k_classify")):
            print(r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
