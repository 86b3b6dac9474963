#!/bin/bash
# cnet node queue kernels per mode under rocprofv3 (kernel stats + trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for m in zc staged; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cn_$m -o run \
        -- python3 tools/node_probe.py $m 3 > gpurun_out/cn_$m.log 2>&1 || exit 1
    grep -i mpps gpurun_out/cn_$m.log
    head -12 gpurun_out/cn_$m/run_kernel_stats.csv | cut -d, -f1-4
done
