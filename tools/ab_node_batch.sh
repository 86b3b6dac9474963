#!/bin/bash
# Node-queue batch / depth A/B: the default bench's node-boundary section at
# CNDP_GPU_BATCH/CNDP_GPU_DEPTH 8192/4 (default), 4096/8, 2048/16, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/${1:-r04an}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for bd in 8192:4 4096:8 2048:16; do
    b=${bd%:*}; d=${bd#*:}
    echo "[$(date +%T)] batch $b depth $d round $r"
    CNDP_GPU_BATCH=$b CNDP_GPU_DEPTH=$d timeout -k 10 240 python3 -u bench.py --steps 10 --extra "" --no-e2e \
        --no-cpu-baseline > $OUT/b${b}_r$r.json 2> $OUT/b${b}_r$r.log || { echo "rc=$? at $b"; exit 1; }
  done
done
echo done
