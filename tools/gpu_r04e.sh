#!/bin/bash
# Round-4 session E: node-queue GPU tests, C4 ablation timings (tools/abbuild.sh -DCD_ABL=<bits>,
# interleaved), then the SQ counters of C4 / C5 (tools/pmc_sq.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04e}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 20 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step pytest_mq 400 python3 -u -m pytest tests/test_gpu_mq.py tests/test_node_graph.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread || exit 1
step ab_c4 600 bash tools/abrun.sh "--config c4 --steps 30 --warmup 5" base a1 a2 a3 a4 a8 a16 a31 || exit 1
step sq 600 bash tools/pmc_sq.sh $TAG c4 c5
echo done
