#!/bin/bash
# Round-4 session AB: the pipelined-chain cnet kernel: parity, then A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04ab}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 14 "$OUT/${TAG}_$name.log" | grep -v amdgpu.ids
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step parity 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "cnet or c4 or c5 or imix or frame_memory or spec" || exit 1
AB='{"defer": {"cnet_tile": 1}, "pipe": {"cnet_tile": 2}}' step ab 500 python3 -u tools/ab_tune.py c4 c5
echo done
