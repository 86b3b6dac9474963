#!/bin/bash
# Round-4 session Q: the device FIB painter (boundary + churn tests), the rx
# node walk, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04q}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 8 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
P="python3 -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread"
step paint 400 $P tests/test_gpu_boundary.py tests/test_gpu_parity.py -k "paint or churn or frame_memory or fib" || exit 1
step rxwalk 300 $P tests/test_node_graph.py -k "rx_node_graph_walk" || exit 1
step pytest 900 $P tests
echo done
