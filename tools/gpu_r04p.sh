#!/bin/bash
# Round-4 session P: the rx node walk with diagnostics, the frame-memory parity test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04p}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 12 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step rxwalk 300 python3 -u -m pytest tests/test_node_graph.py -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "rx_node_graph_walk"
grep -A4 "^DIFF" $OUT/${TAG}_rxwalk.log | head -30
step fmem 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_memory"
echo done
