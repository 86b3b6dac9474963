#!/bin/bash
# Round-4 session N: the node-path GPU tests after the CNDP_MQ_F_REWRITE flag
# fix, then probe8 (window reads by slab allocation / load flavour).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04n}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 4 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step pytest_nodes 400 python3 -u -m pytest tests/test_gpu_mq.py tests/test_node_graph.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread || exit 1
step probe8 400 bash tools/probe8.sh 24
echo done
