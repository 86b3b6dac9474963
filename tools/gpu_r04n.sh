#!/bin/bash
# Round-4 session N: the node-path GPU tests, probe8 (window reads by slab
# allocation / load flavour), then the whole GPU suite and the default bench.
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
step pytest_nodes 400 python3 -u -m pytest tests/test_gpu_mq.py tests/test_node_graph.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step probe8 400 bash tools/probe8.sh 24
cat $OUT/${TAG}_probe8.log
step pytest 600 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_gpu_mq.py --deselect tests/test_node_graph.py
step bench 600 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
echo done
