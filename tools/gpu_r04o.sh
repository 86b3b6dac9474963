#!/bin/bash
# Round-4 session O: node tests again, torch interop check, C4 / C5 on
# uncached / fine-grained frame slabs (interleaved A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04o}
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
step pytest_nodes 400 python3 -u -m pytest tests/test_node_graph.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step cai 120 python3 -u tools/cai_check.py || exit 1
step ab_unc 400 python3 -u tools/ab_uncached.py c4 c5
echo done
