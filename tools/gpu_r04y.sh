#!/bin/bash
# Round-4 session Y: painter tests, then the default bench (with fib_update).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04y}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 4 "$OUT/${TAG}_$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step paint 400 python3 -u -m pytest tests/test_gpu_boundary.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k paint || exit 1
step bench 600 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
grep 'fib update' $OUT/${TAG}_bench.log | cut -c1-600
echo done
