#!/bin/bash
# Round-4 session S: the painter + per-range /16 directory walk: tests, churn A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04s}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 9 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
P="python3 -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread"
step paint 400 $P tests/test_gpu_boundary.py tests/test_gpu_parity.py -k "paint or churn or fib or dir16" || exit 1
step churn_paint 200 python3 -u tools/fib_churn.py || exit 1
CNDP_FIB_PAINT=0 step churn_copy 200 python3 -u tools/fib_churn.py || exit 1
echo done
