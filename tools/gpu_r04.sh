#!/bin/bash
# Round-4 GPU session: pytest -m gpu, then the default bench line.  Every GPU
# step has its own time limit; a crash / fault / timeout stops the script.
# usage: tools/gpu_r04.sh <tag> [tests|bench|all]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04}
WHAT=${2:-all}
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
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
    step pytest 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
    step bench 600 python3 -u bench.py
    grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
fi
echo done
