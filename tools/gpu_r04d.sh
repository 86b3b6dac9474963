#!/bin/bash
# Round-4 session D: GPU tests, the trip-order / table-pointer A/B on
# C4 / C5 / C3 (interleaved builds, tools/abrun.sh), then the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04d}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 6 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step pytest 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
step ab_c4 500 bash tools/abrun.sh "--config c4 --steps 30 --warmup 5" base o0 o0pin
step ab_c5 400 bash tools/abrun.sh "--config c5 --steps 20 --warmup 3" base o0
step ab_c3 300 bash tools/abrun.sh "--config c3 --steps 50 --warmup 5" base o0
step bench 600 python3 -u bench.py
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
echo done
