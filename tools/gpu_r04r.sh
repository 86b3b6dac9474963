#!/bin/bash
# Round-4 session R: FIB churn with / without the device painter; probe8 C5/C4
# window reads at 4, 6 and 8 waves a SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04r}
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
step churn_paint 200 python3 -u tools/fib_churn.py || exit 1
CNDP_FIB_PAINT=0 step churn_copy 200 python3 -u tools/fib_churn.py || exit 1
for b in 4 6 8; do step probe8_bpc$b 200 ./tools/probe8 25 $b 1 || exit 1; done
echo done
