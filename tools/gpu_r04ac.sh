#!/bin/bash
# Round-4 session AC: bench contract test, then the default bench with the
# full-batch parity checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04ac}
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
step contract 400 python3 -u -m pytest tests/test_bench_contract.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
step bench 800 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
grep 'full batch\|parity' $OUT/${TAG}_bench.log | cut -c1-300
echo done
