#!/bin/bash
# Round-4 final evidence on HEAD: the whole GPU suite, smoke, the default bench,
# the headline profile from the bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04final}
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
step pytest 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
step headline 400 bash tools/prof_headline.sh $TAG
python3 tools/kstats.py $OUT/headline_$TAG/prof/run_kernel_stats.csv
echo done
