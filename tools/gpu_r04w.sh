#!/bin/bash
# Round-4 session W: the whole GPU suite, the C4 / C5 bins ablation, then the
# C4 / C5 kernel statistics from the bench command with the window probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04w}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 8 "$OUT/${TAG}_$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step pytest 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
step bins 400 python3 -u tools/ab_c4_bins.py c4 c5 || exit 1
step prof 700 bash tools/gpu_r04v.sh $TAG
echo done
