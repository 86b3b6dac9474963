#!/bin/bash
# Round-4 session T: the LDS-DMA cnet kernel (CNDP_TUNE_CNET_TILE 2): parity,
# then the C4 / C5 A/B against the register-staged kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04t}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 14 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
P="python3 -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
step parity 500 $P tests/test_gpu_parity.py -k "cnet or c4 or c5 or imix or frame_memory or spec" || exit 1
AB_BPC=${AB_BPC:-5,6,7} step ab 500 python3 -u tools/ab_cnet_tile.py c4 c5
echo done
