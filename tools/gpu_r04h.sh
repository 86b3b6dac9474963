#!/bin/bash
# Round-4 session H: the default bench line (node A/B with the cnet
# device-header queue) and the eth_rx node's host-time phases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04h}
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
step bench 600 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
step node_cnet 300 python3 -u tools/node_probe_cnet.py --json $OUT/${TAG}_node_cnet.json
CNDP_GPU_MQ_FLAGS=0 step node_cnet_hosthdr 300 python3 -u tools/node_probe_cnet.py --json $OUT/${TAG}_node_cnet_hosthdr.json
echo done
