#!/bin/bash
# Round-4 session U: default bench (N=1), the two-rank torchrun rehearsal of
# the multi-GPU path (gloo, ranks sharing the box's one GPU), headline profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04u}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 3 "$OUT/${TAG}_$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
step bench 600 python3 -u bench.py || exit 1
grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true
CNDP_DIST_BACKEND=gloo step dist2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-node --no-e2e || exit 1
grep '^{' $OUT/${TAG}_dist2.log > $OUT/${TAG}_dist2.json || true
step headline 400 bash tools/prof_headline.sh $TAG
echo done
