# The one-family regroup's ceiling (bench.py family_group): C4 with the IMIX
# frames reordered inside groups of G frames so IPv4 comes first, interleaved
# with the original order; SPEC=0 also takes the ptype speculation model out
# (a clustered order changes what its passes have to do).
set -e
SPEC=${SPEC:-256}
for r in 1 2; do
for g in 0 128 16777216; do
  CNDP_BENCH_FAMILY_GROUP=$g timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 3 --extra "" --no-node --no-e2e --no-cpu-baseline --no-probe --no-parity --cnet-spec $SPEC > gpurun_out/fg_${SPEC}_${g}_${r}.json 2>> gpurun_out/fg.log
  python -c "import json,sys; d=json.load(open('gpurun_out/fg_${SPEC}_${g}_${r}.json')); print('spec=$SPEC G=$g r=$r', d['roofline']['kernel_ms'], d['ms_per_step'])" >> gpurun_out/fg.txt
done
done
