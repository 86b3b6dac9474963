# The one-family regroup's ceiling (bench.py family_run): C4 with the address
# family drawn once per run of R frames (R = 64: every wave tile one family)
# against the per-frame draw, interleaved; SPEC=0 also takes the ptype
# speculation model out.
set -e
SPEC=${SPEC:-256}
for r in 1 2; do
for g in 0 64 256; do
  CNDP_BENCH_FAMILY_RUN=$g timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 3 --extra "" --no-node --no-e2e --no-cpu-baseline --no-probe --no-parity --cnet-spec $SPEC > gpurun_out/fr_${SPEC}_${g}_${r}.json 2>> gpurun_out/fr.log
  python -c "import json,sys; d=json.load(open('gpurun_out/fr_${SPEC}_${g}_${r}.json')); print('spec=$SPEC run=$g r=$r', d['roofline']['kernel_ms'], d['ms_per_step'])" >> gpurun_out/fr.txt
done
done
