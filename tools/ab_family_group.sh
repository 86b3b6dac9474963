set -e
for r in 1 2; do
for g in 0 128 1024 16777216; do
  CNDP_BENCH_FAMILY_GROUP=$g timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 3 --extra "" --no-node --no-e2e --no-cpu-baseline --no-probe --no-parity > gpurun_out/r06b_fg_${g}_${r}.json 2>> gpurun_out/r06b_fg.log
  python -c "import json,sys; d=json.load(open('gpurun_out/r06b_fg_${g}_${r}.json')); print('G=$g r=$r', d['roofline']['kernel_ms'], d['ms_per_step'])" >> gpurun_out/r06b_fg.txt
done
done
