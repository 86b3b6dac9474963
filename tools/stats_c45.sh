cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for cfg in c4 c5; do
  mkdir -p gpurun_out/s_$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s_$cfg -o run -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-node --extra "" > gpurun_out/s_$cfg/log 2>&1 || exit 1
  find gpurun_out/s_$cfg -name '*kernel_trace.csv' -delete
done
