cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for f in 1.0 0.9 0.0; do
  timeout -k 10 300 python3 bench.py --config c3 --sweep --steps 5 --warmup 2 --no-cpu-baseline --no-parity --in-route-frac $f > gpurun_out/exp_frac_$f.log 2>&1 || exit $?
done
