set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in zc staged; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l3_$m -o run -- python3 tools/node_probe_l3.py $m > gpurun_out/l3_$m.log 2>&1
cat gpurun_out/l3_$m.log | grep -v "^W\|rocprof" | tail -4
f=$(ls gpurun_out/l3_$m/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/l3_$m/run_kernel_stats.csv); head -5 $f | cut -c1-200
done
