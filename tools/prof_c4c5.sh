# Per-kernel statistics of the C4 and C5 bench lines (rocprofv3 --kernel-trace
# --stats), outputs under gpurun_out/prof_<cfg>_<tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-r06}
for cfg in c4 c5; do
  out=gpurun_out/prof_${cfg}_$tag
  mkdir -p $out
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run \
      -- python3 bench.py --config $cfg --steps 40 --no-cpu-baseline --no-e2e --no-node --no-parity --no-probe --extra "" \
      > $out/bench.json 2> $out/bench.log || { echo "profiled bench failed rc=$?"; exit 1; }
  find $out/prof -name '*kernel_trace.csv' -size +20M -delete
done
echo done
