#!/bin/bash
# The headline bench invocation itself under rocprofv3 --kernel-trace --stats:
# the bench JSON line and the kernel statistics of the SAME run, side by side,
# so roofline.frac follows from one record (74 B x 16,777,216 / the profile's
# average duration of the C3 kernel / 8 TB/s).  tools/kstats.py summarises.
# usage: tools/prof_headline.sh [tag]   (outputs under gpurun_out/headline_<tag>)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-r03}
out=gpurun_out/headline_$tag
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run \
    -- python3 bench.py --steps 100 --no-cpu-baseline --no-e2e --no-node --extra "" \
    > $out/bench.json 2> $out/bench.log || { echo "profiled bench failed rc=$?"; exit 1; }
find $out/prof -name '*kernel_trace.csv' -size +20M -delete
echo done
