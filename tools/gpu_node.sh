#!/bin/bash
# node-path check: the mq tests, then the bench's node-boundary rates (C3 line only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mq.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mq_tests.log 2>&1 || { tail -30 gpurun_out/mq_tests.log; exit 1; }
tail -2 gpurun_out/mq_tests.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --extra "" > gpurun_out/node_bench.log 2>&1 || exit 1
grep -o '"node_boundary".*' gpurun_out/node_bench.log | head -c 1500
