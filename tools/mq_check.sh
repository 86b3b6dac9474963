#!/bin/bash
# node-queue check: the mq + graph-node GPU tests, then the ip4_lookup and cnet queue probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mq.py tests/test_node_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_mq.log 2>&1; r=$?
tail -3 gpurun_out/pytest_mq.log
[ $r -eq 0 ] || exit 1
bash tools/l3_probe.sh && bash tools/cnet_probe.sh
