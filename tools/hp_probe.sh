#!/bin/bash
# zero-copy node queues over a 4 KiB-page pool and a 2 MiB-THP pool
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cat /sys/kernel/mm/transparent_hugepage/enabled
for m in zc zc_hp zc zc_hp; do
    timeout -k 10 120 python3 tools/node_probe_l3.py $m 2>&1 | grep Mpps || exit 1
    timeout -k 10 120 python3 tools/node_probe.py $m 3 2>&1 | grep Mpps || exit 1
done
