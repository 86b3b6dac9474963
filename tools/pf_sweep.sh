#!/bin/bash
# staged node-queue host loops: prefetch distance sweep (needs a CNDP_MQ_PF getenv hook in mq_create, not in the product)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rep in 1 2; do for pf in 8 16 32; do
  echo "pf=$pf"; CNDP_MQ_PF=$pf timeout -k 10 120 python3 tools/node_probe_l3.py staged 2>&1 | grep Mpps || exit 1
  CNDP_MQ_PF=$pf timeout -k 10 120 python3 tools/node_probe.py staged 3 2>&1 | grep Mpps || exit 1
done; done
