#!/bin/bash
# C4 with the speculation chunk lists on (default) and off: kernel timeline
# of each, then interleaved step times.  Diagnostic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/c4_timeline.sh c4 2>&1 | tail -6 || exit 1
for r in 1 2; do
    for l in 1 0; do
        timeout -k 10 300 python3 bench.py --config c4 --steps 30 --warmup 3 --spec-lists $l --no-e2e --no-cpu-baseline \
            --no-imix --no-parity --no-node > gpurun_out/sl_${l}_$r.log 2>&1 || { echo "run failed"; exit 1; }
        echo "lists=$l run $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sl_${l}_$r.log | head -1)"
    done
done
