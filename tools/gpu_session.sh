#!/bin/bash
# One GPU-box session (diagnostic driver for gpurun): the named steps in order,
# each under its own time limit, outputs under gpurun_out/<tag>_<step>.log.
# A fault, abort, segfault or time limit (rc 124/134/137/139) ends the session;
# a failing test run (rc 1) ends it too unless KEEP_GOING=1.
#   tools/gpu_session.sh <tag> <step>...
# steps:
#   smoke            __graft_entry__.smoke()
#   pytest[:expr]    pytest -m gpu (optionally -k expr)
#   bench[:args]     python bench.py <args, comma-separated>   (JSON line -> <tag>_bench.json)
#   headline         the headline bench under rocprofv3 --kernel-trace --stats (tools/prof_headline.sh)
#   prof:<cfg>       bench --config <cfg> under rocprofv3 --kernel-trace --stats
#   pmc:<cfg>        calibrated counter passes over bench --config <cfg> (tools/pmc_cal.sh)
#   ab:<args>|<builds>  tools/abrun.sh with bench args and library builds (comma-separated)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=$1
shift
run() { # name timeout cmd...
    local name=$1 to=$2
    shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 6 "$OUT/${TAG}_$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"
        exit $rc
    fi
    if [ $rc -ne 0 ] && [ "${KEEP_GOING:-0}" != 1 ]; then
        echo "rc=$rc in $name: stopping"
        exit $rc
    fi
    return 0
}
for st in "$@"; do
    case "$st" in
    smoke)
        run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest*)
        k=${st#pytest}
        k=${k#:}
        if [ -n "$k" ]; then
            run pytest 1100 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
                --timeout-method thread -k "$k"
        else
            run pytest 1100 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
                --timeout-method thread
        fi ;;
    bench*)
        a=${st#bench}
        a=${a#:}
        run bench 900 python3 -u bench.py ${a//,/ }
        grep '^{' $OUT/${TAG}_bench.log > $OUT/${TAG}_bench.json || true ;;
    headline)
        run headline 500 bash tools/prof_headline.sh $TAG
        python3 tools/kstats.py $OUT/headline_$TAG/prof/run_kernel_stats.csv ;;
    prof:*)
        c=${st#prof:}
        run prof_$c 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$c -o run \
            -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-e2e \
            --no-node --extra ""
        find $OUT/${TAG}_prof_$c -name '*kernel_trace.csv' -size +20M -delete
        python3 tools/kstats.py $(find $OUT/${TAG}_prof_$c -name '*kernel_stats.csv') ;;
    pmc:*)
        c=${st#pmc:}
        run pmc_$c 900 bash tools/pmc_cal.sh ${c//,/ } ;;
    ab:*)
        x=${st#ab:}
        run ab 1100 bash tools/abrun.sh "${x%%|*}" $(echo "${x#*|}" | tr , ' ') ;;
    *)
        echo "unknown step $st"
        exit 2 ;;
    esac
done
echo "session $TAG done"
