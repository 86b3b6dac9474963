#!/bin/bash
# Round-4 session C: probe7 (C5 fetch-order sweep, known-byte timings), the
# counter calibration passes over probe7 and the C4 / C5 bench kernels, and
# rocprofv3 --stats of the default bench command (headline evidence).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r04c}
WHAT=${2:-probe,node,fib,cal,prof}
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] >>> $name"
    timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] <<< $name rc=$rc"
    tail -n 30 "$OUT/${TAG}_$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"; exit $rc
    fi
    return $rc
}
case ",$WHAT," in *,probe,*) step probe7 300 ./tools/probe7 || exit 1;; esac
case ",$WHAT," in *,node,*) step node_cnet 300 python3 -u tools/node_probe_cnet.py --json $OUT/${TAG}_node_cnet.json;; esac
case ",$WHAT," in *,fib,*) step fib_latency 300 python3 -u tools/fib_latency.py --json $OUT/${TAG}_fib_latency.json;; esac
case ",$WHAT," in *,cal,*) step cal 900 bash tools/pmc_cal.sh probe c4 c5;; esac
case ",$WHAT," in *,prof,*) step headline 500 bash tools/prof_headline.sh $TAG;; esac
echo done
