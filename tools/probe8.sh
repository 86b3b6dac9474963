#!/bin/bash
# probe8 (diagnostic): window-read time by slab allocation and load flavour,
# then one rocprofv3 --pmc pass for the L2's request sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/p8
mkdir -p $OUT
LG=${1:-24}
echo "[$(date +%T)] time"
timeout -k 10 180 ./tools/probe8 $LG > $OUT/time.log 2>&1
rc=$?
cat $OUT/time.log
[ $rc -ne 0 ] && { echo "probe8 rc=$rc"; exit $rc; }
echo "[$(date +%T)] req"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d $OUT/req -o run -- ./tools/probe8 $LG > $OUT/req.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/pmc_seq.py $(find $OUT/req -name "*counter_collection.csv") > $OUT/req_summary.txt 2>&1
head -60 $OUT/req_summary.txt
