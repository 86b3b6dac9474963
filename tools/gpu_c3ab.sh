#!/bin/bash
# A/B (diagnostic): parity on the "dpp" build (tools/abbuild.sh dpp
# -DCNDP_STREAM_DPP=1 -DCNDP_CNET_DPP=1) and, for the cnet tests, on the "inl"
# build (-DCNDP_SPEC_INLINE=1); then C3 / C4 / C5 timings against the default
# build ("base"), dpp640 = dpp with 640-thread blocks at 5 waves per SIMD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
L=$PWD/cndp_amd/lib
CNDP_GPU_LIB=$L/libcndp_gpu_dpp.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    -m "gpu and not slow" -x -q --timeout 300 -p no:cacheprovider > gpurun_out/parity_dpp.log 2>&1 \
    || { echo "parity dpp rc=$?"; tail -30 gpurun_out/parity_dpp.log; exit 1; }
tail -1 gpurun_out/parity_dpp.log
CNDP_GPU_LIB=$L/libcndp_gpu_inl.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    -m "gpu and not slow" -x -q --timeout 300 -p no:cacheprovider -k "cnet or spec" > gpurun_out/parity_inl.log 2>&1 \
    || { echo "parity inl rc=$?"; tail -30 gpurun_out/parity_inl.log; exit 1; }
tail -1 gpurun_out/parity_inl.log
tools/abrun.sh "--config c3 --steps 50 --warmup 5" base dpp || exit 1
tools/abrun.sh "--config c3 --steps 50 --warmup 5 --bpc 3" dpp || exit 1
tools/abrun.sh "--config c4 --steps 30 --warmup 3" base dpp inl dpp640 || exit 1
tools/abrun.sh "--config c5 --steps 20 --warmup 3" base dpp
