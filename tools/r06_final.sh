#!/bin/bash
# Round 6, final GPU call on the library at HEAD: HBM traffic of this build
# (two --pmc passes -> profiles/pmc_traffic.json), then the whole GPU test
# suite, smoke, the default bench line and a rocprofv3 --stats run
# (tools/gpu_check.sh), then the round-5 library on the odd-size host
# batches (the copies before round 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc.sh || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
STEPS=pytest,smoke,bench,prof bash tools/gpu_check.sh || exit $?
if [ -f xrs_amd/variants/libxrs_hip_r05.so ]; then
  XRS_LIB=xrs_amd/variants/libxrs_hip_r05.so AMD_LOG_LEVEL=1 timeout -k 10 600 python -u tools/bench_host.py odd \
    > gpurun_out/r06_bench_host_odd_r05lib.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06_bench_host_odd_r05lib.log
  echo "DMA buffer failed lines (round-5 library): $(grep -c 'DMA buffer failed' gpurun_out/r06_bench_host_odd_r05lib.log || true)"
fi
