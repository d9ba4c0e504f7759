#!/bin/bash
# Round 5, robustness campaign on the final library: the registered-memory
# tests with a longer fuzz followed by the shards and queue tests in one
# process (each GPU test synchronizes the device in teardown), a fresh grid
# fuzz campaign, the 60 s registered-caller soak and the N = 8 rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XRS_FUZZ_SEEDS=16 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_registered.py tests/test_gpu_shards.py tests/test_gpu_queue.py \
    > gpurun_out/r05_final_registered.log 2>&1
rc=$?; tail -3 gpurun_out/r05_final_registered.log; [ $rc -eq 0 ] || exit $rc
XRS_FUZZ_SEEDS=60 XRS_FUZZ_BASE=90000 XRS_FUZZ_GRID=1 timeout -k 10 500 \
    python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_fuzz.py > gpurun_out/r05_final_fuzz_grid_60seeds.log 2>&1
rc=$?; tail -3 gpurun_out/r05_final_fuzz_grid_60seeds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/sync_bench stress 60 32 > gpurun_out/r05_final_stress_60s.log 2>&1
rc=$?; tail -2 gpurun_out/r05_final_stress_60s.log; [ $rc -eq 0 ] || exit $rc
bash tools/rehearse_n8.sh
