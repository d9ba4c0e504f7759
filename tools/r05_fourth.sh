#!/bin/bash
# Round 5, fourth GPU call, on the final library: the registered-memory fuzz
# (sync and queue table mode), a fresh fuzz campaign of the batched API on
# full grids with large vects, a 60 s 32-thread soak of the queue and the
# shared codec with registered callers and registry churn, and the N = 8
# bench rehearsal on one card.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XRS_FUZZ_SEEDS=8 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_registered.py > gpurun_out/r05_registered_fuzz.log 2>&1
rc=$?; tail -3 gpurun_out/r05_registered_fuzz.log; [ $rc -eq 0 ] || exit $rc
XRS_FUZZ_SEEDS=100 XRS_FUZZ_BASE=60000 XRS_FUZZ_GRID=1 XRS_FUZZ_BIG=1 timeout -k 10 600 \
    python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_fuzz.py > gpurun_out/r05_fuzz_grid_big_100seeds.log 2>&1
rc=$?; tail -3 gpurun_out/r05_fuzz_grid_big_100seeds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/sync_bench stress 60 32 > gpurun_out/r05_stress_reg_60s.log 2>&1
rc=$?; tail -3 gpurun_out/r05_stress_reg_60s.log; [ $rc -eq 0 ] || exit $rc
bash tools/rehearse_n8.sh
