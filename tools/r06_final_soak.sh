#!/bin/bash
# Round 6, robustness campaign on the final library: a fresh grid fuzz
# campaign, the 60 s soak (every op on two queues replaced every second, the
# plain API, registered callers, registration churn, and now asynchronous
# submit / poll / wait), and the N = 8 one-card rehearsal of bench.py (its
# config5 split and xgmi need-set plan are new this round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    "tests/gpu_registered_cases.py::test_unregister_free_reuse_then_pageable_copy" \
    > gpurun_out/r06_reuse_child.log 2>&1
rc=$?; tail -3 gpurun_out/r06_reuse_child.log; [ $rc -eq 0 ] || exit $rc
XRS_FUZZ_SEEDS=60 XRS_FUZZ_BASE=120000 XRS_FUZZ_GRID=1 timeout -k 10 500 \
    python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_fuzz.py > gpurun_out/r06_final_fuzz_grid_60seeds.log 2>&1
rc=$?; tail -3 gpurun_out/r06_final_fuzz_grid_60seeds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/sync_bench stress 60 32 > gpurun_out/r06_final_stress_60s.log 2>&1
rc=$?; tail -2 gpurun_out/r06_final_stress_60s.log; [ $rc -eq 0 ] || exit $rc
bash tools/rehearse_n8.sh
timeout -k 10 600 python -u tools/bench_host.py odd > gpurun_out/r06_bench_host_odd_b.log 2>&1 &&
  grep '^{' gpurun_out/r06_bench_host_odd_b.log
