#!/bin/bash
# Round 5, third GPU call: the queue's single-launch table mode over
# registered vects (indirect-row kernels): its tests and the C++ port, the
# per-stripe rates with and without registered vects, then HBM traffic of this
# library (two --pmc passes) and, with that traffic in place, the whole GPU
# test suite, smoke, the default bench line and a rocprofv3 --stats run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
gate() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_registered.py tests/test_gpu_queue.py -s > gpurun_out/r05_third_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_third_tests.log; gate $rc
timeout -k 10 300 ./tests/cpp/build/xrs_test > gpurun_out/r05_cpp_tests.log 2>&1
rc=$?; grep -E "queue|FAIL|passed|failed" gpurun_out/r05_cpp_tests.log | tail -8; gate $rc
: > gpurun_out/r05_sync_bench.log
for mode in queue queuereg; do
  timeout -k 10 120 ./tools/sync_bench 4096 $mode 50 1 8 32 >> gpurun_out/r05_sync_bench.log 2>&1
  rc=$?; gate $rc
done
for mode in syncmt syncmtreg; do
  timeout -k 10 120 ./tools/sync_bench 4096 $mode 1 8 32 >> gpurun_out/r05_sync_bench.log 2>&1
  rc=$?; gate $rc
done
grep '^{' gpurun_out/r05_sync_bench.log
bash tools/gpu_pmc.sh || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
STEPS=pytest,smoke,bench,prof bash tools/gpu_check.sh
