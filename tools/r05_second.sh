#!/bin/bash
# Round 5, second GPU call: the persistent kernel's per-call cost without
# fences in the slot reset, the C++ port (queue coalescing), the queue's
# in-flight limit with and without registered vects, then the whole GPU test
# suite, smoke, the default bench line and a rocprofv3 --stats run
# (tools/gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
gate() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
timeout -k 10 240 python -u tools/wsp_call_overhead.py > gpurun_out/r05_wsp_overhead.log 2>&1
rc=$?; grep n= gpurun_out/r05_wsp_overhead.log; gate $rc
timeout -k 10 300 ./tests/cpp/build/xrs_test > gpurun_out/r05_cpp_tests.log 2>&1
rc=$?; grep -E "queue|FAIL|PASS" gpurun_out/r05_cpp_tests.log; gate $rc
: > gpurun_out/r05_queue_inflight.log
for inf in 4 8; do
  for mode in queue queuereg; do
    XRS_QUEUE_INFLIGHT=$inf XRS_QUEUE_BATCHES=$((inf + 2)) timeout -k 10 120 ./tools/sync_bench 4096 $mode 50 32 \
        >> gpurun_out/r05_queue_inflight.log 2>&1
    rc=$?; gate $rc
  done
done
grep '^{' gpurun_out/r05_queue_inflight.log
STEPS=pytest,smoke,bench,prof bash tools/gpu_check.sh
