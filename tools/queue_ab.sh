#!/bin/bash
# Batching-queue A/B on one GPU box: the queue's GPU tests, then
# tools/sync_bench (T concurrent per-stripe callers) across policies, worker
# counts and completion waits.  Output: gpurun_out/q_*.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${QTEST:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/q_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
SIZES=${SIZES:-4096}
CONFIGS=${CONFIGS:-"free:2 free:3 free:4 timer:2 free:2:block"}
THREADS=${THREADS:-"1 8 32 64"}
for size in $SIZES; do
  for cfg in $CONFIGS; do
    IFS=: read -r pol w sync <<< "$cfg"
    echo "size=$size policy=$pol workers=$w sync=${sync:-spin}"
    XRS_QUEUE_POLICY=$pol XRS_QUEUE_WORKERS=$w XRS_QUEUE_SYNC=${sync:-spin} \
      timeout -k 10 120 tools/sync_bench $size queue 50 $THREADS || exit $?
  done
done > gpurun_out/q_ab.log 2>&1
rc=$?; cat gpurun_out/q_ab.log; exit $rc
