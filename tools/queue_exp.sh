#!/bin/bash
# Batching-queue experiments (tools/sync_bench): the queue's GPU tests, then
# CONFIGS of policy:launchers:inflight, THREADS callers, SIZES vects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${QTEST:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/q_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
CONFIGS=${CONFIGS:-"free:1:4 free:1:6 free:2:4 timer:1:4"}
THREADS=${THREADS:-"1 8 16 32 48"}
SIZES=${SIZES:-4096}
for size in $SIZES; do
for cfg in $CONFIGS; do
  IFS=: read -r pol w inf <<< "$cfg"
  echo "size=$size policy=$pol launchers=$w inflight=$inf"
  XRS_QUEUE_POLICY=$pol XRS_QUEUE_WORKERS=$w XRS_QUEUE_INFLIGHT=$inf \
    timeout -k 10 90 tools/sync_bench $size queue 50 $THREADS
  rc=$?
  echo "rc=$rc"
  [ $rc -eq 0 ] || break 2
done
done > gpurun_out/qexp_ab.log 2>&1
cat gpurun_out/qexp_ab.log
