#!/bin/bash
# Round 6, first GPU call: the unregister -> free -> reuse test (C++, logged
# with AMD_LOG_LEVEL=1, then the Python twin and the registered suite), the
# persistent-slot tests after the reset change, the DMA rectangle probe, and
# the per-stripe 4 KiB caller sweep (32..256 callers, plain and registered).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
o=gpurun_out
step() { echo "== $*"; }
step reuse C++ && AMD_LOG_LEVEL=1 timeout -k 10 180 ./tests/cpp/build/xrs_test TestRegistered_UnregisterFreeReuse \
    > $o/r06_reuse_cpp.log 2>&1 &&
  tail -3 $o/r06_reuse_cpp.log &&
  step pytest && timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_kernel_resources.py tests/test_gpu_registered.py tests/test_gpu_edge.py tests/test_gpu_shards.py \
    > $o/r06_pytest_a.log 2>&1 &&
  tail -3 $o/r06_pytest_a.log &&
  step dma probe && AMD_LOG_LEVEL=1 timeout -k 10 180 ./tools/dma_rect_probe > $o/r06_dma_rect_probe.log 2>&1 &&
  tail -2 $o/r06_dma_rect_probe.log &&
  step sweep && : > $o/r06_callers.log &&
  for mode in queue queuereg; do
    timeout -k 10 240 ./tools/sync_bench 4096 $mode 50 32 64 128 256 >> $o/r06_callers.log 2>&1 || exit 1
  done &&
  for mode in syncmt syncmtreg; do
    timeout -k 10 240 ./tools/sync_bench 4096 $mode 32 64 128 256 >> $o/r06_callers.log 2>&1 || exit 1
  done &&
  grep '^{' $o/r06_callers.log
