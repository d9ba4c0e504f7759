#!/bin/bash
# Round 6, second GPU call: the rest of the first call (edge + shard tests,
# the C++ suite under host ASan, the DMA rectangle probe, the per-stripe 4 KiB
# caller sweep) and the 4-lost staged Reconst A/B at 1 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
o=gpurun_out
step() { echo "== $*"; }
step pytest && timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    -m gpu tests/test_gpu_queue_async.py tests/test_gpu_edge.py tests/test_gpu_shards.py tests/test_cpp.py \
    > $o/r06_pytest_b.log 2>&1 &&
  tail -3 $o/r06_pytest_b.log &&
  step dma probe && AMD_LOG_LEVEL=1 timeout -k 10 180 ./tools/dma_rect_probe > $o/r06_dma_rect_probe.log 2>&1 &&
  tail -2 $o/r06_dma_rect_probe.log &&
  step 4-lost A/B && VAR=XRS_STAGED_WS VALS=,512,256 CASE=reconst_4 SIZE=1048576 ROUNDS=11 \
    timeout -k 10 300 python -u tools/env_ab.py > $o/r06_4lost_ws_ab.log 2>&1 &&
  VAR=XRS_STAGED_EARLY VALS=0,1 CASE=reconst_4 SIZE=1048576 ROUNDS=11 \
    timeout -k 10 300 python -u tools/env_ab.py >> $o/r06_4lost_ws_ab.log 2>&1 &&
  VAR=XRS_WSP VALS=0,512 CASE=reconst_4 SIZE=1048576 ROUNDS=11 \
    timeout -k 10 300 python -u tools/env_ab.py >> $o/r06_4lost_ws_ab.log 2>&1 &&
  cat $o/r06_4lost_ws_ab.log | grep '^{' &&
  step sweep && : > $o/r06_callers.log &&
  for mode in queue queuereg; do
    timeout -k 10 240 ./tools/sync_bench 4096 $mode 50 32 64 128 256 >> $o/r06_callers.log 2>&1 || exit 1
  done &&
  for mode in queueasync queueasyncreg; do
    for win in 4 16; do
      timeout -k 10 240 ./tools/sync_bench 4096 $mode 50 $win 8 32 64 >> $o/r06_callers.log 2>&1 || exit 1
    done
  done &&
  for mode in syncmt syncmtreg; do
    timeout -k 10 240 ./tools/sync_bench 4096 $mode 32 64 128 256 >> $o/r06_callers.log 2>&1 || exit 1
  done &&
  grep '^{' $o/r06_callers.log
