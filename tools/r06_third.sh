#!/bin/bash
# Round 6, third GPU call: the host pipeline's DMA-clean copies (codec.cpp
# copy_rows): the host / odd / group / queue tests with
# runtime logging (every "DMA buffer failed" line counted), the DMA probe's
# fixed 1-D leg, bench_host aligned vs odd rates, and the per-stripe queue
# sweeps (async window, mixed registered + plain at 1 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
o=gpurun_out
step() { echo "== $*"; }
step logged tests && AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 \
    --timeout-method thread -m gpu tests/test_gpu_host.py tests/test_gpu_odd.py tests/test_gpu_group.py \
    tests/test_gpu_queue.py tests/test_gpu_registered.py > $o/r06_host_logged.log 2>&1 &&
  tail -2 $o/r06_host_logged.log &&
  echo "DMA buffer failed lines: $(grep -c 'DMA buffer failed' $o/r06_host_logged.log || true)" &&
  step dma probe && AMD_LOG_LEVEL=1 timeout -k 10 180 ./tools/dma_rect_probe > $o/r06_dma_rect_probe2.log 2>&1 &&
  grep ' 1D ' $o/r06_dma_rect_probe2.log | head -30 &&
  step bench_host && timeout -k 10 600 python -u tools/bench_host.py pipeline > $o/r06_bench_host.log 2>&1 &&
  AMD_LOG_LEVEL=1 timeout -k 10 600 python -u tools/bench_host.py odd > $o/r06_bench_host_odd.log 2>&1 &&
  grep '^{' $o/r06_bench_host.log $o/r06_bench_host_odd.log &&
  echo "DMA buffer failed lines (odd bench): $(grep -c 'DMA buffer failed' $o/r06_bench_host_odd.log || true)"
