#!/bin/bash
# Round 6, fourth GPU call: per-stripe 4 KiB through the asynchronous queue
# calls after registered tickets release their slots at completion (window x
# callers, plain and registered, XRS_QUEUE_BATCHES 6 and 12), and the 1 MiB
# mixed registered + plain queue batch against all-plain and
# all-registered.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
o=gpurun_out/r06_async_sweep.log
: > $o
for mode in queueasyncreg queueasync; do
  for win in 8 16 32; do
    timeout -k 10 200 ./tools/sync_bench 4096 $mode 50 $win 4 8 16 >> $o 2>&1 || { echo "rc=$? $mode $win"; tail -5 $o; exit 1; }
  done
done
XRS_QUEUE_BATCHES=12 timeout -k 10 200 ./tools/sync_bench 4096 queueasyncreg 50 16 4 8 16 >> $o 2>&1 || exit 1
XRS_QUEUE_BATCHES=12 XRS_QUEUE_INFLIGHT=8 timeout -k 10 200 ./tools/sync_bench 4096 queueasyncreg 50 16 4 8 16 >> $o 2>&1 || exit 1
grep '^{' $o
m=gpurun_out/r06_mixed_1m.log
: > $m
for mode in queue queuereg queuemixed; do
  timeout -k 10 200 ./tools/sync_bench 1048576 $mode 50 8 >> $m 2>&1 || { echo "rc=$? $mode"; tail -5 $m; exit 1; }
done
grep '^{' $m
# the round-5 library (xrs_amd/variants/libxrs_hip_r05.so, built from
# f20d09e) on the same odd-size host batches: the copies before round 6
if [ -f xrs_amd/variants/libxrs_hip_r05.so ]; then
  XRS_LIB=xrs_amd/variants/libxrs_hip_r05.so AMD_LOG_LEVEL=1 timeout -k 10 600 python -u tools/bench_host.py odd \
    > gpurun_out/r06_bench_host_odd_r05lib.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06_bench_host_odd_r05lib.log
  echo "DMA buffer failed lines (round-5 library): $(grep -c 'DMA buffer failed' gpurun_out/r06_bench_host_odd_r05lib.log || true)"
fi
