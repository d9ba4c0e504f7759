#!/bin/bash
# Per-stripe calls at 64 KiB and 1 MiB vects, plain and registered vects:
# the batching queue (32 callers) and the plain API on one codec (32 / 8
# threads), tools/sync_bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r05_reg_sizes.log
: > $out
for sz in 65536 1048576; do
  for mode in queue queuereg; do
    timeout -k 10 120 ./tools/sync_bench $sz $mode 50 32 >> $out 2>&1 || { echo "rc=$? $sz $mode"; tail -5 $out; exit 1; }
  done
  for mode in syncmt syncmtreg; do
    timeout -k 10 120 ./tools/sync_bench $sz $mode 8 32 >> $out 2>&1 || { echo "rc=$? $sz $mode"; tail -5 $out; exit 1; }
  done
done
grep '^{' $out
