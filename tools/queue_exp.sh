#!/bin/bash
# Batching-queue experiments (tools/sync_bench): CONFIGS of
# policy:workers:sync:spin_ns, THREADS callers, 4 KiB vects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-"free:6:block:0 free:6:spin:2000"}
THREADS=${THREADS:-"16 32 48"}
SIZE=${SIZE:-4096}
for cfg in $CONFIGS; do
  IFS=: read -r pol w sync spin <<< "$cfg"
  echo "policy=$pol workers=$w sync=$sync spin_ns=$spin"
  XRS_QUEUE_POLICY=$pol XRS_QUEUE_WORKERS=$w XRS_QUEUE_SYNC=$sync XRS_QUEUE_SPIN_NS=$spin \
    timeout -k 10 60 tools/sync_bench $SIZE queue 50 $THREADS
  rc=$?
  echo "rc=$rc"
  [ $rc -eq 0 ] || break
done > gpurun_out/qexp_ab.log 2>&1
cat gpurun_out/qexp_ab.log
