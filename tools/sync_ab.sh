#!/bin/bash
# Per-stripe sync calls (tools/sync_bench SIZE sync, and the reference's
# benchmark matrix `ref`): default completion wait vs XRS_SYNC_WAIT=block,
# interleaved ROUNDS times.  Output: gpurun_out/sync_ab.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for w in spin block; do
    for size in ${SIZES:-4096 65536 1048576}; do
      echo "round=$r wait=$w size=$size"
      XRS_SYNC_WAIT=$w timeout -k 10 60 tools/sync_bench $size sync || exit $?
    done
    if [ "${REF:-1}" = 1 ]; then
      echo "round=$r wait=$w ref"
      XRS_SYNC_WAIT=$w timeout -k 10 120 tools/sync_bench ref || exit $?
    fi
  done
done > gpurun_out/sync_ab.log 2>&1
rc=$?; cat gpurun_out/sync_ab.log; exit $rc
