#!/bin/bash
# Interleaved A/B of the 12+4 lost-parity Reconst patterns: library default
# vs XRS_STAGED_CT=0 (runtime-count kernels), at 4 KiB and 1 MiB vects.
# GB/s of accounted bytes, (d + lost) * S per stripe (tools/env_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CASES:-mixed_12 mixed_13 mixed_14 mixed_0-13 mixed_0-12 mixed_0-1-13 mixed_0-1-12-13}; do
  for sz in 4096 1048576; do
    VAR=XRS_STAGED_CT VALS=,0 CASE=$c SIZE=$sz ROUNDS=${ROUNDS:-11} timeout -k 10 120 \
      python tools/env_ab.py || exit $?
  done
done
