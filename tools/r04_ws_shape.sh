#!/bin/bash
# Round 4: wave-specialised staged kernel, chunks per block (XRS_STAGED_WS) x
# block order (XRS_WS_ORDER) at 256 KiB - 1 MiB vects, interleaved A/B
# (tools/env_ab.py VAR=MULTI), GB/s of the bytes each launch moves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ws_shape.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
V=",XRS_STAGED_WS=256,XRS_STAGED_WS=256+XRS_WS_ORDER=64,XRS_STAGED_WS=256+XRS_WS_ORDER=32,XRS_STAGED_WS=256+XRS_WS_ORDER=16,XRS_STAGED_WS=512+XRS_WS_ORDER=32,XRS_STAGED_WS=512+XRS_WS_ORDER=16"
for size in 1048576 2097152 524288 262144; do
  for c in reconst_2 reconst_3 mixed_0-13 mixed_13 mixed_12; do
    ab VAR=MULTI VALS=$V CASE=$c SIZE=$size ROUNDS=11
  done
done
grep -v amdgpu.ids $out
