#!/bin/bash
# Round 4: BASELINE config 4 (Update, Replace(4) @ 8 MiB) against the block
# order (XRS_BLOCK_ORDER) and the pair kernel's block size (XRS_PAIR_BLOCK),
# interleaved A/B (tools/env_ab.py), GB/s of the bytes each launch moves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c4_order.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for c in update replace_4; do
  ab VAR=XRS_BLOCK_ORDER VALS=,8,16,64,128,256,0 CASE=$c SIZE=8388608 ROUNDS=11
  ab VAR=XRS_PAIR_BLOCK VALS=,128,512,1024 CASE=$c SIZE=8388608 ROUNDS=11
done
grep -v amdgpu.ids $out
