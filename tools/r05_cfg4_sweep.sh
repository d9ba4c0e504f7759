#!/bin/bash
# Config 4 (Update / Replace(4) @ 8 MiB, 64 stripes) launch-knob sweep:
# XCD block order K and the pair kernel's block size, interleaved A/B
# (tools/env_ab.py), Encode @ 8 MiB beside them for reference.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r05_cfg4_sweep.log
: > $out
run() { timeout -k 10 120 env "$@" python -u tools/env_ab.py >> $out 2>&1 || { echo "rc=$? $*"; tail -5 $out; exit 1; }; }
for c in update replace_4 encode; do
  echo "== $c XRS_BLOCK_ORDER" >> $out
  run VAR=XRS_BLOCK_ORDER VALS=32,0,8,16,64,128,256,full CASE=$c SIZE=8388608 STRIPES=64 ROUNDS=11
done
echo "== replace_4 XRS_PAIR_BLOCK" >> $out
run VAR=XRS_PAIR_BLOCK VALS=256,128 CASE=replace_4 SIZE=8388608 STRIPES=64 ROUNDS=11
grep -E '^==|^\{' $out
