#!/bin/bash
# Round 4: block order K (XRS_ENC_WS_ORDER) for the wave-specialised Encode,
# T = 128 / 256, against the pair kernel (first value), bytes moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/encws_order.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for T in 128 256; do
  V=""
  for k in 0 4 8 16 32 64 128 256; do V="$V,XRS_ENC_WS=$T+XRS_ENC_WS_ORDER=$k"; done
  for size in 4096 65536 1048576; do
    ab VAR=MULTI VALS="$V" CASE=encode SIZE=$size ROUNDS=5
  done
done
for size in 16384 262144 4194304 4100; do
  ab VAR=MULTI VALS=",XRS_ENC_WS=128,XRS_ENC_WS=256" CASE=encode SIZE=$size ROUNDS=7
done
grep -v amdgpu.ids $out
exit 0
