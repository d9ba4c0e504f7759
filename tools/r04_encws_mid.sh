#!/bin/bash
# Round 4: the wave-specialised Encode, T = 128 / 256 x block order (default
# K, plain), against the pair kernel from 4 KiB to 384 KiB vects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/encws_mid.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
V=",XRS_ENC_WS=128,XRS_ENC_WS=128+XRS_ENC_WS_ORDER=0,XRS_ENC_WS=256,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=0"
for size in 4096 8192 32768 65536 131072 262144 393216; do
  ab VAR=MULTI VALS=$V CASE=encode SIZE=$size ROUNDS=9
done
grep -v amdgpu.ids $out
exit 0
