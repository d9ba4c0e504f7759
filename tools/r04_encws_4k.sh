#!/bin/bash
# Round 4: the wave-specialised Encode at the sizes it might take over:
# 4 KiB (the headline) with the orders the sweep liked, then 128 KiB - 1 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/encws_4k.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
ab VAR=MULTI VALS=",XRS_ENC_WS=128+XRS_ENC_WS_ORDER=16,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=16,XRS_ENC_WS=128,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=4" \
   CASE=encode SIZE=4096 ROUNDS=15
for size in 131072 524288 786432 1048576; do
  ab VAR=MULTI VALS=",XRS_ENC_WS=128,XRS_ENC_WS=256,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=0" CASE=encode SIZE=$size ROUNDS=9
done
grep -v amdgpu.ids $out
exit 0
