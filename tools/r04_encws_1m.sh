#!/bin/bash
# Round 4: settle the wave-specialised Encode at 1 MiB vects (the bench's
# dominant launch): pair (plain order) vs enc_ws T = 256 in two block orders,
# long interleaved runs in two separate processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/encws_1m.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 200 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
V=",XRS_ENC_WS=256,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=0,XRS_ENC_WS=256+XRS_ENC_WS_ORDER=128"
for rep in 1 2; do
  ab VAR=MULTI VALS=$V CASE=encode SIZE=1048576 ROUNDS=21 STRIPES=512
done
ab VAR=MULTI VALS=$V CASE=encode SIZE=2097152 ROUNDS=11
ab VAR=MULTI VALS=$V CASE=encode SIZE=524288 ROUNDS=11
grep -v amdgpu.ids $out
exit 0
