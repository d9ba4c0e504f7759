#!/bin/bash
# Round 4: the persistent staged kernel with 256-chunk tiles and two blocks
# per CU (XRS_WSP=256 XRS_WSP_PER_CU=2: the same lanes per CU as 512-chunk
# tiles, two independent tile streams) against the defaults, 2 and 3 lost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wsp256.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
V=",XRS_WSP=256+XRS_WSP_PER_CU=2,XRS_WSP=512,XRS_WSP=256+XRS_WSP_PER_CU=2+XRS_WS_ORDER=64"
for size in 1048576 524288 2097152; do
  ab VAR=MULTI VALS=$V CASE=reconst_3 SIZE=$size ROUNDS=7
  ab VAR=MULTI VALS=$V CASE=reconst_2 SIZE=$size ROUNDS=7
done
ab VAR=MULTI VALS=$V CASE=reconst_3 SIZE=262144 ROUNDS=7
grep -v amdgpu.ids $out
exit 0
