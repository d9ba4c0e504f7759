#!/bin/bash
# Round 4: the persistent staged kernel forced (XRS_WSP=512) for 4 lost data
# vects (default: the one-wave compile-time kernel) and 3 lost (default: the
# one-shot 256-chunk wave-specialised kernel), bytes moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wsp_lost4.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for size in 1048576 524288 2097152; do
  ab VAR=MULTI VALS=",XRS_WSP=512,XRS_WSP=512+XRS_WS_ORDER=128" CASE=reconst_4 SIZE=$size ROUNDS=7
done
grep -v amdgpu.ids $out
exit 0
