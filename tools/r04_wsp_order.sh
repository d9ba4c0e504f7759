#!/bin/bash
# Round 4: block (tile) order for the persistent staged kernel at 1 MiB vects:
# XRS_WS_ORDER = K logical tiles per XCD per group, default (128) first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wsp_order.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
W=XRS_WSP=512
V=",$W,$W+XRS_WS_ORDER=8,$W+XRS_WS_ORDER=16,$W+XRS_WS_ORDER=32,$W+XRS_WS_ORDER=64,$W+XRS_WS_ORDER=256,$W+XRS_WS_ORDER=0"
for size in 1048576 2097152; do
  for c in reconst_2 reconst_3; do
    ab VAR=MULTI VALS=$V CASE=$c SIZE=$size ROUNDS=7
  done
done
grep -v amdgpu.ids $out
exit 0
