#!/bin/bash
# Round 4: block order of the wave-specialised staged kernel (XRS_WS_ORDER,
# logical blocks per XCD per group) for 2-3 lost data vects at 4 KiB - 1 MiB
# vects, and the one-wave 4-lost kernel (XRS_BLOCK_ORDER); interleaved A/B,
# GB/s of the bytes each launch moves (tools/env_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ws_order.log
: > $out
ab() { echo "== $*" | tee -a $out; env "$@" timeout -k 10 120 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
ab VAR=XRS_WS_ORDER VALS=,4,8,16,32,64,0 CASE=reconst_2 SIZE=1048576 ROUNDS=15
ab VAR=XRS_WS_ORDER VALS=,4,8,16,32,64,0 CASE=reconst_3 SIZE=1048576 ROUNDS=15
ab VAR=XRS_BLOCK_ORDER VALS=,4,8,16,32,64,0 CASE=reconst_4 SIZE=1048576 ROUNDS=15
ab VAR=XRS_WS_ORDER VALS=,4,8,16,64 CASE=mixed_0-13 SIZE=1048576 ROUNDS=15
ab VAR=XRS_WS_ORDER VALS=,4,8,16,64 CASE=reconst_2 SIZE=262144 ROUNDS=15
ab VAR=XRS_WS_ORDER VALS=,4,8,16,64 CASE=reconst_2 SIZE=4096 ROUNDS=15
ab VAR=XRS_WS_ORDER VALS=,4,8,16,64 CASE=reconst_3 SIZE=4096 ROUNDS=15
cat $out
