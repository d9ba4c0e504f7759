#!/bin/bash
# Round 4: XCD start rotation of the block order (BlockOrder.rot: XCD x begins
# its K blocks of each group at (x * rot) % K, so the XCDs' concurrent blocks
# sit at different offsets of their vects) for the staged kernels
# (XRS_WS_ROT) and ReconstOne (XRS_ORDER_ROT), default first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  XRS_WS_ROT=24 XRS_ORDER_ROT=24 timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_order.py \
      -k "full_grid or persistent or order" -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/rot_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/rot_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/rot_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  P="XRS_WSP=512+XRS_WS_ORDER=32"
  ab VAR=MULTI VALS=",XRS_WS_ROT=4,XRS_WS_ROT=8,XRS_WS_ROT=16,XRS_WS_ROT=32,XRS_WS_ROT=48,$P,$P+XRS_WS_ROT=4,$P+XRS_WS_ROT=12" \
     CASE=reconst_2 SIZE=1048576 ROUNDS=7
  ab VAR=MULTI VALS=",XRS_WS_ROT=8,XRS_WS_ROT=16,XRS_WS_ROT=32" CASE=reconst_3 SIZE=1048576 ROUNDS=7
  ab VAR=MULTI VALS=",XRS_WS_ROT=8,XRS_WS_ROT=16,XRS_WS_ROT=32" CASE=reconst_2 SIZE=262144 ROUNDS=7
  ab VAR=MULTI VALS=",XRS_ORDER_ROT=4,XRS_ORDER_ROT=8,XRS_ORDER_ROT=16" CASE=reconst_one SIZE=1048576 ROUNDS=7
  ab VAR=MULTI VALS=",XRS_ORDER_ROT=4,XRS_ORDER_ROT=8,XRS_ORDER_ROT=16" CASE=update SIZE=8388608 ROUNDS=7
  grep -v amdgpu.ids $out
fi
exit 0
