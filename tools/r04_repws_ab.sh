#!/bin/bash
# Round 4: the wave-specialised Replace (XRS_REP_WS=1; rep_ws_kernel is in
# commit b73a498 only: within +-3%, removed) against the
# accumulating pair kernel: oracle tests forced, then an interleaved A/B
# (bytes moved), Replace(1 / 4 / 8) at 4 KiB, 64 KiB and 8 MiB vects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XRS_REP_WS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_edge.py tests/test_gpu_fuzz.py \
    -k "replace or Replace" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/repws_tests.log 2>&1
rc=$?; tail -2 gpurun_out/repws_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/repws_ab.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for size in 4096 65536 8388608; do
  for c in replace_1 replace_4 replace_8; do
    ab VAR=XRS_REP_WS VALS=0,1 CASE=$c SIZE=$size ROUNDS=7
  done
done
grep -v amdgpu.ids $out
exit 0
