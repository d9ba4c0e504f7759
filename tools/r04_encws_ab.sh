#!/bin/bash
# Round 4: the wave-specialised Encode (XRS_ENC_WS = T chunks per block of 2T
# lanes) against the pair kernel: oracle tests with it forced, then an
# interleaved A/B (tools/env_ab.py, GB/s of the bytes each launch moves).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  for T in 128 256 512; do
    XRS_ENC_WS=$T timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_edge.py tests/test_gpu_order.py \
        -k "encode or Encode" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/encws_tests_$T.log 2>&1
    rc=$?; echo "T=$T"; tail -2 gpurun_out/encws_tests_$T.log; [ $rc -eq 0 ] || exit $rc
  done
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/encws_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  for size in 4096 65536 1048576; do
    ab VAR=XRS_ENC_WS VALS=,128,256,512 CASE=encode SIZE=$size ROUNDS=9
  done
  grep -v amdgpu.ids $out
fi
exit 0
