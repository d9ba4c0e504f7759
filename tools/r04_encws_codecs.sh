#!/bin/bash
# Round 4: the wave-specialised Encode forced (XRS_ENC_WS=256) for the other
# d+4 compile-time codecs: oracle tests, then an interleaved A/B against the
# pair kernel (bytes moved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "compile_time_shapes" -q -x -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/encws_codecs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/encws_codecs_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/encws_codecs.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for codec in 8,4 10,4 14,4 16,4 20,4; do
  for size in 4096 65536 1048576; do
    ab VAR=XRS_ENC_WS VALS=0,256 CASE=encode SIZE=$size CODEC=$codec ROUNDS=7
  done
done
grep -v amdgpu.ids $out
exit 0
