#!/bin/bash
# Round 4: the wave-specialised Encode on ragged halves (XRS_ENC_WS_RAGGED=1:
# overlapping last chunk, as the pair kernel): oracle tests, then an
# interleaved A/B against the pair kernel at odd vect sizes (bytes moved).
# Needs tools/r04_encws_ragged.patch applied to xrs_amd/csrc/kernels.hip (not
# run in round 4: no GPU box was free at the end of the round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XRS_ENC_WS_RAGGED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_odd.py tests/test_gpu_edge.py \
    -k "encode or Encode or odd or ragged" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/encws_ragged_tests.log 2>&1
rc=$?; tail -2 gpurun_out/encws_ragged_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/encws_ragged.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
for size in 4100 4098 2052 65540 262146; do
  ab VAR=XRS_ENC_WS_RAGGED VALS=0,1 CASE=encode SIZE=$size ROUNDS=9
done
grep -v amdgpu.ids $out
exit 0
