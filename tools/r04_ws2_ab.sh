#!/bin/bash
# Round 4: the two-pass wave-specialised staged kernel (XRS_STAGED_WS2) against
# the default: full-grid oracle tests, then an interleaved A/B
# (tools/env_ab.py, GB/s of the bytes each launch moves).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py -k "full_grid" -q -x -p no:cacheprovider \
      --timeout 300 --timeout-method thread > gpurun_out/ws2_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/ws2_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/ws2_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  for size in 1048576 262144 4096; do
    for c in reconst_2 reconst_3 mixed_12 mixed_13 mixed_0-13; do
      ab VAR=XRS_STAGED_WS2 VALS=,512,256,512o6,256o6 CASE=$c SIZE=$size ROUNDS=15
    done
  done
  grep -v amdgpu.ids $out
fi
exit 0
