#!/bin/bash
# Round 4: early-b stage 3 in the wave-specialised staged kernel (XRS_WS_EARLYB,
# default on) against the round-2 form (=0): staged-kernel oracle tests, then an
# interleaved A/B (tools/env_ab.py, GB/s of the bytes each launch moves).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_dispatch.py tests/test_gpu_order.py \
      -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/eb_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/eb_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/eb_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 120 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  for size in 1048576 262144 65536 4096; do
    for c in reconst_2 reconst_3 mixed_12 mixed_13 mixed_0-13; do
      ab VAR=XRS_WS_EARLYB VALS=,0 CASE=$c SIZE=$size ROUNDS=21
    done
  done
  grep -v amdgpu.ids $out
fi
exit 0
