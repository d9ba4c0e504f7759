#!/bin/bash
# Round 4: the LDS-DMA staged kernel (XRS_STAGED_GLDS=1) against the default:
# full-grid oracle tests, then an interleaved A/B (tools/env_ab.py, GB/s of
# the bytes each launch moves).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -k "full_grid and glds" -v -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/glds_tests.log 2>&1
  rc=$?; tail -8 gpurun_out/glds_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/glds_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  for size in 1048576 262144 4096; do
    for c in reconst_2 reconst_4 mixed_13 mixed_0-13; do
      ab VAR=XRS_STAGED_GLDS VALS=,1,18 CASE=$c SIZE=$size ROUNDS=11
    done
  done
  grep -v amdgpu.ids $out
fi
exit 0
