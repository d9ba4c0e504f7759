#!/bin/bash
# Round 4: the persistent wave-specialised staged kernel (staged_wsp_kernel,
# the default for 2 lost from 256 KiB halves; XRS_WSP=0 the one-shot kernel):
# oracle tests with multi-tile blocks and concurrent streams, then an
# interleaved A/B (tools/env_ab.py, GB/s of the bytes each launch moves).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_dispatch.py -k "persistent or staged_patterns" -v -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/wsp_tests.log 2>&1
  rc=$?; tail -8 gpurun_out/wsp_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/wsp_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  # one-shot (XRS_WSP=0) vs the default (persistent for 2 lost from 256 KiB halves)
  for size in 524288 786432 1048576 1572864 2097152 4194304 8388608; do
    ab VAR=XRS_WSP VALS=0, CASE=reconst_2 SIZE=$size ROUNDS=9
  done
  grep -v amdgpu.ids $out
fi
exit 0
