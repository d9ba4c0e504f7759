#!/bin/bash
# Round 4: the persistent counter-fed Encode (XRS_ENC_WSP=T; the kernel,
# enc_wsp_kernel, is in commit 416ee77 only: slower at every size, removed) against the
# default launch: oracle tests forced (also with 24-block grids, so blocks
# take many tiles), then an interleaved A/B, bytes moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab}
if [[ $STEPS == *tests* ]]; then
  for env in "XRS_ENC_WSP=512" "XRS_ENC_WSP=256" "XRS_ENC_WSP=512 XRS_WSP_GRID=24"; do
    env $env timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "encode_batched_vs_oracle" \
        -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/encwsp_tests.log 2>&1
    rc=$?; echo "$env"; tail -2 gpurun_out/encwsp_tests.log; [ $rc -eq 0 ] || exit $rc
  done
fi
if [[ $STEPS == *ab* ]]; then
  out=gpurun_out/encwsp_ab.log
  : > $out
  ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
  V=",XRS_ENC_WSP=512,XRS_ENC_WSP=256+XRS_WSP_PER_CU=2,XRS_ENC_WSP=512+XRS_ENC_WS_ORDER=128"
  for size in 1048576 2097152 524288 8388608 4096; do
    ab VAR=MULTI VALS=$V CASE=encode SIZE=$size ROUNDS=9
  done
  grep -v amdgpu.ids $out
fi
exit 0
