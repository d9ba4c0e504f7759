#!/bin/bash
# End-of-round refresh of the per-config tables with the
# final library: every BASELINE config, other codecs, the reference's matrix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/bench_configs.py c2 c3 c4 c5 rows multi > gpurun_out/final_configs.log 2>&1 || exit $?
timeout -k 10 300 python tools/refbench.py > gpurun_out/final_refbench.log 2>&1 || exit $?
timeout -k 10 500 python tools/bench_configs.py others_ab > gpurun_out/final_others_ab.log 2>&1 || exit $?
echo done
