#!/bin/bash
# Round 6, final validation after the registered cases moved to child
# processes: PMC passes of this library, the GPU suite, smoke, bench,
# rocprofv3 --stats; then (only if nothing faulted) the standalone
# host-memory-churn reproducer (tools/fault_repro.cpp).  Any GPU fault ends
# the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
faulted() { grep -q -i "illegal memory access\|memory access fault" "$@" 2>/dev/null; }
bash tools/gpu_pmc.sh || exit $?
STEPS=pytest bash tools/gpu_check.sh
if faulted gpurun_out/pytest_gpu.log; then echo "GPU fault in the suite: stopping"; exit 1; fi
STEPS=smoke,bench,prof bash tools/gpu_check.sh || exit $?
timeout -k 10 240 ./tools/fault_repro both 300 > gpurun_out/r06_fault_repro.log 2>&1
echo "fault_repro both rc=$?"; tail -3 gpurun_out/r06_fault_repro.log
if faulted gpurun_out/r06_fault_repro.log || grep -q FAULT gpurun_out/r06_fault_repro.log; then exit 1; fi
timeout -k 10 240 ./tools/fault_repro_q queue 150 > gpurun_out/r06_fault_repro_q.log 2>&1
echo "fault_repro queue rc=$?"; tail -3 gpurun_out/r06_fault_repro_q.log
exit 0
