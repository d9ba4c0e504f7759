#!/bin/bash
# Round 6, final-library parity campaign: 120 fresh big-vect fuzz seeds
# (128 KiB - 1 MiB vects), 24 registered-memory fuzz seeds (sync and queue
# table mode, child process), then the full GPU suite once more.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
faulted() { grep -q -i "illegal memory access\|memory access fault" "$@" 2>/dev/null; }
XRS_FUZZ_SEEDS=120 XRS_FUZZ_BASE=200000 XRS_FUZZ_BIG=1 timeout -k 10 600 \
    python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_fuzz.py > gpurun_out/r06_fuzz_big_120seeds.log 2>&1
rc=$?; tail -2 gpurun_out/r06_fuzz_big_120seeds.log; [ $rc -eq 0 ] || exit $rc
faulted gpurun_out/r06_fuzz_big_120seeds.log && exit 1
XRS_FUZZ_SEEDS=24 timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread \
    -p no:cacheprovider "tests/test_gpu_registered.py::test_registered_case_in_child[test_registered_fuzz_vs_oracle]" \
    > gpurun_out/r06_registered_fuzz_24seeds.log 2>&1
rc=$?; tail -2 gpurun_out/r06_registered_fuzz_24seeds.log; [ $rc -eq 0 ] || exit $rc
STEPS=pytest bash tools/gpu_check.sh
echo "fault lines: $(grep -c -i 'illegal memory access' gpurun_out/pytest_gpu.log || true)"
