#!/bin/bash
# Round 5, first GPU call: the new tests (queue coalescing, registered-memory
# per-stripe calls, persistent-kernel counter slots) and smoke, the
# persistent kernel's per-call cost (item 6), the per-stripe rates with and without
# registered vects, the staged large-half investigation
# (item 2: rates, then rocprofv3 --pmc passes) and the parked ragged-half
# Encode A/B (item 5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# a failed test (rc 1) does not stop the measurements; a crash, abort or time
# limit (124, 134, 137, 139, or > 128) ends the call
gate() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernel_resources.py tests/test_gpu_registered.py \
    "tests/test_gpu_queue.py::test_queue_coalesces_barrier_released_callers" \
    "tests/test_gpu_edge.py::test_reconst_persistent_counter_slots_reused" \
    "tests/test_gpu_edge.py::test_reconst_persistent_concurrent_streams" \
    "tests/test_gpu_edge.py::test_reconst_batched_persistent_vs_oracle" \
    -s > gpurun_out/r05_first_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_first_tests.log; grep "queue:" gpurun_out/r05_first_tests.log; gate $rc
timeout -k 10 300 ./tests/cpp/build/xrs_test > gpurun_out/r05_cpp_tests.log 2>&1
rc=$?; tail -20 gpurun_out/r05_cpp_tests.log; gate $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05_smoke.log | tail -20; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_sync_bench.log
for mode in queue queuereg; do
  timeout -k 10 120 ./tools/sync_bench 4096 $mode 50 1 8 32 >> gpurun_out/r05_sync_bench.log 2>&1 || { echo "sync_bench $mode rc=$?"; tail gpurun_out/r05_sync_bench.log; exit 1; }
done
for mode in syncmt syncmtreg; do
  timeout -k 10 120 ./tools/sync_bench 4096 $mode 1 8 32 >> gpurun_out/r05_sync_bench.log 2>&1 || { echo "sync_bench $mode rc=$?"; tail gpurun_out/r05_sync_bench.log; exit 1; }
done
grep '^{' gpurun_out/r05_sync_bench.log
timeout -k 10 240 python -u tools/wsp_call_overhead.py > gpurun_out/r05_wsp_overhead.log 2>&1
rc=$?; grep n= gpurun_out/r05_wsp_overhead.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/staged_big_cases.py > gpurun_out/r05_staged_big.log 2>&1
rc=$?; grep '^{' gpurun_out/r05_staged_big.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05_staged_big.log; exit $rc; }
export CASES=A,C,D,E,F,G,H
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum \
    TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE -d gpurun_out/r05_pmc_bigA -o pmc --output-format csv -- \
    python tools/staged_big_cases.py > gpurun_out/r05_pmc_bigA.log 2>&1
rc=$?; echo "pmc A rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05_pmc_bigA.log; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
    TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum GRBM_GUI_ACTIVE -d gpurun_out/r05_pmc_bigB -o pmc \
    --output-format csv -- python tools/staged_big_cases.py > gpurun_out/r05_pmc_bigB.log 2>&1
rc=$?; echo "pmc B rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05_pmc_bigB.log; exit $rc; }
python tools/pmc_generic.py gpurun_out/r05_pmc_bigA gpurun_out/r05_pmc_bigB > gpurun_out/r05_staged_big_pmc.jsonl
cat gpurun_out/r05_staged_big_pmc.jsonl
unset CASES
bash tools/r04_encws_ragged.sh
