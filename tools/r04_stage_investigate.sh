#!/bin/bash
# Round 4: the staged multi-loss Reconst gap at 1 MiB vects.
#  1. tools/stage_probe: pure memory patterns (Encode-like, staged-like with and
#     without in-place write-backs, read-only) at 4 KiB / 64 KiB / 1 MiB vects;
#  2. two rocprofv3 --pmc passes over tools/staged_pmc_cases.py: EA read/write
#     request counts and queue levels (mean latency = LEVEL / REQ), DRAM credit
#     and tag stalls, for the staged kernels at 4 KiB and 1 MiB and the Encode
#     launches beside them;
#  3. tools/qlat_probe once (the wait-value variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-probe,pmc,qlat}
if [[ $STEPS == *probe* ]]; then
  timeout -k 10 180 ./tools/stage_probe 20 > gpurun_out/stage_probe.log 2>&1
  rc=$?; echo "stage_probe rc=$rc"; cat gpurun_out/stage_probe.log | tail -70; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *pmc* ]]; then
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum \
      TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_stA -o pmc --output-format csv -- \
      python tools/staged_pmc_cases.py > gpurun_out/pmc_stA.log 2>&1
  rc=$?; echo "pmc A rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/pmc_stA.log; exit $rc; }
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
      TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_stB -o pmc \
      --output-format csv -- python tools/staged_pmc_cases.py > gpurun_out/pmc_stB.log 2>&1
  rc=$?; echo "pmc B rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/pmc_stB.log; exit $rc; }
  python tools/pmc_generic.py gpurun_out/pmc_stA gpurun_out/pmc_stB > gpurun_out/staged_pmc_counters.jsonl
  cat gpurun_out/staged_pmc_counters.jsonl
fi
if [[ $STEPS == *qlat* ]]; then
  timeout -k 10 120 ./tools/qlat_probe > gpurun_out/qlat.log 2>&1
  rc=$?; echo "qlat rc=$rc"; tail -40 gpurun_out/qlat.log
fi
exit 0
