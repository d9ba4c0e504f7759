#!/bin/bash
# Round 4: HBM bytes per staged launch (FETCH_SIZE / WRITE_SIZE passes over
# tools/staged_pmc_cases.py) with the persistent 2-lost kernel in place, vs
# the bytes each launch must move (the JSON lines of staged_pmc_cases.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/wsp_pmc_fetch -o pmc --output-format csv -- \
    python tools/staged_pmc_cases.py > gpurun_out/wsp_pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/wsp_pmc_fetch.log; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wsp_pmc_write -o pmc --output-format csv -- \
    python tools/staged_pmc_cases.py > gpurun_out/wsp_pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/wsp_pmc_write.log; exit $rc; }
{ grep '^{' gpurun_out/wsp_pmc_fetch.log; python tools/pmc_by_kernel.py gpurun_out/wsp_pmc_fetch gpurun_out/wsp_pmc_write; } \
    > gpurun_out/wsp_pmc.txt
cat gpurun_out/wsp_pmc.txt
exit 0
