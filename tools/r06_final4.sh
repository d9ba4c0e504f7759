#!/bin/bash
# Round 6, validation of the rebuilt library (header comment changed, so a
# new source digest and sha256): PMC passes keyed to it, then the GPU suite,
# smoke, bench (reading the fresh PMC traffic) and rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc.sh || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
STEPS=pytest,smoke,bench,prof bash tools/gpu_check.sh
