#!/bin/bash
# Two rocprofv3 --pmc passes over bench.py (counters only: no trace domains),
# then HBM bytes per launch -> gpurun_out/pmc_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config5-stripes 0 --host-mib 0 --xgmi-stripes 0 --ramp-seconds 0.3 --no-parity"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- $B \
  > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch pass rc=$?"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- $B \
  > gpurun_out/pmc_write.log 2>&1 || { echo "write pass rc=$?"; tail -20 gpurun_out/pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_traffic.json
cat gpurun_out/pmc_traffic.json
