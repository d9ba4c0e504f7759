#!/bin/bash
# A short bench line (no CPU baseline, config5, host path, queue or xGMI keys)
# to check the roofline and its PMC traffic provenance on the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --config5-stripes 0 \
  --host-mib 0 --queue-callers --xgmi-stripes 0 --ramp-seconds 1 \
  > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?
echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_quick.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], r["frac"], r["traffic"], r["traffic_source"])
PY
