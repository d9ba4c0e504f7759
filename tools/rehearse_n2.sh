#!/bin/bash
# Two ranks on the one card (XRS_REHEARSAL=1): the N > 1 bench path end to
# end (split, gloo bracket, config5, host_e2e, parity leg on both ranks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
XRS_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 \
  --config5-stripes 512 --host-mib 64 --ramp-seconds 1 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?
echo "n2 rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_n2.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_n2.json").read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], d["shared_gpu"], d["parity"]["bitexact"], d["parity"]["all_ranks"],
      d["per_stripe_queue"], d["config5"]["encode"]["gibps"])
PY
