#!/bin/bash
# Eight ranks on the one card (XRS_REHEARSAL=1, XRS_XGMI_SELF=1): the N = 8
# bench path the driver's 8-GPU run takes, end to end with small batches:
# 8-rank gloo start-up, the per-rank stripe split, the config5 agreement over
# ranks, config4, host_e2e, the xgmi_repair child (its peers are the same
# device here), and the oracle parity leg on every rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
XRS_REHEARSAL=1 XRS_XGMI_SELF=1 timeout -k 10 420 python bench.py --gpus 8 --steps 30 --warmup 2 \
  --enc-stripes 1024 --rec-stripes 8 --config5-stripes 64 --config5-steps 2 --host-mib 64 \
  --config4-stripes 4 --config4-steps 2 --xgmi-stripes 8 --ramp-seconds 0.5 \
  > gpurun_out/bench_n8.json 2> gpurun_out/bench_n8.err
rc=$?
echo "n8 rc=$rc"
[ $rc -eq 0 ] || { tail -30 gpurun_out/bench_n8.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_n8.json").read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "value", d["value"], "shared_gpu", d["shared_gpu"],
      "ranks", len(d["rank_devices"]), "parity", d["parity"]["bitexact"], d["parity"]["all_ranks"])
print("config5", d["config5"]["stripes_total"], d["config5"]["roundtrip_ok_ranks"])
print("xgmi", json.dumps(d["xgmi_repair"])[:400])
print("library", d["library"]["built_from_tree"])
PY
