#!/bin/bash
# Round 4: the persistent 2-lost kernel's default range also takes lost data +
# parity patterns (nl = nn = 2): one-shot (XRS_WSP=0) vs default, GB/s of
# accounted bytes (d + lost) * S (tools/env_ab.py mixed_*); then tile orders
# for the forced persistent kernel at 2-8 MiB vects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wsp_mixed.log
: > $out
ab() { echo "== $*" >> $out; env "$@" timeout -k 10 150 python tools/env_ab.py >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }; }
XRS_TRACE_PRINT=1 timeout -k 10 60 python - >> $out 2>&1 <<'PY'
import torch, xrs_amd
x = xrs_amd.XRS(12, 4)
s = torch.cuda.current_stream().cuda_stream
S, n = 1 << 20, 8
b = torch.zeros(n * 16 * S, dtype=torch.uint8, device="cuda")
for lost in ([0, 13], [1, 13], [0, 12], [0, 1]):
    has = [i for i in range(16) if i not in lost]
    xrs_amd.trace_kernels(True)
    x.reconst_batched(b.data_ptr(), S, S, 16 * S, n, has, lost, s)
    torch.cuda.synchronize()
    xrs_amd.trace_kernels(False)
    print("kernels", lost, list(xrs_amd.traced_kernels()))
PY
for size in 1048576 524288; do
  for c in mixed_0-13 mixed_1-13 mixed_0-12; do
    ab VAR=XRS_WSP VALS=0, CASE=$c SIZE=$size ROUNDS=9
  done
done
# larger vects: the persistent kernel forced, K = 128 / 256 / the default (tiles of one half)
for size in 8388608 4194304 2097152; do
  ab VAR=MULTI VALS="XRS_WSP=0,XRS_WSP=512,XRS_WSP=512+XRS_WS_ORDER=128,XRS_WSP=512+XRS_WS_ORDER=256,XRS_WSP=512+XRS_WS_ORDER=64" \
     CASE=reconst_2 SIZE=$size ROUNDS=7
done
grep -v amdgpu.ids $out
exit 0
