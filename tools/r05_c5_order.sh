set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 env VAR=XRS_BLOCK_ORDER VALS=128,0,32,64,256,512,full CASE=encode SIZE=1048576 STRIPES=8192 ROUNDS=5 \
  python -u tools/env_ab.py > gpurun_out/r05_c5_order.log 2>&1
rc=$?; cat gpurun_out/r05_c5_order.log | grep '^{'; exit $rc
