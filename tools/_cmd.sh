set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_order.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_order.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_order.log; exit $rc
