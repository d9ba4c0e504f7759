set -u
mkdir -p gpurun_out
timeout -k 10 200 tools/kbench rw > gpurun_out/kbench_rw.log 2>&1 || exit $?
timeout -k 10 200 tools/kbench rw xcd > gpurun_out/kbench_rw_xcd.log 2>&1 || exit $?
cat gpurun_out/kbench_rw.log gpurun_out/kbench_rw_xcd.log
