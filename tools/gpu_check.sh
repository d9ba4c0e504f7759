#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, a rocprofv3 kernel
# trace.  Every GPU step has its own time limit; a crash/timeout ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
if [[ $STEPS == *counters* ]]; then
  run counters 120 rocprofv3 -L || true
fi
if [[ $STEPS == *pytest* ]]; then
  run pytest_gpu 1200 python -u -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider \
      --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [[ $STEPS == *bench* ]]; then
  run bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
fi
if [[ $STEPS == *prof* ]]; then
  # 40 timed steps after a 2 s soak: the dominant launch's --stats average is
  # then within a fraction of a percent of the line's HIP-event timing
  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 40 --warmup 2 --no-cpu-baseline --config5-stripes 0 --host-mib 0 --ramp-seconds 2 \
      --xgmi-stripes 0 --config4-stripes 0 --queue-callers || exit $?
fi
exit 0
