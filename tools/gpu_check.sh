#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout/abort stops the script there.
# Plain test failures (pytest exit 1) do not stop the later steps.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
stop_on_fault() {  # $1 = exit status, $2 = step name
    case "$1" in
        0|1) return 0 ;;
        *) echo "STOP: $2 exited $1 (fault/timeout) -- no further GPU steps"; exit "$1" ;;
    esac
}
echo "== pytest -m gpu"; date
timeout -k 10 1200 python -u -m pytest tests -m gpu -q ${PYTEST_X--x} -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu_$TAG.log; stop_on_fault $rc pytest
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; tail -3 $OUT/smoke_$TAG.log; stop_on_fault $rc smoke
echo "== bench"; date
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cat $OUT/bench_$TAG.json; tail -3 $OUT/bench_$TAG.err; stop_on_fault $rc bench
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"; date
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
      python3 bench.py --steps ${PROF_STEPS:-30} --warmup 2 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err
  rc=$?; tail -2 $OUT/prof_$TAG.err; stop_on_fault $rc rocprof
  find $OUT/prof_$TAG -name "*stats*" | head
fi
echo "== done"; date
