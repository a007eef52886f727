#!/bin/bash
# One iteration on the GPU box: a subset of the GPU tests, then bench lines per workload.
#   TESTS="tests/test_gpu_parity.py ..."  (default: the parity core; "none" skips)
#   BENCH="udp64 imix quic"               (workloads; "none" skips)
#   TAG=name                              (output directory gpurun_out/$TAG)
# Every GPU step runs under its own time limit; a fault, abort or timeout ends the script.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
stop() { case "$1" in 0) return 0 ;; 1) [ "${2#pytest}" != "$2" ] && return 0 ;; esac; echo "STOP: $2 exited $1"; exit "$1"; }
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_semantics.py tests/test_gpu_workloads.py}
if [ "$TESTS" != "none" ]; then
  echo "== pytest $TESTS"; date
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest.txt 2>&1
  rc=$?; tail -3 $OUT/pytest.txt; stop $rc pytest
fi
for W in ${BENCH:-udp64}; do
  [ "$W" = none ] && break
  case $W in
    udp64) ARGS="--steps 300 --warmup 5" ;;
    imix) ARGS="--workload imix --steps 3 --warmup 1" ;;
    quic) ARGS="--workload quic --steps 5 --warmup 1" ;;
    imix10m) ARGS="--workload imix10m --shard 0/8 --steps 1 --warmup 1" ;;
    *) ARGS="$W" ;;
  esac
  echo "== bench $W"; date
  timeout -k 10 600 python bench.py $ARGS --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > $OUT/bench_${W%% *}.json 2> $OUT/bench_${W%% *}.err
  rc=$?; stop $rc "bench $W"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpkt/s', d['ms_per_step'], 'ms/step', 'kernel', r['frac'], 'step', r['step_frac'], d['stage_ms_per_step'])" $OUT/bench_${W%% *}.json "$W"
done
echo "== done"; date
