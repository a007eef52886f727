#!/bin/bash
# The round's GPU evidence in one gpurun call: GPU parity tests, smoke, one bench line per
# workload (BASELINE.json configs[1], [2], [4], the streaming and the strict modes), then the
# rocprofv3 kernel-trace statistics and FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh).
# Usage: TAG=r02 [STAGES="test bench prof"] [WORKLOADS=...] bash tools/gpu_round.sh
# Every GPU step has its own time limit; a fault, abort or timeout stops the script there
# (plain test failures, exit 1, do not).
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
stop_on_fault() {
    case "$1" in
        0|1) return 0 ;;
        *) echo "STOP: $2 exited $1 (fault/timeout) -- no further GPU steps"; exit "$1" ;;
    esac
}
STAGES=${STAGES:-test bench prof}
if [[ " $STAGES " == *" test "* ]]; then
  echo "== pytest -m gpu"; date
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.txt 2>&1
  rc=$?; tail -4 $OUT/pytest_gpu.txt; stop_on_fault $rc pytest
  echo "== smoke"; date
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
  rc=$?; tail -1 $OUT/smoke.txt; stop_on_fault $rc smoke
fi
if [[ " $STAGES " == *" bench "* ]]; then
  for W in ${BENCHES:-udp64 stream imix quic strict imix10m imix_plugins quic_plugins}; do
    case $W in
      udp64) ARGS="" ;;  # the driver's default invocation
      stream) ARGS="--mode stream --steps 50 --warmup 3 --no-cpu-baseline --no-e2e" ;;
      imix) ARGS="--workload imix --steps 3 --warmup 1 --no-cpu-baseline --no-e2e" ;;
      quic) ARGS="--workload quic --steps 5 --warmup 1 --no-cpu-baseline --no-e2e" ;;
      strict) ARGS="--strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify" ;;
      imix10m) ARGS="--workload imix10m --shard 0/8 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e" ;;
      imix_plugins) ARGS="--workload imix --plugins dns,http,tls --steps 3 --warmup 1 --no-cpu-baseline --no-e2e" ;;
      quic_plugins) ARGS="--workload quic --plugins quic --steps 5 --warmup 1 --no-cpu-baseline --no-e2e" ;;
    esac
    echo "== bench $W"; date
    timeout -k 10 500 python bench.py $ARGS > $OUT/bench_$W.json 2> $OUT/bench_$W.err
    rc=$?; cut -c1-300 $OUT/bench_$W.json; tail -2 $OUT/bench_$W.err; stop_on_fault $rc "bench $W"
  done
fi
if [[ " $STAGES " == *" prof "* ]]; then
  TAG=$TAG PMC=${PMC:-0} WORKLOADS="${PROF_WORKLOADS:-udp64 imix quic imix_plugins quic_plugins}" bash tools/gpu_profile.sh
  rc=$?; stop_on_fault $rc profile
fi
echo "== round done"; date
