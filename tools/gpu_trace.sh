#!/bin/bash
# Kernel traces of bench.py (no PMC) per workload, each followed by its step timeline
# (tools/trace_gaps.py: per-kernel durations and the idle gap before each kernel).
# Usage: TAG=r5a WORKLOADS="udp64 stream" bash tools/gpu_trace.sh
# Every GPU step has its own time limit; a fault, abort or timeout stops the script there.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-trace}
mkdir -p $OUT
export TMPDIR=/tmp
for W in ${WORKLOADS:-udp64}; do
  case $W in
    udp64) ARGS="--steps 30 --warmup 3"; FIRST="k_bin<" ;;
    stream) ARGS="--mode stream --steps 20 --warmup 3"; FIRST="k_bin<" ;;
    imix) ARGS="--workload imix --steps 2 --warmup 1"; FIRST=k_finish ;;
    quic) ARGS="--workload quic --steps 3 --warmup 1"; FIRST=k_finish ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  echo "== kernel trace $W"; date
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$W -o run -- \
      python3 bench.py $ARGS ${BENCH_ARGS:-} --no-cpu-baseline --no-e2e > $OUT/kt_$W.json 2> $OUT/kt_$W.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/kt_$W.err; echo "STOP: kernel trace $W exited $rc"; exit $rc; }
  f=$(find $OUT/kt_$W -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_gaps.py "$f" $FIRST 3 > $OUT/gaps_$W.txt || true
  head -c 400 $OUT/kt_$W.json; echo
done
echo "== done"; date
