#!/bin/bash
# round 3: full GPU suite, then the plugin benches and the plugin-free imix/quic lines
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03o}
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 240 --timeout-method thread \
      > $OUT/pytest_gpu.txt 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.txt
  [ $rc = 0 ] || { grep -E "FAIL|Error|error" $OUT/pytest_gpu.txt | head -20; echo "STOP: tests rc=$rc"; exit 1; }
fi
TAG=${TAG:-r03o} SKIP_TESTS=1 RUNS="imix dns,http,tls 2 0;quic quic 3 0" bash tools/gpu_r03n.sh || exit 1
for W in imix quic; do
  timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_$W.json 2>$OUT/bench_$W.err
  rc=$?; python3 -c "
import json; d=json.load(open('$OUT/bench_$W.json')); print('$W', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"; stop $rc "bench $W"
done
echo "== done"; date
