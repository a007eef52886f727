#!/bin/bash
# round 3 (session 2): state at HEAD -- GPU tests, smoke, the default bench line, the plugin
# benches with the host walk's phase trace
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03m
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
echo "== pytest -m gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.txt; stop $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -1 $OUT/smoke.txt; stop $rc smoke
echo "== bench default"; date
timeout -k 10 400 python bench.py > $OUT/bench_udp64.json 2> $OUT/bench_udp64.err
rc=$?; cut -c1-400 $OUT/bench_udp64.json; stop $rc "bench udp64"
for W in "imix dns,http,tls 2 0" "quic quic 3 0" "imix dns,http,tls 2 1" "quic quic 3 1"; do set -- $W
  echo "== bench $1 plugins $2 walk threads $4"; date
  IPXG_WALK_TRACE=1 timeout -k 10 500 python bench.py --workload $1 --plugins $2 --steps $3 --warmup 1 --no-cpu-baseline --no-e2e \
      --walk-threads $4 > $OUT/bench_$1_plugins_t$4.json 2> $OUT/bench_$1_plugins_t$4.err
  rc=$?; cut -c1-300 $OUT/bench_$1_plugins_t$4.json; tail -3 $OUT/bench_$1_plugins_t$4.err; stop $rc "bench $1 plugins"
done
echo "== done"; date
