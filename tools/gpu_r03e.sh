#!/bin/bash
# round 3: the follow test, the plugin benches with the host walk's phase trace, then the
# profile passes of tools/gpu_r03c.sh.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03e
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_stdplugins.py -k follow -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $OUT/pytest_follow.txt 2>&1
rc=$?; tail -2 $OUT/pytest_follow.txt; stop $rc pytest
for W in "imix_plugins:--workload imix --plugins config --steps 3 --warmup 1" \
         "quic_plugins:--workload quic --plugins config --steps 5 --warmup 1"; do
  N=${W%%:*}; A=${W#*:}
  IPXG_WALK_TRACE=1 timeout -k 10 400 python bench.py $A --no-cpu-baseline --no-e2e > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; grep "walk ms" $OUT/bench_$N.err; stop $rc "bench $N"
done
bash tools/gpu_r03c.sh
