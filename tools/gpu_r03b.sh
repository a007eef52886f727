#!/bin/bash
# round 3, second GPU pass: the new GPU tests (plugins on the workloads, follow_packets, the
# bench-exact size parity, the export gather), then bench lines: imix / quic with and without
# their process plugins, configs[3]'s per-GPU shard (imix10m --shard 0/8), udp64.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03b
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_stdplugins.py tests/test_ref_plugins.py tests/test_gpu_parity.py tests/test_shard.py tests/test_strict.py \
    tests/test_gpu_workloads.py tests/test_gpu_semantics.py::test_bench_size_parity tests/test_gpu_semantics.py::test_wide_walk_ext_and_gre_edges -m gpu -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread > $OUT/pytest_new.txt 2>&1
rc=$?; tail -15 $OUT/pytest_new.txt; stop $rc pytest
for W in "udp64:--steps 50 --warmup 3 --no-cpu-baseline --no-e2e" \
         "imix:--workload imix --steps 3 --warmup 1 --no-cpu-baseline --no-e2e" \
         "imix_plugins:--workload imix --plugins config --steps 3 --warmup 1 --no-cpu-baseline --no-e2e" \
         "quic:--workload quic --steps 5 --warmup 1 --no-cpu-baseline --no-e2e" \
         "quic_plugins:--workload quic --plugins config --steps 5 --warmup 1 --no-cpu-baseline --no-e2e" \
         "imix10m_shard:--workload imix10m --shard 0/8 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"; do
  N=${W%%:*}; A=${W#*:}
  echo "== bench $N"; date
  timeout -k 10 400 python bench.py $A > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; cut -c1-400 $OUT/bench_$N.json; tail -2 $OUT/bench_$N.err; stop $rc "bench $N"
done

echo "== membench"; date
timeout -k 10 120 tools/membench/membench 10000000 64 2048 > $OUT/membench.txt 2>&1
timeout -k 10 120 tools/membench/membench 10000000 64 1024 >> $OUT/membench.txt 2>&1
cat $OUT/membench.txt
echo "== done"; date
