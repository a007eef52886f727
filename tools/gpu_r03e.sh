#!/bin/bash
# round 3: the whole GPU suite on HEAD, the plugin benches with the host walk's phase trace, an
# A/B of k_fin_list probing the table (default) vs k_reduce probing it (variants/finres.so) on
# udp64 / quic / imix, then the profile passes of tools/gpu_r03c.sh.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03e
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.txt; stop $rc pytest
for W in "imix_plugins:--workload imix --plugins config --steps 3 --warmup 1" \
         "quic_plugins:--workload quic --plugins config --steps 5 --warmup 1"; do
  N=${W%%:*}; A=${W#*:}
  IPXG_WALK_TRACE=1 timeout -k 10 400 python bench.py $A --no-cpu-baseline --no-e2e > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; grep "walk ms" $OUT/bench_$N.err; stop $rc "bench $N"
done
for rep in 1 2; do
  for W in "udp64:--steps 100 --warmup 5" "quic:--workload quic --steps 10 --warmup 2" "imix:--workload imix --steps 3 --warmup 1"; do
    N=${W%%:*}; A=${W#*:}
    for v in default finres; do
      if [ $v = default ]; then L=""; else L="IPXG_LIB=$PWD/ipfixprobe_amd/variants/$v.so"; fi
      env $L timeout -k 10 300 python bench.py $A --no-cpu-baseline --no-e2e > $OUT/ab_${N}_${v}_$rep.json 2> $OUT/ab_${N}_${v}_$rep.err
      rc=$?; python3 -c "import json; d=json.load(open('$OUT/ab_${N}_${v}_$rep.json')); print('$N $v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
      stop $rc "ab $N $v"
    done
  done
done
bash tools/gpu_r03c.sh
