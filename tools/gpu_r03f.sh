#!/bin/bash
# round 3: GPU suite after the k_fin_list deferral fix, plugin benches (pageable walk copies,
# packed flow order) with the walk trace, k_reduce phase probes on quic / imix, and the SQ
# counters of the strict replay (issue- vs latency-bound).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03f
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.txt; stop $rc pytest
for W in "imix_plugins:--workload imix --plugins config --steps 3 --warmup 1" \
         "quic_plugins:--workload quic --plugins config --steps 5 --warmup 1"; do
  N=${W%%:*}; A=${W#*:}
  IPXG_WALK_TRACE=1 timeout -k 10 400 python bench.py $A --no-cpu-baseline --no-e2e > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; grep "walk ms" $OUT/bench_$N.err; python3 -c "import json; d=json.load(open('$OUT/bench_$N.json')); print(d['value'], d['plugins']['host_walk'])"; stop $rc "bench $N"
done
for W in quic imix; do
  IPXG_TUNING=1 IPXG_LIB=$PWD/ipfixprobe_amd/variants/probe.so timeout -k 10 300 python tools/probe_reduce.py $W \
      > $OUT/probe_$W.txt 2>&1
  rc=$?; cat $OUT/probe_$W.txt | tail -6; stop $rc "probe $W"
done
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD \
    --kernel-trace --output-format csv -d $OUT/pmc_strict -o run -- python3 bench.py --strict 17 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e \
    > $OUT/pmc_strict.json 2> $OUT/pmc_strict.err
rc=$?; stop $rc "pmc strict"
python3 tools/pmc_summary.py $OUT/pmc_strict | grep -i strict
echo "== done"
