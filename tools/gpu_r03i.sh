#!/bin/bash
# round 3: strict parity (one and several workgroups) + bench sweep over workgroups per XCD;
# strict memory-pipeline counters; plugin benches with the first-packet-ordered walk layout.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_strict.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_strict.txt 2>&1
rc=$?; tail -4 $OUT/pytest_strict.txt; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/pytest_strict.txt | head -20; echo "STOP: strict tests rc=$rc"; exit 1; }
for W in 0 4 8 16 32; do
  IPXG_STRICT_WGS=$W timeout -k 10 300 python bench.py --strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify > $OUT/bench_strict_w$W.json 2> $OUT/bench_strict_w$W.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict_w$W.json')); print('strict wgs=$W', d['value'], d['ms_per_step'], d['verify'])"; stop $rc "bench strict $W"
done
for W in 0 8; do
  IPXG_STRICT_WGS=$W IPXG_TUNING=1 IPXG_LIB=$PWD/ipfixprobe_amd/variants/probe.so timeout -k 10 200 python tools/probe_strict.py 17 > $OUT/probe_strict_w$W.txt 2>&1
  rc=$?; tail -5 $OUT/probe_strict_w$W.txt; stop $rc "probe strict"
done
timeout -k 10 600 python -u -m pytest tests/test_ref_plugins.py tests/test_stdplugins.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_plugins.txt 2>&1
rc=$?; tail -2 $OUT/pytest_plugins.txt; [ $rc = 0 ] || { echo "STOP: plugin tests rc=$rc"; exit 1; }
for W in "imix_plugins:--workload imix --plugins config --steps 3 --warmup 1" \
         "quic_plugins:--workload quic --plugins config --steps 5 --warmup 1"; do
  N=${W%%:*}; A=${W#*:}
  IPXG_WALK_TRACE=1 timeout -k 10 400 python bench.py $A --no-cpu-baseline --no-e2e > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; grep "walk ms" $OUT/bench_$N.err; python3 -c "import json; d=json.load(open('$OUT/bench_$N.json')); print(d['value'], d['plugins']['host_walk'])"; stop $rc "bench $N"
done
timeout -k 10 -s KILL 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $OUT/pmc_strict_ta -o run -- python3 bench.py --strict 17 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
    > $OUT/pmc_strict_ta.json 2> $OUT/pmc_strict_ta.err
rc=$?; stop $rc "pmc strict ta"
echo "== done"
