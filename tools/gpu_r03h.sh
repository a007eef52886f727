#!/bin/bash
# round 3: strict replay scheduler probes with and without the sweep pruning; plugin walk trace
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03h
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
for PR in 1 0; do
  IPXG_STRICT_PRUNE=$PR IPXG_TUNING=1 IPXG_LIB=$PWD/ipfixprobe_amd/variants/probe.so timeout -k 10 200 python tools/probe_strict.py 17 \
      > $OUT/probe_strict_$PR.txt 2>&1
  rc=$?; echo "prune=$PR"; tail -6 $OUT/probe_strict_$PR.txt; stop $rc "probe strict $PR"
done
IPXG_WALK_TRACE=1 timeout -k 10 400 python bench.py --workload imix --plugins config --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_imix_plugins.json 2> $OUT/bench_imix_plugins.err
rc=$?; grep "walk ms" $OUT/bench_imix_plugins.err; python3 -c "import json; d=json.load(open('$OUT/bench_imix_plugins.json')); print(d['value'], d['plugins']['host_walk'])"; stop $rc "bench imix plugins"
echo "== done"
