#!/bin/bash
# round 3: strict suite at the new default (12 x 256-lane workgroups per XCD) + lane/workgroup sweep
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03k
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_strict.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $OUT/pytest_strict.txt 2>&1
rc=$?; tail -2 $OUT/pytest_strict.txt; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/pytest_strict.txt | head; echo "STOP: strict tests rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --strict 17 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --verify > $OUT/bench_strict.json 2> $OUT/bench_strict.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict.json')); print('strict default', d['value'], d['ms_per_step'], d['verify'])"; stop $rc "bench strict"
for C in "256 10" "256 14" "128 16" "128 24" "128 32"; do set -- $C
  IPXG_STRICT_MW_LANES=$1 IPXG_STRICT_WGS=$2 timeout -k 10 300 python bench.py --strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_strict_l$1_w$2.json 2> $OUT/bench_strict_l$1_w$2.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict_l$1_w$2.json')); print('strict lanes=$1 wgs=$2', d['value'], d['ms_per_step'])"; stop $rc "bench strict $1 $2"
done
IPXG_STRICT_WGS=12 IPXG_TUNING=1 IPXG_LIB=$PWD/ipfixprobe_amd/variants/probe.so timeout -k 10 200 python tools/probe_strict.py 17 > $OUT/probe_strict.txt 2>&1
rc=$?; tail -6 $OUT/probe_strict.txt; stop $rc "probe strict"
echo "== done"
