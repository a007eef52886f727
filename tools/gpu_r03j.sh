#!/bin/bash
# round 3: strict multi-workgroup tuning -- workgroups per XCD x lanes per workgroup, body-phase probes
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03j
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
IPXG_STRICT_MW_LANES=256 timeout -k 10 600 python -u -m pytest tests/test_strict.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread -k multi \
    > $OUT/pytest_strict256.txt 2>&1
rc=$?; tail -2 $OUT/pytest_strict256.txt; [ $rc = 0 ] || { echo "STOP: strict tests rc=$rc"; exit 1; }
for L in 768 256; do for W in 2 4 6 8 12 16; do
  IPXG_STRICT_MW_LANES=$L IPXG_STRICT_WGS=$W timeout -k 10 300 python bench.py --strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_strict_l${L}_w$W.json 2> $OUT/bench_strict_l${L}_w$W.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict_l${L}_w$W.json')); print('strict lanes=$L wgs=$W', d['value'], d['ms_per_step'])"; stop $rc "bench strict $L $W"
done; done
for C in "768 0" "768 4" "256 8"; do set -- $C
  IPXG_STRICT_MW_LANES=$1 IPXG_STRICT_WGS=$2 IPXG_TUNING=1 IPXG_LIB=$PWD/ipfixprobe_amd/variants/probe.so timeout -k 10 200 python tools/probe_strict.py 17 > $OUT/probe_strict_l$1_w$2.txt 2>&1
  rc=$?; echo "probe lanes=$1 wgs=$2"; tail -6 $OUT/probe_strict_l$1_w$2.txt; stop $rc "probe strict"
done
echo "== done"
