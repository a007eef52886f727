#!/bin/bash
# round 3: strict replay lanes x workgroups sweep, two passes (A/B noise)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03l
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
for R in 1 2; do
for C in "128 12" "128 16" "128 20" "256 8" "256 12" "256 16" "768 6"; do set -- $C
  IPXG_STRICT_MW_LANES=$1 IPXG_STRICT_WGS=$2 timeout -k 10 300 python bench.py --strict 17 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_strict_l$1_w$2_$R.json 2> $OUT/bench_strict_l$1_w$2_$R.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict_l$1_w$2_$R.json')); print('strict lanes=$1 wgs=$2 pass=$R', d['value'], d['ms_per_step'])"; stop $rc "bench strict $1 $2"
done; done
echo "== done"
