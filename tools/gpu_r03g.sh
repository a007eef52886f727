#!/bin/bash
# round 3: strict replay with provably idle-free sweep steps left out of the DAG -- strict
# parity tests, then the strict bench at the reference default (s=17).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_strict.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_strict.txt 2>&1
rc=$?; tail -4 $OUT/pytest_strict.txt; [ $rc = 0 ] || { echo "STOP: strict tests rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_strict.json 2> $OUT/bench_strict.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench_strict.json')); print(d['value'], d['ms_per_step'], d['verify'])"; stop $rc "bench strict"
echo "== done"
