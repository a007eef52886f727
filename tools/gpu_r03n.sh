#!/bin/bash
# round 3: plugin-bridge tests and the configs[2]/[4] plugin benches (walk trace)
#   RUNS="workload plugins steps walk_threads[;...]"  (default: imix and quic, default and 1 thread)
#   SKIP_TESTS=1  benches only;  ENVX="VAR=value ..." extra environment;  SFX: output name suffix
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03n}
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_stdplugins.py tests/test_ref_plugins.py tests/test_plugins.py -m gpu -q -x \
      -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_plugins.txt 2>&1
  rc=$?; tail -3 $OUT/pytest_plugins.txt
  [ $rc = 0 ] || { grep -E "FAIL|Error|error" $OUT/pytest_plugins.txt | head -20; echo "STOP: plugin tests rc=$rc"; exit 1; }
fi
IFS=';' read -ra LIST <<< "${RUNS:-imix dns,http,tls 2 0;quic quic 3 0;imix dns,http,tls 2 1;quic quic 3 1}"
for W in "${LIST[@]}"; do
  set -- $W
  F=$OUT/bench_$1_plugins_t$4${SFX:-}
  echo "== bench $1 plugins $2 walk threads $4 ${ENVX:-}"; date
  IPXG_WALK_TRACE=1 env ${ENVX:-} timeout -k 10 500 python bench.py --workload $1 --plugins $2 --steps $3 --warmup 1 \
      --no-cpu-baseline --no-e2e --walk-threads $4 > $F.json 2> $F.err
  rc=$?
  python3 -c "
import json; d=json.load(open('$F.json')); h=d['plugins']['host_walk']
print('$1 t=$4', d['value'], d['ms_per_step'], 'walk ms/step', h['ms_per_step'], 'stages', d['stage_ms_per_step'])"
  grep "plugin walk" $F.err; stop $rc "bench $1 plugins"
done
echo "== done"; date
