#!/bin/bash
# A/B bench lines: TESTS="tests/x.py ..." (GPU tests first, optional), then for each workload in
# WORKLOADS and each entry of VARS ("name:ENV=1" for an environment knob, or a
# variants/<name>.so library, or base) one bench.py line.  Every step has its own time limit; a
# failure stops the script.
set -u
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
  tail -1 $OUT/pytest.txt
fi
for W in ${WORKLOADS:-udp64}; do
  case $W in
    udp64) ARGS="--steps 300 --warmup 5" ;;
    stream) ARGS="--mode stream --steps 300 --warmup 5" ;;
    imix) ARGS="--workload imix --steps 3 --warmup 1" ;;
    quic) ARGS="--workload quic --steps 5 --warmup 1" ;;
    strict) ARGS="--strict 17 --steps 3 --warmup 1" ;;
  esac
  for V in ${VARS:-base}; do
    name=${V%%:*}; E=""; L=""
    case $V in
      base) ;;
      *:*) E=${V#*:} ;;
      *) L=ipfixprobe_amd/variants/$V.so ;;
    esac
    env $E IPXG_TUNING=1 IPXG_LIB=$L timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-e2e > $OUT/${W}_$name.json 2> $OUT/${W}_$name.err || { tail -5 $OUT/${W}_$name.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/${W}_$name.json "$W $name"
  done
done
