#!/bin/bash
# A/B of library variants (tools/variants.sh) on bench workloads, one summary line each:
#   LIBS="default fin4" WORKLOADS="quic imix" bash tools/ab_lib.sh
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ab
mkdir -p $O
for rep in ${REPS:-1}; do
for w in ${WORKLOADS:-quic imix}; do
for lib in ${LIBS:-default}; do
  case $w in
    udp64) ARGS="--steps 300 --warmup 3" ;;
    *) ARGS="--workload $w --steps 3 --warmup 1" ;;
  esac
  if [ $lib = default ]; then unset IPXG_LIB IPXG_TUNING; else export IPXG_LIB=$PWD/ipfixprobe_amd/variants/$lib.so IPXG_TUNING=1; fi
  timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-e2e > $O/${w}_${lib}_$rep.json 2> $O/${w}_${lib}_$rep.err \
      || { echo "$w $lib failed"; tail -3 $O/${w}_${lib}_$rep.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${w}_${lib}_$rep.json')); print('%-6s %-8s %9.1f %8.4f' % ('$w', '$lib', d['value'], d['ms_per_step']), d['stage_ms_per_step'])"
done
done
done
