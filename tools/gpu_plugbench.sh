#!/bin/bash
# Plugin bench lines (bench.py --plugins config) per workload and library variant:
# WORKLOADS="quic imix" VARS="base old ..." (variants/<name>.so), TAG=...
set -u
OUT=gpurun_out/${TAG:-plug}
mkdir -p $OUT
for W in ${WORKLOADS:-quic}; do
  for V in ${VARS:-base}; do
    L=""; [ "$V" != base ] && L=ipfixprobe_amd/variants/$V.so
    IPXG_TUNING=1 IPXG_LIB=$L timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 1 --plugins config --no-cpu-baseline --no-e2e > $OUT/${W}_$V.json 2> $OUT/${W}_$V.err
    rc=$?; [ $rc -ne 0 ] && { tail -4 $OUT/${W}_$V.err; echo "STOP: $W $V exited $rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['plugins']['host_walk'])" $OUT/${W}_$V.json "$W $V"
  done
done
