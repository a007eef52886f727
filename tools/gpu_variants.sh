#!/bin/bash
# Bench lines for compile-time variants of libipxg.so (tools/variants.sh builds them into
# ipfixprobe_amd/variants/<name>.so): VARIANTS="base nohash ..." (base = the in-tree library),
# WORKLOADS="udp64 imix".  Timing-experiment builds need IPXG_TUNING=1 (set here).  Every run has
# its own time limit; a fault, abort or timeout stops the script there.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
for W in ${WORKLOADS:-udp64}; do
  case $W in
    udp64) ARGS="--steps 300 --warmup 5" ;;
    imix) ARGS="--workload imix --steps 3 --warmup 1" ;;
    quic) ARGS="--workload quic --steps 5 --warmup 1" ;;
  esac
  for V in ${VARIANTS:-base}; do
    LIB=""; [ "$V" != base ] && LIB=ipfixprobe_amd/variants/$V.so
    echo "== $W $V"; date
    IPXG_TUNING=1 IPXG_LIB=$LIB timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-e2e \
        > $OUT/${W}_$V.json 2> $OUT/${W}_$V.err
    rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/${W}_$V.err; echo "STOP: $W $V exited $rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mpkt/s', d['ms_per_step'], 'ms/step', d['stage_ms_per_step'])" \
        $OUT/${W}_$V.json "$W $V"
  done
done
echo "== done"; date
