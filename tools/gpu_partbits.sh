#!/bin/bash
# udp64 bench lines at forced partition counts (IPXG_PART_BITS, a setup_bins tuning knob):
# PBS="7 9" TAG=name bash tools/gpu_partbits.sh.  Each run under its own time limit.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pb}
mkdir -p $OUT
for PB in ${PBS:-7 9}; do
  echo "== part bits $PB"; date
  IPXG_PART_BITS=$PB timeout -k 10 300 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-e2e \
      > $OUT/udp64_pb$PB.json 2> $OUT/udp64_pb$PB.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/udp64_pb$PB.err; echo "STOP: part bits $PB exited $rc"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pb', sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" \
      $OUT/udp64_pb$PB.json $PB
done
echo "== done"
