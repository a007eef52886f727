#!/bin/bash
# Plugin lines in byte and 16-byte unit offsets on one box (the host walk varies across boxes).
set -u
OUT=gpurun_out/plugab; mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline --no-e2e > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['plugins']['host_walk']; print(sys.argv[2], d['value'], d['ms_per_step'], h['ms_per_step'], h['overlapped_batches_per_step'])" $OUT/$name.json $name; }
for r in 1 2; do
  run imix_plug_bytes$r --workload imix --plugins dns,http,tls --steps 3 --warmup 1 --offsets bytes
  run imix_plug_units$r --workload imix --plugins dns,http,tls --steps 3 --warmup 1 --offsets units --packets 14285715 --batches 7
  run quic_plug_bytes$r --workload quic --plugins quic --steps 3 --warmup 1 --offsets bytes
  run quic_plug_units$r --workload quic --plugins quic --steps 3 --warmup 1 --offsets units
done
