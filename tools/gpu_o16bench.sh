set -u
OUT=gpurun_out/o16b; mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" --no-cpu-baseline --no-e2e > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('step_frac'), d['stage_ms_per_step'])" $OUT/$name.json $name; }
run quic4x5 --workload quic --steps 5 --warmup 1 --offsets bytes
run quic2x10 --workload quic --steps 5 --warmup 1 --packets 10000000 --batches 2 --offsets units
run imix10x10 --workload imix --steps 3 --warmup 1 --offsets bytes
run imix7x14 --workload imix --steps 3 --warmup 1 --packets 14285715 --batches 7 --offsets units
run udp64 --steps 300 --warmup 5
run imix10m_bytes --workload imix10m --shard 0/8 --steps 2 --warmup 1 --offsets bytes
run imix10m_units --workload imix10m --shard 0/8 --steps 2 --warmup 1
run quic_plug_units --workload quic --plugins config --steps 3 --warmup 1
run imix_plug_units --workload imix --plugins config --steps 2 --warmup 1
