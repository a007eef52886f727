#!/bin/bash
# bench.py once per library variant (ipfixprobe_amd/variants/*.so), one line each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in ${VARIANTS:-$(ls ipfixprobe_amd/variants/*.so)}; do
  name=$(basename $v .so)
  IPXG_TUNING=1 IPXG_LIB=$PWD/$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "$name: exit $rc"; tail -3 gpurun_out/var_$name.err; exit $rc; fi
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/var_$name.json'))
print('%-10s %8.1f Mpkt/s  step %.4f ms  stages %s' % ('$name', d['value'], d['ms_per_step'], d['stage_ms_per_step']))"
  grep -h verify gpurun_out/var_$name.err || true
done
