#!/bin/bash
# bench.py once per environment setting (tuning knobs read by the engine, e.g.
# IPXG_PART_BITS=7), one summary line each:
#   SETTINGS="IPXG_PART_BITS=7 IPXG_PART_BITS=8 IPXG_BIN_GRID=512" bash tools/env_sweep.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for s in ${SETTINGS:-IPXG_PART_BITS=8}; do
  tag=$(echo "$s" | tr '=,' '__')
  env "$s" timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} \
      > gpurun_out/env_$tag.json 2> gpurun_out/env_$tag.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "$s: exit $rc"; tail -3 gpurun_out/env_$tag.err; exit $rc; fi
  python3 -c "
import json; d=json.load(open('gpurun_out/env_$tag.json'))
print('%-22s %8.1f Mpkt/s  step %.4f ms  stages %s' % ('$s', d['value'], d['ms_per_step'], d['stage_ms_per_step']))"
done
