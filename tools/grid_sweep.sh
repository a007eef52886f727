#!/bin/bash
# bench.py once per k_bin grid size (IPXG_BIN_GRID), one summary line each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for g in ${GRIDS:-256 512 768 1024 1536 2048}; do
  IPXG_BIN_GRID=$g timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/grid_$g.json 2> gpurun_out/grid_$g.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "grid $g: exit $rc"; tail -3 gpurun_out/grid_$g.err; exit $rc; fi
  python3 -c "
import json; d=json.load(open('gpurun_out/grid_$g.json'))
print('grid %-5s %8.1f Mpkt/s  step %.4f ms  stages %s' % ('$g', d['value'], d['ms_per_step'], d['stage_ms_per_step']))"
done
