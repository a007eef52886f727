#!/bin/bash
# PMC passes over bench.py (each counter group in its own run, kernel trace only --
# MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ, <= 4 TCC counters per pass).
# Usage: TAG=r01d [SETS="FETCH_SIZE;WRITE_SIZE;..."] [BENCH_ARGS=...] bash tools/gpu_pmc.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; TAG=${TAG:-r01}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/pmc_list_$TAG.txt 2>&1 || true
DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
IFS=';' read -ra SETS_ARR <<< "${SETS:-$DEFAULT}"
for C in "${SETS_ARR[@]}"; do
  N=$(echo $C | tr ' ' '_')
  echo "== pmc $C"; date
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$TAG/$N -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pmc_${TAG}_$N.json 2> $OUT/pmc_${TAG}_$N.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $C exited $rc"; tail -3 $OUT/pmc_${TAG}_$N.err; [ $rc -gt 1 ] && exit $rc; fi
done
echo done
