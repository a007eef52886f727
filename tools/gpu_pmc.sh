#!/bin/bash
# PMC passes for the bench's dominant kernel (each counter group in its own run, kernel
# trace only -- MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; TAG=${TAG:-r01}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/pmc_list_$TAG.txt 2>&1 || true
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"; do
  N=$(echo $C | tr ' ' '_')
  echo "== pmc $C"; date
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$TAG/$N -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_${TAG}_$N.json 2> $OUT/pmc_${TAG}_$N.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $C exited $rc"; tail -3 $OUT/pmc_${TAG}_$N.err; [ $rc -gt 1 ] && exit $rc; fi
done
echo done
