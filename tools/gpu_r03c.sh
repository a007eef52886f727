#!/bin/bash
# round 3, profiles: rocprofv3 kernel-trace statistics per workload, and per workload the PMC
# passes FETCH_SIZE, WRITE_SIZE and the L2->fabric read requests split by size
# (TCC_EA0_RDREQ_32B/64B/128B: settles how many bytes FETCH_SIZE's requests carry).
# Each pass its own run, kernel trace only (no --sys-trace with --pmc).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p $OUT
stop() { echo "STOP: $1 exited $2"; exit "$2"; }
for W in ${WORKLOADS:-udp64 quic imix}; do
  case $W in
    udp64) ARGS="--steps 30 --warmup 3" ;;
    quic) ARGS="--workload quic --steps 5 --warmup 1" ;;
    imix) ARGS="--workload imix --steps 3 --warmup 1" ;;
  esac
  echo "== kernel trace $W"; date
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$W -o run -- \
      python3 bench.py $ARGS --no-cpu-baseline --no-e2e > $OUT/kt_$W.json 2> $OUT/kt_$W.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/kt_$W.err; stop "kernel trace $W" $rc; }
  for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"; do
    N=$(echo $C | tr ' ' '_')
    echo "== pmc $W $N"; date
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$W/$N -o run -- \
        python3 bench.py $ARGS --no-cpu-baseline --no-e2e > $OUT/pmc_${W}_$N.json 2> $OUT/pmc_${W}_$N.err
    rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_${W}_$N.err; stop "pmc $W $N" $rc; }
  done
done
echo "== done"; date
