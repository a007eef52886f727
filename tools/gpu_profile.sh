#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of bench.py per workload, then PMC
# passes (FETCH_SIZE / WRITE_SIZE, each its own run) for the HBM traffic of every kernel.
# Usage: TAG=r02 [WORKLOADS="udp64 imix quic"] [PMC=1] bash tools/gpu_profile.sh
# Every GPU step has its own time limit; a fault, abort or timeout stops the script there.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/prof_${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP: $1 exited $2"; exit "$2"; }
for W in ${WORKLOADS:-udp64 imix quic}; do
  case $W in
    udp64) ARGS="--steps 30 --warmup 3" ;;
    gather) ARGS="--gather --steps 30 --warmup 3" ;;
    stream) ARGS="--mode stream --steps 20 --warmup 3" ;;
    imix) ARGS="--workload imix --steps 3 --warmup 1" ;;
    quic) ARGS="--workload quic --steps 5 --warmup 1" ;;
    imix_plugins) ARGS="--workload imix --plugins dns,http,tls --steps 2 --warmup 1" ;;
    quic_plugins) ARGS="--workload quic --plugins quic --steps 3 --warmup 1" ;;
    imix10m) ARGS="--workload imix10m --shard 0/8 --steps 2 --warmup 1" ;;
  esac
  echo "== kernel trace $W"; date
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$W -o run -- \
      python3 bench.py $ARGS --no-cpu-baseline --no-e2e --no-two-engines > $OUT/kt_$W.json 2> $OUT/kt_$W.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/kt_$W.err; stop "kernel trace $W" $rc; }
  if [ "${PMC:-1}" = "1" ]; then
    # (each pass its own run: FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2; the fabric
    # read requests by size settle how many bytes FETCH_SIZE's requests moved)
    for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"; do
      N=$(echo $C | tr ' ' '_')
      echo "== pmc $W $N"; date
      timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$W/$N -o run -- \
          python3 bench.py $ARGS --no-cpu-baseline --no-e2e --no-two-engines > $OUT/pmc_${W}_$N.json 2> $OUT/pmc_${W}_$N.err
      rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_${W}_$N.err; stop "pmc $W $N" $rc; }
    done
  fi
done
echo "== done"; date
