#!/bin/bash
# Round evidence, part A: the GPU suite and smoke, then PMC passes per workload (FETCH_SIZE,
# WRITE_SIZE, L2 fabric read requests by size -- each its own run) summarised with
# tools/pmc_summary.py into gpurun_out/$TAG/pmc_summary[_<workload>].json.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest -m gpu"; date
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
      > $OUT/pytest_gpu.txt 2>&1
  rc=$?; tail -2 $OUT/pytest_gpu.txt; stop $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
  rc=$?; tail -1 $OUT/smoke.txt; stop $rc smoke
fi
for W in ${WORKLOADS:-udp64 imix quic imix10m}; do
  case $W in
    udp64) ARGS="--steps 30 --warmup 3" ;;
    imix) ARGS="--workload imix --steps 2 --warmup 1" ;;
    quic) ARGS="--workload quic --steps 3 --warmup 1" ;;
    imix10m) ARGS="--workload imix10m --shard 0/8 --steps 1 --warmup 1" ;;
  esac
  for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
    N=$(echo $C | cut -d' ' -f1)
    echo "== pmc $W $N"; date
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$W/$N -o run -- \
        python3 bench.py $ARGS --no-cpu-baseline --no-e2e --no-two-engines > $OUT/pmc_${W}_$N.json 2> $OUT/pmc_${W}_$N.err
    rc=$?; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_${W}_$N.err; stop $rc "pmc $W $N"; }
  done
  S=pmc_summary_$W.json; [ $W = udp64 ] && S=pmc_summary.json
  python3 tools/pmc_summary.py $OUT/pmc_$W $OUT/$S $OUT/pmc_${W}_FETCH_SIZE.json || exit 1
done
echo "== done"; date
