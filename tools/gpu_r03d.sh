#!/bin/bash
# round 3: A/B of k_bin's narrow-walk head loads (IPXG_BIN_XPOSE: contiguous 1 KB loads +
# LDS transpose when a wave's frames are back to back) on udp64, with a parity check of the
# variant first.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03d
mkdir -p $OUT
stop() { case "$1" in 0|1) return 0 ;; *) echo "STOP: $2 exited $1"; exit "$1" ;; esac; }
IPXG_LIB=$PWD/ipfixprobe_amd/variants/xpose.so timeout -k 10 600 python -u -m pytest tests/test_gpu_semantics.py \
    -k "bench_size or stream_parity" -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_xpose.txt 2>&1
rc=$?; tail -3 $OUT/pytest_xpose.txt; stop $rc pytest
for rep in 1 2; do
  for v in default xpose xpose2 base2; do
    if [ $v = default ]; then L=""; else L="IPXG_LIB=$PWD/ipfixprobe_amd/variants/$v.so"; fi
    env $L timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e \
        > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err
    rc=$?; python3 -c "import json,sys; d=json.load(open('$OUT/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stage_ms_per_step'])"
    stop $rc "bench $v"
  done
done
echo "== done"
