#!/bin/bash
# round-3 first GPU pass: GPU parity tests, then the stall/issue counters of k_bin / k_reduce
#  on udp64.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.txt
[ $rc -gt 1 ] && { echo "STOP pytest rc=$rc"; exit $rc; }
timeout -k 10 120 rocprofv3 -L > $OUT/pmc_list.txt 2>&1 || true
TAG=r03a SETS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR;TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum;FETCH_SIZE;WRITE_SIZE" bash tools/gpu_pmc.sh
