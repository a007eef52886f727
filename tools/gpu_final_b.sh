#!/bin/bash
# Round evidence, part B: rocprofv3 kernel-trace statistics per workload (tools/gpu_profile.sh,
# no PMC), then one bench line per workload (tools/gpu_round.sh) -- the lines read the PMC
# summaries part A left in profiles/<round>/.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-final} PMC=0 WORKLOADS="${PROF_WORKLOADS:-udp64 imix quic imix_plugins quic_plugins imix10m}" \
    bash tools/gpu_profile.sh || exit $?
TAG=${TAG:-final} STAGES=bench bash tools/gpu_round.sh
