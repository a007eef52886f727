set -u
TAG=r02i STAGES="test bench" BENCHES="udp64 imix quic" bash tools/gpu_round.sh || exit $?
IPXG_LIB=ipfixprobe_amd/variants/probe.so timeout -k 10 300 python tools/probe_slow.py quic > gpurun_out/r02i/probe_slow.txt 2>&1 || { tail -5 gpurun_out/r02i/probe_slow.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r02i/probe_slow.txt | head -5
