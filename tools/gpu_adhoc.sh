set -u
mkdir -p gpurun_out/r02k
for W in imix quic; do
IPXG_LIB=ipfixprobe_amd/variants/probe.so timeout -k 10 300 python tools/probe_slow.py $W > gpurun_out/r02k/probe_$W.txt 2>&1 || { tail -5 gpurun_out/r02k/probe_$W.txt; exit 3; }
echo "== $W"; grep -v amdgpu.ids gpurun_out/r02k/probe_$W.txt
done
