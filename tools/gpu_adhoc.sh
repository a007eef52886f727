set -u
mkdir -p gpurun_out/r02f
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r02f/pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/r02f/pytest_gpu.txt; [ $rc -gt 1 ] && exit $rc
IPXG_LIB=ipfixprobe_amd/variants/probe.so timeout -k 10 300 python tools/probe_slow.py quic > gpurun_out/r02f/probe_slow.txt 2>&1 || { tail -5 gpurun_out/r02f/probe_slow.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r02f/probe_slow.txt | head -5
IPXG_LIB=ipfixprobe_amd/variants/probe.so timeout -k 10 300 python tools/probe_bin.py > gpurun_out/r02f/probe_bin.txt 2>&1 || { tail -5 gpurun_out/r02f/probe_bin.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r02f/probe_bin.txt
for W in quic imix; do
timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r02f/bench_$W.json 2> gpurun_out/r02f/bench_$W.err || exit $?
python -c "
import json; d=json.load(open('gpurun_out/r02f/bench_$W.json')); print('$W', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
