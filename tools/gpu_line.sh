set -u
mkdir -p gpurun_out/r5l
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_semantics.py tests/test_gpu_ahead.py tests/test_gpu_async.py > gpurun_out/r5l/pytest.txt 2>&1 || { tail -30 gpurun_out/r5l/pytest.txt; exit 1; }
tail -2 gpurun_out/r5l/pytest.txt
for v in base noline lnt ct0; do
  case $v in
    base) E=""; L="";;
    noline) E="IPXG_NO_LINE=1"; L="";;
    lnt) E=""; L=ipfixprobe_amd/variants/lnt.so;;
    ct0) E=""; L=ipfixprobe_amd/variants/ct0.so;;
  esac
  env $E IPXG_TUNING=1 IPXG_LIB=$L timeout -k 10 200 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/r5l/udp64_$v.json 2> gpurun_out/r5l/udp64_$v.err || { tail -5 gpurun_out/r5l/udp64_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" gpurun_out/r5l/udp64_$v.json $v
done
