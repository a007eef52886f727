set -u
mkdir -p gpurun_out/r02n
timeout -k 10 400 python -u -m pytest tests/test_strict.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02n/pytest_strict.txt 2>&1; rc=$?; tail -3 gpurun_out/r02n/pytest_strict.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --strict 17 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify > gpurun_out/r02n/bench_strict.json 2> gpurun_out/r02n/bench_strict.err || { tail -3 gpurun_out/r02n/bench_strict.err; exit 3; }
python -c "
import json; d=json.load(open('gpurun_out/r02n/bench_strict.json')); print(d['value'], d['ms_per_step'], d['verify'], d['strict'])"
