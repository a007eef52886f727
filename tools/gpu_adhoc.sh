set -u
O=gpurun_out/r02nt2
mkdir -p $O
for rep in 1 2; do
for lib in default aux0; do
  if [ $lib = default ]; then unset IPXG_LIB; else export IPXG_LIB=$PWD/ipfixprobe_amd/variants/$lib.so IPXG_TUNING=1; fi
  timeout -k 10 300 python bench.py --steps 300 --warmup 3 --no-cpu-baseline --no-e2e > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err || { tail -3 $O/${lib}_$rep.err; exit 3; }
  python -c "
import json; d=json.load(open('$O/${lib}_$rep.json')); print('$lib', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
done
