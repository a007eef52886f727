set -u
export TMPDIR=/tmp
O=gpurun_out/r02nt
mkdir -p $O
for lib in default aux0; do
  if [ $lib = default ]; then unset IPXG_LIB; else export IPXG_LIB=$PWD/ipfixprobe_amd/variants/$lib.so; fi
  for W in imix quic; do
    A="--workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
    timeout -k 10 300 python bench.py $A > $O/${lib}_$W.json 2> $O/${lib}_$W.err || { tail -3 $O/${lib}_$W.err; exit 3; }
    python -c "
import json; d=json.load(open('$O/${lib}_$W.json')); print('$lib $W', d['value'], d['stage_ms_per_step'])"
    timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_${lib}_$W/FETCH_SIZE -o run -- \
        python3 bench.py $A > /dev/null 2> $O/pmc_${lib}_$W.err || { tail -3 $O/pmc_${lib}_$W.err; exit 4; }
    python tools/pmc_summary.py $O/pmc_${lib}_$W | grep k_bin
  done
done
