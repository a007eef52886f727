#!/bin/bash
# Build tuning variants of libipxg.so (compile-time knobs of ipxg_ingest.hip) into
# ipfixprobe_amd/variants/<name>.so; bench.py picks one with IPXG_LIB=<path>.
#   tools/variants.sh name "-DIPXG_BIN_K=4 -DIPXG_BIN_WAVES=5" [name2 "flags2" ...]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ipfixprobe_amd/variants"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  tmp=$(mktemp -d /tmp/ipxg_var_XXXX)
  mkdir -p "$tmp/ipfixprobe_amd" "$tmp/include"
  cp -r "$ROOT/ipfixprobe_amd/csrc" "$tmp/ipfixprobe_amd/"
  cp "$ROOT/include/ipxg.h" "$tmp/include/"
  rm -rf "$tmp/ipfixprobe_amd/csrc/build"
  make -s -C "$tmp/ipfixprobe_amd/csrc" -j8 OPT="-O3 $flags" > "$tmp/build.log" 2>&1 || { cat "$tmp/build.log"; exit 1; }
  cp "$tmp/ipfixprobe_amd/libipxg.so" "$ROOT/ipfixprobe_amd/variants/$name.so"
  rm -rf "$tmp"
  echo "built variants/$name.so ($flags)"
done
