#!/bin/bash
# Round 6 A/B of the streamed reduce (IPXG_STREAM=1: k_reduce_stream beside k_bin) against the
# default (k_reduce after k_bin), udp64, one box; the knobs of ipxg_engine.cpp: IPXG_STREAM_GRID,
# IPXG_PROG_MODE (1 sc1 record stores, 2 per-tile publish), IPXG_PUB_EVERY, IPXG_RS_SLEEP,
# IPXG_RS_EXP (1 no fold, 2 no record loads: timing only), IPXG_RS_LOWPRI.  Summaries:
# python3 tools/bline.py gpurun_out/<TAG>/*.json  (profiles/r06/stream_ab.txt)
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-stream_ab}; mkdir -p $O
B="python -u bench.py --steps 200 --no-cpu-baseline --no-e2e"
timeout -k 10 100 $B > $O/ns.json 2>/dev/null
IPXG_STREAM=1 timeout -k 10 100 $B --verify > $O/stream.json 2>/dev/null
for m in 0 1 2 3; do IPXG_STREAM=1 IPXG_STREAM_GRID=768 IPXG_PROG_MODE=$m timeout -k 10 100 $B > $O/g768_m$m.json 2>/dev/null; done
for pe in 1 2 8; do IPXG_STREAM=1 IPXG_PUB_EVERY=$pe timeout -k 10 100 $B > $O/pe$pe.json 2>/dev/null; done
for sl in 1 16 64; do IPXG_STREAM=1 IPXG_RS_SLEEP=$sl timeout -k 10 100 $B > $O/sl$sl.json 2>/dev/null; done
for x in 1 2; do IPXG_STREAM=1 IPXG_RS_EXP=$x timeout -k 10 100 $B > $O/x$x.json 2>/dev/null; done
IPXG_STREAM=1 IPXG_RS_LOWPRI=1 timeout -k 10 100 $B > $O/lowpri.json 2>/dev/null
IPXG_BIN_GRID=512 timeout -k 10 100 $B > $O/ns512.json 2>/dev/null
