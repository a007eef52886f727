#!/bin/bash
# LDS op throughput table (tools/ldsbench): every op at 390 entries (a udp64 k_reduce partition's
# flows) and 2048 (the whole table)
cd "$(dirname "$0")"
for n in 390 2048; do for op in 0 1 2 3 4 5 6 7 8 9 10 11 12 13; do timeout -k 5 60 ./ldsbench $op 4096 $n || exit 1; done; done
