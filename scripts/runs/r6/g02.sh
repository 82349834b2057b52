#!/bin/bash
# Round 6, call g02: how much of the 128x128 1x1 GEMM is epilogue -- the l3.conv3 shape (M 250880, N 1024) at
# K = 64 / 128 / 256 with and without the statistics epilogue, forced 128x128 tile (TileCfg 1)
set -o pipefail
O=gpurun_out/r6/g02
mkdir -p $O
for K in 64 128 256 512; do
  for kind in fwd fwdns dgrad_add dgrad; do
    timeout -k 10 120 python3 scripts/gemm_stall.py 250880 $K 1024 $kind 40 1 >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
  done
done
grep ok $O/timing.txt
