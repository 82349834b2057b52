#!/bin/bash
# Round 6, call g10: tile shape vs write rate for the write-dominated stage-3 1x1 GEMMs (N = 1024): forced tiles
# 128x128 / 256x128 (8 waves) / 256x128w4 / 128x256w4 / 256x256, and the streaming kernel forced on
set -o pipefail
O=gpurun_out/r6/g10
mkdir -p $O
for s in "250880 64 1024 fwd" "250880 256 1024 fwd" "250880 256 1024 dgrad_add" "250880 256 1024 dgrad" "62720 512 2048 fwd"; do
  for tile in 1 4 5 6 8; do
    timeout -k 10 120 python3 scripts/gemm_stall.py $s 40 $tile >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
  done
  STALL_STREAM=1 timeout -k 10 120 python3 scripts/gemm_stall.py $s 40 0 | sed "s/^/stream=1 /" >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
done
grep ok $O/timing.txt
