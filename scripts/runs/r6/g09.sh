#!/bin/bash
# Round 6, call g09: persistent register-stored 1x1 GEMM tiles (gemm_direct.hip gemm_direct_persist_kernel) -- numerics,
# per-shape timing staged / direct / persistent (2, 3 blocks per CU; register-staged and buffer-DMA main loops)
set -o pipefail
O=gpurun_out/r6/g09
mkdir -p $O
DLA_GEMM_PERSIST=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_direct.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
SH=("250880 256 1024 fwd" "250880 256 1024 dgrad_add" "62720 512 2048 fwd" "62720 512 2048 dgrad_add" "1003520 256 512 fwd" "250880 512 1024 fwd" "1003520 512 256 fwd" "1003520 512 128 dgrad_add")
for s in "${SH[@]}"; do
  for v in "0 0 -1" "1 0 -1" "1 2 -1" "1 3 -1" "1 2 6" "1 0 6"; do
    set -- $v
    DLA_GEMM_DIRECT=$1 DLA_GEMM_PERSIST=$2 STALL_PIPE=$3 timeout -k 10 120 python3 scripts/gemm_stall.py $s 40 | sed "s/^/direct=$1 persist=$2 pipe=$3 /" >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
  done
done
grep ok $O/timing.txt
