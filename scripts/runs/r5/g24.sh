#!/bin/bash
# Round 5, call g24: main-loop pipeline sweep of the register-staged 1x1 GEMM shapes (K <= 512, stages 2-4)
set -o pipefail
O=gpurun_out/r5/g24
mkdir -p $O
cd scripts && timeout -k 10 400 python -u bench_gemm_pipes.py > ../$O/pipes.jsonl 2> ../$O/err.log || { tail ../$O/err.log; exit 1; }
cd .. && cut -c1-400 $O/pipes.jsonl
