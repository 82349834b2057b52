#!/bin/bash
set -o pipefail
O=gpurun_out/g27; mkdir -p $O
timeout -k 10 120 python3 scripts/uninit_ops.py > $O/ops.log 2>&1 || { tail -20 $O/ops.log; exit 1; }
grep -v Warn $O/ops.log | grep -E "s2|1x1|gemm_nt"
