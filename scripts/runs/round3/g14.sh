#!/bin/bash
# Round 3, call 14: tr_frag without the per-read v_bfi (every k-major MFMA operand read now waits with a
# counted lgkmcnt instead of right behind the read) + the halo weight gradient's 2-step fragment pipeline:
# the GEMM / conv / halo numerics tests, the halo micro-bench, end-to-end bench x2 and a kernel profile.
set -o pipefail
O=gpurun_out/g14; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo_wgrad.py tests/test_gpu_gemm.py tests/test_gpu_gemm_stream.py tests/test_gpu_conv3x3.py tests/test_gpu_conv.py tests/test_gpu_conv3x3_autograd.py tests/test_gpu_stem.py tests/test_gpu_linear.py tests/test_gpu_bn_epilogue.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python -u scripts/bench_halo_wgrad.py > $O/halo_wgrad.log 2>&1 || { tail -20 $O/halo_wgrad.log; exit 1; }
grep '^{' $O/halo_wgrad.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || { tail -30 $O/bench_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log | tee -a $O/ab.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g14prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
T=$(find /tmp/g14prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
S=$(find /tmp/g14prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
head -40 $O/ksum.md
