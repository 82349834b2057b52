#!/bin/bash
# Round 3, call 12: the persistent streaming 1x1 GEMM (csrc/kernels/gemm_stream.hip): numerics tests, the
# per-layer stream-vs-tile micro-benchmark at bs1024 shapes, end-to-end A/B (DLA_GEMM_STREAM=0 / 1).
set -o pipefail
O=gpurun_out/g12; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_stream.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u scripts/bench_gemm_stream.py --out $O/layers.jsonl > $O/layers.log 2>&1 || { tail -30 $O/layers.log; exit 1; }
cat $O/layers.jsonl
for i in 1 2; do
  for m in 0 1; do
    DLA_GEMM_STREAM=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_s${m}_$i.log 2>&1 || { tail -30 $O/bench_s${m}_$i.log; exit 1; }
    echo "stream=$m $(grep -o '"ms_per_step": [0-9.]*' $O/bench_s${m}_$i.log)" | tee -a $O/ab.txt
  done
done
