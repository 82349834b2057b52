#!/bin/bash
# auto 256x256 tiles for compute-bound shapes: full GPU suite, then interleaved whole-step A/B
# (DLA_TILE256=0 vs default), HIP-graph and batch-1024 probes
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5b/full_gpu.log 2>&1 || { echo "GPU suite failed"; tail -40 gpurun_out/r5b/full_gpu.log; exit 1; }
tail -2 gpurun_out/r5b/full_gpu.log
for i in 1 2; do
  for t in 1 0; do
    DLA_TILE256=$t timeout -k 10 300 python bench.py > gpurun_out/r5b/bench_t${t}_${i}.log 2>&1 || { tail -20 gpurun_out/r5b/bench_t${t}_${i}.log; exit 1; }
    echo "tile256=$t $(grep -o '"value": [0-9.]*' gpurun_out/r5b/bench_t${t}_${i}.log)" | tee -a gpurun_out/r5b/ab.txt
  done
done
timeout -k 10 300 python bench.py --graph on > gpurun_out/r5b/bench_graph.log 2>&1 && echo "graph $(grep -o '"value": [0-9.]*' gpurun_out/r5b/bench_graph.log)" | tee -a gpurun_out/r5b/ab.txt
timeout -k 10 300 python bench.py --batch 1024 --steps 20 > gpurun_out/r5b/bench_b1024.log 2>&1 && echo "b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r5b/bench_b1024.log)" | tee -a gpurun_out/r5b/ab.txt
