#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/vrank_ring_timing.py --world 8 --channels 7 --graph --out gpurun_out/vrank_ring_pipe_graph_c7.jsonl > gpurun_out/r2n_c7.log 2>&1 && cat gpurun_out/r2n_c7.log || { tail -30 gpurun_out/r2n_c7.log; exit 1; }
timeout -k 10 300 python scripts/vrank_ring_timing.py --world 8 --channels 1 --graph --out gpurun_out/vrank_ring_pipe_graph_c1.jsonl > gpurun_out/r2n_c1.log 2>&1 && cat gpurun_out/r2n_c1.log
