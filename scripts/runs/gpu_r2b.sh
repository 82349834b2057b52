#!/bin/bash
# Per-layer conv roofline benchmark + steady-state kernel profile of the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u scripts/bench_layers.py --out gpurun_out/layers_r2b.jsonl > gpurun_out/layers_r2b.log 2>&1 || { echo "layers rc=$?"; tail -30 gpurun_out/layers_r2b.log; exit 1; }
tail -16 gpurun_out/layers_r2b.log
bash scripts/gpu_bench_prof.sh r2b || { echo "prof rc=$?"; tail -20 gpurun_out/prof_r2b.log; exit 1; }
grep metric gpurun_out/bench_r2b.log
head -40 gpurun_out/ksum_r2b.md
