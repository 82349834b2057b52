#!/bin/bash
# per-GPU cost of the N>1 gradient path at the bs1024 default: forced 1-rank collective (gather ->
# fp32 staging -> RCCL all-reduce on the comm stream -> cast back) vs the N=1 pass-through, interleaved
set -o pipefail
mkdir -p gpurun_out/r5p
for i in 1 2; do
  for f in 1 0; do
    timeout -k 10 300 python bench.py --force_comm $f > gpurun_out/r5p/bench_fc${f}_$i.log 2>&1 || { tail -20 gpurun_out/r5p/bench_fc${f}_$i.log; exit 1; }
    echo "force_comm=$f $(grep -o '"value": [0-9.]*' gpurun_out/r5p/bench_fc${f}_$i.log | head -1) $(grep -o '"allreduce_ms_per_step": [0-9.]*' gpurun_out/r5p/bench_fc${f}_$i.log)" | tee -a gpurun_out/r5p/ab.txt
  done
done
