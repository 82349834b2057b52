#!/bin/bash
# cost of the N>1 gradient data path on one GPU: forced 1-rank collectives (fp32 staging, bucketed
# ncclAllReduce on the comm stream, overlapped with backward) vs the N=1 pass-through
set -o pipefail
mkdir -p gpurun_out
for f in 0 1 0 1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --force_comm $f > gpurun_out/r3e.log 2>&1 && echo "force_comm=$f $(grep -o '"value": [0-9.]*\|"allreduce_ms_per_step": [0-9.]*' gpurun_out/r3e.log | tr '\n' ' ')"
done
