#!/bin/bash
# Round 5, call g59: 512x128 vs 128x128 at smaller batches (Cout-128 3x3 at 28x28): where the auto threshold belongs
set -o pipefail
O=gpurun_out/r5/g59
mkdir -p $O
for n in 256 512 768; do
  PROBE_N=$n timeout -k 10 150 python -u scripts/probe_tile512.py | sed "s/^{/{\"N\": $n, /" >> $O/probe.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
cat $O/probe.jsonl
