#!/bin/bash
# Round 5, call g44: stem forward main-loop pipeline A/B (0 / 2 / 3 / 4 / 5) on the stem op alone, x2 each
set -o pipefail
O=gpurun_out/r5/g44
mkdir -p $O
for i in 1 2; do
  for p in 2 3 4 5 0; do
    timeout -k 10 200 python -u scripts/ab_call.py "set_mfma_pipeline($p)" scripts/bench_stem.py >> $O/p$p.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
for p in 2 3 4 5 0; do echo "pipe $p: $(grep -o '"fwd_ms": [0-9.]*' $O/p$p.jsonl | tr '\n' ' ')"; done
