#!/bin/bash
# Round 5, call g09: localise the fp32 GoogLeNet gradient difference (native vs stock fp32) op by op
set -o pipefail
O=gpurun_out/r5/g09
mkdir -p $O
timeout -k 10 200 python -u scripts/fp32_op_parity.py > $O/fp32_ops.jsonl 2> $O/fp32_ops.err || { tail $O/fp32_ops.err; exit 1; }
cat $O/fp32_ops.jsonl
