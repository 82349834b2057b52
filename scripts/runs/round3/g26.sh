#!/bin/bash
# Round 3, call 26: localise the uninitialised-memory dependence of the ResNet-18 native step to a block.
set -o pipefail
O=gpurun_out/g26; mkdir -p $O
timeout -k 10 120 python3 scripts/uninit_blocks.py --model resnet18 > $O/r18.log 2>&1 || { tail -20 $O/r18.log; exit 1; }
grep -v Warn $O/r18.log | grep "^layer"
