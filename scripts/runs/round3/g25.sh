#!/bin/bash
# Round 3, call 25: uninitialised-memory probe (NaN-filled allocations) of the native training step,
# ResNet-18 / ResNet-50, with the late weight gradients off and on.
set -o pipefail
O=gpurun_out/g25; mkdir -p $O
for m in resnet18 resnet50; do
  for d in 0 3x3; do
    DLA_WGRAD_DEFER=$d timeout -k 10 120 python3 scripts/uninit_probe.py --model $m > $O/${m}_$d.log 2>&1 || { tail -20 $O/${m}_$d.log; exit 1; }
    echo "== $m defer=$d"; grep -v Warning $O/${m}_$d.log | grep -E "step|RESULT"
  done
done
