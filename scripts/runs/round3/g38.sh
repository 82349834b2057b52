#!/bin/bash
# Round 3, call 38: the late 3x3 weight gradients on the other models: GoogLeNet bs128 (HIP graph) and
# bs512 eager, ResNet-152 bs256, ResNet-18 bs512; DLA_WGRAD_DEFER=0 vs 3x3, 2 rounds.
set -o pipefail
O=gpurun_out/g38; mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  for i in 1 2; do
    for d in 0 3x3; do
      DLA_WGRAD_DEFER=$d timeout -k 10 300 python3 bench.py "$@" > $O/${tag}_${d}_$i.log 2>&1 || { tail -20 $O/${tag}_${d}_$i.log; return 1; }
      echo "$tag defer=$d $(grep -o '"value": [0-9.]*' $O/${tag}_${d}_$i.log)" | tee -a $O/ab.txt
    done
  done
}
run gnet128g --model googlenet --batch 128 --graph on --steps 30 --warmup 10 || exit 1
run gnet512 --model googlenet --batch 512 --steps 20 --warmup 5 || exit 1
run r152 --model resnet152 --batch 256 --steps 15 --warmup 5 || exit 1
run r18 --model resnet18 --batch 512 --steps 20 --warmup 5 || exit 1
