#!/bin/bash
# model-zoo bench lines on the final round-2 kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r5n
run() { tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 5 "$@" > gpurun_out/r5n/models_$tag.log 2>&1; rc=$?; echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5n/models_$tag.log | head -1)"; return $rc; }
run resnet18 --model resnet18 --batch 512 || exit $?
run resnet34 --model resnet34 --batch 512 || exit $?
run resnet50_b512 --batch 512 || exit $?
run resnet101 --model resnet101 --batch 256 || exit $?
run resnet152 --model resnet152 --batch 256 || exit $?
run googlenet128_graph --model googlenet --batch 128 --graph on || exit $?
run googlenet512 --model googlenet --batch 512 || exit $?
