#!/bin/bash
# profile refresh after the 256x256 tiles at the new default (ResNet-50, per-GPU batch 1024):
# bench + kernel-trace summary, MFMA-busy counter pass, and the other models' bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r5g
bash scripts/gpu_bench_prof.sh r5g || { echo "bench/prof failed"; tail -20 gpurun_out/prof_r5g.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_r5g.log | cut -c1-200
cd $R && bash scripts/gpu_pmc_mfma.sh || { echo "pmc failed"; tail -20 gpurun_out/pmc_mfma.log; exit 1; }
cd $R
run() { tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 5 "$@" > gpurun_out/r5g/models_$tag.log 2>&1; rc=$?; echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5g/models_$tag.log | head -1)"; return $rc; }
run resnet50_b512 --batch 512 || exit $?
run googlenet128_graph --model googlenet --batch 128 --graph on || exit $?
run googlenet512 --model googlenet --batch 512 || exit $?
run resnet18 --model resnet18 --batch 512 || exit $?
run resnet34 --model resnet34 --batch 512 || exit $?
run resnet101 --model resnet101 --batch 256 || exit $?
run resnet152 --model resnet152 --batch 256 || exit $?
