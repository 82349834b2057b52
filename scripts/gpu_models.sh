#!/bin/bash
# bench.py across the model zoo on one GPU (each run under its own time limit; stop at the first crash)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$R/miopen_db
run() { tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 5 "$@" > gpurun_out/models_$tag.log 2>&1; rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/models_$tag.log; return $rc; }
run googlenet128 --model googlenet --batch 128 || exit $?
run googlenet256 --model googlenet --batch 256 || exit $?
run resnet152 --model resnet152 --batch 256 || exit $?
run resnet18 --model resnet18 --batch 256 || exit $?
run resnet50_graph --graph on || exit $?
run resnet50_torch --kernels torch --precision autocast --conv miopen || exit $?
