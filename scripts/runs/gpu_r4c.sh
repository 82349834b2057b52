#!/bin/bash
# other models on the current code: ResNet-101/152 (bs256), ResNet-18/34 (bs512), GoogLeNet autocast, ResNet-50 bs128 graph
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4c_records.jsonl
run() { timeout -k 10 300 python bench.py "$@" > gpurun_out/r4c.log 2>&1 && grep metric gpurun_out/r4c.log >> gpurun_out/r4c_records.jsonl && echo "$* -> $(grep -o '"value": [0-9.]*' gpurun_out/r4c.log | head -1)" || { echo "FAILED $*"; tail -5 gpurun_out/r4c.log; }; }
run --model resnet152 --batch 256 --steps 10 --warmup 5
run --model resnet101 --batch 256 --steps 10 --warmup 5
run --model resnet18 --batch 512 --steps 20 --warmup 5
run --model resnet34 --batch 512 --steps 20 --warmup 5
run --model googlenet --batch 128 --steps 20 --warmup 5 --precision autocast
run --batch 128 --graph on --steps 30 --warmup 10
