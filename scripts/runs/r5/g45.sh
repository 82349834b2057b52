#!/bin/bash
# Round 5, call g45: the other models on the final round-5 kernels (bf16 native path, one MI355X): ResNet-18/34/101/152,
# GoogLeNet (eager bs512, HIP graph bs128), and ResNet-152 at the BASELINE config #5 batch (1280)
set -o pipefail
O=gpurun_out/r5/g45
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
b() { run 400 python bench.py --steps 10 --warmup 4 "$@" >> $O/models.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }; }
b --model resnet18 --batch 512
b --model resnet34 --batch 512
b --model resnet101 --batch 256
b --model resnet152 --batch 256
b --model googlenet --batch 512
b --model googlenet --batch 128 --graph on
b --model resnet152 --batch 1280
python3 - <<'PY'
import json
for l in open("gpurun_out/r5/g45/models.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["model"], d["config"].get("per_gpu_batch"), d["config"].get("graph", ""), round(d["value"]), round(d["ms_per_step"], 2))
PY
