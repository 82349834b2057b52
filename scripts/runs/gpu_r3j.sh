#!/bin/bash
# record: ResNet-50 default bench x3, GoogLeNet bs128 graph / bs512 eager, ResNet-50 graph
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3j_records.jsonl
for i in 1 2 3; do timeout -k 10 300 python bench.py > gpurun_out/r3j.log 2>&1 && grep metric gpurun_out/r3j.log >> gpurun_out/r3j_records.jsonl; done
timeout -k 10 300 python bench.py --graph on > gpurun_out/r3j.log 2>&1 && grep metric gpurun_out/r3j.log >> gpurun_out/r3j_records.jsonl
timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on > gpurun_out/r3j.log 2>&1 && grep metric gpurun_out/r3j.log >> gpurun_out/r3j_records.jsonl
timeout -k 10 300 python bench.py --model googlenet --batch 512 > gpurun_out/r3j.log 2>&1 && grep metric gpurun_out/r3j.log >> gpurun_out/r3j_records.jsonl
python3 -c "
import json
for l in open('gpurun_out/r3j_records.jsonl'):
    d=json.loads(l); print(d['config']['model'], d['config']['per_gpu_batch'], 'graph' if d['config']['hip_graph'] else 'eager', d['value'], d['ms_per_step'])
"
