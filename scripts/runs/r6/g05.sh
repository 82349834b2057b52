#!/bin/bash
# Round 6, call g05: fp32 MFMA convolutions (conv_f32.hip) -- numerics vs float64, per-layer time vs MIOpen at the
# GoogLeNet bs128 shapes, then the fp32 GoogLeNet bench line (native convs) and the fp32 path test
set -o pipefail
O=gpurun_out/r6/g05
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_f32.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 400 python -u scripts/bench_conv_f32.py --out $O/layers.jsonl > $O/layers.log 2>&1 || { tail -20 $O/layers.log; exit 1; }
tail -1 $O/layers.log
timeout -k 10 300 python bench.py --model googlenet --precision fp32 --batch 128 --steps 20 --warmup 5 > $O/gnet_fp32.jsonl 2> $O/gnet.err || { tail $O/gnet.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gnet_fp32.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['conv1x1'], d['vs_baseline'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32_path.py -x -q --timeout 300 --timeout-method thread > $O/fp32_path.txt 2>&1 || { tail -30 $O/fp32_path.txt; exit 1; }
tail -2 $O/fp32_path.txt
