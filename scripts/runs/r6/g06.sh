#!/bin/bash
# Round 6, call g06: fp32 conv main loop, double vs single LDS buffer, per layer vs MIOpen; fp32 GoogLeNet line
set -o pipefail
O=gpurun_out/r6/g06
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_f32.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 500 python -u scripts/bench_conv_f32.py --out $O/layers.jsonl > $O/layers.log 2>&1 || { tail -20 $O/layers.log; exit 1; }
tail -1 $O/layers.log
timeout -k 10 300 python bench.py --model googlenet --precision fp32 --batch 128 --steps 20 --warmup 5 > $O/gnet_fp32.jsonl 2> $O/gnet.err || { tail $O/gnet.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gnet_fp32.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['conv1x1'])"
