#!/bin/bash
# Round 6, call g18: the other models on the final kernels (deferred block-final apply on), one box
set -o pipefail
O=gpurun_out/r6/g18
mkdir -p $O
export MIOPEN_USER_DB_PATH=$(pwd)/miopen_db
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.jsonl').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['config'].get('global_batch'), d['telemetry']['before_timed']['gfxclk_mhz'])"
}
run resnet18_bs512 --model resnet18 --batch 512
run resnet34_bs512 --model resnet34 --batch 512
run resnet101_bs256 --model resnet101 --batch 256
run resnet152_bs256 --model resnet152 --batch 256
run resnet152_bs1280 --model resnet152 --batch 1280
run googlenet_bs512 --model googlenet --batch 512
run googlenet_bs128_graph --model googlenet --batch 128 --graph on
run resnet50_bs1280 --model resnet50 --batch 1280
