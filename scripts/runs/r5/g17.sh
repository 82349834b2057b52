#!/bin/bash
# Round 5, call g17: the 64-channel halo 3x3 conv (fwd + dgrad) with its 18 fragment steps software-pipelined
# (next step's LDS reads issued before this step's MFMAs) -- numerics, per-shape timing, a step A/B needs none
set -o pipefail
O=gpurun_out/r5/g17
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_conv3x3_autograd.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_tiles.jsonl 2> $O/conv_tiles.err || { tail $O/conv_tiles.err; exit 1; }
cut -c1-300 $O/conv_tiles.jsonl
run 200 python -u bench.py --steps 15 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-200 $O/bench.jsonl
