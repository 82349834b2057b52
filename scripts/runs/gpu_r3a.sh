#!/bin/bash
# other configs: GoogLeNet with torch autocast (fp32 master weights, bf16 autocast), ResNet-152
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 --precision autocast > gpurun_out/r3a_gnet_autocast.log 2>&1 && grep metric gpurun_out/r3a_gnet_autocast.log | cut -c1-250 || tail -20 gpurun_out/r3a_gnet_autocast.log
timeout -k 10 300 python bench.py --model resnet152 --batch 256 --steps 10 --warmup 5 > gpurun_out/r3a_r152.log 2>&1 && grep metric gpurun_out/r3a_r152.log | cut -c1-250 || tail -20 gpurun_out/r3a_r152.log
timeout -k 10 300 python bench.py --model resnet101 --batch 256 --steps 10 --warmup 5 > gpurun_out/r3a_r101.log 2>&1 && grep metric gpurun_out/r3a_r101.log | cut -c1-250 || tail -20 gpurun_out/r3a_r101.log
