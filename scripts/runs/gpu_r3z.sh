#!/bin/bash
# fused fan-in: inception unit tests (incl. strided grouped BN) + GoogLeNet bs128 graph profile + records
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inception.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3z_tests.log | head -20; tail -20 gpurun_out/r3z_tests.log; exit 1; }
tail -1 gpurun_out/r3z_tests.log
bash scripts/gpu_bench_prof.sh r3z_gnet --model googlenet --batch 128 --graph on || exit 1
grep -E "GPU wall" gpurun_out/ksum_r3z_gnet.md | head -2
grep metric gpurun_out/bench_r3z_gnet.log >> gpurun_out/r3z_records.jsonl
timeout -k 10 300 python bench.py --model googlenet --batch 512 > gpurun_out/r3z_g512.log 2>&1 && grep metric gpurun_out/r3z_g512.log >> gpurun_out/r3z_records.jsonl
cut -c1-160 gpurun_out/r3z_records.jsonl
