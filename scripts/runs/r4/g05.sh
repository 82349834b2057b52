#!/bin/bash
# Round 4, call g05: auto 256x256 tiles from K = 256 (was K >= 1024) -- GEMM tests, then interleaved A/B x3
set -o pipefail
O=gpurun_out/g05
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm_stream.py \
  > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_k256.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_tile256_min_k(1024)" bench.py --steps 15 --warmup 5 >> $O/ab_k1024.jsonl 2>> $O/ab.err || exit 1
done
