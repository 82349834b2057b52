#!/bin/bash
# Round 4, call g05: auto 256x256 tiles from K = 256 (was K >= 1024) and the stem forward on the streaming
# kernel -- GEMM / stem tests, then interleaved A/B (new / old tile threshold / stem on the tile kernel) x2
set -o pipefail
O=gpurun_out/g05
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm_stream.py tests/test_gpu_stem.py \
  > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_new.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_tile256_min_k(1024)" bench.py --steps 15 --warmup 5 >> $O/ab_k1024.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_stem_stream(0)" bench.py --steps 15 --warmup 5 >> $O/ab_stem_tile.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 400 rocprofv3 --kernel-trace -d $O/prof -o trace -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 1
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 5 --out $O/ksum > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 5 --out $O/timeline.md > /dev/null || exit 1
