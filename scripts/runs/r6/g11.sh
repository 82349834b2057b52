#!/bin/bash
# Round 6, call g11: 256x256 tiles for the statistics forwards from K = 256 / 512 (DLA_TILE256_MIN_K_STATS) -- GEMM and
# batch tests under the new policy, then the driver bench interleaved x3 (default 1024 / 512 / 256)
set -o pipefail
O=gpurun_out/r6/g11
mkdir -p $O
DLA_TILE256_MIN_K_STATS=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bench_batch.py tests/test_gpu_bn_epilogue.py -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2 3; do
  for k in 1024 256 512; do
    DLA_TILE256_MIN_K_STATS=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$k.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
  echo "round $i done"
done
python3 - <<'PY'
import json
for k in (1024, 512, 256):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g11/b{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v], [d["step_ms"]["p50"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
