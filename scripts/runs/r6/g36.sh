#!/bin/bash
# Round 6, call g36: 256x256 statistics forwards stored from registers (DLA_GEMM256_DIRECT) -- tests,
# driver bench interleaved x3 against the staged epilogue
set -o pipefail
O=gpurun_out/r6/g36
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm256_direct.py tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2 3; do
  for v in 0 1; do
    DLA_GEMM256_DIRECT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$v.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g36/b{k}.jsonl") if l.startswith("{")]
    print("gemm256_direct", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
