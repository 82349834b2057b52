#!/bin/bash
# Round 6, call g15: the fused conv1 apply for K up to 2048 (stages 3-4; DLA_APPLY_MAX_K) -- tests, then the driver
# bench interleaved x2 with 512 (default) / 1024 / 2048
set -o pipefail
O=gpurun_out/r6/g15
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_apply.py -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test.txt | head -20; tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2; do
  for k in 512 2048 1024; do
    DLA_APPLY_MAX_K=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$k.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
  echo "round $i done"
done
python3 - <<'PY'
import json
for k in (512, 1024, 2048):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g15/b{k}.jsonl") if l.startswith("{")]
    print("max_k", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v], [d["step_ms"]["p50"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
