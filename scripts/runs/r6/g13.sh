#!/bin/bash
# Round 6, call g13: deferred block-final BN apply written by the next bottleneck's conv1 GEMM (gemm_apply.hip) --
# kernel + model tests, then the driver bench interleaved x2 with DLA_DEFER_APPLY=0 / 1
set -o pipefail
O=gpurun_out/r6/g13
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_apply.py -x -v --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test.txt | head -20; tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_act.py tests/test_gpu_bench_batch.py tests/test_gpu_stem_bn_fused.py -x -q --timeout 200 --timeout-method thread > $O/test2.txt 2>&1 || { tail -30 $O/test2.txt; exit 1; }
tail -1 $O/test2.txt
for i in 1 2; do
  for d in 0 1; do
    DLA_DEFER_APPLY=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$d.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
  echo "round $i done"
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g13/b{k}.jsonl") if l.startswith("{")]
    print("defer", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v], [d["step_ms"]["p50"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
