#!/bin/bash
# Round 6, call g25: the stem forward on the persistent streaming GEMM (DLA_STEM_STREAM) -- tests, driver bench
# interleaved x3
set -o pipefail
O=gpurun_out/r6/g25
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem_stream.py tests/test_gpu_gemm_stream.py -x -v --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test.txt | head -20; tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
DLA_STEM_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_stem_bn_fused.py tests/test_gpu_bench_batch.py -x -q --timeout 200 --timeout-method thread > $O/test2.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test2.txt | head -20; tail -30 $O/test2.txt; exit 1; }
tail -1 $O/test2.txt
for i in 1 2 3; do
  for m in 0 1; do
    DLA_STEM_STREAM=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$m.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g25/b{k}.jsonl") if l.startswith("{")]
    print("stem_stream", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
