#!/bin/bash
# Round 5, call g60: K = 256 data gradients with the fused identity addend on the streaming kernel (one block per
# CU): GEMM GPU tests, then same-box step A/B against DLA_STREAM_ADD256=0, interleaved x3
set -o pipefail
O=gpurun_out/r5/g60
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_stream.py tests/test_gpu_gemm.py tests/test_gpu_bn_epilogue.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  DLA_STREAM_ADD256=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/off.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/on.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  echo "pair $i done"
done
python3 - <<'PY'
import json
for k in ("off", "on"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g60/{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v], [d.get("telemetry", {}).get("after_timed", {}).get("gfxclk_mhz") for d in v])
PY
