#!/bin/bash
# Round 6, call g16: options measured neutral / slower before the deferred apply, re-measured on the new step:
# BN-backward partials in the streaming dgrad epilogue (DLA_BN_EPILOGUE=stream) and register-stored 128x128 tiles
# (DLA_GEMM_DIRECT=1); driver bench interleaved x3
set -o pipefail
O=gpurun_out/r6/g16
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/base.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_BN_EPILOGUE=stream timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/epi_stream.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_GEMM_DIRECT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/direct.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  echo "round $i done"
done
python3 - <<'PY'
import json
for k in ("base", "epi_stream", "direct"):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g16/{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
