#!/bin/bash
# Round 6, call g20: stride-2 subsample written by the fused conv1 apply (DLA_APPLY_SUBSAMPLE) -- driver bench
# interleaved x3
set -o pipefail
O=gpurun_out/r6/g20
mkdir -p $O
for i in 1 2 3; do
  for m in 0 1; do
    DLA_APPLY_SUBSAMPLE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$m.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g20/b{k}.jsonl") if l.startswith("{")]
    print("sub", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
