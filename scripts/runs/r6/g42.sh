#!/bin/bash
# Round 6, call g42: the 256x256 statistics-forward threshold (DLA_TILE256_MIN_K_STATS) re-checked on the final step
set -o pipefail
O=gpurun_out/r6/g42
mkdir -p $O
for i in 1 2 3; do
  for k in 256 512 1024; do
    DLA_TILE256_MIN_K_STATS=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$k.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (256, 512, 1024):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g42/b{k}.jsonl") if l.startswith("{")]
    print("min_k_stats", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
