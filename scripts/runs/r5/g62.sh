#!/bin/bash
# Round 5, call g62: BN reduction-pass block target (DLA_BN_RED_BLOCKS) re-checked after the last-to-first BN order:
# step A/B 512 / 1024 (default) / 2048, interleaved x2
set -o pipefail
O=gpurun_out/r5/g62
mkdir -p $O
for i in 1 2; do
  for b in 512 1024 2048; do
    DLA_BN_RED_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$b.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
  echo "round $i done"
done
python3 - <<'PY'
import json
for b in (512, 1024, 2048):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g62/b{b}.jsonl") if l.startswith("{")]
    print(b, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
PY
