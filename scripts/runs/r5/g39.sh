#!/bin/bash
# Round 5, call g39: same-box A/B of the dual-kernel swizzle (new default vs DLA_DUAL_SWZ=1 variant), interleaved x4
set -o pipefail
O=gpurun_out/r5/g39
mkdir -p $O
V=$(pwd)/variants/_C_swz1.so
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/new.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_EXT_SO=$V DLA_ALLOW_STALE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
for k in ("new", "old"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g39/{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
PY
