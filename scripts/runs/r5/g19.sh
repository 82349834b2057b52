#!/bin/bash
# Round 5, call g19: in-step A/B of the smallest K for the auto 256x256 GEMM / conv tiles (default 1024 vs 512
# vs 256), interleaved x3 on one box, at the shipped bs1280 step
set -o pipefail
O=gpurun_out/r5/g19
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
for i in 1 2 3; do
  for k in 1024 512 256; do
    run 240 python -u scripts/ab_call.py "set_tile256_min_k($k)" bench.py --steps 15 --warmup 5 >> $O/k$k.jsonl 2>> $O/err.log \
      || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (1024, 512, 256):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g19/k{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
PY
