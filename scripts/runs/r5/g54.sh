#!/bin/bash
# Round 5, call g54: 512x128 conv tile for the Cout-128 3x3 passes (then opt-in): conv GPU tests, stage-2 timing vs 128x128, step A/B
set -o pipefail
O=gpurun_out/r5/g54
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_tile_policy.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/probe_tile512.py > $O/probe.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
cat $O/probe.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/off.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_TILE512=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/on.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  echo "pair $i done"
done
python3 - <<'PY'
import json
for k in ("off", "on"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g54/{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
PY
