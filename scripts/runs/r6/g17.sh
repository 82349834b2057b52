#!/bin/bash
# Round 6, call g17: 128x256 weight-gradient tiles for the Cout-128 3x3 convs (DLA_WGRAD_W4) -- tests, isolated
# timing at the stage-2 bs1280 shapes, driver bench interleaved x2
set -o pipefail
O=gpurun_out/r6/g17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test.txt | head -20; tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 300 python scripts/wgrad_w4_ab.py > $O/timing.jsonl 2> $O/timing.err || { tail $O/timing.err; exit 1; }
cat $O/timing.jsonl
for i in 1 2; do
  for m in 0 1; do
    DLA_WGRAD_W4=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$m.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g17/b{k}.jsonl") if l.startswith("{")]
    print("w4", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
