#!/bin/bash
# Round 6, call g32: per-direction halo conv variant (DLA_HALO_V=3: v2 forward, v1 data gradient) -- halo tests,
# driver bench interleaved x3 against the default v1
set -o pipefail
O=gpurun_out/r6/g32
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k "halo" --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2 3; do
  for v in 1 3; do
    DLA_HALO_V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$v.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (1, 3):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g32/b{k}.jsonl") if l.startswith("{")]
    print("halo_v", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
