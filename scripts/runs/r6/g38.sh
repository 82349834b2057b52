#!/bin/bash
# Round 6, call g38: the variant-1 halo forward with statistics stored from registers (dla_mfma.h epilogue_direct) --
# halo tests, driver bench interleaved x3: default (v2 forward staged, v1 dgrad direct) vs v1 forward direct
set -o pipefail
O=gpurun_out/r6/g38
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k "halo" --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b0.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_HALO_V=1 DLA_HALO_DIRECT_FWD=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b1.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g38/b{k}.jsonl") if l.startswith("{")]
    print("v1_direct_fwd", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
