#!/bin/bash
# Round 6, call g03: register-stored 128x128 1x1 GEMM tiles (gemm_direct.hip): numerics vs the staged kernel and
# fp32 torch, per-shape timing direct vs staged (production dispatch), then the driver bench A/B interleaved
set -o pipefail
O=gpurun_out/r6/g03
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_direct.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
SH=("250880 256 1024 fwd" "250880 256 1024 dgrad_add" "62720 512 2048 fwd" "62720 512 2048 dgrad_add" "1003520 512 128 dgrad_add" "1003520 256 512 fwd" "250880 512 1024 fwd" "1003520 512 256 fwd")
for s in "${SH[@]}"; do
  for d in 0 1; do
    DLA_GEMM_DIRECT=$d timeout -k 10 120 python3 scripts/gemm_stall.py $s 40 | sed "s/^/direct=$d /" >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
  done
done
cat $O/timing.txt
for i in 1 2; do
  for d in 0 1; do
    DLA_GEMM_DIRECT=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$d.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for d in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g03/b{d}.jsonl") if l.startswith("{")]
    print("direct", d, [round(x["value"]) for x in v], [x["ms_per_step"] for x in v], [x["telemetry"]["before_timed"]["gfxclk_mhz"] for x in v])
PY
