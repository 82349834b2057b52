#!/bin/bash
# Round 5, call g18: shared MFMA main loops with the next fragment half read before this half's MFMAs
# (kstep_mfma, <= 16 fragments) vs the previous schedule (variants/_C_pre0.so, DLA_KSTEP_PRE_FRAGS=0):
# numerics, the 3x3 and 1x1 shape tables, and the bs1280 step interleaved x3
set -o pipefail
O=gpurun_out/r5/g18
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
V=$(pwd)/variants/_C_pre0.so
run 600 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_gemm.py tests/test_gpu_conv3x3_autograd.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_new.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
DLA_EXT_SO=$V run 300 python -u scripts/bench_conv_tiles.py > $O/conv_old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm_new.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
DLA_EXT_SO=$V run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm_old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_new.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_EXT_SO=$V run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r5/g18"
for k in ("new", "old"):
    v = [json.loads(l) for l in open(f"{O}/ab_{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
for f in ("conv", ):
    n = [json.loads(l) for l in open(f"{O}/{f}_new.jsonl")]
    o = [json.loads(l) for l in open(f"{O}/{f}_old.jsonl")]
    for a, b in zip(n, o):
        print("conv C", a["C"], {k: (b[k], a[k]) for k in ("fwd_auto", "dgrad_auto", "wgrad")})
PY
