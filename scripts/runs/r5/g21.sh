#!/bin/bash
# Round 5, call g21: streaming 1x1 GEMM with both k-halves' fragments read before the MFMAs (one wave per SIMD)
# vs HEAD (variants/_C_pre0.so): numerics, the bs1280 1x1 shape table (incl. forced stream), step A/B x3
set -o pipefail
O=gpurun_out/r5/g21
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
V=$(pwd)/variants/_C_pre0.so
run 600 python -u -m pytest tests/test_gpu_gemm_stream.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm_new.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
DLA_EXT_SO=$V DLA_ALLOW_STALE=1 run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm_old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_new.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_EXT_SO=$V DLA_ALLOW_STALE=1 run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r5/g21"
for k in ("new", "old"):
    v = [json.loads(l) for l in open(f"{O}/ab_{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
n = [json.loads(l) for l in open(f"{O}/gemm_new.jsonl") if l.startswith("{")]
o = [json.loads(l) for l in open(f"{O}/gemm_old.jsonl") if l.startswith("{")]
for a, b in zip(n, o):
    print({k: a[k] for k in list(a)[:4]}, "| old", {k: b[k] for k in b if "ms" in k or "stream" in k}, "| new", {k: a[k] for k in a if "ms" in k or "stream" in k})
PY
