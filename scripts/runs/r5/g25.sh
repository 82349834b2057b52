#!/bin/bash
# Round 5, call g25: persistent register-staged 1x1 GEMM (next tile's first k-step loaded during the last
# k-step + epilogue) -- numerics, per-shape table with it off / 2 / 3 blocks per CU, step A/B x3, pipeline sweep
set -o pipefail
O=gpurun_out/r5/g25
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bench_batch.py tests/test_gpu_conv.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for p in 0 2 3; do
  DLA_GEMM_PERSIST=$p run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm_p$p.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_p2.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_GEMM_PERSIST=0 run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_p0.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r5/g25"
for k in ("p2", "p0"):
    v = [json.loads(l) for l in open(f"{O}/ab_{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
t = {p: [json.loads(l) for l in open(f"{O}/gemm_p{p}.jsonl") if l.startswith("{")] for p in (0, 2, 3)}
tot = {p: 0.0 for p in t}
for rows in zip(*t.values()):
    a = rows[0]
    for p, r in zip(t, rows):
        tot[p] += r["auto_ms"] * r["calls"]
    print(a["kind"], a["M"], a["K"], a["N"], a["calls"], [r["auto_ms"] for r in rows])
print("sum auto ms/step by persist", {p: round(v, 3) for p, v in tot.items()})
PY
cd scripts && timeout -k 10 300 python -u bench_gemm_pipes.py > ../$O/pipes.jsonl 2>> ../$O/err.log || exit 0
