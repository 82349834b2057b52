#!/bin/bash
# Round 5, call g33: register-staged row-major LDS tiles in the XOR-swizzled 128-byte layout (bank conflicts of the
# padded rows) -- numerics, 1x1 shape table, 3x3 table, step x3
set -o pipefail
O=gpurun_out/r5/g33
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py tests/test_gpu_stem.py tests/test_gpu_bench_batch.py \
  tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_tiles.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
for i in 1 2 3; do
  run 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
grep metric $O/bench.jsonl | cut -c1-200
python3 - <<'PY'
import json
O = "gpurun_out/r5/g33"
old = {(d["kind"], d["M"], d["K"], d["N"]): d for d in map(json.loads, open("gpurun_out/r5/g33/none"))}
tn = to = 0.0
for l in open(f"{O}/gemm.jsonl"):
    d = json.loads(l)
    o = old.get((d["kind"], d["M"], d["K"], d["N"]))
    if o:
        tn += d["auto_ms"] * d["calls"]; to += o["auto_ms"] * o["calls"]
        print(d["kind"], d["M"], d["K"], d["N"], d["calls"], o["auto_ms"], "->", d["auto_ms"])
print("1x1 sum ms/step", round(to, 3), "->", round(tn, 3))
for l in open(f"{O}/conv_tiles.jsonl"):
    d = json.loads(l); print("3x3 C", d["C"], {k: d[k] for k in ("fwd_auto", "dgrad_auto", "wgrad")})
PY
