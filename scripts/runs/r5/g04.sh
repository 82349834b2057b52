#!/bin/bash
# Round 5, call g04: fusion-off launch groups (GPU test + the verdict's forced world-1 measurements, ResNet-50
# bs1280 and ResNet-152 bs256, fused vs per-tensor), and the 1x1 GEMM shape table with a hipBLASLt column
set -o pipefail
O=gpurun_out/r5/g04
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 600 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log
run 300 python -u bench.py --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/r50_fusion_off_times.csv > $O/r50_fusion_off.jsonl 2> $O/r50_fusion_off.err || { tail $O/r50_fusion_off.err; exit 1; }
run 300 python -u bench.py --force_comm 1 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/r50_fusion_on_times.csv > $O/r50_fusion_on.jsonl 2> $O/r50_fusion_on.err || exit 1
run 300 python -u bench.py --model resnet152 --batch 256 --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/r152_fusion_off_times.csv > $O/r152_fusion_off.jsonl 2> $O/r152_fusion_off.err || exit 1
run 300 python -u bench.py --model resnet152 --batch 256 --force_comm 1 --steps 10 --warmup 3 --phases 5 \
  > $O/r152_fusion_on.jsonl 2> $O/r152_fusion_on.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5/g04/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["value"], d["ms_per_step"], "comm", d.get("allreduce_ms_per_step"), d.get("latency_breakdown_ms"))
PY
run 400 python -u scripts/bench_gemm_bs1280.py --out $O/gemm_bs1280.jsonl > $O/gemm.log 2>&1 || { tail $O/gemm.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r5/g04/gemm_bs1280.jsonl"):
    d = json.loads(l)
    print(d["kind"], d["M"], d["K"], d["N"], d["calls"], "auto", round(d["auto_ms"], 4), "hipblaslt", round(d["hipblaslt_ms"], 4))
PY
