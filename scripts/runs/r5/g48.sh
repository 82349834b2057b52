#!/bin/bash
# Round 5, call g48: BN row blocks last-to-first for the forward apply and backward reductions (MALL reuse):
# BN GPU tests, then same-box A/B against the DLA_BN_REV=0 variant, interleaved x4
set -o pipefail
O=gpurun_out/r5/g48
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn_act.py tests/test_gpu_bn_epilogue.py tests/test_gpu_stem_bn_fused.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$(pwd)/variants/_C_norev.so
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/new.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_EXT_SO=$V DLA_ALLOW_STALE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/old.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  echo "pair $i done"
done
python3 - <<'PY'
import json
for k in ("new", "old"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g48/{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v])
PY
