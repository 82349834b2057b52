#!/bin/bash
# Record of a past call: the switch it A/Bs was removed from the sources after measuring slower (profiles/r4/README.md).
# Round 4, call g19: relu(BN2) normalised on load, in the MFMA operand registers (no LDS pass) -- kernel + model tests, then
# interleaved A/B x2 (default = lazy off / lazy on)
set -o pipefail
O=gpurun_out/g19
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lazy_bn.py \
  tests/test_gpu_gemm_dual.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.LAZY_BN_ACT = True" bench.py \
    --steps 15 --warmup 5 >> $O/ab_lazyon.jsonl 2>> $O/ab.err || exit 1
done
python - <<'PY'
import json
for f in ("ab_default", "ab_lazyon"):
    for l in open(f"gpurun_out/g19/{f}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"])
PY
