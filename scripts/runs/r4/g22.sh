#!/bin/bash
# Round 4, call g22: the kBN one-pass kernel (stage 1, block-final BN apply fused) with register-held weights and
# a 4-stage ring (160 KB LDS) vs the LDS weight panel + 3 stages -- bitwise check, then interleaved A/B x3
set -o pipefail
O=gpurun_out/g22
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 200 python -u - > $O/check.log 2>&1 <<'PY' || { cat $O/check.log; exit 1; }
import torch
from distributed_learning_amd.ops import _ext
C = _ext.require()
co, ci = 256, 64
for M in (65536, 100003, 4014080):
    g = torch.Generator().manual_seed(M)
    dout = torch.randn(M, co, generator=g).to("cuda", torch.bfloat16)
    ybn = (torch.randn(M, co, generator=g) * 2 + 0.5).to("cuda", torch.bfloat16)
    x = torch.randn(M, ci, generator=g).to("cuda", torch.bfloat16)
    w = (torch.randn(co, ci, generator=g) * co ** -0.5).to("cuda", torch.bfloat16)
    mask = torch.randint(0, 256, ((M * co + 7) // 8,), generator=g, dtype=torch.uint8).to("cuda")
    gamma = (torch.rand(co, generator=g) + 0.5).to("cuda")
    ws = torch.zeros(7 * co, device="cuda")
    ws[:co] = ybn.float().mean(0)
    ws[co:2 * co] = (ybn.float().var(0, unbiased=False) + 1e-5).rsqrt()
    C.bn_act_bwd(dout, None, mask, ybn, ws, gamma, 2, False, None, False)
    C.set_dualbn_form(0); a = C.conv1x1_dual(dout, x, w, torch.float32, ybn, ws, mask)
    C.set_dualbn_form(1); b = C.conv1x1_dual(dout, x, w, torch.float32, ybn, ws, mask)
    C.set_dualbn_form(0)
    torch.cuda.synchronize()
    ok = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    print(M, "bitwise" if ok else "MISMATCH")
    assert ok
PY
cat $O/check.log
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_panel.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_dualbn_form(1)" bench.py --steps 15 --warmup 5 >> $O/ab_wreg4.jsonl 2>> $O/ab.err || exit 1
done
python - <<'PY'
import json
for f in ("ab_panel", "ab_wreg4"):
    for l in open(f"gpurun_out/g22/{f}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"])
PY
