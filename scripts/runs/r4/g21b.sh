#!/bin/bash
# Round 4, call g21b: repeat of g21 (3 pairs) -- 4-stage ring for the Cout-512 one-pass gradient kernel -- bitwise check against the 3-stage
# form, then interleaved A/B x2 (default 3 / 4 stages)
set -o pipefail
O=gpurun_out/g21b
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 200 python -u - > $O/check.log 2>&1 <<'PY' || { cat $O/check.log; exit 1; }
import torch
from distributed_learning_amd.ops import _ext
C = _ext.require()
for M, ci in ((50001, 128), (131072, 256), (1003520, 128), (40003, 256)):
    g = torch.Generator().manual_seed(M)
    dy = torch.randn(M, 512, generator=g).to("cuda", torch.bfloat16)
    x = torch.randn(M, ci, generator=g).to("cuda", torch.bfloat16)
    w = (torch.randn(512, ci, generator=g) * 0.05).to("cuda", torch.bfloat16)
    C.set_dual512_stages(3); a = C.conv1x1_dual(dy, x, w, torch.float32)
    C.set_dual512_stages(4); b = C.conv1x1_dual(dy, x, w, torch.float32)
    C.set_dual512_stages(3)
    torch.cuda.synchronize()
    ok = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    print(M, ci, "bitwise" if ok else "MISMATCH")
    assert ok
PY
cat $O/check.log
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_ns3.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_dual512_stages(4)" bench.py --steps 15 --warmup 5 >> $O/ab_ns4.jsonl 2>> $O/ab.err || exit 1
done
python - <<'PY'
import json
for f in ("ab_ns3", "ab_ns4"):
    for l in open(f"gpurun_out/g21b/{f}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"])
PY
