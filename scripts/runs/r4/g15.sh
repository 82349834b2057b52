#!/bin/bash
# Round 4, call g15: the N > 1 path on the final tree at a batch where the one-pass 1x1 kernels and the BN
# hand-off engage (2 ranks on one GPU over the IPC transport, per-rank batch 256): JSON line, and the two ranks'
# parameters / fp32 masters / gradients compared bitwise
set -o pipefail
O=gpurun_out/g15
mkdir -p $O/ck
timeout -k 10 600 python -u bench.py --gpus 2 --same_device 1 --batch 256 --steps 6 --warmup 2 --check_dir $O/ck \
  > $O/two_ranks.jsonl 2> $O/two_ranks.err || { tail -30 $O/two_ranks.err; exit 1; }
grep metric $O/two_ranks.jsonl | cut -c1-300
timeout -k 10 120 python - <<'PY' > $O/ranks_bitwise.txt 2>&1
import torch
a = torch.load("gpurun_out/g15/ck/rank0.pt", weights_only=True)
b = torch.load("gpurun_out/g15/ck/rank1.pt", weights_only=True)
bad = [(k, n) for k in ("params", "masters", "grads") for n in a[k] if not torch.equal(a[k][n], b[k][n])]
print({"compared": sum(len(a[k]) for k in ("params", "masters", "grads")), "differ": bad[:10], "ok": not bad})
PY
cat $O/ranks_bitwise.txt
rm -rf $O/ck
