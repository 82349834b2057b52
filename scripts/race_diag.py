#!/usr/bin/env python3
"""Diagnose a race-replay mismatch: run scripts/race_replay.py concurrently twice and once serialised,
then print per-tensor max differences and the per-step losses (nondeterminism vs a race)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(out, extra):
    env = dict(os.environ)
    env.update(extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "race_replay.py"), out] + sys.argv[2:],
                       env=env, capture_output=True, text=True, timeout=120)
    print(r.stdout.strip()[-400:], r.stderr.strip()[-600:] if r.returncode else "")
    return torch.load(out, weights_only=True)


def cmp(a, b, tag):
    diff = [(k, (a[k].float() - b[k].float()).abs().max().item()) for k in a if not torch.equal(a[k], b[k])]
    print(f"{tag}: {len(diff)} of {len(a)} tensors differ; losses {a['__losses__'].tolist()} vs {b['__losses__'].tolist()}")
    for k, d in diff[:12]:
        print(f"   {k}: max |diff| {d:.3e}")


d = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
ser = {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1"}
runs = {"c1": {}, "c2": {}, "s1": ser, "s2": ser, "k": {"AMD_SERIALIZE_KERNEL": "3"}, "b": {"HIP_LAUNCH_BLOCKING": "1"}}
res = {n: run(f"{d}/{n}.pt", e) for n, e in runs.items()}
for n in runs:
    if n != "c1":
        cmp(res["c1"], res[n], f"c1 vs {n}")
