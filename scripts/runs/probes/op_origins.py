"""Attribute small torch ops (fill_/copy_/add/...) in a training step to their Python call sites.

Runs the bench model for a few steps under torch.profiler with Python stacks, then prints, per op
name, the most frequent innermost framework call sites. Diagnostics only."""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from distributed_learning_amd.data import SyntheticBatches  # noqa: E402
from distributed_learning_amd.models import get_spec  # noqa: E402
from distributed_learning_amd.ops import nn as dnn  # noqa: E402
from distributed_learning_amd.ops.loss import cross_entropy  # noqa: E402
from distributed_learning_amd.ops.optim import FusedSGD  # noqa: E402
from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer  # noqa: E402
from distributed_learning_amd.parallel import context as ctxmod  # noqa: E402

OPS = set(sys.argv[1].split(",")) if len(sys.argv) > 1 else {"aten::fill_", "aten::copy_", "aten::zero_", "aten::add",
                                                            "aten::add_", "aten::zeros", "aten::contiguous"}
c = ctxmod.init(backend="nccl")
dev = c.device
torch.backends.cudnn.benchmark = True
dnn.set_backend("native")
dnn.set_native_conv(True)
spec = get_spec("resnet50")
model = spec.build().to(dev).to(memory_format=torch.channels_last)
dnn.bf16_weights(model)
model = PipelinedFusedDP(model, make_reducer("immediate", "builtin", native=True), 25 << 20, dev)
opt = FusedSGD(model.module.parameters(), lr=0.01, momentum=0.5, master_weights=True)
data = SyntheticBatches(int(os.environ.get("BS", "64")), spec.input_shape, spec.num_classes, dev,
                        dtype=torch.bfloat16, channels_last=True)


def step():
    x, y = data.next()
    opt.zero_grad(set_to_none=True)
    loss = cross_entropy(model(x), y)
    loss.backward()
    model.sync_gradients()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
path = "/tmp/op_origins_trace.json"
prof.export_chrome_trace(path)
ev = json.load(open(path))["traceEvents"]
py = [e for e in ev if e.get("cat") == "python_function" and "dur" in e]
ops = [e for e in ev if e.get("cat") == "cpu_op" and e.get("name") in OPS]
by_tid = collections.defaultdict(list)
for e in py:
    by_tid[e["tid"]].append(e)
counts = collections.Counter()
for o in ops:
    t0 = o["ts"]
    frames = [e for e in by_tid[o["tid"]] if e["ts"] <= t0 <= e["ts"] + e["dur"]]
    frames.sort(key=lambda e: e["ts"])
    names = [f["name"] for f in frames if "distributed_learning_amd" in f["name"] or "bench" in f["name"]
             or "torch/autograd" in f["name"]]
    counts[(o["name"], " <- ".join(n.split("/")[-1] for n in names[-3:][::-1]))] += 1
for (name, site), n in counts.most_common(40):
    print(f"{n:5d}  {name:18s} {site}")
