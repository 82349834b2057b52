import sys, torch, torch.nn as nn
sys.path.insert(0, ".")
from distributed_learning_amd.ops.bn_act import fused_bn_act
from distributed_learning_amd.models.resnet import Bottleneck
from distributed_learning_amd.ops import nn as dnn
dev = torch.device("cuda:0")
torch.manual_seed(0)
def rel(a, b): return float((a - b).norm() / (b.norm() + 1e-30))
for shape in [(8, 2048, 7, 7), (2, 2048, 7, 7), (8, 64, 56, 56)]:
    C = shape[1]
    bn = nn.BatchNorm2d(C).to(dev); bn2 = nn.BatchNorm2d(C).to(dev); bn2.load_state_dict(bn.state_dict())
    x = torch.randn(shape, device=dev).contiguous(memory_format=torch.channels_last)
    r = torch.randn(shape, device=dev).contiguous(memory_format=torch.channels_last)
    for mode in ["randn", "avgpool"]:
        x1 = x.clone().requires_grad_(True); r1 = r.clone().requires_grad_(True)
        x2 = x.clone().requires_grad_(True); r2 = r.clone().requires_grad_(True)
        y1 = fused_bn_act(x1, bn, True, r1)
        y2 = torch.relu(bn2(x2) + r2)
        if mode == "randn":
            g = torch.randn(shape, device=dev)
            y1.backward(g); y2.backward(g)
        else:
            y1.mean((2, 3)).pow(2).sum().backward(); y2.mean((2, 3)).pow(2).sum().backward()
        print(shape, mode, "y", rel(y1, y2), "dx", rel(x1.grad, x2.grad), "dr", rel(r1.grad, r2.grad),
              "dg", rel(bn.weight.grad, bn2.weight.grad), "db", rel(bn.bias.grad, bn2.bias.grad), flush=True)
        bn.weight.grad = None; bn.bias.grad = None; bn2.weight.grad = None; bn2.bias.grad = None
# one bottleneck block
for ds in [False, True]:
    torch.manual_seed(1)
    inp, planes = (2048, 512) if not ds else (1024, 512)
    down = None
    from distributed_learning_amd.models.resnet import Downsample
    if ds: down = Downsample(inp, planes * 4, 2)
    b1 = Bottleneck(inp, planes, 2 if ds else 1, down).to(dev).to(memory_format=torch.channels_last)
    import copy
    b2 = copy.deepcopy(b1)
    x = torch.randn(8, inp, 14 if ds else 7, 14 if ds else 7, device=dev).contiguous(memory_format=torch.channels_last)
    outs = []
    for be, b in (("native", b1), ("torch", b2)):
        dnn.set_backend(be)
        xx = x.clone().requires_grad_(True)
        y = b(xx)
        y.mean((2, 3)).pow(2).sum().backward()
        outs.append((y, xx.grad, b.conv1.weight.grad, b.conv3.weight.grad))
    print("block ds=", ds, [rel(a, c) for a, c in zip(outs[0], outs[1])], flush=True)
