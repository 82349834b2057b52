import sys, torch
sys.path.insert(0, ".")
from distributed_learning_amd.models import resnet50
from distributed_learning_amd.ops import nn as dnn
dev = torch.device("cuda:0")
def run(order):
    torch.manual_seed(0)
    ms = [resnet50().to(dev).to(memory_format=torch.channels_last) for _ in order]
    for m in ms[1:]: m.load_state_dict(ms[0].state_dict())
    x = torch.randn(8, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    for be, m in zip(order, ms):
        dnn.set_backend(be); out = m(x); out.float().pow(2).mean().backward()
    a, b = ms
    for n in ["layer4.2.bn3.bias", "layer4.2.conv3.weight", "layer3.5.conv2.weight", "conv1.weight"]:
        ga, gb = dict(a.named_parameters())[n].grad, dict(b.named_parameters())[n].grad
        print(order, n, float((ga - gb).norm() / gb.norm()), flush=True)
run(("torch", "torch"))
run(("native", "native"))
run(("native", "torch"))
torch.backends.cudnn.deterministic = True
run(("torch", "torch"))
run(("native", "torch"))
