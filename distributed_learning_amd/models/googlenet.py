"""GoogLeNet (Inception v1) with the torchvision-v0.6 layout, defined locally.

The reference loads it with ``torch.hub.load('pytorch/vision:v0.6.0', 'googlenet',
pretrained=False, init_weights=False)`` and wraps it so the loss uses ``log_softmax(output[0])``
(/root/reference/src/network.py:33-54). The hub needs network access, which neither this
container nor the GPU box has, so the architecture is re-declared here with the same module
names, registration order, shapes and v0.6 quirks:

* ``BasicConv2d`` = conv(bias=False) + BN(eps=1e-3) + ReLU;
* branch3 of every Inception block uses a 3x3 (not 5x5) conv — the torchvision v0.6 layout;
* aux heads (``aux1`` after 4a, ``aux2`` after 4d) are *computed* in training mode but their
  outputs are not part of the returned logits, so ~6.38M parameters receive no gradient — the
  "unused parameter" case the reference's ``OurDist._find_unused`` handles
  (/root/reference/src/ourdist.py:137-156).

Totals: 187 parameter tensors / 13,004,888 parameters with aux heads,
173 / 6,624,904 without.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import nn as dnn
from ..ops.pool import MaxPool2d, global_avg_pool


class BasicConv2d(nn.Module):
    def __init__(self, cin: int, cout: int, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kw)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x):
        return dnn.conv_bn_act(x, self.conv, self.bn, relu=True)


class Inception(nn.Module):
    def __init__(self, cin, ch1x1, ch3x3red, ch3x3, ch5x5red, ch5x5, pool_proj):
        super().__init__()
        self.branch1 = BasicConv2d(cin, ch1x1, kernel_size=1)
        self.branch2 = nn.Sequential(BasicConv2d(cin, ch3x3red, kernel_size=1),
                                     BasicConv2d(ch3x3red, ch3x3, kernel_size=3, padding=1))
        self.branch3 = nn.Sequential(BasicConv2d(cin, ch5x5red, kernel_size=1),
                                     BasicConv2d(ch5x5red, ch5x5, kernel_size=3, padding=1))
        self.branch4 = nn.Sequential(MaxPool2d(kernel_size=3, stride=1, padding=1, ceil_mode=True),
                                     BasicConv2d(cin, pool_proj, kernel_size=1))

    def forward(self, x):
        if dnn.get_backend() == "native" and dnn.native_conv() and x.is_cuda:
            from ..ops import inception as ninc

            if ninc.supported(self, x):  # no concat copy, no autograd sum of x's four gradients
                return ninc.inception_forward(self, x)
        if dnn.get_backend() == "native" and dnn.native_conv_f32() and x.is_cuda:
            from ..ops import inception_f32

            if inception_f32.supported(self, x):  # the three 1x1 convs on x as one fp32 GEMM, one BN pass
                return inception_f32.forward(self, x)
        return torch.cat([self.branch1(x), self.branch2(x), self.branch3(x), self.branch4(x)], 1)


class InceptionAux(nn.Module):
    def __init__(self, cin, num_classes):
        super().__init__()
        self.conv = BasicConv2d(cin, 128, kernel_size=1)
        self.fc1 = nn.Linear(2048, 1024)
        self.fc2 = nn.Linear(1024, num_classes)

    def forward(self, x):
        x = F.adaptive_avg_pool2d(x, (4, 4))
        x = self.conv(x)
        x = torch.flatten(x, 1)
        x = F.relu(dnn.linear(x, self.fc1), inplace=True)
        x = F.dropout(x, 0.7, training=self.training)
        return dnn.linear(x, self.fc2)


class GoogLeNet(nn.Module):
    def __init__(self, num_classes: int = 1000, aux_logits: bool = True):
        super().__init__()
        self.aux_logits = aux_logits
        self.conv1 = BasicConv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.maxpool1 = MaxPool2d(3, stride=2, ceil_mode=True)
        self.conv2 = BasicConv2d(64, 64, kernel_size=1)
        self.conv3 = BasicConv2d(64, 192, kernel_size=3, padding=1)
        self.maxpool2 = MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception3a = Inception(192, 64, 96, 128, 16, 32, 32)
        self.inception3b = Inception(256, 128, 128, 192, 32, 96, 64)
        self.maxpool3 = MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception4a = Inception(480, 192, 96, 208, 16, 48, 64)
        self.inception4b = Inception(512, 160, 112, 224, 24, 64, 64)
        self.inception4c = Inception(512, 128, 128, 256, 24, 64, 64)
        self.inception4d = Inception(512, 112, 144, 288, 32, 64, 64)
        self.inception4e = Inception(528, 256, 160, 320, 32, 128, 128)
        self.maxpool4 = MaxPool2d(2, stride=2, ceil_mode=True)
        self.inception5a = Inception(832, 256, 160, 320, 32, 128, 128)
        self.inception5b = Inception(832, 384, 192, 384, 48, 128, 128)
        if aux_logits:
            self.aux1 = InceptionAux(512, num_classes)
            self.aux2 = InceptionAux(528, num_classes)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout(0.2)
        self.fc = nn.Linear(1024, num_classes)
        self.last_aux = None

    def forward(self, x):
        # conv + BN + ReLU + ceil-mode max-pool as one fused op on the native path (the full-
        # resolution activations of conv1 and conv3 are never written)
        x = dnn.conv_bn_act_maxpool(x, self.conv1.conv, self.conv1.bn, self.maxpool1)
        x = self.conv2(x)
        x = dnn.conv_bn_act_maxpool(x, self.conv3.conv, self.conv3.bn, self.maxpool2)
        x = self.inception3a(x)
        x = self.inception3b(x)
        x = self.maxpool3(x)
        x = self.inception4a(x)
        aux1 = self.aux1(x) if (self.aux_logits and self.training) else None
        x = self.inception4b(x)
        x = self.inception4c(x)
        x = self.inception4d(x)
        aux2 = self.aux2(x) if (self.aux_logits and self.training) else None
        x = self.inception4e(x)
        x = self.maxpool4(x)
        x = self.inception5a(x)
        x = self.inception5b(x)
        x = global_avg_pool(x) if isinstance(self.avgpool, nn.AdaptiveAvgPool2d) else torch.flatten(self.avgpool(x), 1)
        x = self.dropout(x)
        x = dnn.linear(x, self.fc)
        # Reference semantics: only output[0] (main logits) enters the loss (network.py:41). The aux
        # outputs are kept detached: holding their autograd graph would keep the previous step's
        # AccumulateGrad nodes alive across iterations (and across a HIP-graph capture boundary).
        self.last_aux = tuple(a.detach() if a is not None else None for a in (aux2, aux1))
        return x


def googlenet(num_classes: int = 1000, aux_logits: bool = True) -> GoogLeNet:
    return GoogLeNet(num_classes, aux_logits)
