"""ResNet-18/34/50/101/152 defined locally (no torchvision on the GPU box, no network).

The reference has no ResNet (SURVEY.md §0 mismatch table); BASELINE.json names ResNet-18 CIFAR,
ResNet-50 and ResNet-152 configs. Parameter registration order and shapes follow the standard
ImageNet ResNet layout (conv1, bn1, layer1..4, fc; bottleneck conv1/bn1/conv2/bn2/conv3/bn3 then
downsample) so gradient bucket layouts are comparable with the torchvision layout the survey
recomputed (R18 62 tensors / 11,689,512 params, R50 161 / 25,557,032,
R152 467 / 60,192,808).

MI355X-first choices:
  * ``channels_last`` (NHWC) activations: every 1x1 convolution is a plain [N*H*W, Cin] x
    [Cin, Cout] GEMM, which is what the MFMA GEMM path consumes without a transpose.
  * Conv -> BN -> ReLU (-> residual add) are expressed through :mod:`distributed_learning_amd.ops.nn`
    so the fused HIP BN+ReLU(+add) kernels replace three memory-bound passes with one when the
    native backend is selected (``set_backend('native')``), and stock PyTorch ops otherwise.
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from .. import knobs
from ..ops import nn as dnn
from ..ops.bn_act import deferral_scope, ensure
from ..ops.pool import MaxPool2d, global_avg_pool


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = dnn.conv_bn_act(x, self.conv1, self.bn1, relu=True)
        if self.downsample is not None:  # one apply pass for relu(bn2(conv2) + bn_d(conv_d))
            return dnn.conv_bn_add_conv_bn_act(out, self.conv2, self.bn2, x, self.downsample[0], self.downsample[1])
        return dnn.conv_bn_act(out, self.conv2, self.bn2, relu=True, residual=x)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)  # stride on the 3x3 (ResNet v1.5)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.downsample = downsample
        self.stride = stride
        self.defer_output = False  # set by ResNet for every bottleneck followed by another

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # conv1 forwards x as a second output that feeds the identity branch (or the downsample conv),
        # so the two gradients of the block input are summed inside conv1's dgrad GEMM epilogue
        # instead of by an elementwise add (native path; a plain alias otherwise)
        if self.downsample is not None and self.downsample[0].stride == (2, 2):
            # stride-2 downsample: conv1's fork also yields x[:, :, ::2, ::2], whose compact gradient
            # it adds at the even pixels in its dgrad epilogue (no zero-filled scatter)
            out, xa, xs = dnn.conv_bn_act_fork(x, self.conv1, self.bn1, relu=True, subsample=True)
        else:
            out, xa = dnn.conv_bn_act_fork(x, self.conv1, self.bn1, relu=True)
            xs = None
        # a block whose output goes straight into the next bottleneck (ResNet.forward) leaves the final apply
        # pass to that block's conv1 GEMM (ops/bn_act.py PendingApply); nothing else may observe it. The same for
        # bn2, whose only consumer is conv3 (the streaming GEMM applies it at stages 1-2)
        observed = bool(self._forward_hooks or self._forward_pre_hooks or nn.modules.module._global_forward_hooks)
        defer = self.defer_output and not observed
        out = dnn.conv_bn_act(out, self.conv2, self.bn2, relu=True, defer=not observed and knobs.flag("DEFER_MID"))
        if self.downsample is None:
            return dnn.conv_bn_act(out, self.conv3, self.bn3, relu=True, residual=xa, defer=defer)
        # the shortcut BN is applied inside the block's final apply pass (never materialised)
        ds_conv, ds_bn = self.downsample[0], self.downsample[1]
        if xs is not None:
            return dnn.conv_bn_add_conv_bn_act(out, self.conv3, self.bn3, xs, ds_conv, ds_bn, presubsampled=True,
                                               defer=defer)
        return dnn.conv_bn_add_conv_bn_act(out, self.conv3, self.bn3, xa, ds_conv, ds_bn, defer=defer)


class Downsample(nn.Sequential):
    """1x1 strided conv + BN on the identity path (registered as ``downsample.0/.1``)."""

    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__(conv1x1(cin, cout, stride), nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return dnn.conv_bn_act(x, self[0], self[1], relu=False)

    def forward_presubsampled(self, xs: torch.Tensor) -> torch.Tensor:
        """Same result for an input already subsampled by the conv's stride."""
        return dnn.conv_bn_act(xs, self[0], self[1], relu=False, presubsampled=True)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 cifar_stem: bool = False, zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        if cifar_stem:  # 32x32 inputs: 3x3/s1 stem, no max-pool
            self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        else:
            self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.Identity() if cifar_stem else MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        self._chain_bottlenecks()

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = Downsample(self.inplanes, planes * block.expansion, stride)
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def _chain_bottlenecks(self) -> None:
        """Mark every bottleneck whose output feeds another bottleneck (all but the network's last)."""
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        for b, nxt in zip(blocks, blocks[1:]):
            if isinstance(b, Bottleneck):
                b.defer_output = isinstance(nxt, Bottleneck)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = dnn.conv_bn_act_maxpool(x, self.conv1, self.bn1, self.maxpool)
        # block outputs consumed only by the next bottleneck's conv1 may be written by that conv's GEMM
        # (deferral_scope: anything still unwritten at its exit is materialised)
        with deferral_scope():
            x = self.layer1(x)
            x = self.layer2(x)
            x = self.layer3(x)
            x = self.layer4(x)
            ensure(x)
        x = global_avg_pool(x) if isinstance(self.avgpool, nn.AdaptiveAvgPool2d) else torch.flatten(self.avgpool(x), 1)
        return dnn.linear(x, self.fc)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)
