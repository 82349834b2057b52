"""BasicNet: the reference's MNIST CNN (/root/reference/src/network.py:7-30).

conv(1->32,3) -> relu -> conv(32->64,3) -> relu -> maxpool2 -> dropout .25 -> fc 9216->128 ->
relu -> dropout .5 -> fc 128->10. The reference applies ``log_softmax`` inside forward and uses
``nll_loss``; here forward returns logits and the fused log-softmax+NLL loss
(:func:`distributed_learning_amd.ops.loss.cross_entropy`) computes the identical value.
1,199,882 parameters in 8 tensors.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicNet(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        x = self.dropout2(x)
        return self.fc2(x)


def basicnet(num_classes: int = 10) -> BasicNet:
    return BasicNet(num_classes)
