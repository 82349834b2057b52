"""Model zoo (all defined locally: no torchvision / torch.hub on the GPU box).

Registry keys include the reference's ``model_type`` names (``mnist`` -> BasicNet, ``imagenet`` ->
GoogLeNet; /root/reference/src/config.py:7) plus the BASELINE.json models.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, Tuple

import torch.nn as nn

from .basicnet import BasicNet, basicnet
from .googlenet import GoogLeNet, googlenet
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152


@dataclass(frozen=True)
class ModelSpec:
    name: str
    build: Callable[[], nn.Module]
    input_shape: Tuple[int, int, int]  # C, H, W
    num_classes: int
    dataset: str  # synthetic template / loader family


MODELS: Dict[str, ModelSpec] = {
    "mnist": ModelSpec("basicnet", lambda: basicnet(10), (1, 28, 28), 10, "mnist"),
    "basicnet": ModelSpec("basicnet", lambda: basicnet(10), (1, 28, 28), 10, "mnist"),
    "imagenet": ModelSpec("googlenet", lambda: googlenet(1000), (3, 224, 224), 1000, "imagenet"),
    "googlenet": ModelSpec("googlenet", lambda: googlenet(1000), (3, 224, 224), 1000, "imagenet"),
    "googlenet_noaux": ModelSpec("googlenet_noaux", lambda: googlenet(1000, aux_logits=False), (3, 224, 224), 1000,
                                 "imagenet"),
    "resnet18": ModelSpec("resnet18", lambda: resnet18(1000), (3, 224, 224), 1000, "imagenet"),
    # torchvision-style resnet18(num_classes=10) on 32x32 inputs (11,181,642)
    "resnet18_cifar": ModelSpec("resnet18_cifar", lambda: resnet18(10), (3, 32, 32), 10, "cifar10"),
    # CIFAR-adapted stem (3x3/s1 conv, no max-pool)
    "resnet18_cifar_stem": ModelSpec("resnet18_cifar_stem", lambda: resnet18(10, cifar_stem=True), (3, 32, 32), 10,
                                     "cifar10"),
    "resnet34": ModelSpec("resnet34", lambda: resnet34(1000), (3, 224, 224), 1000, "imagenet"),
    "resnet50": ModelSpec("resnet50", lambda: resnet50(1000), (3, 224, 224), 1000, "imagenet"),
    "resnet101": ModelSpec("resnet101", lambda: resnet101(1000), (3, 224, 224), 1000, "imagenet"),
    "resnet152": ModelSpec("resnet152", lambda: resnet152(1000), (3, 224, 224), 1000, "imagenet"),
}


def get_spec(name: str) -> ModelSpec:
    try:
        return MODELS[name]
    except KeyError:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}") from None


def create_network(name: str) -> nn.Module:
    return get_spec(name).build()


__all__ = ["MODELS", "ModelSpec", "get_spec", "create_network", "BasicNet", "GoogLeNet", "ResNet", "basicnet",
           "googlenet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152"]
