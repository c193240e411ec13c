"""The reference's model zoo, restated for FedDF's teacher replay and the
parity fixtures (fedsim/models/simple_models.py:23-256, utils.py:49-62).

FedSim's ``model_def`` is any ``nn.Module``; these three are the ones its CLI
and tests name (``SimpleMLP`` = McMahan's 2NN on MNIST, ``SimpleCNN`` on MNIST,
``SimpleCNN2(num_classes=100)`` on CIFAR-100).  They keep the reference's
parameter registration order (hence its ``parameters_to_vector`` layout: the
P of each model, e.g. SimpleCNN2(num_classes=100) P = 1 085 668) and its
forward op by op, including the leading ``resize`` leaf module.

``Resize`` stands in for ``torchvision.transforms.Resize`` (torchvision is not
part of this image): no parameters, the identity when the input already has
the target height and width (what torchvision's resize returns at the native
size), else an antialiased bilinear resample.  Its shape test is data-dependent
Python, so ``torch.fx`` cannot trace through it -- exactly like torchvision's
own; the teacher replay (teacher_program.py) keeps such parameterless foreign
modules as leaves instead of giving up on the whole model.
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
from torch import nn
from torch.nn import functional as F

__all__ = ["Resize", "SimpleMLP", "SimpleCNN", "SimpleCNN2", "get_output_size"]


def get_output_size(in_size: int, pad: Union[int, str], kernel: int, stride: int) -> int:
    """Spatial size after a kernel along one axis ("same" keeps it)."""
    if pad == "same":
        return in_size
    return (in_size + 2 * pad - kernel) // stride + 1


class Resize(nn.Module):
    """Parameterless spatial resize to ``size`` = (height, width)."""

    def __init__(self, size: Tuple[int, int]):
        super().__init__()
        self.size = (int(size[0]), int(size[1]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if tuple(x.shape[-2:]) == self.size:
            return x
        lead = x.shape[:-2]
        y = x.reshape(-1, 1, *x.shape[-2:]) if x.dim() != 4 else x
        y = F.interpolate(y, size=self.size, mode="bilinear", align_corners=False,
                          antialias=True)
        return y.reshape(*lead, *self.size)


def _classifier(features: int, num_classes: Optional[int]) -> Optional[nn.Linear]:
    return nn.Linear(features, num_classes) if num_classes is not None and num_classes > 0 \
        else None


class SimpleMLP(nn.Module):
    """2NN: resize, flatten, two ReLU layers of ``feature_size``, classifier
    (simple_models.py:23-77)."""

    def __init__(self, num_classes=10, num_channels=1, in_height=28, in_width=28,
                 feature_size=200):
        super().__init__()
        self.feature_size = feature_size
        self.resize = Resize((in_height, in_width))
        self.fc1 = nn.Linear(num_channels * in_height * in_width, feature_size)
        self.fc2 = nn.Linear(feature_size, feature_size)
        self.classifier = _classifier(feature_size, num_classes)

    def get_features(self, x):
        x = self.resize(x)
        x = x.view(x.shape[0], -1)
        return F.relu(self.fc2(F.relu(self.fc1(x))))

    def forward(self, x):
        x = self.get_features(x)
        return x if self.classifier is None else self.classifier(x)


class SimpleCNN(nn.Module):
    """Two 5x5 convs (padding 1), each ReLU + 2x2/2 max-pool with padding 1,
    then one ReLU layer and the classifier (simple_models.py:80-162)."""

    def __init__(self, num_classes=10, num_channels=1, in_height=28, in_width=28,
                 num_filters1=32, num_filters2=64, feature_size=512):
        super().__init__()
        self.feature_size = feature_size
        self.resize = Resize((in_height, in_width))
        self.conv1 = nn.Conv2d(num_channels, num_filters1, kernel_size=5, stride=1, padding=1)
        self.conv2 = nn.Conv2d(num_filters1, num_filters2, kernel_size=5, stride=1, padding=1)
        # the reference sizes both axes from in_height (simple_models.py:119-129)
        side = in_height
        for _ in range(2):
            side = get_output_size(get_output_size(side, 1, 5, 1), 1, 2, 2)
        self.fc = nn.Linear(num_filters2 * side * side, feature_size)
        self.classifier = _classifier(feature_size, num_classes)

    def get_features(self, x):
        x = self.resize(x)
        x = F.max_pool2d(F.relu(self.conv1(x)), kernel_size=2, stride=2, padding=1)
        x = F.max_pool2d(F.relu(self.conv2(x)), kernel_size=2, stride=2, padding=1)
        x = x.view(x.shape[0], -1)
        return F.relu(self.fc(x))

    def forward(self, x):
        x = self.get_features(x)
        return x if self.classifier is None else self.classifier(x)


class SimpleCNN2(nn.Module):
    """McMahan's CIFAR CNN: two 5x5 "same" convs with ReLU, a (0,1,0,1) zero
    pad, LRN(size 4, alpha 0.001/9) and a 3x3/2 max-pool around each (in the
    reference's order), then 384- and 192-wide ReLU layers and the classifier
    (simple_models.py:165-256)."""

    def __init__(self, num_classes=10, num_channels=3, in_height=24, in_width=24,
                 num_filters1=64, num_filters2=64, hidden_size=384, feature_size=192):
        super().__init__()
        self.feature_size = feature_size
        self.resize = Resize((in_height, in_width))
        self.conv1 = nn.Conv2d(num_channels, num_filters1, kernel_size=5, stride=1,
                               padding="same")
        self.conv2 = nn.Conv2d(num_filters1, num_filters2, kernel_size=5, stride=1,
                               padding="same")
        side = get_output_size(in_height, 0, 3, 2)  # conv1 keeps it; pool1 (pad 0)
        side = get_output_size(side, 1, 2, 2)       # conv2 keeps it; as the reference sizes pool2
        self.fc1 = nn.Linear(num_filters2 * side * side, hidden_size)
        self.fc2 = nn.Linear(hidden_size, feature_size)
        self.classifier = _classifier(feature_size, num_classes)

    def get_features(self, x):
        x = self.resize(x)
        x = F.relu(self.conv1(x))
        x = F.pad(x, (0, 1, 0, 1), value=0)
        x = F.local_response_norm(x, size=4, alpha=0.001 / 9)
        x = F.max_pool2d(x, kernel_size=3, stride=2, padding=0)
        x = F.relu(self.conv2(x))
        x = F.local_response_norm(x, size=4, alpha=0.001 / 9)
        x = F.pad(x, (0, 1, 0, 1), value=0)
        x = F.max_pool2d(x, kernel_size=3, stride=2, padding=0)
        x = x.view(x.shape[0], -1)
        return F.relu(self.fc2(F.relu(self.fc1(x))))

    def forward(self, x):
        x = self.get_features(x)
        return x if self.classifier is None else self.classifier(x)
