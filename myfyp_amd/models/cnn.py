"""CNNs for the CIFAR-shaped configs (BASELINE configs 3-5; not in the reference).

Inputs are ``uint8`` images ``[N, H, W, C]`` (or ``[N, H, W]``) as stored by the datasets; the
model converts to ``NCHW`` float and scales by ``input_scale`` (1/255 by default — unlike the
reference MLP, raw 0..255 inputs destabilise BN-free conv stacks). Outputs are log-probabilities.
On MI355X the convolutions run channels-last in bf16 under autocast (MIOpen) and the whole train
step is captured in a HIP graph by the learner.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F


def _to_nchw(x: torch.Tensor, scale: float) -> torch.Tensor:
    if x.dim() == 3:
        x = x.unsqueeze(-1)
    if x.shape[-1] in (1, 3) and x.shape[1] not in (1, 3):
        x = x.permute(0, 3, 1, 2)
    return x.float() * scale


class LeNet5(torch.nn.Module):
    """LeNet-5: conv(5)→pool→conv(5)→pool→fc120→fc84→fc10."""

    def __init__(self, in_channels: int = 3, num_classes: int = 10, image_size: int = 32, input_scale: float = 1 / 255, lr_rate: float = 0.01, seed: Optional[int] = None) -> None:
        super().__init__()
        if seed is not None:
            torch.manual_seed(seed)
        self.input_scale = input_scale
        self.lr_rate = lr_rate
        self.conv1 = torch.nn.Conv2d(in_channels, 6, 5)
        self.conv2 = torch.nn.Conv2d(6, 16, 5)
        s = ((image_size - 4) // 2 - 4) // 2
        self.fc1 = torch.nn.Linear(16 * s * s, 120)
        self.fc2 = torch.nn.Linear(120, 84)
        self.fc3 = torch.nn.Linear(84, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = _to_nchw(x, self.input_scale)
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = x.flatten(1)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return torch.log_softmax(self.fc3(x).float(), dim=1)

    def optimizer_spec(self) -> dict:
        return {"name": "sgd", "lr": self.lr_rate, "momentum": 0.9}


class _BasicBlock(torch.nn.Module):
    def __init__(self, cin: int, cout: int, stride: int) -> None:
        super().__init__()
        self.conv1 = torch.nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = torch.nn.BatchNorm2d(cout)
        self.conv2 = torch.nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = torch.nn.BatchNorm2d(cout)
        self.shortcut = torch.nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = torch.nn.Sequential(torch.nn.Conv2d(cin, cout, 1, stride, bias=False), torch.nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))


class ResNet18(torch.nn.Module):
    """CIFAR ResNet-18 (3x3 stem, no max-pool), 11.2M parameters."""

    def __init__(self, in_channels: int = 3, num_classes: int = 10, input_scale: float = 1 / 255, lr_rate: float = 0.05, seed: Optional[int] = None) -> None:
        super().__init__()
        if seed is not None:
            torch.manual_seed(seed)
        self.input_scale = input_scale
        self.lr_rate = lr_rate
        self.conv1 = torch.nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False)
        self.bn1 = torch.nn.BatchNorm2d(64)
        cfg = [(64, 1), (128, 2), (256, 2), (512, 2)]
        layers = []
        cin = 64
        for cout, stride in cfg:
            layers += [_BasicBlock(cin, cout, stride), _BasicBlock(cout, cout, 1)]
            cin = cout
        self.layers = torch.nn.Sequential(*layers)
        self.fc = torch.nn.Linear(512, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = _to_nchw(x, self.input_scale)
        x = F.relu(self.bn1(self.conv1(x)))
        x = self.layers(x)
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return torch.log_softmax(self.fc(x).float(), dim=1)

    def optimizer_spec(self) -> dict:
        return {"name": "sgd", "lr": self.lr_rate, "momentum": 0.9, "weight_decay": 5e-4}
