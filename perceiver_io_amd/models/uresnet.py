"""U-ResNet CNN of the LArTPC experiment (reference ``uresnet.py``, SURVEY #35).

In the reference it is constructed by ``run.py:103`` but its use in ``forward`` is commented
out (``run.py:109-110``), so it contributes parameters (and optimizer state) only.  It is a
plain PyTorch/MIOpen convolution network — not a kernel target (SURVEY K-18) — kept with the
same ``state_dict`` names so ``run.py`` checkpoints (``uresnet.*`` keys) load.

Architecture: 3 stem 3×3 conv-BN-ReLU; 4 encoder stages of two bottleneck residual blocks
(the first strided ×2, channels ×2); 4 decoder stages of (bottleneck, 3×3 transposed conv ×2)
with U-Net skip concatenations; a 3-conv head and a 1×1 classifier producing raw class scores
(the ``softmax`` LogSoftmax module exists but, as in the reference, is not applied).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    """Two 3×3 conv-BN layers with an identity (or projected) shortcut."""
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample=None):
        super().__init__()
        self.conv1, self.bn1 = conv3x3(inplanes, planes, stride), nn.BatchNorm2d(planes)
        self.conv2, self.bn2 = conv3x3(planes, planes), nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample, self.stride = downsample, stride

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + (x if self.downsample is None else self.downsample(x)))


class Bottleneck(nn.Module):
    """1×1 → 3×3 (strided) → 1×1 conv-BN branch, 1×1 strided projection shortcut when stride > 1."""

    def __init__(self, inplanes: int, planes: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(inplanes, planes, 1, bias=False), nn.BatchNorm2d(planes)
        self.conv2, self.bn2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False), nn.BatchNorm2d(planes)
        self.conv3, self.bn3 = nn.Conv2d(planes, planes, 1, bias=False), nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.stride = stride
        self.shortcut = nn.Conv2d(inplanes, planes, 1, stride=stride, bias=False) if stride > 1 else None

    def forward(self, x):
        skip = x if self.shortcut is None else self.shortcut(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(skip + y)


class DoubleResNet(nn.Module):
    def __init__(self, inplanes: int, planes: int, stride: int = 1):
        super().__init__()
        self.res1 = Bottleneck(inplanes, planes, stride)
        self.res2 = Bottleneck(planes, planes, 1)

    def forward(self, x):
        return self.res2(self.res1(x))


class ConvTransposeLayer(nn.Module):
    def __init__(self, inplanes: int, outplanes: int, stride: int = 2):
        super().__init__()
        self.res = Bottleneck(inplanes, inplanes, stride=1)
        self.deconv = nn.ConvTranspose2d(inplanes, outplanes, kernel_size=3, stride=2, padding=1, bias=False)

    def forward(self, x, output_size):
        return self.deconv(self.res(x), output_size=output_size)


def _conv_bn_relu(owner: nn.Module, idx: int, cin: int, cout: int):
    setattr(owner, f"conv{idx}", nn.Conv2d(cin, cout, kernel_size=3, stride=1, padding=1, bias=True))
    setattr(owner, f"bn{idx}", nn.BatchNorm2d(cout))
    setattr(owner, f"relu{idx}", nn.ReLU(inplace=True))


class UResNet(nn.Module):
    def __init__(self, num_classes: int = 3, input_channels: int = 3, inplanes: int = 16, showsizes: bool = False):
        super().__init__()
        self.inplanes = p = inplanes
        self._showsizes = showsizes
        for i, cin in ((1, input_channels), (2, p), (3, p)):
            _conv_bn_relu(self, i, cin, p)
        for i in range(1, 5):
            setattr(self, f"enc_layer{i}", DoubleResNet(p * 2 ** (i - 1), p * 2 ** i, stride=2))
        self.dec_layer4 = ConvTransposeLayer(p * 16, p * 8)
        for i in (3, 2, 1):
            setattr(self, f"dec_layer{i}", ConvTransposeLayer(p * 2 ** i * 2, p * 2 ** (i - 1)))
        self.nkernels = k = 16
        for i, cin, cout in ((10, p, k), (11, k, 2 * k), (12, 2 * k, k)):
            _conv_bn_relu(self, i, cin, cout)
        self.conv13 = nn.Conv2d(k, num_classes, kernel_size=1, stride=1, padding=0, bias=True)
        self.softmax = nn.LogSoftmax(dim=1)
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                with torch.no_grad():
                    m.weight.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                with torch.no_grad():
                    m.weight.fill_(1)
                    m.bias.zero_()

    def _cbr(self, i, x):
        return getattr(self, f"relu{i}")(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))

    def forward(self, x):
        x0 = self._cbr(3, self._cbr(2, self._cbr(1, x)))
        skips = [x0]
        for i in range(1, 5):
            skips.append(getattr(self, f"enc_layer{i}")(skips[-1]))
        y = skips[4]
        for i in (4, 3, 2, 1):
            y = getattr(self, f"dec_layer{i}")(y, output_size=skips[i - 1].size())
            if i > 1:
                y = torch.cat([y, skips[i - 1]], 1)
        y = self._cbr(12, self._cbr(11, self._cbr(10, y)))
        return self.conv13(y)
