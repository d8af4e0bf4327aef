"""ReCoNet — drop-in for the reference's model.py (imported by pipeline.py via `from lib import ReCoNet`).

Same nested nn.Sequential names as model.py:5-116 (`encoder.layers.0.layers.0.layers.1.weight`, ...).
Encoder: 9x9 3->48, 3x3/s2 48->96, 3x3/s2 96->192 (reflect pad, IN, ReLU), 4 ResLayers with
ReLU AFTER the residual add (model.py:55-60); Decoder: nearest x2 -> 3x3 192->96, nearest x2 ->
3x3 96->48 (IN, ReLU), 9x9 48->3 + Tanh.  Runs as libnst_hip kernels.  Both variants run: the
InstanceNorm one the pipeline builds (`ReCoNet()`, pipeline.py:602) and `ReCoNet(frn=True)` (FRN + TLU,
frn.py:7-78; the engine keeps TLU outputs shifted by tau, nst_api.cpp frn_layer).
"""
import torch
from torch import nn

from ._lib import NST_ARCH_RECONET, NST_ARCH_RECONET_FRN
from .engine import StylizationNet


class TLU(nn.Module):
    """frn.py:7-23: max(x, tau), tau [1, C, 1, 1] (initialised to 0)."""

    def __init__(self, num_features):
        super().__init__()
        self.num_features = num_features
        self.tau = nn.Parameter(torch.zeros(1, num_features, 1, 1))


class FRN(nn.Module):
    """frn.py:26-78: x * rsqrt(mean(x^2 over H, W) + |eps|), then weight * x + bias; eps a buffer [1]
    (is_eps_leanable=False, the only form model.py builds)."""

    def __init__(self, num_features, eps=1e-6):
        super().__init__()
        self.num_features = num_features
        self.init_eps = eps
        self.weight = nn.Parameter(torch.ones(1, num_features, 1, 1))
        self.bias = nn.Parameter(torch.zeros(1, num_features, 1, 1))
        self.register_buffer("eps", torch.tensor([eps]))


class ConvLayer(nn.Module):
    """model.py:5-15: Sequential(ReflectionPad2d, Conv2d) — index 1 holds the conv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.layers = nn.Sequential(nn.ReflectionPad2d(kernel_size // 2),
                                    nn.Conv2d(in_channels, out_channels, kernel_size, stride))


class ConvNormLayer(nn.Module):
    """model.py:18-40: Sequential(ConvLayer, InstanceNorm2d[, ReLU]) or Sequential(ConvLayer, FRN[, TLU])."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, activation=True, frn=False):
        super().__init__()
        layers = [ConvLayer(in_channels, out_channels, kernel_size, stride),
                  FRN(out_channels) if frn else nn.InstanceNorm2d(out_channels, affine=True)]
        if activation:
            layers.append(TLU(out_channels) if frn else nn.ReLU(inplace=True))
        self.layers = nn.Sequential(*layers)


class ResLayer(nn.Module):
    """model.py:43-60."""

    def __init__(self, in_channels, out_channels, kernel_size, frn=False):
        super().__init__()
        self.branch = nn.Sequential(
            ConvNormLayer(in_channels, out_channels, kernel_size, 1, frn=frn),
            ConvNormLayer(out_channels, out_channels, kernel_size, 1, activation=False, frn=frn))
        self.activation = TLU(out_channels) if frn else nn.ReLU(inplace=True)


class ConvTanhLayer(nn.Module):
    """model.py:63-72."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.layers = nn.Sequential(ConvLayer(in_channels, out_channels, kernel_size, stride), nn.Tanh())


class Encoder(nn.Module):
    def __init__(self, frn=False):
        super().__init__()
        self.layers = nn.Sequential(
            ConvNormLayer(3, 48, 9, 1, frn=frn), ConvNormLayer(48, 96, 3, 2, frn=frn),
            ConvNormLayer(96, 192, 3, 2, frn=frn),
            ResLayer(192, 192, 3, frn=frn), ResLayer(192, 192, 3, frn=frn),
            ResLayer(192, 192, 3, frn=frn), ResLayer(192, 192, 3, frn=frn))


class Decoder(nn.Module):
    def __init__(self, frn=False):
        super().__init__()
        self.layers = nn.Sequential(
            nn.Upsample(scale_factor=2), ConvNormLayer(192, 96, 3, 1, frn=frn),
            nn.Upsample(scale_factor=2), ConvNormLayer(96, 48, 3, 1, frn=frn),
            ConvTanhLayer(48, 3, 9, 1))


class ReCoNet(StylizationNet):
    ARCH = NST_ARCH_RECONET

    def __init__(self, frn=False):
        super().__init__()
        if frn:
            self.ARCH = NST_ARCH_RECONET_FRN
        self.encoder = Encoder(frn=frn)
        self.decoder = Decoder(frn=frn)
