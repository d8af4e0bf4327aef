"""ReCoNet — drop-in for the reference's model.py (imported by pipeline.py via `from lib import ReCoNet`).

Same nested nn.Sequential names as model.py:5-116 (`encoder.layers.0.layers.0.layers.1.weight`, ...).
Encoder: 9x9 3->48, 3x3/s2 48->96, 3x3/s2 96->192 (reflect pad, IN, ReLU), 4 ResLayers with
ReLU AFTER the residual add (model.py:55-60); Decoder: nearest x2 -> 3x3 192->96, nearest x2 ->
3x3 96->48 (IN, ReLU), 9x9 48->3 + Tanh.  Runs as libnst_hip kernels.  Only the InstanceNorm
variant the pipeline builds (`ReCoNet()`, frn=False, pipeline.py:602) has an engine path.
"""
from torch import nn

from ._lib import NST_ARCH_RECONET, NstError
from .engine import StylizationNet


class ConvLayer(nn.Module):
    """model.py:5-15: Sequential(ReflectionPad2d, Conv2d) — index 1 holds the conv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.layers = nn.Sequential(nn.ReflectionPad2d(kernel_size // 2),
                                    nn.Conv2d(in_channels, out_channels, kernel_size, stride))


class ConvNormLayer(nn.Module):
    """model.py:18-40 (InstanceNorm variant): Sequential(ConvLayer, InstanceNorm2d[, ReLU])."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, activation=True, frn=False):
        super().__init__()
        if frn:
            raise NstError("ReCoNet(frn=True) has no engine path (the pipeline builds frn=False)")
        layers = [ConvLayer(in_channels, out_channels, kernel_size, stride),
                  nn.InstanceNorm2d(out_channels, affine=True)]
        if activation:
            layers.append(nn.ReLU(inplace=True))
        self.layers = nn.Sequential(*layers)


class ResLayer(nn.Module):
    """model.py:43-60."""

    def __init__(self, in_channels, out_channels, kernel_size, frn=False):
        super().__init__()
        self.branch = nn.Sequential(
            ConvNormLayer(in_channels, out_channels, kernel_size, 1, frn=frn),
            ConvNormLayer(out_channels, out_channels, kernel_size, 1, activation=False, frn=frn))
        self.activation = nn.ReLU(inplace=True)


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
        self.encoder = Encoder(frn=frn)
        self.decoder = Decoder(frn=frn)
