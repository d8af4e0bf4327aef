"""Johnson fast-style TransformerNet — drop-in for the reference's transformer_net.py.

Same constructor (no arguments), submodule names and parameter shapes as
transformer_net.py:4-99, so `.pth` checkpoints (candy/mosaic/rain_princess/udnie) load
unchanged; `forward` runs the whole net as libnst_hip kernels (see engine.py).
Architecture (transformer_net.py:29-41): 9x9 conv 3->32, 3x3/s2 32->64, 3x3/s2 64->128
(each ReflectionPad + InstanceNorm(affine) + ReLU), 5 residual blocks (no ReLU after the add),
two nearest-x2-upsample 3x3 convs 128->64->32 (IN + ReLU), 9x9 conv 32->3.
"""
from torch import nn

from ._lib import NST_ARCH_JOHNSON
from .engine import StylizationNet


class ConvLayer(nn.Module):
    """transformer_net.py:44-54 — reflection pad (kernel//2) is fused into the conv kernel."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride)


class UpsampleConvLayer(ConvLayer):
    """transformer_net.py:79-99 — nearest x2 upsample folded into the conv's input addressing."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, upsample=None):
        super().__init__(in_channels, out_channels, kernel_size, stride)
        self.upsample = upsample


class ResidualBlock(nn.Module):
    """transformer_net.py:57-76: conv-IN-ReLU-conv-IN, + residual."""

    def __init__(self, channels):
        super().__init__()
        self.conv1 = ConvLayer(channels, channels, kernel_size=3, stride=1)
        self.in1 = nn.InstanceNorm2d(channels, affine=True)
        self.conv2 = ConvLayer(channels, channels, kernel_size=3, stride=1)
        self.in2 = nn.InstanceNorm2d(channels, affine=True)


class TransformerNet(StylizationNet):
    ARCH = NST_ARCH_JOHNSON

    def __init__(self):
        super().__init__()
        self.conv1 = ConvLayer(3, 32, kernel_size=9, stride=1)
        self.in1 = nn.InstanceNorm2d(32, affine=True)
        self.conv2 = ConvLayer(32, 64, kernel_size=3, stride=2)
        self.in2 = nn.InstanceNorm2d(64, affine=True)
        self.conv3 = ConvLayer(64, 128, kernel_size=3, stride=2)
        self.in3 = nn.InstanceNorm2d(128, affine=True)
        for i in range(1, 6):
            setattr(self, f"res{i}", ResidualBlock(128))
        self.deconv1 = UpsampleConvLayer(128, 64, kernel_size=3, stride=1, upsample=2)
        self.in4 = nn.InstanceNorm2d(64, affine=True)
        self.deconv2 = UpsampleConvLayer(64, 32, kernel_size=3, stride=1, upsample=2)
        self.in5 = nn.InstanceNorm2d(32, affine=True)
        self.deconv3 = ConvLayer(32, 3, kernel_size=9, stride=1)
