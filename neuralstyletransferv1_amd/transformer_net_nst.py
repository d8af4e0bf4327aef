"""NST_Train TransformerNet — drop-in for the reference's transformer_net_nst.py.

Same submodule names/shapes as transformer_net_nst.py:12-127 (`down1.conv.weight`, ...,
`up1.conv.weight` [ConvTranspose2d: in,out,3,3], `final.weight`).  Forward semantics
(transformer_net_nst.py:95-127): ReflectionPad2d(40) -> zero-padded convs -> 5 residual
blocks -> two ConvTranspose2d(3, s2, p1, op1) + IN + ReLU -> 9x9 conv -> centre crop to HxW;
all fused into libnst_hip kernels (the pad-40 reflection and the crop are address maps).
"""
from torch import nn

from ._lib import NST_ARCH_NST
from .engine import StylizationNet


class ConvBlock(nn.Module):
    """transformer_net_nst.py:12-25: Conv2d(padding=k//2) + InstanceNorm2d(affine) + ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding=None):
        super().__init__()
        if padding is None:
            padding = kernel_size // 2
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding)
        self.norm = nn.InstanceNorm2d(out_channels, affine=True)


class ResidualBlock(nn.Module):
    """transformer_net_nst.py:28-43."""

    def __init__(self, channels):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, 3, stride=1, padding=1)
        self.norm1 = nn.InstanceNorm2d(channels, affine=True)
        self.conv2 = nn.Conv2d(channels, channels, 3, stride=1, padding=1)
        self.norm2 = nn.InstanceNorm2d(channels, affine=True)


class UpsampleBlock(nn.Module):
    """transformer_net_nst.py:46-59: ConvTranspose2d + IN + ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, output_padding):
        super().__init__()
        self.conv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                                       output_padding=output_padding)
        self.norm = nn.InstanceNorm2d(out_channels, affine=True)


class TransformerNet(StylizationNet):
    ARCH = NST_ARCH_NST
    PAD = 40  # ReflectionPad2d(40), transformer_net_nst.py:74

    def __init__(self):
        super().__init__()
        self.down1 = ConvBlock(3, 32, kernel_size=9, stride=1)
        self.down2 = ConvBlock(32, 64, kernel_size=3, stride=2)
        self.down3 = ConvBlock(64, 128, kernel_size=3, stride=2)
        for i in range(1, 6):
            setattr(self, f"res{i}", ResidualBlock(128))
        self.up1 = UpsampleBlock(128, 64, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.up2 = UpsampleBlock(64, 32, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.final = nn.Conv2d(32, 3, kernel_size=9, stride=1, padding=4)
