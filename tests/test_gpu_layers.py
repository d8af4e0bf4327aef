"""Teacher-forced per-layer parity of the 16-bit paths, bf16 (throughput) and fp16 (the benchmarked kernels).

Every op of the program is recomputed on the CPU from the engine's own stored input (captured by
nst_forward_capture) with the bf16 mode's rounding points (oracle/bf16_layers.py), so each kernel
is checked alone: conv_ws9 (first layer), conv_ws2 (down-convs), conv_wstat (residual trunk, plain
and with the fused residual join), conv_wphase (x2 up-convs), conv_out9 (output conv + decode +
truncation), and on ReCoNet (InstanceNorm and FRN/TLU) the generic bf16 kernels.  Bars (tests/layer_check.py): stored bf16
outputs within 1 bf16 ulp (or 4e-6 of the layer's max |value| where the sum cancels), <= 0.1 % of
elements 1 ulp off (measured <= 0.03 %), IN statistics within 1e-5, joined residual streams bit-exact, raw fp32 output
within 5e-6, u8 frames >= 99.99 % identical and never more than 1 LSB off.
"""
import numpy as np
import pytest
import torch

import layer_check as LC
from neuralstyletransferv1_amd import synthetic

pytestmark = pytest.mark.gpu


def _net(arch, seed, dtype="bf16"):
    m = synthetic.build_module(arch)
    m.load_state_dict(synthetic.make_state_dict(arch, seed))
    m = m.to("cuda").eval()
    if dtype == "fp16m2":  # NST_DT_F16M with residual blocks 1 and 2 split (NST_KSEL_F16M_TWO_BLOCKS)
        dtype = "fp16m"
        m.kernel_select = frozenset(["f16m_two_blocks"])
    m.compute_dtype = dtype
    return m


def _report(recs):
    for r in recs:
        print({k: (round(v, 7) if isinstance(v, float) else v) for k, v in r.items()})


@pytest.mark.parametrize("arch,n,h,w,preset", [
    ("johnson", 2, 70, 90, "imagenet_255"),   # ragged tiles everywhere, output fit (72x92 conv output)
    ("johnson", 1, 33, 47, "caffe_bgr"),      # frame narrower than one first-layer tile's halo
    ("johnson", 1, 64, 96, "imagenet_255"),   # u8 output path (output size == input size)
    ("nst", 1, 72, 100, "raw_01"),            # zero padding, pre-reflect 40, ConvTranspose phases, crop
    ("reconet", 1, 61, 90, "tanh"),           # 48/96/192 channels: generic bf16 kernels + tanh output
    ("reconet_frn", 1, 61, 90, "tanh"),       # FRN + TLU: mean-square statistics, tau folded into biases / shifts
])
@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp16m", "fp16m2"])
def test_16bit_layers_small(arch, n, h, w, preset, dtype):
    if dtype.startswith("fp16m") and arch.startswith("reconet"):
        pytest.skip("NST_DT_F16M is built for the Johnson / NST nets")
    frames = synthetic.make_frames(n, h, w, seed=40 + h)
    recs = LC.check_layers(_net(arch, 11, dtype), frames, preset, acc=torch.float64)
    _report(recs)
    # fp16m: the split residual blocks run unfused (+1 op: the join writing the fp16 stream; two blocks: +2, the
    # first join writing x_1 in fp32)
    extra = {"fp16m": 1, "fp16m2": 2}.get(dtype, 0)
    assert len(recs) == (14 if arch.startswith("reconet") else 16) + extra
    if extra:  # the split-precision head: ~22-bit products (measured rel error reported)
        assert sum(1 for r in recs if "split_rel" in r) == 3 + 2 * extra


def test_bf16_layers_1080p():
    """configs[1]'s frame size, every output row of every layer."""
    frames = synthetic.make_frames(1, 1080, 1920, seed=1000)
    recs = LC.check_layers(_net("johnson", 0), frames, "imagenet_255")
    _report(recs)
    modes = {r["layer"]: r["mode"] for r in recs}
    # the benchmarked kernels are the ones checked: ws9, ws2, wstat, wphase, out9
    assert modes["conv1.conv2d"] == 7 and modes["conv2.conv2d"] == 6 and modes["res3.conv1.conv2d"] == 4
    assert modes["deconv1.conv2d"] == 5 and modes["deconv3.conv2d"] == 3


def test_fp16_layers_1080p():
    """fp16 mode at configs[1]'s frame size, every output row of every layer; each layer's largest
    stored |value| is reported (the fp16 range check: stored conv outputs must stay below 65504)."""
    frames = synthetic.make_frames(1, 1080, 1920, seed=1000)
    recs = LC.check_layers(_net("johnson", 0, "fp16"), frames, "imagenet_255")
    _report(recs)
    assert max(r.get("absmax", 0.0) for r in recs) < 65504


def test_fp16m_layers_1080p():
    """NST_DT_F16M at configs[1]'s frame size: the split-precision head (first layer, down-convs, first residual
    block: fp32 outputs against the conv of the same operand, exact / with the fp16 weights), the join and the fp16
    trunk / up-convs / output conv, every output row of every layer."""
    frames = synthetic.make_frames(1, 1080, 1920, seed=1000)
    recs = LC.check_layers(_net("johnson", 0, "fp16m"), frames, "imagenet_255")
    _report(recs)
    modes = {r["layer"]: r["mode"] for r in recs}
    assert modes["conv1.conv2d"] == 7 and modes["conv2.conv2d"] == 6 and modes["conv3.conv2d"] == 6
    assert modes["res1.conv1.conv2d"] == 8 and modes["res1.conv2.conv2d"] == 8 and modes["res2.conv1.conv2d"] == 4
    assert modes["res3.conv1.conv2d"] == 4 and modes["deconv1.conv2d"] == 5 and modes["deconv3.conv2d"] == 3
    assert max(r.get("split_rel", 0.0) for r in recs) <= LC.SPLIT_REL


def test_bf16_layers_4k_bands():
    """configs[3]'s 3840x2160 frame: every layer on its first, middle and last 16 output rows
    (all columns, so the first and last tile columns too)."""
    frames = synthetic.make_frames(1, 2160, 3840, seed=2000)
    recs = LC.check_layers(_net("johnson", 0), frames, "imagenet_255", bands=[(0.0, 16), (0.5, 16), (1.0, 16)])
    _report(recs)
    assert all(r["elements"] > 0 for r in recs)
