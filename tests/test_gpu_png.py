"""GPU PNG encoder (csrc/png_enc.hip, nst_png_encode_u8) replacing the host's Image.fromarray(out).save(path)
(/root/reference/pipeline.py:2099-2119; PNG is the default --image_ext, :2170).  PNG is lossless, so the bar is the
decoded pixels: every file must decode to the frame's exact bytes through zlib (Adler-32 checked by zlib), with
every chunk CRC-32 recomputed here, and through Pillow (the reference's decoder, also its --input_dir reader)."""
import ctypes
import io
import struct
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

from neuralstyletransferv1_amd import _lib, pngio, synthetic


def _chunks(data: bytes):
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    p, out = 8, []
    while p < len(data):
        n, = struct.unpack(">I", data[p:p + 4])
        kind, body = data[p + 4:p + 8], data[p + 8:p + 8 + n]
        crc, = struct.unpack(">I", data[p + 8 + n:p + 12 + n])
        assert crc == zlib.crc32(kind + body) & 0xFFFFFFFF, kind
        out.append((kind, body))
        p += 12 + n
    assert p == len(data)
    return out


def _decode_strict(data: bytes) -> np.ndarray:
    """chunk CRCs, IHDR, the zlib stream (zlib checks the Adler-32), the Up filter undone in numpy"""
    ch = _chunks(data)
    assert [k for k, _ in ch] == [b"IHDR", b"IDAT", b"IEND"]
    w, h, depth, color, comp, filt, inter = struct.unpack(">IIBBBBB", ch[0][1])
    assert (depth, comp, filt, inter) == (8, 0, 0, 0)
    c = {0: 1, 2: 3, 6: 4}[color]
    raw = zlib.decompress(ch[1][1])
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + w * c)
    assert (rows[:, 0] == 2).all()
    img = np.cumsum(rows[:, 1:].astype(np.uint64), axis=0, dtype=np.uint64).astype(np.uint8)  # mod-256 prefix sums
    return img.reshape(h, w, c) if c > 1 else img.reshape(h, w)


def _frames(kind: str, n: int, h: int, w: int, c: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, (n, h, w, c), dtype=np.uint8)
    if kind == "flat":  # long runs: 258-byte matches back to back, length codes of every size
        a = np.zeros((n, h, w, c), np.uint8)
        a[:, :, : w // 2] = 7
        a[:, h // 3:, :, 0] = 200
        return a
    if kind == "bands":  # runs of every length 1..300 within each scanline
        a = np.zeros((n, h, w * c), np.uint8)
        x, v = 0, 0
        while x < w * c:
            L = int(rng.integers(1, 300))
            a[:, :, x:x + L] = v
            x, v = x + L, (v + 37) % 256
        a[:, 1::2] = a[:, 1::2] ^ 1
        return a.reshape(n, h, w, c)
    f = synthetic.make_frames(n, h, w, seed=seed)  # smooth gradients + shapes + noise
    return f if c == 3 else np.ascontiguousarray(np.repeat(f[..., :1], c, axis=-1))


def test_png_bound_and_workspace_validate_without_gpu():
    L = _lib.lib()
    v = ctypes.c_size_t()
    assert L.nst_png_bound(1080, 1920, 3, ctypes.byref(v)) == 0
    assert v.value >= 8 + 25 + 12 + 2 + 1080 * (1920 * 3 + 6) + 2 + 4 + 12
    assert L.nst_png_bound(1080, 1920, 2, ctypes.byref(v)) == -1
    assert L.nst_png_bound(4, 30000, 3, ctypes.byref(v)) == -1  # a stored scanline block holds <= 65535 bytes
    assert L.nst_png_workspace_bytes(0, 8, 8, 3, ctypes.byref(v)) == -1
    assert L.nst_png_encode_u8(None, 1, 8, 8, 3, None, 0, None, None, 0, None) == -1


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,h,w,c", [
    ("synthetic", 3, 64, 96, 3),      # 16-byte rows: the dwordx4 walk
    ("synthetic", 2, 37, 51, 3),      # ragged rows: the byte walk
    ("noise", 2, 40, 64, 3),          # dynamic blocks larger than stored: the stored fallback
    ("flat", 2, 70, 200, 3),
    ("bands", 2, 9, 512, 3),
    ("synthetic", 2, 33, 40, 1),
    ("synthetic", 1, 20, 36, 4),
    ("flat", 1, 1, 1, 3),
    ("noise", 1, 130, 7, 1),          # the header alone outweighs every scanline
    ("noise", 1, 2, 65534, 1),        # the widest scanline: a 65,535-byte stored block (LEN = 0xffff)
    ("synthetic", 1, 2160, 3840, 3),  # 4K (configs[3])
])
def test_gpu_png_decodes_to_the_frames(kind, n, h, w, c):
    fr = _frames(kind, n, h, w, c, seed=h * w + c)
    files = pngio.png_bytes_gpu(torch.from_numpy(fr).cuda())
    assert len(files) == n
    for j, data in enumerate(files):
        want = fr[j] if c > 1 else fr[j, ..., 0]
        assert np.array_equal(_decode_strict(data), want), j
        im = Image.open(io.BytesIO(data))
        im.load()
        assert np.array_equal(np.asarray(im), want), j


@pytest.mark.gpu
def test_gpu_png_1080p_batch_and_size():
    """the bench shape: 8 distinct 1080p frames in one call; files decode exactly and compress (smooth content)"""
    fr = synthetic.make_frames(8, 1080, 1920, seed=300)
    x = torch.from_numpy(fr).cuda()
    files = pngio.png_bytes_gpu(x)
    for j, data in enumerate(files):
        assert np.array_equal(_decode_strict(data), fr[j]), j
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(files[0]))), fr[0])
    raw = 1080 * (1920 * 3 + 1)
    ratio = np.mean([len(d) for d in files]) / raw
    host = np.mean([len(pngio.encode_png(f)) for f in fr[:2]]) / raw
    print(f"gpu png size / raw {ratio:.3f}, host Z_RLE writer {host:.3f}")
    assert ratio < 1.0
    # repeatable: the same frames give the same bytes (no order-dependent atomics reach the output)
    again = pngio.png_bytes_gpu(x)
    assert again == files


@pytest.mark.gpu
def test_gpu_png_styled_output_through_the_engine():
    """a stylized batch (the CLI's real input to the writer) through the encoder equals Pillow's decode of itself"""
    from neuralstyletransferv1_amd.transformer_net import TransformerNet
    net = TransformerNet()
    net.load_state_dict(synthetic.make_state_dict("johnson", 0))
    net = net.cuda().eval()
    net.compute_dtype = "bf16"
    eng = net.engine(torch.device("cuda", 0))
    out = eng.stylize_u8(torch.from_numpy(synthetic.make_frames(2, 136, 240, seed=9)).cuda(), "imagenet_255")
    files = pngio.png_bytes_gpu(out)
    host = out.cpu().numpy()
    for j, data in enumerate(files):
        assert np.array_equal(np.asarray(Image.open(io.BytesIO(data))), host[j])


@pytest.mark.gpu
def test_gpu_png_rejects_small_workspace_and_stride():
    x = torch.zeros((1, 8, 8, 3), dtype=torch.uint8, device="cuda")
    L = _lib.lib()
    bound, wsb = ctypes.c_size_t(), ctypes.c_size_t()
    assert L.nst_png_bound(8, 8, 3, ctypes.byref(bound)) == 0
    assert L.nst_png_workspace_bytes(1, 8, 8, 3, ctypes.byref(wsb)) == 0
    out = torch.empty(bound.value, dtype=torch.uint8, device="cuda")
    sizes = torch.empty(1, dtype=torch.int64, device="cuda")
    ws = torch.empty(wsb.value, dtype=torch.uint8, device="cuda")
    args = (x.data_ptr(), 1, 8, 8, 3, out.data_ptr())
    assert L.nst_png_encode_u8(*args, bound.value, sizes.data_ptr(), ws.data_ptr(), wsb.value - 1, None) == -5
    assert L.nst_png_encode_u8(*args, bound.value - 16, sizes.data_ptr(), ws.data_ptr(), wsb.value, None) == -1
    assert L.nst_png_encode_u8(*args, bound.value, sizes.data_ptr(), ws.data_ptr(), wsb.value, None) == 0
    torch.cuda.synchronize()
