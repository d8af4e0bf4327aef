"""Fast lossless PNG writer for styled frames (SURVEY.md §8(f)4 frame I/O).

The reference saves every styled frame with Pillow's PNG encoder at its defaults (pipeline.py:2099-2119:
`Image.fromarray(...).save(path)`, zlib level 6 with per-row adaptive filter selection).  On 1080p frames that
encoder is the CLI's bottleneck (≈0.5-0.75 s of one core per frame on noisy content).  PNG is lossless, so any
valid encoder yields the same pixels; this one writes

  * every scanline with the "Up" filter (type 2: byte minus the byte above; vectorised in numpy, one pass),
  * one IDAT holding a zlib stream deflated with Z_RLE (run-length matches + Huffman coding: the flat regions of
    a frame collapse into runs of zeros after the Up filter), level 1,
  * IHDR (8-bit RGB, no interlace) and IEND; no ancillary chunks (Pillow writes none for these frames either).

File sizes land within a few percent of Pillow's level-6 files; decoding returns the identical uint8 array
(tests/test_host.py checks with Pillow).  zlib releases the GIL while it deflates, so a thread pool scales.

`encode_png_gpu` builds the same kind of file on the GPU (csrc/png_enc.hip, nst_png_encode_u8): Up filter, one
deflate block per scanline with dynamic Huffman codes built per frame from its run-length tokens (a stored block
where that is smaller), Adler-32 and CRC-32 on the device.  The owner rank copies finished files to the host and
only writes bytes (`--png_writer gpu`).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_SIG = b"\x89PNG\r\n\x1a\n"


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(data, zlib.crc32(kind)) & 0xFFFFFFFF)


def encode_png(rgb: np.ndarray, level: int = 1) -> bytes:
    """uint8 HxWx3 (or HxW grey) -> PNG bytes."""
    a = np.ascontiguousarray(rgb)
    if a.dtype != np.uint8 or a.ndim not in (2, 3) or (a.ndim == 3 and a.shape[2] not in (3, 4)):
        raise ValueError(f"encode_png: need uint8 HxW, HxWx3 or HxWx4, got {a.dtype} {a.shape}")
    h, w = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    color = {1: 0, 3: 2, 4: 6}[ch]
    rows = a.reshape(h, w * ch)
    filt = np.empty((h, 1 + w * ch), np.uint8)
    filt[:, 0] = 2  # Up
    filt[0, 1:] = rows[0]
    np.subtract(rows[1:], rows[:-1], out=filt[1:, 1:])  # uint8 wrap-around = the filter's mod-256 difference
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, zlib.Z_RLE)
    idat = co.compress(filt) + co.flush()
    ihdr = struct.pack(">IIBBBBB", w, h, 8, color, 0, 0, 0)
    return _SIG + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", idat) + _chunk(b"IEND", b"")


def write_png(path, rgb: np.ndarray, level: int = 1) -> None:
    data = encode_png(rgb, level)
    with open(path, "wb") as f:
        f.write(data)


_png_ws = {}  # (device, n, h, w, c) -> workspace tensor, reused across groups


def encode_png_gpu(frames_u8):
    """uint8 frames [n,h,w,c] (c in 1, 3, 4) on an MI355X -> (files [n, stride] uint8, sizes [n] int64), both on
    the device, on the current stream: file j is files[j, :sizes[j]].  No CPU path: the library must be loaded."""
    import ctypes

    import torch

    from . import _lib
    _lib.require_gpu_tensor(frames_u8, "encode_png_gpu frames")
    x = frames_u8 if frames_u8.dim() == 4 else frames_u8[..., None]
    if x.dtype != torch.uint8 or x.dim() != 4:
        raise ValueError(f"encode_png_gpu: need uint8 [n,h,w,c], got {frames_u8.dtype} {tuple(frames_u8.shape)}")
    x = x.contiguous()
    n, h, w, c = x.shape
    L = _lib.lib()
    bound, wsb = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(L.nst_png_bound(h, w, c, ctypes.byref(bound)), "nst_png_bound")
    _lib.check(L.nst_png_workspace_bytes(n, h, w, c, ctypes.byref(wsb)), "nst_png_workspace_bytes")
    key = (x.device, n, h, w, c)
    ws = _png_ws.get(key)
    if ws is None:
        if len(_png_ws) > 4:
            _png_ws.clear()
        ws = _png_ws[key] = torch.empty(wsb.value, dtype=torch.uint8, device=x.device)
    files = torch.empty((n, bound.value), dtype=torch.uint8, device=x.device)
    sizes = torch.empty(n, dtype=torch.int64, device=x.device)
    _lib.check(L.nst_png_encode_u8(x.data_ptr(), n, h, w, c, files.data_ptr(), bound.value, sizes.data_ptr(),
                                   ws.data_ptr(), wsb.value, _lib.stream_ptr(x.device)), "nst_png_encode_u8")
    ws.record_stream(torch.cuda.current_stream(x.device))
    return files, sizes


def png_bytes_gpu(frames_u8) -> list:
    """encode_png_gpu, copied to the host: one bytes object (a complete PNG file) per frame."""
    files, sizes = encode_png_gpu(frames_u8)
    sz = sizes.cpu().tolist()
    host = files.cpu().numpy()
    return [host[j, :sz[j]].tobytes() for j in range(len(sz))]
