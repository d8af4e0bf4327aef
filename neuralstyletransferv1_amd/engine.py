"""Engine handle + the nn.Module base class shared by the three stylization nets.

`StylizationNet` keeps the reference's Module surface (`Net()`, `.to(device)`,
`.load_state_dict(sd, strict=False)`, `.eval()`, `net(X)`), so the reference's callers
(pipeline.py:597-619 model load, :1449-1485 `model(x_in)`) work unchanged, but its
parameters are only containers: `forward` packs them once into a libnst_hip handle and
runs the whole network as hand-written HIP kernels on the caller's stream.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import torch
from torch import nn

from . import _lib
from ._lib import NstError, NstParam, check, lib

_DTYPES = {"fp32": _lib.NST_DT_F32, "float32": _lib.NST_DT_F32, "bf16": _lib.NST_DT_BF16, "bfloat16": _lib.NST_DT_BF16,
           "fp16": _lib.NST_DT_F16, "float16": _lib.NST_DT_F16, "fp32s": _lib.NST_DT_F32S, "fp16m": _lib.NST_DT_F16M}


class Engine:
    """One packed checkpoint on one device (owns an nst_handle and a reusable workspace)."""

    def __init__(self, arch: int, state: Dict[str, torch.Tensor], dtype: str, device: torch.device,
                 kernel_flags: int = 0):
        if device.type != "cuda":
            raise NstError("libnst_hip runs on MI355X (cuda) devices only; there is no CPU path")
        self.arch = arch
        self.dtype = _DTYPES[dtype]
        self.device = device
        host = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in state.items()}
        names = list(host.keys())
        arr = (NstParam * len(names))()
        self._keep = []
        for i, k in enumerate(names):
            b = k.encode()
            self._keep.append(b)
            arr[i].name = b
            arr[i].data = ctypes.cast(host[k].data_ptr(), ctypes.POINTER(ctypes.c_float))
            arr[i].numel = host[k].numel()
        h = ctypes.c_void_p()
        dev_index = device.index if device.index is not None else torch.cuda.current_device()
        check(lib().nst_create_ex(arch, arr, len(names), self.dtype, dev_index, kernel_flags, ctypes.byref(h)),
              "nst_create")
        self._h = h
        self._keep = None
        self._ws: Optional[torch.Tensor] = None
        # NST_DT_F16M's +-1 LSB bar rests on an exact first-layer operand (the io_preset encode folded into the
        # first layer's weights over raw bytes); inputs where that fold does not hold (float32 tensors, a
        # zero-padded first layer with an offset preset, no_fold) run on an NST_DT_F32S twin of the same weights
        self._f16m_src = (host, kernel_flags) if self.dtype == _lib.NST_DT_F16M else None
        self._twin: Optional["Engine"] = None
        self._exact: Dict[Tuple[int, int], bool] = {}
        # NST_RANGE_CHECK=1: every forward checks for values that left the compute dtype's range (NST_E_RANGE; a
        # synchronising debug aid for the fp16 / split modes, off by default).  Set once here; set_range_check
        # overrides it and carries over to the fp32s twin
        self._range_check = False
        if os.environ.get("NST_RANGE_CHECK", "0") == "1":
            self.set_range_check(True)

    def _for_input(self, x_fmt: int, pid: int) -> "Engine":
        """The engine that runs this input format and preset: self, or the fp32s twin (see __init__)."""
        if self._f16m_src is None:
            return self
        key = (x_fmt, pid)
        if key not in self._exact:
            ex = ctypes.c_int()
            check(lib().nst_input_exact(self._h, x_fmt, pid, ctypes.byref(ex)), "nst_input_exact")
            self._exact[key] = bool(ex.value)
        if self._exact[key]:
            return self
        if self._twin is None:
            host, flags = self._f16m_src
            self._twin = Engine(self.arch, host, "fp32s", self.device, flags & ~_lib.KSEL["f16m_two_blocks"])
            self._twin.set_range_check(self._range_check)  # the parent's current setting
        return self._twin

    def forward_into(self, x: torch.Tensor, x_fmt: int, n: int, h: int, w: int, pid: int, y: torch.Tensor,
                     y_fmt: int) -> None:
        """nst_forward of a device batch into y on the current stream (workspace managed here), on the engine
        that holds this mode's bar for the input (_for_input)."""
        e = self._for_input(x_fmt, pid)
        ws = e.workspace(n, h, w)
        check(lib().nst_forward(e._h, x.data_ptr(), x_fmt, n, h, w, pid, y.data_ptr(), y_fmt, ws.data_ptr(),
                                ws.numel(), _lib.stream_ptr(self.device)), "nst_forward")

    def set_range_check(self, enable: bool) -> None:
        """nst_set_range_check on this engine and on its fp32s twin (inputs routed to the twin are checked too)."""
        self._range_check = bool(enable)
        check(lib().nst_set_range_check(self._h, 1 if enable else 0), "nst_set_range_check")
        if self._twin is not None:
            self._twin.set_range_check(enable)

    def set_stream_split(self, k: int) -> None:
        """nst_set_stream_split: run each batch as k sub-batches on the library's internal streams (1 = whole)."""
        check(lib().nst_set_stream_split(self._h, int(k)), "nst_set_stream_split")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().nst_destroy(h)
            except Exception:
                pass
            self._h = None

    def layer_names(self):
        return [lib().nst_layer_name(self._h, i).decode() for i in range(lib().nst_num_layers(self._h))]

    def profile_begin(self) -> None:
        check(lib().nst_profile_begin(self._h), "nst_profile_begin")

    def profile_end(self):
        """-> list of (layer_name, total_ms, launches); call after synchronising the stream."""
        names = self.layer_names()
        n = len(names)
        ms = (ctypes.c_float * n)()
        cnt = (ctypes.c_int * n)()
        check(lib().nst_profile_end(self._h, n, ms, cnt), "nst_profile_end")
        return [(names[i], float(ms[i]), int(cnt[i])) for i in range(n)]

    def output_hw(self, h: int, w: int) -> Tuple[int, int]:
        oh, ow = ctypes.c_int(), ctypes.c_int()
        check(lib().nst_output_hw(self._h, h, w, ctypes.byref(oh), ctypes.byref(ow)), "nst_output_hw")
        return oh.value, ow.value

    def workspace(self, n: int, h: int, w: int) -> torch.Tensor:
        """The cached workspace, grown on demand.  It is handed to kernels on whichever stream is
        current, so it is recorded on that stream (the caching allocator then never reuses its bytes
        while work queued there may still touch them, also after it is replaced)."""
        need = ctypes.c_size_t()
        check(lib().nst_workspace_bytes(self._h, n, h, w, ctypes.byref(need)), "nst_workspace_bytes")
        if self._ws is None or self._ws.numel() < need.value:
            self._ws = torch.empty(max(need.value, 256), dtype=torch.uint8, device=self.device)
        self._ws.record_stream(torch.cuda.current_stream(self.device))
        return self._ws

    def op_descs(self, n: int, h: int, w: int):
        """Wiring and geometry of every op of the handle's program (nst_op_describe)."""
        out = []
        for i in range(lib().nst_num_ops(self._h)):
            d = _lib.NstOpDesc()
            check(lib().nst_op_describe(self._h, n, h, w, i, ctypes.byref(d)), "nst_op_describe")
            out.append(d.as_dict())
        return out

    def forward_capture(self, x: torch.Tensor, x_fmt: str, preset: str, y_fmt: str):
        """nst_forward_capture: run the batch and return (y, ops, captures); captures[i] =
        {"act": raw conv output of op i [n,oh,ow,cout_stride] (bf16/fp32), "res": joined residual
        stream it wrote or None, "stats": [n,cout_stride,2] fp32 {scale, shift} or None}."""
        _lib.require_gpu_tensor(x, "input")
        x = x.contiguous()
        if x_fmt == "u8":
            n, h, w, _ = x.shape
            xf = _lib.NST_IO_U8_NHWC
        else:
            n, _, h, w = x.shape
            xf = _lib.NST_IO_F32_NCHW
        oh, ow = self.output_hw(h, w)
        if y_fmt == "u8":
            y = torch.empty((n, oh, ow, 3), dtype=torch.uint8, device=self.device)
            yf = _lib.NST_IO_U8_NHWC
        else:
            y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=self.device)
            yf = _lib.NST_IO_F32_NCHW
        ops = self.op_descs(n, h, w)
        half = torch.bfloat16 if self.dtype == _lib.NST_DT_BF16 else torch.float16

        def dt_of(esz):  # a 2-byte activation is the handle's 16-bit format, a 4-byte one fp32
            return torch.float32 if esz == 4 else half
        caps = []
        k = len(ops)
        act, res, st = (ctypes.c_void_p * k)(), (ctypes.c_void_p * k)(), (ctypes.c_void_p * k)()
        for i, d in enumerate(ops):
            c = {"act": None, "res": None, "stats": None}
            if d["dst"] != _lib.NST_BUF_OUTPUT:
                c["act"] = torch.empty((n, d["out_h"], d["out_w"], d["cout_stride"]), dtype=dt_of(d["elem_bytes"]),
                                       device=self.device)
                act[i] = c["act"].data_ptr()
                if d["kind"] == 0:
                    c["stats"] = torch.empty((n, d["cout_stride"], 2), dtype=torch.float32, device=self.device)
                    st[i] = c["stats"].data_ptr()
                if d["res_out"] >= 0:
                    c["res"] = torch.empty((n, d["in_h"], d["in_w"], d["cin_stride"]), dtype=dt_of(d["res_elem_bytes"]),
                                           device=self.device)
                    res[i] = c["res"].data_ptr()
            caps.append(c)
        ws = self.workspace(n, h, w)
        check(lib().nst_forward_capture(self._h, x.data_ptr(), xf, n, h, w, _lib.PRESETS[preset], y.data_ptr(), yf,
                                        ws.data_ptr(), ws.numel(), act, res, st, _lib.stream_ptr(self.device)),
              "nst_forward_capture")
        return y, ops, caps

    def forward_tensor(self, x: torch.Tensor) -> torch.Tensor:
        """Raw model tensor in, raw model tensor out: [n,3,h,w] fp32 -> [n,3,oh,ow] fp32."""
        _lib.require_gpu_tensor(x, "input")
        if x.dim() != 4 or x.shape[1] != 3:
            raise NstError(f"expected [N,3,H,W] input, got {tuple(x.shape)}")
        x = x.to(self.device, torch.float32).contiguous()
        n, _, h, w = x.shape
        oh, ow = self.output_hw(h, w)
        y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=self.device)
        self.forward_into(x, _lib.NST_IO_F32_NCHW, n, h, w, 0, y, _lib.NST_IO_F32_NCHW)
        return y

    def stylize_u8(self, frames: torch.Tensor, preset: str) -> torch.Tensor:
        """uint8 RGB frames [n,h,w,3] -> stylized uint8 frames [n,h,w,3] (preset, clamp, truncation fused).

        Output is always the content size: when the net's output size differs
        (Johnson/ReCoNet with h or w not divisible by 4) the raw output is decoded and
        bilinearly fitted as pipeline.py:1512-1516 does.
        """
        _lib.require_gpu_tensor(frames, "frames")
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
            raise NstError(f"expected uint8 [N,H,W,3] frames, got {frames.dtype} {tuple(frames.shape)}")
        if preset not in _lib.PRESETS or preset == "none":
            raise NstError(f"unknown io_preset {preset!r}")
        frames = frames.contiguous()
        n, h, w, _ = frames.shape
        oh, ow = self.output_hw(h, w)
        out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=self.device)
        st = _lib.stream_ptr(self.device)
        pid = _lib.PRESETS[preset]
        if (oh, ow) == (h, w):
            self.forward_into(frames, _lib.NST_IO_U8_NHWC, n, h, w, pid, out, _lib.NST_IO_U8_NHWC)
            return out
        y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=self.device)
        self.forward_into(frames, _lib.NST_IO_U8_NHWC, n, h, w, pid, y, _lib.NST_IO_F32_NCHW)
        check(lib().nst_decode_resize_u8(y.data_ptr(), n, oh, ow, pid, out.data_ptr(), h, w, st),
              "nst_decode_resize_u8")
        return out


def capture_u8(engine: "Engine", frames: torch.Tensor, preset: str):
    """HIP-graph capture of engine.stylize_u8(frames, preset) for a loop over fixed input / output buffers (a video
    loop refilling `frames` in place, the benchmark): returns (replay, out) -- replay() re-runs the whole forward (the
    layer launches, IN reductions and decode) as one graph launch into `out`.  The forward is warmed up on a side
    stream first (plans, workspace, persistent-kernel CU counts are host state set up on first use), as
    torch.cuda.graphs requires."""
    dev = frames.device
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            engine.stylize_u8(frames, preset)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = engine.stylize_u8(frames, preset)
    return g.replay, out


class StylizationNet(nn.Module):
    """Base of the drop-in TransformerNet / ReCoNet modules (parameters = containers)."""

    ARCH: int = -1

    def __init__(self):
        super().__init__()
        # "fp32": parity mode (exact-f32 MFMA); "bf16": throughput mode (bf16 MFMA, fp32 accumulate);
        # "fp16": fp16 MFMA at the bf16 rate (11 significant bits); "fp32s": fp32 activations with
        # every conv operand split into an fp16 hi/lo pair (two fp16 MFMAs per K step, ~22 bits): the
        # parity mode's +-1 LSB at a quarter of its MFMA cycles; "fp16m": the split-fp16 arithmetic on the layers
        # whose rounding reaches the frame most (first layer, down-convs, first residual block), fp16 elsewhere:
        # 1080p frames within +-1 LSB at ~3/4 of the fp16 rate (Johnson / NST nets)
        self.compute_dtype = "fp32"
        # kernel selection (names of _lib.KSEL): e.g. {"no_wstat"} runs the residual trunk on the
        # generic kernel instead of the weight-stationary one; empty = the fastest mapping
        self.kernel_select = frozenset()
        self._engines: Dict[Tuple[str, int, str, int], Tuple[tuple, Engine]] = {}

    def _param_key(self) -> tuple:
        return tuple((p.data_ptr(), p._version) for p in self.state_dict().values())

    def engine(self, device: Optional[torch.device] = None, dtype: Optional[str] = None) -> Engine:
        """Packed handle for the current parameters (re-packed after load_state_dict / in-place edits)."""
        if device is None:
            device = next(self.parameters()).device
            if device.type != "cuda":
                raise NstError("move the module (or pass a device) to an MI355X first: there is no CPU path")
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        dtype = dtype or self.compute_dtype
        if dtype not in _DTYPES:
            raise NstError(f"compute_dtype must be fp32, fp32s, fp16m, bf16 or fp16, got {dtype!r}")
        flags = 0
        for name in self.kernel_select:
            if name not in _lib.KSEL:
                raise NstError(f"unknown kernel_select entry {name!r} (known: {sorted(_lib.KSEL)})")
            flags |= _lib.KSEL[name]
        key = (device.type, device.index, dtype, flags)
        pk = self._param_key()
        hit = self._engines.get(key)
        if hit is not None and hit[0] == pk:
            return hit[1]
        eng = Engine(self.ARCH, self.state_dict(), dtype, device, flags)
        self._engines[key] = (pk, eng)
        return eng

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        _lib.require_gpu_tensor(X, "X")
        return self.engine(X.device).forward_tensor(X)

    def stylize_frames(self, frames_u8: torch.Tensor, io_preset: str) -> torch.Tensor:
        """Fused frame path: uint8 [N,H,W,3] on device -> stylized uint8 [N,H,W,3]."""
        _lib.require_gpu_tensor(frames_u8, "frames")
        return self.engine(frames_u8.device).stylize_u8(frames_u8, io_preset)

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda() invalidate packed handles
        self._engines = {}
        return super()._apply(fn, *args, **kwargs)
