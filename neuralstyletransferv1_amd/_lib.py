"""ctypes binding of libnst_hip.so (C ABI declared in include/nst_hip.h).

The product path has no fallback: if the library is missing or cannot be loaded,
`lib()` raises, and every stylization entry point fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime first so libnst_hip binds to the same one)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NST_HIP_LIB", os.path.join(_HERE, "libnst_hip.so"))

NST_OK = 0
NST_ARCH_JOHNSON, NST_ARCH_NST, NST_ARCH_RECONET, NST_ARCH_RECONET_FRN = 0, 1, 2, 3
NST_DT_F32, NST_DT_BF16, NST_DT_F16, NST_DT_F32S, NST_DT_F16M = 0, 1, 2, 3, 4
# kernel dtypes of the NST_DT_F16M split-precision layers (nst_op_desc.kernel_dtype)
NST_KDT_SW_O32, NST_KDT_SW_O16, NST_KDT_SPLIT_O32, NST_KDT_SPLIT_O16, NST_KDT_SPLITO_O32 = 16, 17, 18, 19, 20
NST_VGG_GENERIC_ONLY = 0x1
NST_IO_F32_NCHW, NST_IO_U8_NHWC = 0, 1
PRESETS = {
    "none": 0,
    "tanh": 1,
    "imagenet_01": 2,
    "imagenet_255": 3,
    "caffe_bgr": 4,
    "raw_255": 5,
    "raw_01": 6,
}

# every symbol include/nst_hip.h declares (tests check the library exports all of them)
EXPORTED_SYMBOLS = (
    "nst_last_error", "nst_version", "nst_create", "nst_destroy", "nst_output_hw",
    "nst_workspace_bytes", "nst_forward", "nst_decode_resize_u8", "nst_lab_create",
    "nst_lab_destroy", "nst_lab_ema_u8", "nst_blend_u8", "nst_gram", "nst_profile_begin",
    "nst_profile_end", "nst_num_layers", "nst_layer_name", "nst_blend_models_u8", "nst_blend_models_lab_u8",
    "nst_mask_feather", "nst_create_ex", "nst_num_ops", "nst_op_describe", "nst_forward_capture",
    "nst_gram_workspace_bytes", "nst_vgg_create", "nst_vgg_create_ex", "nst_vgg_destroy", "nst_gatys_buffer_bytes", "nst_vgg_features",
    "nst_gatys_targets", "nst_gatys_grad", "nst_adam_step", "nst_gatys_grad_capture",
    "nst_seg_create", "nst_seg_destroy", "nst_seg_num_classes", "nst_seg_workspace_bytes", "nst_seg_forward",
    "nst_seg_mask_scratch_bytes", "nst_seg_mask", "nst_resize_create", "nst_resize_destroy",
    "nst_resize_scratch_bytes", "nst_resize_u8", "nst_blend_mask8_u8",
    "nst_region_masks", "nst_region_feather", "nst_region_rotate", "nst_region_bbox", "nst_region_scratch_floats",
    "nst_region_composite_u8", "nst_region_crop_input", "nst_region_resize", "nst_region_morph",
    "nst_region_morph_scratch_floats", "nst_gray_u8", "nst_flow_scratch_floats", "nst_flow_farneback",
    "nst_flow_fuse", "nst_motion_alpha", "nst_flow_downscale_gray", "nst_flow_upscale", "nst_resize_area_u8",
    "nst_flow_dis_scratch_bytes", "nst_flow_dis", "nst_set_range_check", "nst_input_exact", "nst_set_stream_split",
    "nst_lab_planes_u8", "nst_lab_ema_planes", "nst_lab_merge_u8",
    "nst_png_bound", "nst_png_workspace_bytes", "nst_png_encode_u8",
)
# region compositor limits / geometry kinds (include/nst_hip.h NST_REGION_*, NST_RG_*)
NST_REGION_MAX, NST_REGION_TERMS, NST_REGION_MAX_SRC = 32, 9, 16
RG_KINDS = {"rects": 0, "diagonal": 1, "voronoi": 2, "radial": 3, "waves": 4, "spiral": 5, "concentric": 6}
NST_GRAM_CHW, NST_GRAM_HWC = 0, 1

# nst_create_ex kernel-selection flags (include/nst_hip.h NST_KSEL_*)
KSEL = {
    "no_wstat": 0x1, "no_wphase": 0x2, "no_ws2": 0x4, "no_ws9": 0x8, "no_kyrot": 0x10, "no_prepad": 0x20,
    "no_persistent": 0x40, "unfused_residual": 0x80, "no_fold": 0x100, "f16m_two_blocks": 0x200,
    "pad_decoder": 0x400, "pad_encoder": 0x800, "pad_48": 0x1000,
}
NST_BUF_INPUT, NST_BUF_OUTPUT = -1, -2


class NstParam(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.POINTER(ctypes.c_float)), ("numel", ctypes.c_int64)]


class NstOpDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "kind", "layer", "src", "dst", "in_norm", "in_relu", "res_buf", "res_norm", "res_out", "relu_out",
        "in_h", "in_w", "conv_h", "conv_w", "out_h", "out_w", "cin_stride", "cout_stride", "kernel_mode",
        "elem_bytes", "in_elem_bytes", "res_elem_bytes", "kernel_dtype")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None
_lock = threading.Lock()


class NstError(RuntimeError):
    """Raised for any non-zero status from libnst_hip (message from nst_last_error)."""


# Sources (and build flags) that determine the residual-trunk kernel's machine code: the key under
# which tools/pmc_summary.py files that kernel's PMC traffic and bench.py looks it up, so unrelated
# library changes do not orphan the measurement (and any change to the kernel does).
TRUNK_KERNEL_SOURCES = ("csrc/conv_wst16.hip", "csrc/conv_ws_common.h", "csrc/conv_impl.h")


def kernel_sha(sources=TRUNK_KERNEL_SOURCES, obj: str = "conv_wstat") -> str:
    """sha256[:16] of a kernel's sources and the build flags of its translation unit `obj` (the key of its PMC
    summary under profiles/)."""
    import hashlib
    import re
    h = hashlib.sha256()
    for rel in sources:
        with open(os.path.join(_HERE, rel), "rb") as f:
            h.update(f.read())
    # the compiler and the code-generation flags of the object's own translation unit: the global
    # HIPCC / ARCH / SLP / CXXFLAGS definitions and target-specific CXXFLAGS / SLP assignments naming that
    # object alone (diagnostic-only rules such as the multi-target NOSCRATCH remark pass do not change code)
    pat = r"(HIPCC|ARCH|SLP|CXXFLAGS) |\$\(BUILD\)/" + re.escape(obj) + r"\.hip\.o: *(CXXFLAGS|SLP) "
    with open(os.path.join(_HERE, "..", "Makefile")) as f:
        h.update("".join(l for l in f if re.match(pat, l)).encode())
    return h.hexdigest()[:16]


def trunk_kernel_sha() -> str:
    return kernel_sha(TRUNK_KERNEL_SOURCES, "conv_wst16")


# the NST_DT_F16M mode's dominant kernel (the split-operand down-conv conv2, conv_ws2.hip)
WS2_KERNEL_SOURCES = ("csrc/conv_ws2.hip", "csrc/conv_ws_common.h", "csrc/conv_impl.h")


def ws2_kernel_sha() -> str:
    return kernel_sha(WS2_KERNEL_SOURCES, "conv_ws2")


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NstError(
                f"libnst_hip.so not found at {LIB_PATH}: build it with `make` (or __graft_entry__.build()); "
                "there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.nst_last_error.restype = ctypes.c_char_p
        L.nst_version.restype = ctypes.c_char_p
        L.nst_create.argtypes = [i, ctypes.POINTER(NstParam), i, i, i, ctypes.POINTER(vp)]
        L.nst_create_ex.argtypes = [i, ctypes.POINTER(NstParam), i, i, i, ctypes.c_uint, ctypes.POINTER(vp)]
        L.nst_num_ops.argtypes = [vp]
        L.nst_num_ops.restype = i
        L.nst_set_range_check.argtypes = [vp, i]
        L.nst_set_range_check.restype = i
        L.nst_set_stream_split.argtypes = [vp, i]
        L.nst_set_stream_split.restype = i
        L.nst_op_describe.argtypes = [vp, i, i, i, i, ctypes.POINTER(NstOpDesc)]
        L.nst_forward_capture.argtypes = [vp, vp, i, i, i, i, i, vp, i, vp, sz, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                          ctypes.POINTER(vp), vp]
        L.nst_vgg_create.argtypes = [ctypes.POINTER(NstParam), i, i, ctypes.POINTER(vp)]
        L.nst_vgg_create_ex.argtypes = [ctypes.POINTER(NstParam), i, i, ctypes.c_uint, ctypes.POINTER(vp)]
        L.nst_vgg_destroy.argtypes = [vp]
        L.nst_vgg_destroy.restype = None
        L.nst_gatys_buffer_bytes.argtypes = [vp, i, i, ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.nst_vgg_features.argtypes = [vp, vp, i, i, ctypes.POINTER(vp), vp, sz, vp]
        L.nst_gatys_targets.argtypes = [vp, vp, vp, i, i, vp, vp, sz, vp]
        L.nst_gatys_grad.argtypes = [vp, vp, i, i, ctypes.POINTER(f), f, f, vp, vp, vp, vp, sz, vp]
        L.nst_gatys_grad_capture.argtypes = [vp, vp, i, i, ctypes.POINTER(f), f, f, vp, vp, vp, vp, sz,
                                             ctypes.POINTER(vp), vp]
        L.nst_gatys_grad_capture.restype = i
        L.nst_adam_step.argtypes = [vp, vp, vp, vp, i, i, f, f, f, f, i, i, i, vp]
        L.nst_destroy.argtypes = [vp]
        L.nst_destroy.restype = None
        L.nst_seg_create.argtypes = [ctypes.POINTER(NstParam), i, i, i, i, ctypes.POINTER(vp)]
        L.nst_seg_destroy.argtypes = [vp]
        L.nst_seg_destroy.restype = None
        L.nst_seg_num_classes.argtypes = [vp]
        L.nst_seg_workspace_bytes.argtypes = [vp, i, i, i, ctypes.POINTER(sz)]
        L.nst_seg_forward.argtypes = [vp, vp, i, i, i, i, vp, vp, vp, sz, vp]
        L.nst_seg_mask_scratch_bytes.argtypes = [i, i, i, ctypes.POINTER(sz)]
        L.nst_seg_mask.argtypes = [vp, i, i, i, ctypes.POINTER(i), i, i, i, i, i, vp, vp, sz, vp]
        L.nst_resize_create.argtypes = [i, i, i, i, i, i, ctypes.POINTER(vp)]
        L.nst_resize_destroy.argtypes = [vp]
        L.nst_resize_destroy.restype = None
        L.nst_resize_scratch_bytes.argtypes = [vp, i, ctypes.POINTER(sz)]
        L.nst_resize_u8.argtypes = [vp, vp, i, i, vp, vp, sz, vp]
        pi, pd, pf = ctypes.POINTER(i), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(f)
        L.nst_region_masks.argtypes = [i, i, i, pi, pd, pd, pd, pi, pd, pd, i, i, vp, vp, vp]
        L.nst_region_feather.argtypes = [vp, i, i, i, pf, i, vp, vp]
        L.nst_region_rotate.argtypes = [vp, i, i, i, ctypes.c_double, vp, vp]
        L.nst_region_bbox.argtypes = [vp, i, i, i, f, vp, vp]
        dbl = ctypes.c_double
        L.nst_region_morph_scratch_floats.argtypes = [i, i, i, ctypes.POINTER(sz)]
        L.nst_region_morph.argtypes = [vp, i, i, i, i, dbl, dbl, dbl, pd, vp, vp, sz, vp]
        L.nst_region_scratch_floats.argtypes = [i, i, i, i, i, ctypes.POINTER(sz)]
        L.nst_region_composite_u8.argtypes = [ctypes.POINTER(vp), pi, pi, i, pi, pi, pf, i, pi, vp, vp, i, i, i, vp,
                                              sz, vp, vp, vp]
        L.nst_region_crop_input.argtypes = [vp, i, i, i, pi, i, i, vp, vp]
        L.nst_region_resize.argtypes = [vp, i, i, i, i, i, i, i, i, vp, vp]
        L.nst_gray_u8.argtypes = [vp, i, i, i, vp, vp]
        L.nst_flow_scratch_floats.argtypes = [i, i, ctypes.POINTER(sz)]
        L.nst_flow_farneback.argtypes = [vp, vp, i, i, dbl, i, i, i, i, dbl, vp, vp, sz, vp]
        L.nst_flow_fuse.argtypes = [vp, vp, vp, i, i, f, f, vp, vp]
        L.nst_motion_alpha.argtypes = [vp, i, i, f, dbl, f, f, vp, vp, vp]
        L.nst_flow_downscale_gray.argtypes = [vp, i, i, i, vp, vp]
        L.nst_flow_upscale.argtypes = [vp, i, i, i, i, f, vp, vp]
        L.nst_resize_area_u8.argtypes = [vp, i, i, i, i, vp, i, i, vp]
        L.nst_flow_dis_scratch_bytes.argtypes = [i, i, i, ctypes.POINTER(sz)]
        L.nst_flow_dis.argtypes = [vp, vp, i, i, i, vp, vp, sz, vp]
        for name in ("nst_gray_u8", "nst_flow_scratch_floats", "nst_flow_farneback", "nst_flow_fuse",
                     "nst_motion_alpha", "nst_flow_downscale_gray", "nst_flow_upscale", "nst_resize_area_u8",
                     "nst_flow_dis_scratch_bytes", "nst_flow_dis"):
            getattr(L, name).restype = i
        for name in ("nst_region_masks", "nst_region_feather", "nst_region_rotate", "nst_region_bbox",
                     "nst_region_morph", "nst_region_morph_scratch_floats",
                     "nst_region_scratch_floats", "nst_region_composite_u8", "nst_region_crop_input",
                     "nst_region_resize"):
            getattr(L, name).restype = i
        L.nst_output_hw.argtypes = [vp, i, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.nst_workspace_bytes.argtypes = [vp, i, i, i, ctypes.POINTER(sz)]
        L.nst_forward.argtypes = [vp, vp, i, i, i, i, i, vp, i, vp, sz, vp]
        L.nst_decode_resize_u8.argtypes = [vp, i, i, i, i, vp, i, i, vp]
        L.nst_lab_create.argtypes = [vp, vp, i, ctypes.POINTER(vp)]
        L.nst_lab_destroy.argtypes = [vp]
        L.nst_lab_destroy.restype = None
        L.nst_lab_ema_u8.argtypes = [vp, vp, vp, i, i, i, i, f, f, i, f, f, vp, i, vp]
        L.nst_lab_planes_u8.argtypes = [vp, vp, i, i, i, i, i, vp, vp]
        L.nst_lab_ema_planes.argtypes = [vp, vp, i, i, i, i, f, f, i, f, f, vp, i, vp]
        L.nst_lab_merge_u8.argtypes = [vp, vp, vp, i, i, i, i, i, vp, vp]
        L.nst_input_exact.argtypes = [vp, i, i, ctypes.POINTER(i)]
        L.nst_png_bound.argtypes = [i, i, i, ctypes.POINTER(sz)]
        L.nst_png_workspace_bytes.argtypes = [i, i, i, i, ctypes.POINTER(sz)]
        L.nst_png_encode_u8.argtypes = [vp, i, i, i, i, vp, sz, vp, vp, sz, vp]
        for name in ("nst_png_bound", "nst_png_workspace_bytes", "nst_png_encode_u8"):
            getattr(L, name).restype = i
        for name in ("nst_lab_planes_u8", "nst_lab_ema_planes", "nst_lab_merge_u8", "nst_input_exact"):
            getattr(L, name).restype = i
        L.nst_blend_u8.argtypes = [vp, vp, vp, i, f, f, vp, i, i, i, vp]
        L.nst_blend_mask8_u8.argtypes = [vp, vp, vp, i, f, f, vp, i, i, i, vp]
        L.nst_blend_mask8_u8.restype = i
        L.nst_gram.argtypes = [vp, i, i, i, i, i, vp, vp, sz, vp]
        L.nst_gram_workspace_bytes.argtypes = [i, i, i, ctypes.POINTER(sz)]
        L.nst_gram_workspace_bytes.restype = i
        L.nst_blend_models_u8.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(i), ctypes.POINTER(f), i, i, i, i, vp,
                                          i, i, vp]
        L.nst_blend_models_u8.restype = i
        L.nst_blend_models_lab_u8.argtypes = [vp, ctypes.POINTER(vp), i, ctypes.POINTER(f), i, f, f, i, i, i, vp, vp]
        L.nst_mask_feather.argtypes = [vp, i, i, i, f, vp, vp, vp]
        L.nst_profile_begin.argtypes = [vp]
        L.nst_profile_end.argtypes = [vp, i, ctypes.POINTER(f), ctypes.POINTER(i)]
        L.nst_num_layers.argtypes = [vp]
        L.nst_num_layers.restype = i
        L.nst_layer_name.argtypes = [vp, i]
        L.nst_layer_name.restype = ctypes.c_char_p
        for name in ("nst_seg_create", "nst_seg_num_classes", "nst_seg_workspace_bytes", "nst_seg_forward",
                     "nst_seg_mask_scratch_bytes", "nst_seg_mask", "nst_resize_create", "nst_resize_scratch_bytes",
                     "nst_resize_u8", "nst_vgg_create", "nst_vgg_create_ex", "nst_gatys_buffer_bytes", "nst_vgg_features", "nst_gatys_targets",
                     "nst_gatys_grad", "nst_adam_step", "nst_create", "nst_create_ex", "nst_op_describe", "nst_forward_capture", "nst_output_hw", "nst_workspace_bytes", "nst_forward", "nst_decode_resize_u8",
                     "nst_lab_create", "nst_lab_ema_u8", "nst_blend_u8", "nst_gram", "nst_profile_begin",
                     "nst_profile_end"):
            getattr(L, name).restype = i
        _lib = L
        return _lib


def check(rc: int, what: str) -> None:
    if rc != NST_OK:
        msg = lib().nst_last_error().decode(errors="replace")
        raise NstError(f"{what} failed ({rc}): {msg}")


def require_gpu_tensor(t: torch.Tensor, what: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise NstError(f"{what} must be a tensor on an MI355X (cuda) device; there is no CPU path")


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
