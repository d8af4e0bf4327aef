/*
 * nst_hip.h — C ABI of libnst_hip.so, the MI355X (gfx950) stylization engine.
 *
 * Drop-in boundary for the reference's per-frame stylization hot path
 * (TrentMahaffey/NeuralStyleTransferV1).  The reference is pure Python/PyTorch;
 * the interfaces these entry points replace are Python call sites, cited per
 * function below.  Plain pointers and sizes only: no torch types cross this ABI.
 * Device pointers are HIP device pointers (e.g. a PyTorch-ROCm tensor's
 * data_ptr()); `stream` is a hipStream_t passed as void* (NULL = default stream).
 *
 * Ownership: the caller owns every input/output/workspace buffer; a handle owns
 * its packed weights (device) and nothing else.  No entry point allocates device
 * memory except nst_create / nst_lab_create (one-time packing/uploads).
 * Threading: calls on one handle must be serialised on one stream; handles on
 * different devices may be used concurrently from different threads/processes.
 * Errors: every int-returning function returns NST_OK (0) or a negative NST_E*
 * code; nst_last_error() returns the calling thread's last message.
 */
#ifndef NST_HIP_H
#define NST_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define NST_OK 0
#define NST_E_INVALID (-1)   /* bad argument / unknown enum */
#define NST_E_PARAM (-2)     /* missing or mis-shaped checkpoint tensor */
#define NST_E_SHAPE (-3)     /* unsupported input/output geometry */
#define NST_E_HIP (-4)       /* HIP runtime error */
#define NST_E_WORKSPACE (-5) /* workspace too small */
#define NST_E_RANGE (-6)     /* nst_set_range_check: a value left the compute dtype's range (non-finite result) */

/* ---- architectures (pipeline.py:72-79 _detect_transformer_type, :598-603 reconet) ---- */
#define NST_ARCH_JOHNSON 0 /* transformer_net.py:4-41 */
#define NST_ARCH_NST 1     /* transformer_net_nst.py:62-127 */
#define NST_ARCH_RECONET 2 /* model.py:107-116 (frn=False, as pipeline.py:602 builds it) */
#define NST_ARCH_RECONET_FRN 3 /* model.py:107-116 with frn=True: FRN + TLU (frn.py:7-78) */

/* ---- compute dtypes ---- */
#define NST_DT_F32 0  /* fp32 "parity" mode: exact-f32 MFMA (v_mfma_f32_16x16x4_f32) */
#define NST_DT_BF16 1 /* bf16 "throughput" mode: bf16 MFMA, fp32 accumulate/statistics */
#define NST_DT_F16 2  /* fp16 mode: fp16 weights/activations, fp16 MFMA at the bf16 rate, fp32 accumulate/statistics;
                         3 more mantissa bits than bf16 (1080p: ~99.95 % of pixels within +-1 LSB of the reference).
                         Stored conv outputs must stay inside the fp16 range (|v| <= 65504) */
#define NST_DT_F32S 3 /* split-fp16 mode: fp32 activations in HBM; each conv operand is split into an fp16 pair
                         v = hi + lo in LDS (weights at pack time), and two v_mfma_f32_16x16x32_f16 per K step give
                         Wh*(xh + xl) + Wl*xh: ~22 significant bits per product (the fp32 parity bar) at a quarter of
                         the exact-f32 MFMA cycles.  Conv inputs must stay inside the fp16 range (|v| <= 65504) */
#define NST_DT_F16M 4 /* split-precision head + fp16 trunk (Johnson / NST nets): the first layer takes the raw bytes
                         (exact) against fp16 hi/lo weight pairs, the two down-convs run split-fp16 operands and
                         weights (Wh*xh + Wh*xl + Wl*xh), the first two residual blocks split-fp16 operands against
                         fp16 weights (Wh*xh + Wh*xl), all with fp32 activations, and the rest of the net runs the
                         fp16 mode's kernels.  The layers whose rounding reaches the frame
                         most (tests/precision_study.py) keep ~22-bit products: 1080p frames within +-1 LSB of the
                         fp32 reference at about 3/4 of the fp16 mode's rate.  ReCoNet: NST_E_INVALID */

/* ---- I/O formats for nst_forward ---- */
#define NST_IO_F32_NCHW 0 /* raw model tensor [n,3,h,w] fp32 (TransformerNet.forward(X) surface) */
#define NST_IO_U8_NHWC 1  /* frames [n,h,w,3] uint8 RGB; io_preset encode/decode + clamp + ToPILImage truncation fused */

/* ---- io presets (pipeline.py:1445-1486; auto table :2518-2523) ---- */
#define NST_PRESET_NONE 0 /* only valid with NST_IO_F32_NCHW on both sides */
#define NST_PRESET_TANH 1
#define NST_PRESET_IMAGENET_01 2
#define NST_PRESET_IMAGENET_255 3
#define NST_PRESET_CAFFE_BGR 4
#define NST_PRESET_RAW_255 5
#define NST_PRESET_RAW_01 6

typedef struct nst_handle nst_handle;
typedef struct nst_lab nst_lab;

/* One checkpoint tensor, by its reference state_dict name (e.g. "res1.conv1.conv2d.weight"). */
typedef struct nst_param {
  const char* name;
  const float* data; /* host fp32, contiguous in the reference's PyTorch layout */
  int64_t numel;
} nst_param;

/* Last error message of the calling thread ("" if none). */
const char* nst_last_error(void);

/* Library version string. */
const char* nst_version(void);

/*
 * Pack a checkpoint for one device.  Replaces model construction + load:
 * `TransformerNet().to(device)` + `_load_checkpoint_compat` (pipeline.py:554-569, 597-619).
 * Every parameter of the architecture must be present (missing -> NST_E_PARAM);
 * unknown names are ignored (load_state_dict(strict=False) semantics).
 */
int nst_create(int arch, const nst_param* params, int n_params, int compute_dtype, int device,
               nst_handle** out);

/*
 * nst_create with kernel-selection flags (0 = the default, fastest mapping for every layer).  Each
 * NST_KSEL_NO_* bit removes one specialised bf16 kernel family so the layer falls back to the
 * generic implicit-GEMM mapping; the tests use this to check the specialised kernels against the
 * generic ones on the same model.  NST_KSEL_UNFUSED_RESIDUAL runs the residual add as its own
 * kernel instead of fusing it into the next conv's fill.  Unknown bits -> NST_E_INVALID.
 */
#define NST_KSEL_NO_WSTAT 0x1             /* residual-trunk weight-stationary conv (conv_wstat.hip) */
#define NST_KSEL_NO_WPHASE 0x2            /* x2 up-conv phase kernel (conv_wphase.hip) */
#define NST_KSEL_NO_WS2 0x4               /* stride-2 down-conv kernel (conv_ws2.hip) */
#define NST_KSEL_NO_WS9 0x8               /* 9x9 first-layer kernel (conv_ws9.hip) */
#define NST_KSEL_NO_KYROT 0x10            /* 9x9 output-conv row-streaming kernel (conv_out9.hip) */
#define NST_KSEL_NO_PREPAD 0x20           /* first layer over the pre-padded encoded frame (conv_prep.hip) */
#define NST_KSEL_NO_PERSISTENT 0x40       /* generic persistent LDS-weight-ring kernels */
#define NST_KSEL_UNFUSED_RESIDUAL 0x80    /* residual add as a separate kernel */
#define NST_KSEL_NO_FOLD 0x100            /* uint8 frames: stage the encoded value instead of the raw byte with the
                                             io_preset encode folded into the first layer's weights */
#define NST_KSEL_F16M_TWO_BLOCKS 0x200    /* NST_DT_F16M: residual blocks 1 AND 2 on the split-operand kernel (wider
                                            precision margin: live max 0.920 instead of 0.958 LSB; ~10 % slower) */
#define NST_KSEL_PAD_DECODER 0x400       /* ReCoNet, 16-bit modes: the decoder's 96-channel stream padded to 128
                                            channels, as the encoder's (default: unpadded) */
#define NST_KSEL_PAD_ENCODER 0x800       /* ReCoNet, 16-bit modes: the encoder's 96-channel map padded to 128 (default:
                                            unpadded) */
#define NST_KSEL_PAD_48 0x1000         /* ReCoNet, 16-bit modes: the decoder's 48-channel output padded to 64 (default:
                                            unpadded) */
#define NST_KSEL_ALL 0x1fff
int nst_create_ex(int arch, const nst_param* params, int n_params, int compute_dtype, int device,
                  unsigned flags, nst_handle** out);
void nst_destroy(nst_handle* h);

/* Output spatial size the architecture produces for an h x w input
 * (Johnson/ReCoNet: 4*ceil(ceil(h/2)/2); NST: centre-cropped back to h x w). */
int nst_output_hw(const nst_handle* h, int in_h, int in_w, int* out_h, int* out_w);

/* Whether nst_forward feeds the first layer the reference's encoded input without any extra rounding for this
 * input format and io_preset (*exact = 1): always in the fp32-activation modes; in the 16-bit modes only for uint8
 * frames whose preset encode folds into the first layer's weights (reflection-padded first layers: every preset;
 * zero-padded ones, the NST net: presets without an offset).  NST_DT_F16M's +-1 LSB bar needs it (the Python
 * engine runs the other combinations on an NST_DT_F32S twin).  Replaces no reference call: a property query. */
int nst_input_exact(const nst_handle* h, int x_fmt, int preset, int* exact);

/* Device workspace nst_forward needs for a batch of n frames of h x w (with the handle's stream split: one slice
 * per sub-batch). */
int nst_workspace_bytes(const nst_handle* h, int n, int in_h, int in_w, size_t* out);

/* Run each nst_forward batch as k sub-batches (1 <= k <= 4) on internal streams forked from and joined back to the
 * caller's stream (events only: the caller's stream order is kept, frames are independent, outputs identical).
 * Default: 2 for the ReCoNet nets in the 16-bit modes and for NST_DT_F32S (their generic kernels' launch gaps and
 * tails are filled by the other sub-batches), 1 otherwise.  Profiling and the range check run a batch whole.  Replaces no reference
 * call: scheduling only. */
int nst_set_stream_split(nst_handle* h, int k);

/*
 * Stylize a batch.  Replaces `model(x_in)` with its io_preset pre/post arithmetic
 * (pipeline.py:1445-1486: preset encode -> .to(device) -> model -> .cpu() -> decode -> clamp(0,1))
 * and, for NST_IO_U8_NHWC output, the ToPILImage truncation `pic.mul(255).byte()`
 * (pipeline.py:1943/2094).  x: [n,3,h,w] f32 or [n,h,w,3] u8; y: [n,3,oh,ow] f32 (raw
 * model output, no preset) or [n,oh,ow,3] u8 (decoded).  U8 output requires
 * nst_output_hw(h,w) == (h,w) (otherwise use F32 output + nst_resize_bilinear_u8).
 */
int nst_forward(nst_handle* h, const void* x, int x_fmt, int n, int in_h, int in_w, int preset,
                void* y, int y_fmt, void* workspace, size_t workspace_bytes, void* stream);

/*
 * Per-layer inspection (parity tests): the handle runs its architecture as a program of ops, each a
 * conv (with the producer's InstanceNorm + ReLU, or the residual join, applied in its fill) or a
 * separate residual add.  nst_op_describe gives op i's wiring and geometry for an n x h x w batch;
 * nst_forward_capture is nst_forward that also copies, after each op i, the activation it wrote
 * (act[i]: [n][out_h][out_w][cout_stride] in the compute dtype, the raw conv output before its
 * InstanceNorm), the joined residual stream it wrote (res[i]: [n][in_h][in_w][cin_stride]) and its
 * layer's InstanceNorm {scale, shift} pairs (stats[i]: [n][cout_stride] float2) into caller-owned
 * device buffers; NULL arrays or NULL entries skip a copy.  The final op writes y and captures nothing.
 * Replaces inspecting intermediate tensors of the reference's module graph (transformer_net.py:29-41).
 */
#define NST_BUF_INPUT (-1)  /* nst_op_desc src: the input frames / tensor */
#define NST_BUF_OUTPUT (-2) /* nst_op_desc dst: y */
typedef struct nst_op_desc {
  int kind;         /* 0 conv, 1 residual add (out = IN_in_norm(src) + r) */
  int layer;        /* conv layer index (nst_layer_name); for a residual add the layer whose IN applies */
  int src, dst;     /* activation buffer ids (0..6) or NST_BUF_INPUT / NST_BUF_OUTPUT */
  int in_norm;      /* layer whose InstanceNorm the fill applies to src, -1 = none */
  int in_relu;      /* ReLU after that InstanceNorm */
  int res_buf;      /* residual stream r joined in (-1 none): operand = IN(src) + r' */
  int res_norm;     /* r' = ReLU(IN_res_norm(r)) if >= 0, else r */
  int res_out;      /* buffer that receives the joined stream (-1 none) */
  int relu_out;     /* ReLU after the join (ReCoNet ResLayer) */
  int in_h, in_w;   /* source extent */
  int conv_h, conv_w; /* conv output extent (before the NST centre crop) */
  int out_h, out_w; /* stored output extent */
  int cin_stride, cout_stride;
  int kernel_mode;  /* internal kernel family (0 generic, 1 phase, 2 x-shift, 3 out9, 4 wstat, 5 wphase, 6 ws2, 7 ws9) */
  int elem_bytes;   /* bytes per element of what the op writes (act[i]): 2 (bf16 / fp16) or 4 (fp32) */
  int in_elem_bytes;  /* bytes per element of src (NST_BUF_INPUT: the staged first-layer operand, 2 or 4) */
  int res_elem_bytes; /* bytes per element of the joined residual stream (res_buf / res_out), 0 if none */
  int kernel_dtype;   /* the op's arithmetic: an NST_DT_* value, or 16 / 17 (fp16 operand x fp16 hi/lo weight
                         pairs, fp32 / fp16 output), 18 / 19 (split fp16 operand and weights, fp32 / fp16 output),
                         20 (split fp16 operand x fp16 weights, fp32 output) */
} nst_op_desc;
int nst_num_ops(const nst_handle* h);
/* Optional range check (the 16-bit and split modes hold operands inside the fp16 range, |v| <= 65504):
 * enabled, every nst_forward zeroes a device flag, checks each layer's InstanceNorm table (an overflowing operand
 * turns into inf, then a non-finite statistic) and an fp32 output for non-finite values, waits for the stream and
 * returns NST_E_RANGE if any was found.  Off by default (no extra launches, no synchronisation). */
int nst_set_range_check(nst_handle* h, int enable);
int nst_op_describe(const nst_handle* h, int n, int in_h, int in_w, int op, nst_op_desc* out);
int nst_forward_capture(nst_handle* h, const void* x, int x_fmt, int n, int in_h, int in_w, int preset,
                        void* y, int y_fmt, void* workspace, size_t workspace_bytes, void* const* act,
                        void* const* res, void* const* stats, void* stream);

/*
 * Decode a raw model output (f32 NCHW [n,3,h,w]) with `preset` + clamp(0,1), resize
 * bilinearly (align_corners=False) to out_h x out_w, truncate to u8 NHWC.
 * Replaces pipeline.py:1512-1516 (F.interpolate to content size) + :1943 ToPILImage.
 */
int nst_decode_resize_u8(const float* y, int n, int h, int w, int preset, uint8_t* out, int out_h,
                         int out_w, void* stream);

/*
 * Multi-model RGB blend (slots A..H, pipeline.py:1872-1879 with parse_blend_weights :502-511):
 * out01 = sum_i w_i * clamp(decode_i(y_i)), each y_i a raw model output f32 NCHW [n,3,h,w] with its
 * own io preset, fitted to out_h x out_w (bilinear, align_corners=False); clamp(0,1); truncate to
 * u8 NHWC.  ys: host array of m (<= 8) device pointers.  Weights are the fp32 values of the slots'
 * Python floats (the caller validates they sum to 1 +- 1e-6, as the reference does).
 */
int nst_blend_models_u8(const float* const* ys, const int* presets, const float* weights, int m, int n,
                        int h, int w, uint8_t* out, int out_h, int out_w, void* stream);

/* ---- LAB temporal smoothing (pipeline.py:1942-1978) ---- */

/* Upload the two 2^24-entry LittleCMS (Pillow) LUTs: rgb2lab[(r<<16)|(g<<8)|b] = {L,a,b}
 * bytes and lab2rgb[(L<<16)|(a<<8)|b] = {r,g,b} bytes (3*2^24 bytes each, host). */
int nst_lab_create(const uint8_t* rgb2lab, const uint8_t* lab2rgb, int device, nst_lab** out);
void nst_lab_destroy(nst_lab* lab);

/*
 * One frame (or a batch processed in frame order) of the LAB EMA:
 * L' = alpha*L + (1-alpha)*prev_L (fp32), prev_L = L', L byte = trunc(clip(L',0,255));
 * optional same EMA on a/b bytes with chroma_alpha.  `state` is a caller-owned device
 * buffer of 3*h*w floats (prev_L, prev_a, prev_b); `first` != 0 seeds it from the frame
 * (pipeline.py:1951-1952 `prev_L = L.copy()`).  rgb in/out: [n,h,w,3] u8 (may alias).
 * alpha/chroma_alpha are the fp32 values of the Python float coefficients.
 */
int nst_lab_ema_u8(const nst_lab* lab, const uint8_t* rgb_in, uint8_t* rgb_out, int n, int h, int w,
                   int smooth_lightness, float alpha, float one_minus_alpha, int smooth_chroma,
                   float chroma_alpha, float one_minus_chroma_alpha, float* state, int first,
                   void* stream);

/*
 * nst_lab_ema_u8 split in three stages for the sharded video pipeline (pipeline.py:1942-1978 with the
 * frames of one sequence stylized on several GPUs): the EMA's only cross-frame dependency is the fp32
 * state of the planes it smooths, so each frame's owner extracts those planes, one rank runs the ordered
 * EMA over the planes alone, and the owner rebuilds RGB from its own frame with the smoothed planes put
 * back.  The three calls give bytes identical to nst_lab_ema_u8 on the same frames in the same order.
 * planes: uint8 [n][np][h*w], np = smooth_lightness + 2*smooth_chroma, planes in the order L, a, b.
 *   nst_lab_planes_u8: rgb [n,h,w,3] -> planes (rgb2lab bytes of the smoothed channels);
 *   nst_lab_ema_planes: planes_in -> planes_out in frame order (may alias), state / first as nst_lab_ema_u8;
 *   nst_lab_merge_u8: rgb + smoothed planes -> rgb_out = lab2rgb(rgb2lab(rgb) with those planes replaced).
 */
int nst_lab_planes_u8(const nst_lab* lab, const uint8_t* rgb_in, int n, int h, int w, int smooth_lightness,
                      int smooth_chroma, uint8_t* planes, void* stream);
int nst_lab_ema_planes(const uint8_t* planes_in, uint8_t* planes_out, int n, int h, int w, int smooth_lightness,
                       float alpha, float one_minus_alpha, int smooth_chroma, float chroma_alpha,
                       float one_minus_chroma_alpha, float* state, int first, void* stream);
int nst_lab_merge_u8(const nst_lab* lab, const uint8_t* rgb_in, const uint8_t* planes, int n, int h, int w,
                     int smooth_lightness, int smooth_chroma, uint8_t* rgb_out, void* stream);

/*
 * Multi-model LAB blend (pipeline.py:1841-1870, --blend_models_lab): L from model A; per pixel
 *   a = trunc(clip(wL * a_A + wab * (sum_i w_i * a_i), 0, 255))  (float32, models B.. in order; same for b)
 * on Pillow's raw LAB bytes (signed a/b stored as uint8), then LAB -> RGB through the LittleCMS
 * tables.  frames: host array of m device pointers to [n,h,w,3] uint8 outputs (A first, each the
 * decoded + clamped + truncated model output, pipeline.py's to_pil(out.clamp(0,1))); the first
 * min(m-1, n_rest) of weights_rest pair with frames[1..] (zip semantics).
 */
int nst_blend_models_lab_u8(const nst_lab* lab, const uint8_t* const* frames, int m, const float* weights_rest,
                            int n_rest, float w_l, float w_ab, int n, int h, int w, uint8_t* out, void* stream);

/*
 * Mask feathering (pipeline.py:349-351 cv2.GaussianBlur(m, (0,0), sigmaX=sigmaY=sigma) then /255,
 * :353): masks [n,h,w] uint8 (after the NEAREST fit and optional invert) -> alpha [n,h,w] f32 in
 * [0,1].  ksize = round(6*sigma+1)|1, separable Gaussian, BORDER_REFLECT_101, uint8 rounding.
 * scratch: n*h*w floats.  sigma = feather_px * 0.5 (> 0; radius <= 1023).
 */
int nst_mask_feather(const uint8_t* mask, int n, int h, int w, float sigma, float* scratch, float* alpha,
                     void* stream);

/*
 * Uniform / masked blend with the original frame (pipeline.py:1984-2092):
 *   mask (optional, [n,h,w] f32 alpha in [0,1]): keep: C = a*S + (1-a)*O; replace: (1-a)*S + a*O; clip
 *   then if 0 <= blend < 1: out = clamp(blend*C + (1-blend)*O, 0, 1); truncate to u8.
 * S and O are u8 NHWC frames read as x/255 (to_tensor).  composite_mode: 0 keep, 1 replace.
 */
int nst_blend_u8(const uint8_t* styled, const uint8_t* orig, const float* mask, int composite_mode,
                 float blend, float one_minus_blend, uint8_t* out, int n, int h, int w,
                 void* stream);
/* nst_blend_u8 with an 8-bit mask [n,h,w] (alpha = m / 255 in fp32, pipeline.py:353): the DeepLab masks of
 * nst_seg_mask / nst_resize_u8 composited straight from HBM (configs[4]) */
int nst_blend_mask8_u8(const uint8_t* styled, const uint8_t* orig, const uint8_t* mask, int composite_mode, float blend,
                       float one_minus_blend, uint8_t* out, int n, int h, int w, void* stream);

/*
 * Live per-layer kernel timing (bench.py roofline): between nst_profile_begin and
 * nst_profile_end every conv launch of nst_forward on this handle is bracketed by a pair of
 * HIP events recorded on the forward's stream.  Call nst_profile_end after synchronising
 * that stream; it returns, per layer index (0..n_layers-1, program order), the summed
 * kernel milliseconds and the launch count, and releases the events.
 */
int nst_profile_begin(nst_handle* h);
int nst_profile_end(nst_handle* h, int n_layers, float* total_ms, int* launches);
/* Number of conv layers of the handle's architecture and a layer's state_dict prefix. */
int nst_num_layers(const nst_handle* h);
const char* nst_layer_name(const nst_handle* h, int layer);

/*
 * Gram matrix G[b] = F[b] F[b]^T / (c*hw) (utils.py:80-83 gram_matrix), F f32 or bf16, G fp32 [n,c,c].
 * layout NST_GRAM_CHW: F [n][c][hw] (the reference's NCHW feature map); NST_GRAM_HWC: F [n][hw][c]
 * (NHWC activations).  MFMA tiles over K slices of hw, slices summed in fixed order: bit-identical
 * across runs.  workspace: nst_gram_workspace_bytes (0 for a single slice).
 */
#define NST_GRAM_CHW 0
#define NST_GRAM_HWC 1
int nst_gram_workspace_bytes(int n, int c, int hw, size_t* out);
int nst_gram(const void* F, int dtype, int layout, int n, int c, int hw, float* G, void* workspace,
             size_t workspace_bytes, void* stream);

/* ---- Gatys optimisation loop (BASELINE.json configs[2]) ----
 * The reference provides only gram_matrix (utils.py:80-83) and preprocess_for_vgg (utils.py:93-96);
 * it has no VGG network, loss or optimiser.  These entry points build the loop the
 * configuration names around them: VGG-19 features (torchvision layout, state_dict keys
 * "features.N.weight"/"features.N.bias", N in {0,2,5,7,10,12,14,16,19,21,23,25,28}), style =
 * MSE of Grams of relu1_1..relu5_1, content = MSE of relu4_2, gradient with respect to the image,
 * Adam on the image.  Images: [1,3,h,w] fp32 in [0,1], h and w multiples of 16; bf16 activations
 * with fp32 accumulation. */
typedef struct nst_vgg nst_vgg;
int nst_vgg_create(const nst_param* params, int n_params, int device, nst_vgg** out);
/* flags: NST_VGG_GENERIC_ONLY runs every conv on the generic implicit-GEMM kernel (conv_vgg.hip) instead of
 * conv2_1 onward on the K-streaming GEMM conv (conv_gemm.hip) — the same arithmetic in another order */
#define NST_VGG_GENERIC_ONLY 0x1
int nst_vgg_create_ex(const nst_param* params, int n_params, int device, unsigned flags, nst_vgg** out);
void nst_vgg_destroy(nst_vgg* v);
/* caller-owned device buffers: workspace (activations, gradients, Grams) and state (targets) */
int nst_gatys_buffer_bytes(const nst_vgg* v, int h, int w, size_t* workspace, size_t* state);
/* forward only: the rectified feature maps relu1_1, relu2_1, relu3_1, relu4_1, relu5_1, relu4_2 (bf16
 * NHWC [h_l][w_l][c_l]) into feats[0..5] (NULL entries skipped) */
int nst_vgg_features(nst_vgg* v, const float* image, int h, int w, void* const* feats, void* workspace,
                     size_t workspace_bytes, void* stream);
/* targets into state: style Grams of `style` (same size as content) and relu4_2 of `content` */
int nst_gatys_targets(nst_vgg* v, const float* content, const float* style, int h, int w, void* state,
                      void* workspace, size_t workspace_bytes, void* stream);
/* losses (device float[3]: total, content, style) of `image` and grad = dL/d(normalised image),
 * fp32 [1,3,h,w]; L = content_weight * mean((F - P)^2) + style_weight * sum_l w_l mean((G_l - A_l)^2),
 * style_layer_weights: host float[5] (NULL = all 1) */
int nst_gatys_grad(nst_vgg* v, const float* image, int h, int w, const float* style_layer_weights,
                   float content_weight, float style_weight, const void* state, float* grad, float* losses,
                   void* workspace, size_t workspace_bytes, void* stream);
/* nst_gatys_grad that also copies dL/dz of each of the 13 convs (z = its pre-activation; bf16 NHWC
 * [h_i][w_i][c_i]) into dz[i] (NULL entries skipped): per-layer checks of the backward pass */
int nst_gatys_grad_capture(nst_vgg* v, const float* image, int h, int w, const float* style_layer_weights,
                           float content_weight, float style_weight, const void* state, float* grad,
                           float* losses, void* workspace, size_t workspace_bytes, void* const* dz,
                           void* stream);
/* torch.optim.Adam step on an image [c=3][hw] (step >= 1 counts updates; bias corrections from it);
 * grad_is_normalised: the gradient is with respect to (x - mean) / std (nst_gatys_grad's), so it is
 * divided by std per channel; clamp01 clamps the image to [0, 1] after the update */
int nst_adam_step(float* x, const float* grad, float* m, float* v, int c, int hw, float lr, float beta1,
                  float beta2, float eps, int step, int clamp01, int grad_is_normalised, void* stream);

/* ---- DeepLab v3+ mask program (BASELINE.json configs[4]) ----
 * The network of modeling/deeplab.py:9-33 as sky_swap.py:143-177 load_deeplab builds it: backbone
 * 'resnet' (ResNet-101, modeling/backbone/resnet.py:45-124), output stride 16, BatchNorm2d in eval mode,
 * ASPP (modeling/aspp.py:34-78), decoder (modeling/decoder.py:7-43).  Parameters by their state_dict
 * names without the "module." prefix (sky_swap.py:150 strips it), e.g. "backbone.layer3.22.conv2.weight",
 * "aspp.global_avg_pool.1.weight", "decoder.last_conv.8.bias"; running_mean / running_var are used,
 * num_batches_tracked is ignored.  NHWC activations in the compute dtype, fp32 accumulation; compute_dtype
 * NST_DT_F32S keeps fp32 activations and splits every conv's operands into fp16 pairs (the split-fp16 GEMM). */
typedef struct nst_seg nst_seg;
int nst_seg_create(const nst_param* params, int n_params, int num_classes, int compute_dtype, int device,
                   nst_seg** out);
void nst_seg_destroy(nst_seg* s);
int nst_seg_num_classes(const nst_seg* s);
int nst_seg_workspace_bytes(const nst_seg* s, int n, int h, int w, size_t* out);
/*
 * DeepLab.forward (deeplab.py:27-33) on a batch.  x: NST_IO_F32_NCHW = the module input [n,3,h,w]
 * (already normalised), or NST_IO_U8_NHWC = frames [n,h,w,3] with sky_swap.py:179-183 preprocess_pil
 * fused.  logits (optional): f32 NCHW [n,nc,h,w] = the module output (bilinear, align_corners=True);
 * pred (optional): u8 [n,h,w] = logits.argmax(1) (sky_swap.py:189-193: the second interpolate to the
 * same size is the identity).
 */
int nst_seg_forward(nst_seg* s, const void* x, int x_fmt, int n, int h, int w, float* logits, uint8_t* pred,
                    void* workspace, size_t workspace_bytes, void* stream);
/*
 * infer_mask's post-processing (sky_swap.py:196-215) on class maps pred [n,h,w] -> mask u8 [n,h,w]:
 * 255 where pred is one of target_ids, MORPH_CLOSE with ones(close_ks, close_ks) (5 in the reference;
 * 0 skips), dilate ones(2e+1), erode ones(2c+1), GaussianBlur(sigma = feather_px / 2) (cv2 restated:
 * parity unpinned).  scratch: nst_seg_mask_scratch_bytes.
 */
int nst_seg_mask_scratch_bytes(int n, int h, int w, size_t* out);
int nst_seg_mask(const uint8_t* pred, int n, int h, int w, const int* target_ids, int n_ids, int close_ks,
                 int expand_px, int contract_px, int feather_px, uint8_t* mask, void* scratch, size_t scratch_bytes,
                 void* stream);

/* ---- image resamplers of the mask / inference_res paths ----
 * NST_RESIZE_PIL_LANCZOS: Pillow Image.resize((ow, oh), Image.LANCZOS) of RGB frames (sky_swap.py:294-301,
 *   pipeline.py:1089-1097 --inference_res): Resample.c's two integer passes, bit-exact.
 * NST_RESIZE_CV_LINEAR: cv2.resize(m, (ow, oh), interpolation=INTER_LINEAR) of u8 images with c channels
 *   (sky_swap.py:321-324 mask upscale): OpenCV's fixed-point taps restated (cv2 absent: parity unpinned).
 * A resampler is made once per (h, w) -> (oh, ow) geometry: its tap tables live on the device. */
#define NST_RESIZE_PIL_LANCZOS 0
#define NST_RESIZE_CV_LINEAR 1
typedef struct nst_resize nst_resize;
int nst_resize_create(int kind, int h, int w, int oh, int ow, int device, nst_resize** out);
void nst_resize_destroy(nst_resize* r);
int nst_resize_scratch_bytes(const nst_resize* r, int n, size_t* out);
int nst_resize_u8(const nst_resize* r, const uint8_t* in, int n, int c, uint8_t* out, void* scratch,
                  size_t scratch_bytes, void* stream);

/* ---- Region-blend compositor (region_blend.py; pipeline.py:1120-1407 --region_optimize and :1720-1839
 * --region_mode) ----
 * The reference's control logic (random.Random draws, blend specs, animations) stays on the host
 * (neuralstyletransferv1_amd/regions.py); these entry points render, feather, rotate and composite. */
#define NST_REGION_MAX 32     /* regions per composite */
#define NST_REGION_TERMS 9    /* models A..H + the original per region */
#define NST_REGION_MAX_SRC 16 /* sources per composite */
/* mask geometry kinds (generate_region_masks, region_blend.py:925-980) */
#define NST_RG_RECTS 0      /* grid_masks / fractal_quad_masks :109-135, 307-364: region k = rects[k] {y1,y2,x1,x2} */
#define NST_RG_DIAGONAL 1   /* diagonal_masks :138-171: ivals[0] = 1 for x+y, 0 for (W-1-x)+y; dvals[3] = its max */
#define NST_RG_VORONOI 2    /* voronoi_masks :174-236: points[k] = (x, y); divisor[k] = sqrt(w_k)+1e-6 or 0 */
#define NST_RG_RADIAL 3     /* radial_masks :367-401: ivals = cx, cy; dvals[0] = rotation; lo/hi = wedge bounds */
#define NST_RG_WAVES 4      /* wave_masks :404-447: ivals[0] = 0 horizontal, 1 vertical, 2 diagonal;
                               dvals = frequency, amplitude, phase */
#define NST_RG_SPIRAL 5     /* spiral_masks :450-485: ivals = cx, cy; dvals = tightness, rotation, max(H, W) */
#define NST_RG_CONCENTRIC 6 /* concentric_masks :488-516: ivals = cx, cy; dvals[3] = r.max() */
/*
 * Hard (unfeathered) region masks [count][h][w] f32 0/1.  n_gen regions were generated (masks k >= n_gen
 * repeat region n_gen-1; n_gen = 0 gives all ones, :977-978).  Band kinds use lo[k] <= t < hi[k].  All
 * double constants are rounded to fp32 as torch rounds a Python float against a float32 tensor.
 * scratch (NST_RG_WAVES only): h*w + 2052 floats.
 */
int nst_region_masks(int kind, int count, int n_gen, const int* ivals, const double* dvals, const double* lo,
                     const double* hi, const int* rects, const double* points, const double* divisor, int h, int w,
                     float* masks, float* scratch, void* stream);
/* feather_mask (:69-102) in place on k planes: F.pad(reflect, ks/2) + the separable Gaussian whose ks (odd,
 * <= 511) host fp32 taps are the reference's normalised torch taps.  scratch: k*h*w floats. */
int nst_region_feather(float* masks, int k, int h, int w, const float* taps, int ks, float* scratch, void* stream);
/* rotate_all_masks (:25-66): cv2.warpAffine(INTER_LINEAR, BORDER_REPLICATE) of each plane about (W/2, H/2)
 * (OpenCV's fixed-point warp restated: cv2 absent, parity unpinned), then each pixel divided by the sum of
 * the rotated planes clamped to 1e-6.  in != out. */
int nst_region_rotate(const float* in, int k, int h, int w, double angle_deg, float* out, void* stream);
/*
 * warp_all_masks_organic (:737-810, --region_morph) of k planes: each plane j warped by cv2.remap(INTER_LINEAR,
 * BORDER_REFLECT; OpenCV's fixed-point remap restated, cv2 absent: parity unpinned) through
 * x + flow_x * max_disp, y + flow_y * max_disp, flows per mode (0 blob, 1 tentacle, 2 wave, 3 pulse; :688-715;
 * frequency is the noise frequency the mode uses, i.e. 2x for tentacle); blob/tentacle fields are
 * _simplex_noise_2d (:604-652) with the numpy PCG64 draws * 1000 in offsets[((j*2 + field)*2 + octave)*2 + xy]
 * (field 0 seeded morph.seed + 100 j, field 1 that + 1000); then the coverage-gap dilations (5/11/21/41 where
 * the sum < 0.1) and the normalisation by the clamped sum.  in != out.
 */
int nst_region_morph_scratch_floats(int k, int h, int w, size_t* out);
int nst_region_morph(const float* in, int k, int h, int w, int mode, double frequency, double time_offset,
                     double max_disp, const double* offsets, float* out, float* scratch, size_t scratch_floats,
                     void* stream);
/* compute_mask_bbox (:1969-1994): bbox[4k..4k+3] = {x1, y1, x2, y2} (exclusive ends) of the values >
 * threshold in plane k, device int buffer; an empty plane leaves {INT_MAX, INT_MAX, -1, -1}. */
int nst_region_bbox(const float* masks, int k, int h, int w, float threshold, int* bbox, void* stream);
/* scratch floats nst_region_composite_u8 needs (crops mode only) */
int nst_region_scratch_floats(int n, int h, int w, int crops, int with_orig, size_t* out);
/*
 * Region composite of a batch of n frames, out u8 NHWC [n,h,w,3] (ToPILImage truncation) and/or out_f32
 * NCHW [n,3,h,w] in [0,1].  Sources s < n_src: f32 NCHW [n,3,src_hw[2s],src_hw[2s+1]] decoded with
 * src_preset[s] (NST_PRESET_NONE for already-decoded images) and bilinearly fitted; source -1 is the
 * original frame orig u8 NHWC [n,h,w,3] (to_tensor).  Region k blends n_terms[k] (<= 9) terms
 * term_src[9k+j] with weights term_w[9k+j] (region_blend = zeros; += w * src in order).
 *   boxes == NULL: composite_regions(_advanced) (:1049-1108, 1589-1679) over full-frame masks [n_regions][h][w],
 *                  sources fitted to (h, w).
 *   boxes != NULL: composite_from_crops (:2186-2294): region k covers the padded bbox boxes[4k..4k+3] =
 *                  {x1,y1,x2,y2}, its sources are fitted to that crop; then the < 0.1 coverage-gap fill
 *                  (original frame, or max-pool dilation 5/11/21 without one); scratch per
 *                  nst_region_scratch_floats.
 */
int nst_region_composite_u8(const float* const* src_y, const int* src_hw, const int* src_preset, int n_src,
                            const int* n_terms, const int* term_src, const float* term_w, int n_regions,
                            const int* boxes, const uint8_t* orig, const float* masks, int n, int h, int w,
                            float* scratch, size_t scratch_floats, uint8_t* out, float* out_f32, void* stream);
/* --region_optimize crop input (pipeline.py:1309-1332): to_tensor(frame)[:, y1:y2, x1:x2] resized bilinearly
 * (align_corners=False) to out_h x out_w when they differ -> f32 NCHW [n,3,out_h,out_w] in [0,1], the
 * nst_forward NST_IO_F32_NCHW input.  box = {x1, y1, x2, y2}. */
int nst_region_crop_input(const uint8_t* frames, int n, int h, int w, const int* box, int out_h, int out_w, float* out,
                          void* stream);
/* the advanced path's low-resolution outputs (pipeline.py:1786-1796): raw output y [n,3,h,w] decoded with
 * preset, fitted to fit_h x fit_w, then resized bilinearly to out_h x out_w -> decoded f32 NCHW */
int nst_region_resize(const float* y, int n, int h, int w, int preset, int fit_h, int fit_w, int out_h, int out_w,
                      float* out, void* stream);

/* ---- Temporal stage (pipeline.py:1884-1940 --flow_ema, :2072-2086 --motion_blend) ---- */
/* pil_rgb.convert("L") (pipeline.py:1100): Pillow's integer luma (r*19595 + g*38470 + b*7471 + 0x8000) >> 16 of
 * frames [n,h,w,3] -> gray [n,h,w] */
int nst_gray_u8(const uint8_t* rgb, int n, int h, int w, uint8_t* gray, void* stream);
/* cv2.calcOpticalFlowFarneback(prev, next, None, pyr_scale, levels, winsize, iterations, poly_n, poly_sigma, 0)
 * (pipeline.py:1896-1899 passes 0.5, 3, 15, 3, 5, 1.1): OpenCV's optflowgf.cpp restated (cv2 absent: parity
 * unpinned).  prev/next u8 [h,w] device, flow f32 [h,w,2] = (dx, dy); scratch per nst_flow_scratch_floats. */
int nst_flow_scratch_floats(int h, int w, size_t* out);
int nst_flow_farneback(const uint8_t* prev, const uint8_t* next, int h, int w, double pyr_scale, int levels,
                       int winsize, int iterations, int poly_n, double poly_sigma, float* flow, float* scratch,
                       size_t scratch_floats, void* stream);
/* DIS optical flow, the reference's default --flow_method (pipeline.py:1904-1914:
 * cv2.DISOpticalFlow_create(cv2.DISOPTICAL_FLOW_PRESET_FAST).calc(prev, next, None)) for n frame pairs: OpenCV's
 * dis_flow.cpp + variational_refinement.cpp restated with PRESET_FAST's parameters (patch 8, stride 4, finest scale 2,
 * 16 gradient-descent iterations, 5 variational refinement iterations; cv2 absent: parity unpinned).  prev/next u8
 * [n,h,w] device, flow f32 [n,h,w,2] = (dx, dy); scratch per nst_flow_dis_scratch_bytes (NST_E_SHAPE for frames too
 * small for the pyramid: min(round(log2(max(h,w)/32)), floor(log2(min(h,w)/8))) < 2). */
int nst_flow_dis_scratch_bytes(int n, int h, int w, size_t* out);
int nst_flow_dis(const uint8_t* prev, const uint8_t* next, int n, int h, int w, float* flow, void* scratch,
                 size_t scratch_bytes, void* stream);
/* --flow_downscale ds (pipeline.py:1886-1892, 1920-1923): gray [h,w] -> [h//ds, w//ds] (floored, as the reference's
 * (W0 // ds, H0 // ds)) by cv2.resize INTER_AREA (restated: integer scales take resizeAreaFast, others the fractional
 * cells of ResizeArea_Invoker), and the small flow [hs,ws,2] back to [h,w,2] by INTER_LINEAR times mul = ds */
int nst_flow_downscale_gray(const uint8_t* gray, int h, int w, int ds, uint8_t* out, void* stream);
/* cv2.resize(img, (out_w, out_h), interpolation=INTER_AREA) of n u8 images [n,h,w,c] (c <= 4), downscaling only
 * (out <= in): the DIS pyramid (cv2.DISOpticalFlow prepareBuffers) and --flow_downscale */
int nst_resize_area_u8(const uint8_t* in, int n, int h, int w, int c, uint8_t* out, int out_h, int out_w, void* stream);
int nst_flow_upscale(const float* flow_small, int hs, int ws, int h, int w, float mul, float* flow, void* stream);
/* flow EMA (pipeline.py:1926-1931 with _warp_with_flow :425-439): out = clip(alpha*curr + (1-alpha)*warp(prev)),
 * warp = cv2.remap(prev, x + dx, y + dy, INTER_LINEAR, BORDER_REPLICATE) restated; curr/prev/out f32 planar
 * [3,h,w] in [0,1], out != prev */
int nst_flow_fuse(const float* curr, const float* prev, const float* flow, int h, int w, float alpha,
                  float one_minus_alpha, float* out, void* stream);
/* motion-adaptive blend alpha (pipeline.py:2073-2080): m = GaussianBlur(clip(|flow| / motion_norm, 0, 1), sigma),
 * alpha = max_alpha - span * m (span = max_alpha - min_alpha as the fp32 the reference multiplies by);
 * alpha/scratch f32 [h,w] */
int nst_motion_alpha(const float* flow, int h, int w, float motion_norm, double sigma, float max_alpha, float span,
                     float* alpha, float* scratch, void* stream);

/* ---- PNG encode on the owner rank (pipeline.py:2099-2119 `Image.fromarray(out).save(path)`, the reference's
 * default --image_ext png at :2170) ----
 * n u8 frames [n,h,w,c] (c = 1 grey, 3 RGB, 4 RGBA; device) -> n complete PNG files, file j at out + j*out_stride,
 * its byte count in sizes[j] (int64, device).  Every scanline carries the Up filter; each scanline is one deflate
 * block (dynamic Huffman codes built per frame from that frame's run-length tokens, or a stored block where that is
 * smaller), the zlib stream's Adler-32 and the chunks' CRC-32 computed on the device.  Lossless: decoders return
 * the frames' bytes exactly, as from Pillow's file.  out_stride >= nst_png_bound; workspace per
 * nst_png_workspace_bytes; out and out_stride 16-byte aligned; w*c + 1 <= 65535. */
int nst_png_bound(int h, int w, int c, size_t* out_stride);
int nst_png_workspace_bytes(int n, int h, int w, int c, size_t* out);
int nst_png_encode_u8(const uint8_t* frames, int n, int h, int w, int c, uint8_t* out, size_t out_stride,
                      int64_t* sizes, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NST_HIP_H */
