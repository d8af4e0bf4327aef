// seg_deeplab.cpp — C ABI of the DeepLab v3+ mask program (BASELINE.json configs[4]):
// the ResNet-101 (output stride 16) + ASPP + decoder network of modeling/deeplab.py:9-33 in eval mode,
// as sky_swap.py:143-177 load_deeplab builds it (backbone 'resnet', BatchNorm2d, pretrained weights
// from the checkpoint), the mask post-processing of sky_swap.py:185-219 infer_mask, and the two image
// resamplers of the mask path (sky_swap.py:294-301 Pillow LANCZOS working-size downscale,
// :321-324 cv2.resize INTER_LINEAR mask upscale).
//
// Program for a batch of n frames at h x w (NHWC, activations in the compute dtype, channel counts
// padded to the GEMM stage width):
//   stem   im2col (normalisation fused) -> 7x7/2 conv as a GEMM + BN + ReLU -> MaxPool(3,2,1)
//   layer1..layer4: Bottleneck = 1x1 + BN + ReLU, 3x3 (stride, dilation) + BN + ReLU,
//          1x1 + BN + (identity | downsample 1x1/s + BN) + ReLU — one conv_gemm launch each, the
//          residual add and ReLU in the third conv's epilogue (resnet.py:23-43)
//   ASPP   four branches written straight into their channel ranges of the 1280-channel concat,
//          the pooled branch as avgpool -> 1x1 GEMM over n "pixels" -> broadcast (align_corners
//          resize of a 1x1 map), then the 1x1 projection + BN + ReLU (Dropout = identity in eval)
//   decoder ASPP output resized (align_corners=True) into channels 0..255 of a 320-channel concat,
//          the low-level 1x1 (256 -> 48, + 16 zero channels) into 256..319, two 3x3 + BN + ReLU,
//          the 1x1 classifier with bias to fp32 logits
//   head   bilinear (align_corners=True) to h x w fused with the argmax over classes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "nst_hip.h"
#include "nst_internal.h"
#include "seg_internal.h"

using namespace nst;

namespace {

size_t al256(size_t v) { return (v + 255) / 256 * 256; }

int upload_bytes(const void* host, size_t bytes, void** dev) {
  *dev = nullptr;
  if (hipMalloc(dev, bytes) != hipSuccess) { set_error("hipMalloc failed"); return NST_E_HIP; }
  if (hipMemcpy(*dev, host, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(*dev);
    *dev = nullptr;
    set_error("hipMemcpy failed");
    return NST_E_HIP;
  }
  return NST_OK;
}

uint16_t to_bf16(float f) {  // round to nearest even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// One Conv2d (+ BatchNorm2d, or + conv bias) as a conv_gemm layer.
struct SegConv {
  int cin = 0, cout = 0, k = 1, stride = 1, dil = 1, pad = 0;
  int cinp = 0;   // channels per tap the GEMM reads (stage-width multiple; weights zero past cin)
  int coutp = 0;  // packed rows (multiple of 128)
  void* w = nullptr;
  float* scale = nullptr;
  float* shift = nullptr;
};

struct Bottleneck {
  SegConv c1, c2, c3, ds;
  bool has_ds = false;
};

using ParamMap = std::map<std::string, const nst_param*>;

const float* find_param(const ParamMap& pm, const std::string& name, int64_t numel, int* rc) {
  auto it = pm.find(name);
  if (it == pm.end() || it->second->numel != numel || !it->second->data) {
    set_error("missing or mis-shaped DeepLab tensor " + name + " (expected " + std::to_string(numel) + " values)");
    *rc = NST_E_PARAM;
    return nullptr;
  }
  return it->second->data;
}

// Pack W[cout][cin][k][k] (fp32) into [coutp/64][stage = tap*nck + cc][64 rows][stage channels] in the
// compute dtype; eval BatchNorm (bn prefix) or a conv bias (bias name) into per-channel scale/shift.
int build_conv(SegConv& L, const ParamMap& pm, const std::string& wname, const std::string& bn,
               const std::string& bias, int dtype, int cinp_override = 0) {
  int rc = NST_OK;
  const int ck = gemm_stage_channels(dtype);
  const int kk = L.k * L.k;
  const float* W = find_param(pm, wname, (int64_t)L.cout * L.cin * kk, &rc);
  if (!W) return rc;
  L.cinp = cinp_override ? cinp_override : (L.cin + ck - 1) / ck * ck;
  L.coutp = (L.cout + 127) / 128 * 128;
  const int nck = L.cinp / ck, nstage = kk * nck;
  const size_t esz = dtype == NST_DT_F32 ? 4 : 2;
  std::vector<uint8_t> pk((size_t)(L.coutp / 64) * nstage * 64 * ck * esz, 0);
  for (int co = 0; co < L.cout; ++co)
    for (int ci = 0; ci < L.cin; ++ci)
      for (int t = 0; t < kk; ++t) {
        const float v = W[((size_t)co * L.cin + ci) * kk + t];
        const int cc = ci / ck, kc = ci % ck, s = t * nck + cc;
        const size_t e = (((size_t)(co / 64) * nstage + s) * 64 + (co % 64)) * ck + kc;
        if (dtype == NST_DT_F32) std::memcpy(&pk[e * 4], &v, 4);
        else {
          const uint16_t b = dtype == NST_DT_F16 ? f32_to_f16_rne(v) : to_bf16(v);
          std::memcpy(&pk[e * 2], &b, 2);
        }
      }
  std::vector<float> sc(L.coutp, 0.f), sh(L.coutp, 0.f);
  if (!bn.empty()) {
    const float* g = find_param(pm, bn + ".weight", L.cout, &rc);
    const float* b = g ? find_param(pm, bn + ".bias", L.cout, &rc) : nullptr;
    const float* m = b ? find_param(pm, bn + ".running_mean", L.cout, &rc) : nullptr;
    const float* v = m ? find_param(pm, bn + ".running_var", L.cout, &rc) : nullptr;
    if (!v) return rc;
    for (int c = 0; c < L.cout; ++c) {  // torch's batch_norm inference terms (float)
      const float inv = 1.0f / std::sqrt(v[c] + 1e-5f);
      sc[c] = inv * g[c];
      sh[c] = b[c] - m[c] * sc[c];
    }
  } else {
    const float* b = bias.empty() ? nullptr : find_param(pm, bias, L.cout, &rc);
    if (!bias.empty() && !b) return rc;
    for (int c = 0; c < L.cout; ++c) {
      sc[c] = 1.f;
      sh[c] = b ? b[c] : 0.f;
    }
  }
  if ((rc = upload_bytes(pk.data(), pk.size(), &L.w)) != NST_OK) return rc;
  if ((rc = upload_bytes(sc.data(), sc.size() * 4, (void**)&L.scale)) != NST_OK) return rc;
  return upload_bytes(sh.data(), sh.size() * 4, (void**)&L.shift);
}

void free_conv(SegConv& L) {
  if (L.w) (void)hipFree(L.w);
  if (L.scale) (void)hipFree(L.scale);
  if (L.shift) (void)hipFree(L.shift);
  L.w = nullptr;
  L.scale = L.shift = nullptr;
}

int out_extent(int in, int k, int s, int d, int p) { return (in + 2 * p - d * (k - 1) - 1) / s + 1; }

}  // namespace

struct nst_seg {
  int device = 0, dtype = NST_DT_BF16, nc = 0, ncs = 0;
  // the GEMM convs' arithmetic: dtype, or NST_DT_F32S with dtype = NST_DT_F32 (the fp32 layout everywhere, each
  // conv's operands split into fp16 pairs in registers: conv_gemm.hip gemm_conv_kernel)
  int gemm_dt = NST_DT_BF16;
  int cache_n = 0, cache_h = 0, cache_w = 0;  // geometry of the cached workspace plan
  size_t cache_partial = 0;
  SegConv stem;
  std::vector<Bottleneck> blocks;  // layer1 (3), layer2 (4), layer3 (23), layer4 (3: multi-grid 1, 2, 4)
  int layer_last[4] = {0, 0, 0, 0};
  SegConv aspp[4], gap, proj, low, dec1, dec2, cls;
};

namespace {

struct SegPlan {
  int n = 0, h = 0, w = 0;
  int h2, w2, h4, w4, h8, w8, h16, w16;
  size_t col, stem, pool, x0, x1, t1, t2, r, lowf, cat5, gapv, gapo, aspo, dcat, d1, d2, logits, partial, end;
};

// launch context: a dry run walks the program only to size the split-K scratch
struct SegRun {
  bool dry = false;
  size_t partial_need = 0;
  float* partial = nullptr;
  size_t partial_bytes = 0;
};

SegPlan seg_plan(const nst_seg* s, int n, int h, int w) {
  SegPlan P;
  P.n = n; P.h = h; P.w = w;
  P.h2 = out_extent(h, 7, 2, 1, 3); P.w2 = out_extent(w, 7, 2, 1, 3);
  P.h4 = out_extent(P.h2, 3, 2, 1, 1); P.w4 = out_extent(P.w2, 3, 2, 1, 1);
  P.h8 = out_extent(P.h4, 3, 2, 1, 1); P.w8 = out_extent(P.w4, 3, 2, 1, 1);
  P.h16 = out_extent(P.h8, 3, 2, 1, 1); P.w16 = out_extent(P.w8, 3, 2, 1, 1);
  const size_t e = s->dtype == NST_DT_F32 ? 4 : 2;
  const size_t p4 = (size_t)n * P.h4 * P.w4, p8 = (size_t)n * P.h8 * P.w8, p16 = (size_t)n * P.h16 * P.w16;
  // largest block tensors: outputs 4*planes, intermediates planes (layer1 at /4 .. layer4 at /16)
  const size_t big = std::max(std::max(p4 * 256, p8 * 512), std::max(p16 * 1024, p16 * 2048)) * e;
  const size_t mid = std::max(std::max(p4 * 64, p4 * 128 /* layer2's first conv1 runs at /4 */),
                              std::max(p8 * 128, std::max(p8 * 256, p16 * 512))) * e;
  size_t o = 0;
  auto take = [&](size_t bytes) { const size_t r = o; o += al256(bytes); return r; };
  P.col = take((size_t)n * P.h2 * P.w2 * s->stem.cinp * e);
  P.stem = take((size_t)n * P.h2 * P.w2 * 64 * e);
  P.pool = take(p4 * 64 * e);
  P.x0 = take(big);
  P.x1 = take(big);
  P.t1 = take(mid);
  P.t2 = take(mid);
  P.r = take(big);
  P.lowf = take(p4 * 256 * e);
  P.cat5 = take(p16 * 1280 * e);
  P.gapv = take((size_t)n * 2048 * e);
  P.gapo = take((size_t)n * 256 * e);
  P.aspo = take(p16 * 256 * e);
  P.dcat = take(p4 * 320 * e);
  P.d1 = take(p4 * 256 * e);
  P.d2 = take(p4 * 256 * e);
  P.logits = take(p4 * s->ncs * 4);
  P.partial = o;
  P.end = o;
  return P;
}

// one conv_gemm launch (or, in a dry run, its split-K scratch need)
hipError_t run(const nst_seg* s, SegRun& R, const SegConv& L, const void* in, int n, int hi, int wi, int cs, void* out,
               int ho, int wo, int out_cs, int out_off, const void* res, int res_cs, int relu, int out_f32,
               int cout_store, hipStream_t st) {
  GemmConvParams p;
  std::memset(&p, 0, sizeof(p));
  p.in = in;
  p.hi = hi; p.wi = wi; p.cs = cs;
  p.cin = L.cinp;
  p.kh = p.kw = L.k;
  p.stride = L.stride; p.dil = L.dil; p.pad = L.pad;
  p.ho = ho; p.wo = wo; p.npix = n * ho * wo;
  p.wpk = L.w; p.scale = L.scale; p.shift = L.shift;
  p.res = res; p.res_cs = res_cs;
  p.relu = relu;
  p.out = out; p.out_cs = out_cs; p.out_off = out_off;
  p.cout_store = cout_store;
  p.out_f32 = out_f32;
  p.ksplit = 1;
  const size_t need = gemm_partial_bytes(s->dtype, p);
  if (R.dry) {
    R.partial_need = std::max(R.partial_need, need);
    return hipSuccess;
  }
  p.partial = (need && need <= R.partial_bytes) ? R.partial : nullptr;
  return launch_gemm_conv(s->gemm_dt, p, st);
}

#define SEG_CHECK(expr)                                                                            \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) { set_error(std::string(#expr) + ": " + hipGetErrorString(_e)); return NST_E_HIP; } \
  } while (0)

int seg_forward_impl(nst_seg* s, const SegPlan& P, SegRun& R, const void* x, int x_u8, float* logits_out,
                     uint8_t* pred, char* ws, hipStream_t st) {
  const int n = P.n;
  const size_t e = s->dtype == NST_DT_F32 ? 4 : 2;
  // stem
  if (!R.dry) SEG_CHECK(launch_seg_stem_im2col(s->dtype, x, x_u8, n, P.h, P.w, P.h2, P.w2, s->stem.cinp, ws + P.col, st));
  SEG_CHECK(run(s, R, s->stem, ws + P.col, n, P.h2, P.w2, s->stem.cinp, ws + P.stem, P.h2, P.w2, 64, 0, nullptr, 0, 1, 0,
                64, st));
  if (!R.dry) SEG_CHECK(launch_seg_maxpool(s->dtype, ws + P.stem, n, P.h2, P.w2, 64, ws + P.pool, P.h4, P.w4, st));
  // residual layers
  const char* cur = ws + P.pool;
  int ch = 64, hh = P.h4, ww = P.w4;
  char* xb[2] = {ws + P.x0, ws + P.x1};
  int xi = 0;
  for (size_t b = 0; b < s->blocks.size(); ++b) {
    const Bottleneck& B = s->blocks[b];
    const int planes = B.c1.cout, outc = B.c3.cout;
    const int ho = out_extent(hh, 3, B.c2.stride, B.c2.dil, B.c2.pad), wo = out_extent(ww, 3, B.c2.stride, B.c2.dil, B.c2.pad);
    SEG_CHECK(run(s, R, B.c1, cur, n, hh, ww, ch, ws + P.t1, hh, ww, planes, 0, nullptr, 0, 1, 0, planes, st));
    SEG_CHECK(run(s, R, B.c2, ws + P.t1, n, hh, ww, planes, ws + P.t2, ho, wo, planes, 0, nullptr, 0, 1, 0, planes, st));
    const void* res = cur;
    if (B.has_ds) {
      SEG_CHECK(run(s, R, B.ds, cur, n, hh, ww, ch, ws + P.r, ho, wo, outc, 0, nullptr, 0, 0, 0, outc, st));
      res = ws + P.r;
    }
    char* dst = (b == (size_t)s->layer_last[0]) ? ws + P.lowf : xb[xi];
    SEG_CHECK(run(s, R, B.c3, ws + P.t2, n, ho, wo, planes, dst, ho, wo, outc, 0, res, outc, 1, 0, outc, st));
    if (dst == xb[xi]) xi ^= 1;
    cur = dst;
    ch = outc; hh = ho; ww = wo;
  }
  // ASPP (input: layer4 output, 2048 channels at /16)
  const int h16 = hh, w16 = ww;
  for (int i = 0; i < 4; ++i)
    SEG_CHECK(run(s, R, s->aspp[i], cur, n, h16, w16, 2048, ws + P.cat5, h16, w16, 1280, 256 * i, nullptr, 0, 1, 0, 256, st));
  if (!R.dry) SEG_CHECK(launch_seg_avgpool(s->dtype, cur, n, h16 * w16, 2048, 2048, ws + P.gapv, st));
  SEG_CHECK(run(s, R, s->gap, ws + P.gapv, n, 1, 1, 2048, ws + P.gapo, 1, 1, 256, 0, nullptr, 0, 1, 0, 256, st));
  if (!R.dry) SEG_CHECK(launch_seg_resize_ac(s->dtype, ws + P.gapo, n, 1, 1, 256, 256, ws + P.cat5, h16, w16, 1280, 1024, st));
  SEG_CHECK(run(s, R, s->proj, ws + P.cat5, n, h16, w16, 1280, ws + P.aspo, h16, w16, 256, 0, nullptr, 0, 1, 0, 256, st));
  // decoder
  SEG_CHECK(run(s, R, s->low, ws + P.lowf, n, P.h4, P.w4, 256, ws + P.dcat, P.h4, P.w4, 320, 256, nullptr, 0, 1, 0, 64, st));
  if (!R.dry) SEG_CHECK(launch_seg_resize_ac(s->dtype, ws + P.aspo, n, h16, w16, 256, 256, ws + P.dcat, P.h4, P.w4, 320, 0, st));
  SEG_CHECK(run(s, R, s->dec1, ws + P.dcat, n, P.h4, P.w4, 320, ws + P.d1, P.h4, P.w4, 256, 0, nullptr, 0, 1, 0, 256, st));
  SEG_CHECK(run(s, R, s->dec2, ws + P.d1, n, P.h4, P.w4, 256, ws + P.d2, P.h4, P.w4, 256, 0, nullptr, 0, 1, 0, 256, st));
  SEG_CHECK(run(s, R, s->cls, ws + P.d2, n, P.h4, P.w4, 256, ws + P.logits, P.h4, P.w4, s->ncs, 0, nullptr, 0, 0, 1,
                s->ncs, st));
  (void)e;
  if (!R.dry && (logits_out || pred))
    SEG_CHECK(launch_seg_upsample_argmax((const float*)(ws + P.logits), n, P.h4, P.w4, s->nc, s->ncs, P.h, P.w, pred,
                                         logits_out, st));
  return NST_OK;
}

// the full plan: the layout above plus the split-K scratch a dry run of the program asks for
SegPlan seg_plan_full(nst_seg* s, int n, int h, int w) {
  SegPlan P = seg_plan(s, n, h, w);
  size_t partial = 0;
  if (s->cache_n == n && s->cache_h == h && s->cache_w == w) {
    partial = s->cache_partial;
  } else {
    SegRun R;
    R.dry = true;
    static char dummy[1];
    (void)seg_forward_impl(s, P, R, dummy, 1, nullptr, nullptr, dummy, nullptr);
    partial = R.partial_need;
    s->cache_n = n; s->cache_h = h; s->cache_w = w; s->cache_partial = partial;
  }
  P.end = P.partial + al256(partial);
  return P;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Resamplers: per-geometry tables computed on the host in double (as Pillow / OpenCV compute them)
struct nst_resize {
  int kind = 0, h = 0, w = 0, oh = 0, ow = 0, device = 0;
  // PIL: bounds + int taps per axis; ybox window of the horizontal pass
  int kx = 0, ky = 0, y0 = 0, th = 0, need_h = 0, need_v = 0;
  void *xb = nullptr, *xk = nullptr, *yb = nullptr, *yk = nullptr;
  // cv2: offsets + short taps
  void *xofs = nullptr, *xa = nullptr, *yofs = nullptr, *ya = nullptr;
};

namespace {

double pil_sinc(double x) {
  if (x == 0.0) return 1.0;
  x = x * M_PI;
  return std::sin(x) / x;
}
double pil_lanczos(double x) {  // Resample.c lanczos_filter, support 3
  if (-3.0 <= x && x < 3.0) return pil_sinc(x) * pil_sinc(x / 3);
  return 0.0;
}

// Resample.c precompute_coeffs + normalize_coeffs_8bpc (PRECISION_BITS = 22)
int pil_coeffs(int in_size, float in0, float in1, int out_size, std::vector<int>& bounds, std::vector<int>& kk) {
  double scale, filterscale;
  filterscale = scale = (double)(in1 - in0) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 3.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  std::vector<double> k((size_t)out_size * ksize, 0.0);
  bounds.assign((size_t)out_size * 2, 0);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double* kp = &k[(size_t)xx * ksize];
    for (int x = 0; x < xmax; ++x) {
      const double wv = pil_lanczos((x + xmin - center + 0.5) * ss);
      kp[x] = wv;
      ww += wv;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) kp[x] /= ww;
    bounds[xx * 2] = xmin;
    bounds[xx * 2 + 1] = xmax;
  }
  kk.assign(k.size(), 0);
  for (size_t i = 0; i < k.size(); ++i)
    kk[i] = k[i] < 0 ? (int)(-0.5 + k[i] * (1 << 22)) : (int)(0.5 + k[i] * (1 << 22));
  return ksize;
}

short sat_short(float v) {  // saturate_cast<short>(float): cvRound (nearest, ties to even) then clamp
  const double r = std::nearbyint((double)v);
  return (short)std::min(32767.0, std::max(-32768.0, r));
}

// OpenCV resize INTER_LINEAR fixed-point tables (imgproc/resize.cpp): fx = (float)((dx+0.5)*scale - 0.5),
// sx = floor(fx), fx -= sx, clamped at the edges; taps saturate_cast<short>((1-fx)*2048), (fx*2048)
void cv_axis(int in, int out, bool clamp_taps, std::vector<int>& ofs, std::vector<short>& taps) {
  const double scale = 1.0 / ((double)out / in);
  ofs.resize(out);
  taps.resize((size_t)out * 2);
  for (int d = 0; d < out; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int sidx = (int)std::floor(f);
    f -= sidx;
    if (clamp_taps) {
      if (sidx < 0) { f = 0; sidx = 0; }
      if (sidx >= in - 1) { f = 0; sidx = in - 1; }
    }
    ofs[d] = sidx;
    taps[2 * d] = sat_short((1.f - f) * 2048.f);
    taps[2 * d + 1] = sat_short(f * 2048.f);
  }
}

}  // namespace

extern "C" {

int nst_seg_create(const nst_param* params, int n_params, int num_classes, int compute_dtype, int device,
                   nst_seg** out) {
  if (!params || n_params <= 0 || !out || num_classes < 2 || num_classes > 256 ||
      (compute_dtype != NST_DT_F32 && compute_dtype != NST_DT_BF16 && compute_dtype != NST_DT_F16 &&
       compute_dtype != NST_DT_F32S)) {
    set_error("nst_seg_create: invalid arguments");
    return NST_E_INVALID;
  }
  *out = nullptr;
  ParamMap pm;
  for (int i = 0; i < n_params; ++i)
    if (params[i].name) pm[params[i].name] = &params[i];
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) { set_error("nst_seg_create: bad device"); return NST_E_INVALID; }
  auto* s = new nst_seg();
  s->device = device;
  s->gemm_dt = compute_dtype;
  if (compute_dtype == NST_DT_F32S) compute_dtype = NST_DT_F32;  // layout, packing and the non-GEMM kernels: fp32
  s->dtype = compute_dtype;
  s->nc = num_classes;
  s->ncs = (num_classes + 3) / 4 * 4;
  const int ck = gemm_stage_channels(compute_dtype);
  int rc = NST_OK;
  auto conv = [&](SegConv& L, int cin, int cout, int k, int stride, int dil, int pad, const std::string& wname,
                  const std::string& bn, const std::string& bias = "", int cinp = 0) {
    if (rc != NST_OK) return;
    L.cin = cin; L.cout = cout; L.k = k; L.stride = stride; L.dil = dil; L.pad = pad;
    rc = build_conv(L, pm, wname, bn, bias, compute_dtype, cinp);
  };
  // stem: the 7x7x3 taps as one K = 147 row (the im2col buffer), padded to the stage width
  {
    auto it = pm.find("backbone.conv1.weight");
    if (it == pm.end() || it->second->numel != 64 * 3 * 49) {
      set_error("missing or mis-shaped DeepLab tensor backbone.conv1.weight");
      rc = NST_E_PARAM;
    } else {
      // reorder [64][3][7][7] -> [64][(ky*7+kx)*3+c] so the im2col row order is tap-major
      std::vector<float> wr((size_t)64 * 147);
      const float* W = it->second->data;
      for (int co = 0; co < 64; ++co)
        for (int c = 0; c < 3; ++c)
          for (int t = 0; t < 49; ++t) wr[(size_t)co * 147 + t * 3 + c] = W[((size_t)co * 3 + c) * 49 + t];
      nst_param tmp{"stem.reordered", wr.data(), (int64_t)wr.size()};
      ParamMap pm2 = pm;
      pm2["stem.reordered"] = &tmp;
      s->stem.cin = 147; s->stem.cout = 64; s->stem.k = 1;
      rc = build_conv(s->stem, pm2, "stem.reordered", "backbone.bn1", "", compute_dtype, (147 + ck - 1) / ck * ck);
    }
  }
  // layer1..3 (resnet.py:67-69, output stride 16: strides 1,2,2, dilation 1) and the multi-grid layer4
  // (:70, :94-111: stride 1, dilations 2*{1,2,4})
  const int nblocks[3] = {3, 4, 23}, planes_of[4] = {64, 128, 256, 512}, stride_of[4] = {1, 2, 2, 1};
  int inplanes = 64;
  for (int l = 0; l < 4 && rc == NST_OK; ++l) {
    const int nb = l < 3 ? nblocks[l] : 3, planes = planes_of[l];
    for (int i = 0; i < nb && rc == NST_OK; ++i) {
      Bottleneck B;
      const std::string pre = "backbone.layer" + std::to_string(l + 1) + "." + std::to_string(i);
      const int stride = i == 0 ? stride_of[l] : 1;
      const int dil = l < 3 ? 1 : 2 * (1 << i);
      conv(B.c1, inplanes, planes, 1, 1, 1, 0, pre + ".conv1.weight", pre + ".bn1");
      conv(B.c2, planes, planes, 3, stride, dil, dil, pre + ".conv2.weight", pre + ".bn2");
      conv(B.c3, planes, planes * 4, 1, 1, 1, 0, pre + ".conv3.weight", pre + ".bn3");
      if (i == 0) {
        B.has_ds = true;
        conv(B.ds, inplanes, planes * 4, 1, stride, 1, 0, pre + ".downsample.0.weight", pre + ".downsample.1");
      }
      inplanes = planes * 4;
      s->blocks.push_back(B);
    }
    s->layer_last[l] = (int)s->blocks.size() - 1;
  }
  // ASPP (aspp.py:43-60, output stride 16: dilations 1, 6, 12, 18)
  const int adil[4] = {1, 6, 12, 18};
  for (int i = 0; i < 4; ++i) {
    const std::string pre = "aspp.aspp" + std::to_string(i + 1);
    conv(s->aspp[i], 2048, 256, i == 0 ? 1 : 3, 1, adil[i], i == 0 ? 0 : adil[i], pre + ".atrous_conv.weight", pre + ".bn");
  }
  conv(s->gap, 2048, 256, 1, 1, 1, 0, "aspp.global_avg_pool.1.weight", "aspp.global_avg_pool.2");
  conv(s->proj, 1280, 256, 1, 1, 1, 0, "aspp.conv1.weight", "aspp.bn1");
  // decoder (decoder.py:19-30); the 304-channel concat is stored as 320 (16 zero channels)
  conv(s->low, 256, 48, 1, 1, 1, 0, "decoder.conv1.weight", "decoder.bn1");
  conv(s->dec1, 304, 256, 3, 1, 1, 1, "decoder.last_conv.0.weight", "decoder.last_conv.1", "", 320);
  conv(s->dec2, 256, 256, 3, 1, 1, 1, "decoder.last_conv.4.weight", "decoder.last_conv.5");
  conv(s->cls, 256, num_classes, 1, 1, 1, 0, "decoder.last_conv.8.weight", "", "decoder.last_conv.8.bias");
  if (prev >= 0) (void)hipSetDevice(prev);
  if (rc != NST_OK) {
    nst_seg_destroy(s);
    return rc;
  }
  *out = s;
  return NST_OK;
}

void nst_seg_destroy(nst_seg* s) {
  if (!s) return;
  free_conv(s->stem);
  for (auto& B : s->blocks) {
    free_conv(B.c1); free_conv(B.c2); free_conv(B.c3); free_conv(B.ds);
  }
  for (auto& L : s->aspp) free_conv(L);
  free_conv(s->gap); free_conv(s->proj); free_conv(s->low); free_conv(s->dec1); free_conv(s->dec2); free_conv(s->cls);
  delete s;
}

int nst_seg_num_classes(const nst_seg* s) { return s ? s->nc : 0; }

int nst_seg_workspace_bytes(const nst_seg* s, int n, int h, int w, size_t* out) {
  if (!s || !out || n <= 0 || h < 8 || w < 8) { set_error("nst_seg_workspace_bytes: invalid arguments"); return NST_E_INVALID; }
  *out = seg_plan_full(const_cast<nst_seg*>(s), n, h, w).end;
  return NST_OK;
}

int nst_seg_forward(nst_seg* s, const void* x, int x_fmt, int n, int h, int w, float* logits, uint8_t* pred,
                    void* workspace, size_t workspace_bytes, void* stream) {
  if (!s || !x || n <= 0 || h < 8 || w < 8 || (x_fmt != NST_IO_F32_NCHW && x_fmt != NST_IO_U8_NHWC)) {
    set_error("nst_seg_forward: invalid arguments (h, w >= 8)");
    return NST_E_INVALID;
  }
  if ((size_t)n * h * w > (size_t)1 << 31) { set_error("nst_seg_forward: batch too large"); return NST_E_SHAPE; }
  const SegPlan P = seg_plan_full(s, n, h, w);
  if (!workspace || workspace_bytes < P.end) { set_error("nst_seg_forward: workspace too small"); return NST_E_WORKSPACE; }
  SegRun R;
  R.partial = (float*)((char*)workspace + P.partial);
  R.partial_bytes = P.end - P.partial;
  return seg_forward_impl(s, P, R, x, x_fmt == NST_IO_U8_NHWC, logits, pred, (char*)workspace, (hipStream_t)stream);
}

int nst_seg_mask_scratch_bytes(int n, int h, int w, size_t* out) {
  if (!out || n <= 0 || h <= 0 || w <= 0) { set_error("nst_seg_mask_scratch_bytes: invalid arguments"); return NST_E_INVALID; }
  const size_t px = (size_t)n * h * w;
  *out = al256(px) * 2 + al256(px * 4);
  return NST_OK;
}

int nst_seg_mask(const uint8_t* pred, int n, int h, int w, const int* target_ids, int n_ids, int close_ks,
                 int expand_px, int contract_px, int feather_px, uint8_t* mask, void* scratch, size_t scratch_bytes,
                 void* stream) {
  if (!pred || !mask || n <= 0 || h <= 0 || w <= 0 || !target_ids || n_ids <= 0 || close_ks < 0 || expand_px < 0 ||
      contract_px < 0 || feather_px < 0) {
    set_error("nst_seg_mask: invalid arguments");
    return NST_E_INVALID;
  }
  size_t need = 0;
  nst_seg_mask_scratch_bytes(n, h, w, &need);
  if (!scratch || scratch_bytes < need) { set_error("nst_seg_mask: scratch too small"); return NST_E_WORKSPACE; }
  const size_t px = (size_t)n * h * w;
  uint8_t* a = (uint8_t*)scratch;
  uint8_t* b = a + al256(px);
  float* ftmp = (float*)(b + al256(px));
  hipStream_t st = (hipStream_t)stream;
  SegIdSet ids;
  std::memset(&ids, 0, sizeof(ids));
  for (int i = 0; i < n_ids; ++i)
    if (target_ids[i] >= 0 && target_ids[i] < 256) ids.bits[target_ids[i] >> 5] |= 1u << (target_ids[i] & 31);
  // sky = OR of (pred == id) * 255 (sky_swap.py:199-202) -> mask
  SEG_CHECK(launch_seg_select(pred, px, ids, mask, st));
  // MORPH_CLOSE = dilate then erode (sky_swap.py:204; always 5x5 there: morph_close_ks never reaches infer_mask)
  if (close_ks > 1) {
    SEG_CHECK(launch_seg_morph(mask, n, h, w, close_ks, 0, a, b, st));
    SEG_CHECK(launch_seg_morph(b, n, h, w, close_ks, 1, a, mask, st));
  }
  if (expand_px > 0) SEG_CHECK(launch_seg_morph(mask, n, h, w, 2 * expand_px + 1, 0, a, mask, st));
  if (contract_px > 0) SEG_CHECK(launch_seg_morph(mask, n, h, w, 2 * contract_px + 1, 1, a, mask, st));
  if (feather_px > 0) {
    SEG_CHECK(hipMemcpyAsync(b, mask, px, hipMemcpyDeviceToDevice, st));
    SEG_CHECK(launch_seg_gauss_u8(b, n, h, w, (float)feather_px * 0.5f, ftmp, mask, st));
  }
  return NST_OK;
}

int nst_resize_create(int kind, int h, int w, int oh, int ow, int device, nst_resize** out) {
  if (!out || h <= 0 || w <= 0 || oh <= 0 || ow <= 0 || (kind != NST_RESIZE_PIL_LANCZOS && kind != NST_RESIZE_CV_LINEAR)) {
    set_error("nst_resize_create: invalid arguments");
    return NST_E_INVALID;
  }
  *out = nullptr;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) { set_error("nst_resize_create: bad device"); return NST_E_INVALID; }
  auto* r = new nst_resize();
  r->kind = kind; r->h = h; r->w = w; r->oh = oh; r->ow = ow; r->device = device;
  int rc = NST_OK;
  if (kind == NST_RESIZE_PIL_LANCZOS) {
    // ImagingResampleInner with box (0, 0, w, h)
    std::vector<int> xb, xk, yb, yk;
    r->kx = pil_coeffs(w, 0.f, (float)w, ow, xb, xk);
    r->ky = pil_coeffs(h, 0.f, (float)h, oh, yb, yk);
    r->need_h = ow != w;
    r->need_v = oh != h;
    r->y0 = 0;
    r->th = h;
    if (r->need_h) {
      const int first = yb[0], last = yb[(size_t)oh * 2 - 2] + yb[(size_t)oh * 2 - 1];
      if (r->need_v) {
        for (int i = 0; i < oh; ++i) yb[(size_t)i * 2] -= first;
        r->y0 = first;
        r->th = last - first;
      }
    }
    if (rc == NST_OK) rc = upload_bytes(xb.data(), xb.size() * 4, &r->xb);
    if (rc == NST_OK) rc = upload_bytes(xk.data(), xk.size() * 4, &r->xk);
    if (rc == NST_OK) rc = upload_bytes(yb.data(), yb.size() * 4, &r->yb);
    if (rc == NST_OK) rc = upload_bytes(yk.data(), yk.size() * 4, &r->yk);
  } else {
    std::vector<int> xo, yo;
    std::vector<short> xa, ya;
    cv_axis(w, ow, true, xo, xa);
    cv_axis(h, oh, false, yo, ya);  // rows are clamped at read time, taps kept (resizeGeneric_Invoker)
    if (rc == NST_OK) rc = upload_bytes(xo.data(), xo.size() * 4, &r->xofs);
    if (rc == NST_OK) rc = upload_bytes(xa.data(), xa.size() * 2, &r->xa);
    if (rc == NST_OK) rc = upload_bytes(yo.data(), yo.size() * 4, &r->yofs);
    if (rc == NST_OK) rc = upload_bytes(ya.data(), ya.size() * 2, &r->ya);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  if (rc != NST_OK) {
    nst_resize_destroy(r);
    return rc;
  }
  *out = r;
  return NST_OK;
}

void nst_resize_destroy(nst_resize* r) {
  if (!r) return;
  for (void* p : {r->xb, r->xk, r->yb, r->yk, r->xofs, r->xa, r->yofs, r->ya})
    if (p) (void)hipFree(p);
  delete r;
}

int nst_resize_scratch_bytes(const nst_resize* r, int n, size_t* out) {
  if (!r || !out || n <= 0) { set_error("nst_resize_scratch_bytes: invalid arguments"); return NST_E_INVALID; }
  *out = r->kind == NST_RESIZE_PIL_LANCZOS && r->need_h && r->need_v ? (size_t)n * r->th * r->ow * 3 : 0;
  return NST_OK;
}

int nst_resize_u8(const nst_resize* r, const uint8_t* in, int n, int c, uint8_t* out, void* scratch,
                  size_t scratch_bytes, void* stream) {
  if (!r || !in || !out || n <= 0 || c <= 0 || (r->kind == NST_RESIZE_PIL_LANCZOS && c != 3)) {
    set_error("nst_resize_u8: invalid arguments (LANCZOS takes RGB, c = 3)");
    return NST_E_INVALID;
  }
  size_t need = 0;
  nst_resize_scratch_bytes(r, n, &need);
  if (scratch_bytes < need || (need && !scratch)) { set_error("nst_resize_u8: scratch too small"); return NST_E_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  if (r->kind == NST_RESIZE_PIL_LANCZOS) {
    if (!r->need_h && !r->need_v) {
      SEG_CHECK(hipMemcpyAsync(out, in, (size_t)n * r->h * r->w * 3, hipMemcpyDeviceToDevice, st));
      return NST_OK;
    }
    SEG_CHECK(launch_resize_pil_u8(in, n, r->h, r->w, (uint8_t*)scratch, r->y0, r->th, out, r->oh, r->ow,
                                   (const int*)r->xb, (const int*)r->xk, r->kx, (const int*)r->yb, (const int*)r->yk,
                                   r->ky, r->need_h, r->need_v, st));
  } else {
    SEG_CHECK(launch_resize_linear_cv_u8(in, n, r->h, r->w, c, out, r->oh, r->ow, (const int*)r->xofs,
                                         (const short*)r->xa, (const int*)r->yofs, (const short*)r->ya, st));
  }
  return NST_OK;
}

}  // extern "C"
