// vgg_gatys.cpp — C ABI of the Gatys optimisation loop (BASELINE.json configs[2]): a VGG-19
// feature extractor (torchvision's `features` layout, state_dict keys features.N.weight/.bias),
// content + Gram style losses, their gradient with respect to the image, and Adam on the image.
//
// The reference ships only the two helpers this path is built around — utils.py:80-83
// gram_matrix and utils.py:93-96 preprocess_for_vgg (there is no VGG network, loss
// or optimiser in it) — so the network and loop follow Gatys et al. (relu1_1..relu5_1 style Grams,
// relu4_2 content) with torch's definitions of each piece; parity is against a torch-CPU
// restatement (oracle/gatys_oracle.py), not the reference ("parity unpinned").
//
// Program (per image, h and w multiples of 16; bf16 activations, fp32 accumulation):
//   forward: conv1_1 (image -> normalised in the fill) .. conv5_1, the 13 convs the loss needs.
//            Block 1 (512x512-scale maps, 64 channels: thousands of tiles) runs on the generic
//            implicit-GEMM kernel, which stores the pre-activation z and lets the consumer apply the
//            ReLU in its fill (unit IN table); conv2_1 .. conv5_1 (128-512 channels on 256^2 .. 32^2
//            maps: a few hundred tiles, 4.6K-long K) run on the K-streaming GEMM conv of the DeepLab
//            program (conv_gemm.hip: small LDS stages, 8 waves per CU, split-K below a wave of the chip)
//            with the ReLU in its epilogue, so they store r = ReLU(z).  Every consumer of a stored map
//            rectifies it or masks with it (ReLU(r) = r, r > 0 <=> z > 0), so both forms serve the
//            pools, Grams, content term and backward masks unchanged;
//   losses:  Grams of ReLU(z) at the 5 style layers (nst_gram, NHWC) vs the style targets, MSE of
//            ReLU(z4_2) vs the content target;
//   backward: the same generic conv kernel over the masked output gradient with flipped,
//            transposed weights, layer by layer down to the image; the style gradient is an MFMA
//            GEMM of ReLU(z) against 4 beta w_l (G - A) / (c^3 hw) fused with the ReLU backward.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "nst_hip.h"
#include "nst_internal.h"
#include "seg_internal.h"

using namespace nst;

namespace {

// features index, cin, cout; pool_after: a MaxPool2d(2) follows this conv's ReLU
struct VggConvDef {
  int idx, cin, cout;
  bool pool_after;
};
const VggConvDef kConvs[13] = {
    {0, 3, 64, false},    {2, 64, 64, true},                                               // block 1
    {5, 64, 128, false},  {7, 128, 128, true},                                             // block 2
    {10, 128, 256, false}, {12, 256, 256, false}, {14, 256, 256, false}, {16, 256, 256, true},  // block 3
    {19, 256, 512, false}, {21, 512, 512, false}, {23, 512, 512, false}, {25, 512, 512, true},  // block 4
    {28, 512, 512, false},                                                                 // conv5_1
};
const int kStyle[5] = {0, 2, 4, 8, 12};  // conv indices of relu1_1, relu2_1, relu3_1, relu4_1, relu5_1
const int kContent = 9;                  // relu4_2
const float kMean[3] = {0.485f, 0.456f, 0.406f}, kStd[3] = {0.229f, 0.224f, 0.225f};  // utils.py:93-96

struct VggConv {
  VggConvDef d;
  int cinp, coutp;
  const ConvKernelInfo *kf = nullptr, *kb = nullptr;  // forward / input-gradient kernels (generic)
  void *wf = nullptr, *wb = nullptr;
  float *bf = nullptr, *bb = nullptr;
  // conv_gemm.hip path: forward (conv2_1 onward) and input gradient (conv2_1 onward)
  bool gemm_f = false, gemm_b = false;
  void *gwf = nullptr, *gwb = nullptr;
  float *gscale = nullptr, *gshift = nullptr, *gzero = nullptr;
};
// the layers that may take the GEMM conv: every conv whose input has >= 64 channels and whose map is at most a
// quarter of the image (conv2_1 onward); input gradients of the same layers
// (NST_VGG_GEMM_F / NST_VGG_GEMM_B: bitmasks of the layers whose forward / input gradient take the GEMM conv, for
// sweeps.  Default: conv5_1 only, both ways (r04 sweep, profiles/r04_s_gatys_sweep.txt: with its operand fragments
// kept live the halo-staged generic kernel beats the GEMM on conv2_1..conv4_4 too: 1.094 -> 1.007 ms per Adam step;
// a GEMM-forward layer must follow a pool, since the GEMM reads a rectified input)
unsigned vgg_gemm_mask(bool fwd) {
  static const unsigned m[2] = {
      [] { const char* e = std::getenv("NST_VGG_GEMM_B"); return e ? (unsigned)std::strtoul(e, nullptr, 0) : 0x1000u; }(),
      [] { const char* e = std::getenv("NST_VGG_GEMM_F"); return e ? (unsigned)std::strtoul(e, nullptr, 0) : 0x1000u; }()};
  return m[fwd ? 1 : 0];
}
bool vgg_gemm_layer(int i) { return ((vgg_gemm_mask(true) | vgg_gemm_mask(false)) >> i) & 1u; }

// W[cout][cin][3][3] fp32 -> the GEMM conv's bf16 fragments [coutp/64][stage = tap*nck + cc][64 rows][64]
// (seg_internal.h GemmConvParams::wpk)
std::vector<uint16_t> pack_gemm(const float* W, int cout, int cin, int coutp) {
  const int ck = gemm_stage_channels(NST_DT_BF16), nck = cin / ck, nstage = 9 * nck;
  std::vector<uint16_t> pk((size_t)(coutp / 64) * nstage * 64 * ck, 0);
  for (int co = 0; co < cout; ++co)
    for (int ci = 0; ci < cin; ++ci)
      for (int t = 0; t < 9; ++t) {
        const int s = t * nck + ci / ck;
        pk[(((size_t)(co / 64) * nstage + s) * 64 + (co % 64)) * ck + ci % ck] =
            f32_to_bf16_rne(W[((size_t)co * cin + ci) * 9 + t]);
      }
  return pk;
}

const ConvKernelInfo* find_vgg(int cinp, int bn, int in_kind, int out_kind) {
  int count = 0;
  const ConvKernelInfo* t = conv_table_vgg(&count);
  for (int i = 0; i < count; ++i)
    if (t[i].cinp == cinp && t[i].bn == bn && t[i].in_kind == in_kind && t[i].out_kind == out_kind) return &t[i];
  return nullptr;
}

size_t al(size_t v) { return (v + 255) / 256 * 256; }

int upload_u16(const std::vector<uint16_t>& h, void** dev) {
  NST_HIP_CHECK(hipMalloc(dev, h.size() * 2));
  NST_HIP_CHECK(hipMemcpy(*dev, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  return NST_OK;
}

}  // namespace

struct nst_vgg {
  int device = 0;
  VggConv conv[13];
  float2* unit = nullptr;  // {1, 0} x 512: the ReLU-only fill table
  float* zero_bias = nullptr;
};

namespace {

// workspace / state plan for an h x w image
struct VggPlan {
  int h = 0, w = 0;
  int ch[13], cw[13];  // conv output extents
  size_t z[13], pool[4], ga, gb, gimg, gram[5], M[5], gram_ws, part, raw, losses, gpart, spart, end;  // workspace offsets
  size_t gpart_bytes;
  size_t sP, sA[5], send;                                                              // state offsets
};

// geometry of one 3x3 / pad 1 conv on the GEMM conv (pointers set by the caller)
GemmConvParams gemm_geom(int cin, int cout, int h, int w) {
  GemmConvParams p;
  std::memset(&p, 0, sizeof(p));
  p.hi = h; p.wi = w; p.cs = cin; p.cin = cin;
  p.kh = p.kw = 3; p.stride = 1; p.dil = 1; p.pad = 1;
  p.ho = h; p.wo = w; p.npix = h * w;
  p.out_cs = cout; p.out_off = 0; p.cout_store = cout;
  p.ksplit = 1;
  return p;
}

VggPlan vgg_plan(int h, int w) {
  VggPlan P;
  P.h = h; P.w = w;
  size_t off = 0;
  int hh = h, ww = w, pi = 0;
  size_t gmax = 0, gws = 0;
  for (int i = 0; i < 13; ++i) {
    P.ch[i] = hh; P.cw[i] = ww;
    const size_t zb = (size_t)hh * ww * kConvs[i].cout * 2;
    P.z[i] = off; off += al(zb);
    gmax = std::max(gmax, zb);
    gmax = std::max(gmax, (size_t)hh * ww * std::max(kConvs[i].cin, 8) * 2);
    if (kConvs[i].pool_after) {
      hh /= 2; ww /= 2;
      P.pool[pi++] = off; off += al((size_t)hh * ww * kConvs[i].cout * 2);
    }
  }
  P.ga = off; off += al(gmax);
  P.gb = off; off += al(gmax);
  P.gimg = off; off += al((size_t)3 * h * w * 4);
  for (int l = 0; l < 5; ++l) {
    const int ci = kStyle[l], c = kConvs[ci].cout;
    P.gram[l] = off; off += al((size_t)c * c * 4);
    P.M[l] = off; off += al((size_t)c * c * 4);
    gws = std::max(gws, gram_workspace_bytes(1, c, P.ch[ci] * P.cw[ci]));
  }
  P.gram_ws = off; off += al(std::max<size_t>(gws, 256));
  P.part = off; off += al(std::max(512, GRAM_DELTA_MAX_PARTS) * 4);
  P.raw = off; off += al(8 * 4);
  P.spart = off; off += al((size_t)5 * GRAM_DELTA_MAX_PARTS * 4);  // the style layers' Gram-reduce partials
  P.losses = off; off += al(4 * 4);
  // split-K scratch of the GEMM-conv layers (forward and input gradient), the largest one
  size_t gp = 0;
  for (int i = 0; i < 13; ++i) {
    if (!vgg_gemm_layer(i)) continue;
    GemmConvParams f = gemm_geom(kConvs[i].cin, kConvs[i].cout, P.ch[i], P.cw[i]);
    GemmConvParams b = gemm_geom(kConvs[i].cout, kConvs[i].cin, P.ch[i], P.cw[i]);
    gp = std::max(gp, std::max(gemm_partial_bytes(NST_DT_BF16, f), gemm_partial_bytes(NST_DT_BF16, b)));
  }
  P.gpart = off; off += al(std::max<size_t>(gp, 256));
  P.gpart_bytes = gp;
  P.end = off;
  size_t so = 0;
  P.sP = so; so += al((size_t)P.ch[kContent] * P.cw[kContent] * 512 * 2);
  for (int l = 0; l < 5; ++l) {
    const int c = kConvs[kStyle[l]].cout;
    P.sA[l] = so; so += al((size_t)c * c * 4);
  }
  P.send = so;
  return P;
}

bool geometry_ok(int h, int w) { return h >= 16 && w >= 16 && h % 16 == 0 && w % 16 == 0; }

// one conv launch of the generic kernel (zero padding 1, stride 1)
hipError_t run_conv(const ConvKernelInfo* k, const void* in, int in_kind, int h, int w, int cs, const float2* in_norm,
                    const void* wpk, const float* bias, int cout_real, int coutp, void* out, hipStream_t st) {
  ConvParams p;
  std::memset(&p, 0, sizeof(p));
  p.in = in;
  p.hs = h; p.ws = w;
  p.cs = cs;
  p.axis_mode = AX_ZERO;
  p.pad = 1;
  p.in_norm = in_norm;
  p.in_relu = in_norm ? 1 : 0;
  for (int c = 0; c < 3; ++c) {  // image layer: (x - mean) / std  (utils.py:93-96)
    p.enc_a[c] = 1.f;
    p.enc_b[c] = in_kind == IN_F32_NCHW ? kMean[c] : 0.f;
    p.enc_d[c] = in_kind == IN_F32_NCHW ? kStd[c] : 1.f;
    p.enc_perm[c] = c;
    p.dec_p[c] = 0.f; p.dec_q[c] = 1.f; p.dec_r[c] = 1.f; p.dec_s[c] = 0.f; p.dec_perm[c] = c;
  }
  p.wpk = wpk;
  p.bias = bias;
  p.hconv = h; p.wconv = w;
  p.oh = h; p.ow = w;
  p.out = out;
  p.cout_real = cout_real;
  p.cout_stride = coutp;
  p.partial = nullptr;
  tile_grid_of(*k, h, w, h, w, &p.tiles_x, &p.tiles_y);
  p.n_cblk = coutp / k->bn;
  k->launch(p, dim3(p.tiles_x * p.tiles_y, p.n_cblk), st);
  return hipGetLastError();
}

#define VGG_CHECK(expr)                                                                           \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess) { set_error(std::string(#expr) + ": " + hipGetErrorString(_e)); return NST_E_HIP; } \
  } while (0)

// forward of the 13 convs (and 4 pools) on image [1,3,h,w] fp32 in [0,1]
int vgg_forward(nst_vgg* v, const VggPlan& P, const float* image, char* ws, hipStream_t st) {
  const void* src = image;
  int src_kind = IN_F32_NCHW, cs = 3, pi = 0;
  const float2* norm = nullptr;
  for (int i = 0; i < 13; ++i) {
    const VggConv& L = v->conv[i];
    if (L.gemm_f) {  // stores r = ReLU(z) (the epilogue's ReLU); the input is a stored r or a pooled map
      GemmConvParams p = gemm_geom(L.d.cin, L.d.cout, P.ch[i], P.cw[i]);
      p.in = src; p.wpk = L.gwf; p.scale = L.gscale; p.shift = L.gshift; p.relu = 1; p.out = ws + P.z[i];
      p.partial = P.gpart_bytes ? (float*)(ws + P.gpart) : nullptr;
      VGG_CHECK(launch_gemm_conv(NST_DT_BF16, p, st));
    } else {
      VGG_CHECK(run_conv(L.kf, src, src_kind, P.ch[i], P.cw[i], cs, norm, L.wf, L.bf, L.d.cout, L.coutp, ws + P.z[i], st));
    }
    if (L.d.pool_after) {
      VGG_CHECK(launch_vgg_pool(ws + P.z[i], P.ch[i], P.cw[i], L.d.cout, ws + P.pool[pi], st));
      src = ws + P.pool[pi++];
      norm = nullptr;  // the pooled map is already rectified
    } else {
      src = ws + P.z[i];
      norm = v->unit;  // ReLU in the consumer's fill
    }
    src_kind = IN_ACT;
    cs = L.d.cout;
  }
  return NST_OK;
}

}  // namespace

extern "C" {

int nst_vgg_create(const nst_param* params, int n_params, int device, nst_vgg** out) {
  return nst_vgg_create_ex(params, n_params, device, 0u, out);
}

int nst_vgg_create_ex(const nst_param* params, int n_params, int device, unsigned flags, nst_vgg** out) {
  if (!params || n_params <= 0 || !out || (flags & ~(unsigned)NST_VGG_GENERIC_ONLY) != 0) {
    set_error("nst_vgg_create: invalid arguments");
    return NST_E_INVALID;
  }
  const bool gemm_ok = (flags & NST_VGG_GENERIC_ONLY) == 0;
  *out = nullptr;
  std::map<std::string, const nst_param*> byname;
  for (int i = 0; i < n_params; ++i)
    if (params[i].name) byname[params[i].name] = &params[i];
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) { set_error("nst_vgg_create: bad device"); return NST_E_INVALID; }
  auto* v = new nst_vgg();
  v->device = device;
  int rc = NST_OK;
  for (int i = 0; i < 13 && rc == NST_OK; ++i) {
    VggConv& L = v->conv[i];
    L.d = kConvs[i];
    const std::string pre = "features." + std::to_string(L.d.idx);
    auto itw = byname.find(pre + ".weight"), itb = byname.find(pre + ".bias");
    const int64_t wn = (int64_t)L.d.cout * L.d.cin * 9;
    if (itw == byname.end() || itb == byname.end() || itw->second->numel != wn || itb->second->numel != L.d.cout) {
      set_error("missing or mis-shaped VGG-19 tensor " + pre + ".weight/.bias");
      rc = NST_E_PARAM;
      break;
    }
    const float* W = itw->second->data;
    L.cinp = i == 0 ? 4 : L.d.cin;
    L.coutp = L.d.cout;
    L.kf = find_vgg(L.cinp, std::min(L.coutp, 128), i == 0 ? IN_F32_NCHW : IN_ACT, OUT_ACT);
    // input gradient: a conv from cout to cin channels with W'[ci][co][ky][kx] = W[co][ci][2-ky][2-kx]
    const int bcinp = L.d.cout, bcoutp = i == 0 ? 16 : L.d.cin;
    L.kb = find_vgg(bcinp, std::min(bcoutp, 128), IN_ACT, i == 0 ? OUT_F32_NCHW : OUT_ACT);
    if (!L.kf || !L.kb) { set_error("no compiled VGG conv kernel for " + pre); rc = NST_E_SHAPE; break; }
    std::vector<float> Wt((size_t)L.d.cin * L.d.cout * 9);
    for (int co = 0; co < L.d.cout; ++co)
      for (int ci = 0; ci < L.d.cin; ++ci)
        for (int t = 0; t < 9; ++t) Wt[((size_t)ci * L.d.cout + co) * 9 + (8 - t)] = W[((size_t)co * L.d.cin + ci) * 9 + t];
    if ((rc = pack_upload_conv(*L.kf, L.d.cin, L.d.cout, 3, W, L.coutp, &L.wf)) != NST_OK) break;
    if ((rc = pack_upload_conv(*L.kb, L.d.cout, L.d.cin, 3, Wt.data(), bcoutp, &L.wb)) != NST_OK) break;
    if ((rc = upload_floats(itb->second->data, L.d.cout, &L.bf)) != NST_OK) break;
    if (gemm_ok && vgg_gemm_layer(i)) {
      L.gemm_f = (vgg_gemm_mask(true) >> i) & 1u;
      L.gemm_b = (vgg_gemm_mask(false) >> i) & 1u;
      const int cpb = (L.d.cin + 127) / 128 * 128;  // input-gradient outputs, padded to the 128-row tile
      std::vector<uint16_t> pf = pack_gemm(W, L.d.cout, L.d.cin, L.d.cout), pb = pack_gemm(Wt.data(), L.d.cin, L.d.cout, cpb);
      std::vector<float> one(512, 1.f), zero(512, 0.f), bias(512, 0.f);
      std::memcpy(bias.data(), itb->second->data, (size_t)L.d.cout * 4);
      if ((rc = upload_u16(pf, &L.gwf)) != NST_OK) break;
      if ((rc = upload_u16(pb, &L.gwb)) != NST_OK) break;
      if ((rc = upload_floats(one.data(), 512, &L.gscale)) != NST_OK) break;
      if ((rc = upload_floats(bias.data(), 512, &L.gshift)) != NST_OK) break;
      if ((rc = upload_floats(zero.data(), 512, &L.gzero)) != NST_OK) break;
    }
  }
  if (rc == NST_OK) {
    std::vector<float> unit(2 * 512), zero(512, 0.f);
    for (int c = 0; c < 512; ++c) { unit[2 * c] = 1.f; unit[2 * c + 1] = 0.f; }
    rc = upload_floats(unit.data(), unit.size(), (float**)&v->unit);
    if (rc == NST_OK) rc = upload_floats(zero.data(), zero.size(), &v->zero_bias);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  if (rc != NST_OK) { nst_vgg_destroy(v); return rc; }
  *out = v;
  return NST_OK;
}

void nst_vgg_destroy(nst_vgg* v) {
  if (!v) return;
  for (auto& L : v->conv) {
    if (L.wf) (void)hipFree(L.wf);
    if (L.wb) (void)hipFree(L.wb);
    if (L.bf) (void)hipFree(L.bf);
    for (void* q : {L.gwf, L.gwb, (void*)L.gscale, (void*)L.gshift, (void*)L.gzero})
      if (q) (void)hipFree(q);
  }
  if (v->unit) (void)hipFree(v->unit);
  if (v->zero_bias) (void)hipFree(v->zero_bias);
  delete v;
}

int nst_gatys_buffer_bytes(const nst_vgg* v, int h, int w, size_t* workspace, size_t* state) {
  if (!v || !workspace || !state || !geometry_ok(h, w)) {
    set_error("nst_gatys_buffer_bytes: invalid arguments (h and w must be multiples of 16)");
    return NST_E_INVALID;
  }
  const VggPlan P = vgg_plan(h, w);
  *workspace = P.end;
  *state = P.send;
  return NST_OK;
}

int nst_vgg_features(nst_vgg* v, const float* image, int h, int w, void* const* feats, void* workspace,
                     size_t workspace_bytes, void* stream) {
  if (!v || !image || !feats || !geometry_ok(h, w)) { set_error("nst_vgg_features: invalid arguments"); return NST_E_INVALID; }
  const VggPlan P = vgg_plan(h, w);
  if (!workspace || workspace_bytes < P.end) { set_error("nst_vgg_features: workspace too small"); return NST_E_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  int rc = vgg_forward(v, P, image, ws, st);
  if (rc != NST_OK) return rc;
  const int which[6] = {kStyle[0], kStyle[1], kStyle[2], kStyle[3], kStyle[4], kContent};
  for (int k = 0; k < 6; ++k) {
    if (!feats[k]) continue;
    const int i = which[k];
    // rectified: (z > 0) * z of the stored map (a stored z, or an r = ReLU(z) the GEMM conv wrote)
    const size_t n = (size_t)P.ch[i] * P.cw[i] * kConvs[i].cout;
    VGG_CHECK(launch_vgg_relu_bwd(ws + P.z[i], ws + P.z[i], nullptr, 0.f, n, feats[k], st));
  }
  return NST_OK;
}

int nst_gatys_targets(nst_vgg* v, const float* content, const float* style, int h, int w, void* state,
                      void* workspace, size_t workspace_bytes, void* stream) {
  if (!v || !content || !style || !state || !geometry_ok(h, w)) {
    set_error("nst_gatys_targets: invalid arguments");
    return NST_E_INVALID;
  }
  const VggPlan P = vgg_plan(h, w);
  if (!workspace || workspace_bytes < P.end) { set_error("nst_gatys_targets: workspace too small"); return NST_E_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  char* sp = (char*)state;
  int rc = vgg_forward(v, P, style, ws, st);
  if (rc != NST_OK) return rc;
  for (int l = 0; l < 5; ++l) {
    const int i = kStyle[l], c = kConvs[i].cout;
    VGG_CHECK(launch_gram(ws + P.z[i], NST_DT_BF16, 1, 1, c, P.ch[i] * P.cw[i], (float*)(sp + P.sA[l]), ws + P.gram_ws, st, 1));
  }
  if ((rc = vgg_forward(v, P, content, ws, st)) != NST_OK) return rc;
  // content target: ReLU(z4_2), stored rectified
  const size_t n = (size_t)P.ch[kContent] * P.cw[kContent] * 512;
  VGG_CHECK(launch_vgg_relu_bwd(ws + P.z[kContent], ws + P.z[kContent], nullptr, 0.f, n, sp + P.sP, st));
  return NST_OK;
}

}  // extern "C"

namespace {
int gatys_grad_impl(nst_vgg* v, const float* image, int h, int w, const float* style_layer_weights, float content_weight,
                    float style_weight, const void* state, float* grad, float* losses, void* workspace,
                    size_t workspace_bytes, void* stream, void* const* dz) {
  if (!v || !image || !state || !grad || !losses || !geometry_ok(h, w)) {
    set_error("nst_gatys_grad: invalid arguments");
    return NST_E_INVALID;
  }
  const VggPlan P = vgg_plan(h, w);
  if (!workspace || workspace_bytes < P.end) { set_error("nst_gatys_grad: workspace too small"); return NST_E_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const char* sp = (const char*)state;
  int rc = vgg_forward(v, P, image, ws, st);
  if (rc != NST_OK) return rc;
  // style: G_l, M_l = 4 beta w_l (G - A) / (c^3 hw), raw sum (G - A)^2
  float sscale[5];
  int snparts[5];
  for (int l = 0; l < 5; ++l) {
    const int i = kStyle[l], c = kConvs[i].cout, hw = P.ch[i] * P.cw[i];
    const float wl = style_layer_weights ? style_layer_weights[l] : 1.f;
    const double k = 4.0 * style_weight * wl / ((double)c * c * c * hw);
    // partials per layer, summed by the loss kernel below (one launch for the five layers)
    const GramDelta gd{(const float*)(sp + P.sA[l]), (float)k, (__bf16*)(ws + P.M[l]),
                       (float*)(ws + P.spart) + (size_t)l * GRAM_DELTA_MAX_PARTS, nullptr};
    snparts[l] = gram_delta_parts(1, c, hw);  // launch_gram's reduce blocks
    VGG_CHECK(launch_gram(ws + P.z[i], NST_DT_BF16, 1, 1, c, hw, (float*)(ws + P.gram[l]), ws + P.gram_ws, st, 1, &gd));
    sscale[l] = (float)(style_weight * wl / ((double)c * c));
  }
  const size_t nc = (size_t)P.ch[kContent] * P.cw[kContent] * 512;
  VGG_CHECK(launch_vgg_losses(ws + P.z[kContent], sp + P.sP, nc, (float*)(ws + P.part), (float*)(ws + P.raw),
                              (float)(content_weight / (double)nc), sscale, losses, st, (const float*)(ws + P.spart),
                              snparts, GRAM_DELTA_MAX_PARTS));
  // backward, top to bottom, through two ping-pong gradient buffers (each step reads `cur` and
  // writes the other one).  `ready`: cur already holds dL/dz of conv i (the pool backward folds the
  // producer's ReLU backward in); otherwise cur holds dL/d ReLU(z_i) (none above conv5_1).
  char* gbuf[2] = {ws + P.ga, ws + P.gb};
  int cur = -1;
  bool ready = false;
  const float cw = (float)(2.0 * content_weight / (double)nc);
  for (int i = 12; i >= 0; --i) {
    const VggConv& L = v->conv[i];
    const int hw = P.ch[i] * P.cw[i], c = L.d.cout;
    if (!ready) {  // dL/dz = ReLU' * (incoming + style GEMM + content term)
      int si = -1;
      for (int l = 0; l < 5; ++l)
        if (kStyle[l] == i) si = l;
      const void* Pc = i == kContent ? sp + P.sP : nullptr;
      const void* gin = cur >= 0 ? gbuf[cur] : nullptr;
      const int nxt = cur < 0 ? 0 : cur ^ 1;
      if (si >= 0) {
        VGG_CHECK(launch_vgg_gram_bwd(ws + P.z[i], gin, Pc, cw, ws + P.M[si], hw, c, gbuf[nxt], st));
      } else if (gin || Pc) {
        VGG_CHECK(launch_vgg_relu_bwd(ws + P.z[i], gin, Pc, cw, (size_t)hw * c, gbuf[nxt], st));
      } else {
        set_error("nst_gatys_grad: no gradient reaches conv " + std::to_string(i));
        return NST_E_SHAPE;
      }
      cur = nxt;
    }
    if (dz && dz[i]) VGG_CHECK(hipMemcpyAsync(dz[i], gbuf[cur], (size_t)hw * c * 2, hipMemcpyDeviceToDevice, st));
    if (i == 0) {  // the normalised image's gradient, fp32 NCHW (nst_adam_step divides by std)
      VGG_CHECK(run_conv(L.kb, gbuf[cur], IN_ACT, P.ch[0], P.cw[0], c, nullptr, L.wb, v->zero_bias, 3, 16, grad, st));
      break;
    }
    if (L.gemm_b) {
      GemmConvParams p = gemm_geom(L.d.cout, L.d.cin, P.ch[i], P.cw[i]);
      p.in = gbuf[cur]; p.wpk = L.gwb; p.scale = L.gscale; p.shift = L.gzero; p.relu = 0; p.out = gbuf[cur ^ 1];
      p.partial = P.gpart_bytes ? (float*)(ws + P.gpart) : nullptr;
      VGG_CHECK(launch_gemm_conv(NST_DT_BF16, p, st));
    } else {
      VGG_CHECK(run_conv(L.kb, gbuf[cur], IN_ACT, P.ch[i], P.cw[i], c, nullptr, L.wb, v->zero_bias, L.d.cin, L.d.cin,
                         gbuf[cur ^ 1], st));
    }
    cur ^= 1;
    const VggConv& Lp = v->conv[i - 1];
    ready = Lp.d.pool_after;
    if (ready) {  // cur = dL/d pool(ReLU(z_{i-1})) -> dL/dz_{i-1}
      VGG_CHECK(launch_vgg_pool_bwd(ws + P.z[i - 1], gbuf[cur], P.ch[i - 1], P.cw[i - 1], Lp.d.cout, gbuf[cur ^ 1], st));
      cur ^= 1;
    }
  }
  return NST_OK;
}
}  // namespace

extern "C" {

int nst_gatys_grad(nst_vgg* v, const float* image, int h, int w, const float* style_layer_weights, float content_weight,
                   float style_weight, const void* state, float* grad, float* losses, void* workspace,
                   size_t workspace_bytes, void* stream) {
  return gatys_grad_impl(v, image, h, w, style_layer_weights, content_weight, style_weight, state, grad, losses,
                         workspace, workspace_bytes, stream, nullptr);
}

int nst_gatys_grad_capture(nst_vgg* v, const float* image, int h, int w, const float* style_layer_weights,
                           float content_weight, float style_weight, const void* state, float* grad, float* losses,
                           void* workspace, size_t workspace_bytes, void* const* dz, void* stream) {
  return gatys_grad_impl(v, image, h, w, style_layer_weights, content_weight, style_weight, state, grad, losses,
                         workspace, workspace_bytes, stream, dz);
}

int nst_adam_step(float* x, const float* grad, float* m, float* v, int c, int hw, float lr, float beta1, float beta2,
                  float eps, int step, int clamp01, int grad_is_normalised, void* stream) {
  if (!x || !grad || !m || !v || c != 3 || hw <= 0 || step < 1) { set_error("nst_adam_step: invalid arguments"); return NST_E_INVALID; }
  const float inv[3] = {grad_is_normalised ? 1.f / kStd[0] : 1.f, grad_is_normalised ? 1.f / kStd[1] : 1.f,
                        grad_is_normalised ? 1.f / kStd[2] : 1.f};
  const float bc1 = (float)(1.0 - std::pow((double)beta1, step)), bc2 = (float)(1.0 - std::pow((double)beta2, step));
  hipError_t e = launch_adam(x, grad, m, v, hw, c * hw, inv, lr, beta1, beta2, eps, bc1, bc2, clamp01, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("adam launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

}  // extern "C"
