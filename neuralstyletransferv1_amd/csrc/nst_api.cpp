// nst_api.cpp — C ABI of libnst_hip.so (declared in include/nst_hip.h).
//
// Host side of the engine: per-architecture layer programs (the reference's module graphs
// transformer_net.py:29-41, transformer_net_nst.py:95-127, model.py:69-116 restated as a
// flat list of conv / residual-add steps), one-time weight packing into MFMA fragment order,
// workspace planning, and kernel sequencing on the caller's stream.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "nst_hip.h"
#include "nst_internal.h"
#include "post_common.h"

namespace nst {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

const ConvKernelInfo* conv_table_bf16(int* count);
const ConvKernelInfo* conv_table_f16(int* count);
const ConvKernelInfo* conv_table_bf16_wl(int* count);
const ConvKernelInfo* conv_table_f32(int* count);
const ConvKernelInfo* conv_table_f32s(int* count);
const ConvKernelInfo* conv_table_out9(int* count);
const ConvKernelInfo* conv_table_wstat(int* count);
const ConvKernelInfo* conv_table_wst16(int* count);
// conv_wst32.hip (32x32x16 variant of the trunk kernel): built only by `make wst32` (A/B builds), so weak here
const ConvKernelInfo* conv_table_wst32(int* count) __attribute__((weak));
static const ConvKernelInfo* table_wst32_or_none(int* count) {
  if (conv_table_wst32 != nullptr) return conv_table_wst32(count);
  *count = 0;
  return nullptr;
}
const ConvKernelInfo* conv_table_wphase(int* count);
const ConvKernelInfo* conv_table_ws2(int* count);
const ConvKernelInfo* conv_table_ws9(int* count);
const ConvKernelInfo* conv_table_ws1s(int* count);

// first match wins: the persistent / LDS-weight-ring table is searched before the plain one
const ConvKernelInfo* find_conv_kernel(int dtype, int mode, int ks, int stride, int cinp, int bn, int in_kind,
                                       int out_kind, int res, bool no_persistent) {
  typedef const ConvKernelInfo* (*TableFn)(int*);
  // 16-bit formats (bf16, fp16) share the specialised tables; an entry matches only its own dtype
  const TableFn tables_16[] = {conv_table_bf16_wl, conv_table_wst16, table_wst32_or_none, conv_table_wstat, conv_table_wphase,
                               conv_table_ws2, conv_table_ws9, conv_table_out9, conv_table_bf16, conv_table_f16,
                               conv_table_ws1s};
  // 4-byte activation formats (fp32, split-fp16): the generic kernels, and the split-fp16 row-streaming output conv
  const TableFn tables_f32[] = {conv_table_out9, conv_table_f32, conv_table_f32s};
  const bool h16 = !f32_storage(dtype);
  const TableFn* tables = h16 ? tables_16 : tables_f32;
  const int ntables = h16 ? 11 : 3;
  for (int ti = (h16 && no_persistent) ? 1 : 0; ti < ntables; ++ti) {
    int count = 0;
    const ConvKernelInfo* t = tables[ti](&count);
    for (int i = 0; i < count; ++i) {
      const ConvKernelInfo& k = t[i];
      if (k.dtype == dtype && k.mode == mode && k.ks == ks && k.stride == stride && k.cinp == cinp && k.bn == bn &&
          k.in_kind == in_kind && k.out_kind == out_kind && k.res == res)
        return &k;
    }
  }
  return nullptr;
}

// ---------------------------------------------------------------------------------------
// Layer descriptions
enum Role { ROLE_IN = 0, ROLE_FINAL = 1 };  // conv followed by InstanceNorm, or the output conv

struct LayerDef {
  std::string conv;  // state_dict prefix of the conv ("conv1.conv2d")
  std::string norm;  // prefix of the InstanceNorm2d, "" for the output conv
  int cin, cout, ks, stride, axis_mode, pad, pre;
  bool convT;
};

struct Layer {
  LayerDef d;
  int cinp, coutp;
  int mode = MODE_STD;                     // conv_kernel mapping chosen for this layer
  const ConvKernelInfo* k_main = nullptr;  // in/out kind of the activation path
  const ConvKernelInfo* k_alt = nullptr;   // image layer: F32 NCHW input; final: F32 NCHW output
  void* wpk = nullptr;
  float* bias = nullptr;
  void* wpk_rev = nullptr;   // MODE_XSHIFT: channel-reversed rows (caffe_bgr decode), see pack_weights
  float* bias_rev = nullptr;
  float* gamma = nullptr;
  float* beta = nullptr;
  float eps = 1e-5f;  // InstanceNorm2d eps, or |FRN.eps|
  int frn = 0;        // statistics: mean / variance (InstanceNorm) or mean square (FRN, frn.py:71)
  bool prepad = false;  // image layer reading the pre-padded encoded input (conv_prep.hip)
  int kdt = 0;                   // the layer's arithmetic (NST_DT_* / NST_KDT_*): the handle's dtype except in NST_DT_F16M
  int in_esz = 2, out_esz = 2;   // activation element bytes it reads / writes
  // image layer over pre-padded uint8 frames: weights / bias with the io_preset encode folded in, per preset
  // (fold_first_layer; nullptr where the fold does not hold), used with the raw-byte staging (ConvParams::enc_raw)
  void* wpk_fold[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  float* bias_fold[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // NST_DT_F32S image layer: the kernel that runs uint8 frames of a folded preset (the split-weight 9x9 kernel over
  // the pre-padded raw bytes, wpk_fold / bias_fold); float frames and unfolded presets keep k_main / k_alt
  const ConvKernelInfo* k_u8fold = nullptr;
};

// Program steps
enum OpKind { OP_CONV = 0, OP_RESADD = 1 };
enum Buf { B_IMG = -1, B_OUT = -2, B_A = 0, B_B = 1, B_C = 2, B_D = 3, B_E = 4, B_F = 5, B_G = 6, NBUF = 7 };
struct Op {
  int kind;
  int layer;     // OP_CONV: layer to run; OP_RESADD: layer whose IN applies to y
  int src, dst;  // buffers
  int in_norm;   // OP_CONV: layer whose IN+ReLU the prologue applies (-1: identity); with res_buf: IN of src, no ReLU
  int r_buf, r_norm, r_relu, relu_out;  // OP_RESADD; OP_CONV with res_buf >= 0: the residual join in the fill
  int res_buf = -1, res_out = -1;       // OP_CONV: residual stream r (joined into the fill) / where it is written
  int out_esz = 0;                      // OP_RESADD: element bytes of the stream it writes (0: the handle's)
};

static int round_up(int v, int a) { return (v + a - 1) / a * a; }
static bool is_reconet(int arch) { return arch == NST_ARCH_RECONET || arch == NST_ARCH_RECONET_FRN; }

// x0_export (with fuse_res): block 1's conv1 also writes x_0 = ReLU(IN_2(C)) from its fill (only the
// weight-stationary trunk kernel does), so block 2's join reads a stored x_0 like every later join
// split_blocks (NST_DT_F16M): the first one or two residual blocks run unfused on the split-operand kernel (fp32
// activations), separate residual adds write x_1 (fp32, when block 2 is split) and the fp16 stream; the later blocks
// are the fused fp16 program from that stored stream (the first of them reads it as is, later joins read it)
static void build_program(int arch, bool fuse_res, bool x0_export, std::vector<LayerDef>& L, std::vector<Op>& P,
                          int split_blocks = 0) {
  L.clear();
  P.clear();
  auto conv = [&](int layer, int src, int dst, int in_norm) {
    P.push_back(Op{OP_CONV, layer, src, dst, in_norm, 0, 0, 0, 0});
  };
  // conv whose fill joins the residual stream: IN(y = src) + r (r itself IN+ReLU of r_norm, lazily)
  auto convres = [&](int layer, int y, int y_norm, int r_buf, int r_norm, int res_out, int relu_out, int dst) {
    Op o{OP_CONV, layer, y, dst, y_norm, r_buf, r_norm, r_norm >= 0 ? 1 : 0, relu_out};
    o.res_buf = r_buf;
    o.res_out = res_out;
    P.push_back(o);
  };
  auto resadd = [&](int layer, int y, int dst, int r_buf, int r_norm, int relu_out) {
    P.push_back(Op{OP_RESADD, layer, y, dst, -1, r_buf, r_norm, r_norm >= 0 ? 1 : 0, relu_out});
  };
  if (arch == NST_ARCH_JOHNSON) {
    // transformer_net.py:4-41
    L.push_back({"conv1.conv2d", "in1", 3, 32, 9, 1, AX_REFLECT, 4, 0, false});
    L.push_back({"conv2.conv2d", "in2", 32, 64, 3, 2, AX_REFLECT, 1, 0, false});
    L.push_back({"conv3.conv2d", "in3", 64, 128, 3, 2, AX_REFLECT, 1, 0, false});
    for (int r = 1; r <= 5; ++r) {
      const std::string p = "res" + std::to_string(r);
      L.push_back({p + ".conv1.conv2d", p + ".in1", 128, 128, 3, 1, AX_REFLECT, 1, 0, false});
      L.push_back({p + ".conv2.conv2d", p + ".in2", 128, 128, 3, 1, AX_REFLECT, 1, 0, false});
    }
    L.push_back({"deconv1.conv2d", "in4", 128, 64, 3, 1, AX_REFLECT_UP2, 1, 0, false});
    L.push_back({"deconv2.conv2d", "in5", 64, 32, 3, 1, AX_REFLECT_UP2, 1, 0, false});
    L.push_back({"deconv3.conv2d", "", 32, 3, 9, 1, AX_REFLECT, 4, 0, false});
  } else if (arch == NST_ARCH_NST) {
    // transformer_net_nst.py:62-127 (zero-padded convs after ReflectionPad2d(40); ConvTranspose ups)
    L.push_back({"down1.conv", "down1.norm", 3, 32, 9, 1, AX_ZERO_PREREFLECT, 4, 40, false});
    L.push_back({"down2.conv", "down2.norm", 32, 64, 3, 2, AX_ZERO, 1, 0, false});
    L.push_back({"down3.conv", "down3.norm", 64, 128, 3, 2, AX_ZERO, 1, 0, false});
    for (int r = 1; r <= 5; ++r) {
      const std::string p = "res" + std::to_string(r);
      L.push_back({p + ".conv1", p + ".norm1", 128, 128, 3, 1, AX_ZERO, 1, 0, false});
      L.push_back({p + ".conv2", p + ".norm2", 128, 128, 3, 1, AX_ZERO, 1, 0, false});
    }
    L.push_back({"up1.conv", "up1.norm", 128, 64, 3, 1, AX_ZINSERT, 1, 0, true});
    L.push_back({"up2.conv", "up2.norm", 64, 32, 3, 1, AX_ZINSERT, 1, 0, true});
    L.push_back({"final", "", 32, 3, 9, 1, AX_ZERO, 4, 0, false});
  } else {
    // model.py:69-116 (FRN at the InstanceNorm's index, frn=True)
    L.push_back({"encoder.layers.0.layers.0.layers.1", "encoder.layers.0.layers.1", 3, 48, 9, 1, AX_REFLECT, 4, 0, false});
    L.push_back({"encoder.layers.1.layers.0.layers.1", "encoder.layers.1.layers.1", 48, 96, 3, 2, AX_REFLECT, 1, 0, false});
    L.push_back({"encoder.layers.2.layers.0.layers.1", "encoder.layers.2.layers.1", 96, 192, 3, 2, AX_REFLECT, 1, 0, false});
    for (int r = 3; r <= 6; ++r) {
      const std::string p = "encoder.layers." + std::to_string(r) + ".branch.";
      L.push_back({p + "0.layers.0.layers.1", p + "0.layers.1", 192, 192, 3, 1, AX_REFLECT, 1, 0, false});
      L.push_back({p + "1.layers.0.layers.1", p + "1.layers.1", 192, 192, 3, 1, AX_REFLECT, 1, 0, false});
    }
    L.push_back({"decoder.layers.1.layers.0.layers.1", "decoder.layers.1.layers.1", 192, 96, 3, 1, AX_REFLECT_UP2, 1, 0, false});
    L.push_back({"decoder.layers.3.layers.0.layers.1", "decoder.layers.3.layers.1", 96, 48, 3, 1, AX_REFLECT_UP2, 1, 0, false});
    L.push_back({"decoder.layers.4.layers.0.layers.1", "", 48, 3, 9, 1, AX_REFLECT, 4, 0, false});
  }
  const int nres = is_reconet(arch) ? 4 : 5;
  const int relu_out = is_reconet(arch) ? 1 : 0;  // ReCoNet ResLayer: ReLU (TLU) after the add
  const int u1 = 3 + 2 * nres, u2 = u1 + 1, fin = u1 + 2;
  conv(0, B_IMG, B_A, -1);
  conv(1, B_A, B_B, 0);
  conv(2, B_B, B_C, 1);
  if (split_blocks > 0) {
    // blocks 1..split_blocks unfused on fp32 activations: x_1 = IN(y) + ReLU(IN_2(C)) (fp32 in F when block 2 is
    // split too), x_2 = IN(y) + x_1; the last split block's sum is the fp16 stream in G; the later blocks are fused
    // from G (the first of them reads it as is)
    conv(3, B_C, B_D, 2);
    conv(4, B_D, B_E, 3);
    if (split_blocks >= 2) {
      resadd(4, B_E, B_F, B_C, 2, relu_out);
      P.back().out_esz = 4;
      conv(5, B_F, B_D, -1);
      conv(6, B_D, B_E, 5);
      resadd(6, B_E, B_G, B_F, -1, relu_out);
    } else {
      resadd(4, B_E, B_G, B_C, 2, relu_out);
    }
    P.back().out_esz = 2;
    int xbuf = B_G;
    for (int r = split_blocks; r < nres; ++r) {
      const int l1 = 3 + 2 * r, l2 = 4 + 2 * r;
      if (r == split_blocks) {
        conv(l1, B_G, B_D, -1);  // x_2 as stored: the fill applies nothing
      } else {
        const int xout = xbuf == B_F ? B_G : B_F;
        convres(l1, B_E, l2 - 2, xbuf, -1, xout, relu_out, B_D);
        xbuf = xout;
      }
      conv(l2, B_D, B_E, l1);
    }
    convres(u1, B_E, u1 - 1, xbuf, -1, -1, relu_out, B_A);
  } else if (!fuse_res) {
    // residual stream lives in B_C; block k's input is C (block 1: IN+ReLU of layer 2, lazily)
    for (int r = 0; r < nres; ++r) {
      const int l1 = 3 + 2 * r, l2 = 4 + 2 * r;
      conv(l1, B_C, B_D, r == 0 ? 2 : -1);
      conv(l2, B_D, B_E, l1);
      resadd(l2, B_E, B_C, B_C, r == 0 ? 2 : -1, relu_out);
    }
    conv(u1, B_C, B_A, -1);
  } else {
    // the residual add x_{k+1} = IN(y_k) + x_k runs inside the NEXT conv's fill, which also writes
    // x_{k+1} (ping-pong F/G) for its own pixels; x_0 = ReLU(IN_2(C)) is either written by block 1's
    // conv1 (x0_export, into F) or applied lazily in block 2's join
    int xbuf = x0_export ? B_F : B_C, xnorm = x0_export ? -1 : 2;
    for (int r = 0; r < nres; ++r) {
      const int l1 = 3 + 2 * r, l2 = 4 + 2 * r;
      if (r == 0) {
        conv(l1, B_C, B_D, 2);
        if (x0_export) P.back().res_out = B_F;
      } else {
        const int xout = ((r & 1) != 0) != x0_export ? B_F : B_G;
        convres(l1, B_E, l2 - 2, xbuf, xnorm, xout, relu_out, B_D);
        xbuf = xout;
        xnorm = -1;
      }
      conv(l2, B_D, B_E, l1);
    }
    convres(u1, B_E, u1 - 1, xbuf, xnorm, -1, relu_out, B_A);
  }
  conv(u2, B_A, B_B, u1);
  conv(fin, B_B, B_OUT, u2);
}

}  // namespace nst

using namespace nst;

struct nst_handle {
  int arch, dtype, device;
  int* range_flag = nullptr;  // nst_set_range_check: device flag raised by check_finite_kernel
  std::vector<Layer> layers;
  std::vector<Op> prog;
  // live profiling (nst_profile_begin/end)
  bool profiling = false;
  struct Rec { int layer; hipEvent_t a, b; };
  std::vector<Rec> recs;
  // nst_set_stream_split: a batch runs as `split` sub-batches on internal streams forked from / joined to the
  // caller's, so one sub-batch's launch gaps and kernel tails are filled by another's kernels
  int split = 1;
  hipStream_t sub[NST_MAX_STREAM_SPLIT] = {};
  hipEvent_t fork = nullptr, join[NST_MAX_STREAM_SPLIT] = {};
};

struct nst_lab {
  int device;
  uint32_t* rgb2lab = nullptr;  // 2^24 x {L, a, b, 0}
  uint32_t* lab2rgb = nullptr;  // 2^24 x {r, g, b, 0}
};

namespace {


// packed weights -> device, in the layer's compute dtype
int upload_weights(int dtype, const std::vector<float>& pk, void** dst);

// Sub-pixel phase weights of an x2 up-conv: output pixel (2y + a, 2x + b) is a 2x2 conv over the
// source grid, window tap (ty, tx); its weight is the sum of the 3x3 taps landing on that source
// pixel: nearest-x2 (a=0: ty0<-{k0}, ty1<-{k1,k2}; a=1: ty0<-{k0,k1}, ty1<-{k2}), or the one
// ConvTranspose2d(s2,p1) tap (a=0: ty0<-k1; a=1: ty0<-k2, ty1<-k0), per axis.
// phase_taps: kernel indices (along one axis) that fall on window position t of phase a
int phase_taps(bool convT, int a, int t, int* ks_out) {
  if (convT) {  // unflipped ConvTranspose indices
    if (a == 0) { if (t == 0) { ks_out[0] = 1; return 1; } return 0; }
    ks_out[0] = t == 0 ? 2 : 0;
    return 1;
  }
  if (a == 0) {
    if (t == 0) { ks_out[0] = 0; return 1; }
    ks_out[0] = 1; ks_out[1] = 2; return 2;
  }
  if (t == 0) { ks_out[0] = 0; ks_out[1] = 1; return 2; }
  ks_out[0] = 2;
  return 1;
}

// weight of output channel co, input channel ci at phase ph = 2a + b, window tap = 2 ty + tx
double phase_weight(const LayerDef& d, const float* W, int co, int ci, int ph, int tap) {
  int ky[2], kx[2];
  const int ny = phase_taps(d.convT, ph >> 1, tap >> 1, ky), nx = phase_taps(d.convT, ph & 1, tap & 1, kx);
  double sum = 0.0;
  for (int yy = 0; yy < ny; ++yy)
    for (int xx = 0; xx < nx; ++xx)
      sum += d.convT ? (double)W[(((size_t)ci * d.cout + co) * d.ks + ky[yy]) * d.ks + kx[xx]]
                     : (double)W[(((size_t)co * d.cin + ci) * d.ks + ky[yy]) * d.ks + kx[xx]];
  return sum;
}

// Pack conv weights into MFMA A-fragment order: [cblk][step (nstep_pack; >= nstep zero)][n-subtile][lane][cpc]
// lane l = (g = l>>4, q = l&15): output channel of row q in subtile t (wave wn, local t):
//   cb*bn + wn*nsub*16 + 4*nsub*(q>>2) + 4*t + (q&3);  K chunk 4*step+g -> (tap, channel chunk).
//
// MODE_PHASE: n-subtile tg = phase*nsub + t (phase (a,b) = (tg/nsub)>>1, &1), tap = (ty,tx) of the
//   phase's 2x2 window on the source grid (phase_weight).
// MODE_XSHIFT: row q = 3*s + c (q < 15) is output channel perm[c] at x-shift s; tap (dy, u) over
//   13 columns carries W[.][.][dy][u - s] when 0 <= u - s < 9.
std::vector<float> pack_weights(const ConvKernelInfo& k, const LayerDef& d, const float* W, int coutp,
                                bool reverse_channels = false) {
  const int ncblk = coutp / k.bn;
  const size_t per_frag = 64 * (size_t)k.cpc;
  std::vector<float> out((size_t)ncblk * k.nstep_pack * k.nsubt * per_frag, 0.f);
  auto w_at = [&](int co, int ci, int dy, int dx) -> double {
    if (d.convT)  // ConvTranspose2d weight [cin][cout][kh][kw], flipped for the zero-inserted conv
      return W[(((size_t)ci * d.cout + co) * d.ks + (d.ks - 1 - dy)) * d.ks + (d.ks - 1 - dx)];
    return W[(((size_t)co * d.cin + ci) * d.ks + dy) * d.ks + dx];
  };
  for (int cb = 0; cb < ncblk; ++cb)
    for (int s = 0; s < k.nstep; ++s)
      for (int tg = 0; tg < k.nsubt; ++tg)
        for (int lane = 0; lane < 64; ++lane) {
          const int q = lane & 15, g = lane >> 4;
          // korder 1 (persistent kernels): packed step s runs chunk group s / taps of tap s % taps
          const int taps = k.nchunk / k.nch;
          const int sl = k.korder ? (s % taps) * (k.nch / 4) + s / taps : s;
          const int i = 4 * sl + g;
          float* dst = &out[((((size_t)cb * k.nstep_pack + s) * k.nsubt + tg) * 64 + lane) * k.cpc];
          if (i >= k.nchunk) continue;
          const int tap = i / k.nch, c = i % k.nch;
          if (k.mode == MODE_PHASE) {
            const int ph = tg / k.nsub, t = tg % k.nsub;
            const int co = cb * k.bn + 4 * k.nsub * (q >> 2) + 4 * t + (q & 3);
            if (co >= d.cout) continue;
            for (int j = 0; j < k.cpc; ++j) {
              const int ci = c * k.cpc + j;
              if (ci < d.cin) dst[j] = (float)phase_weight(d, W, co, ci, ph, tap);
            }
          } else if (k.mode == MODE_XSHIFT) {
            if (q >= 15) continue;
            const int sft = q / 3, ch = q % 3;
            const int co = reverse_channels ? 2 - ch : ch;
            const int dy = tap / k.kp, u = tap % k.kp, dx = u - sft;
            if (dx < 0 || dx >= d.ks || co >= d.cout) continue;
            for (int j = 0; j < k.cpc; ++j) {
              const int ci = c * k.cpc + j;
              if (ci < d.cin) dst[j] = (float)w_at(co, ci, dy, dx);
            }
          } else {
            const int wn = tg / k.nsub, t = tg % k.nsub;
            const int co = cb * k.bn + wn * k.nsub * 16 + 4 * k.nsub * (q >> 2) + 4 * t + (q & 3);
            if (co >= d.cout) continue;
            const int dy = tap / k.kp, dxp = tap % k.kp;
            for (int j = 0; j < k.cpc; ++j) {
              int dx, ci;
              if (k.pair) { dx = 2 * dxp + (j >= 4 ? 1 : 0); ci = j & 3; }
              else { dx = dxp; ci = c * k.cpc + j; }
              if (dx < d.ks && ci < d.cin) dst[j] = (float)w_at(co, ci, dy, dx);
            }
          }
        }
  return out;
}

// Split-weight layouts (ConvKernelInfo::split_w): every 16-bit weight fragment f of the plain packing becomes
// the pair (hi, lo) = (RNE16(w), w - RNE16(w)) — hi as its exact fp32 value, lo left in fp32 for
// upload_weights(NST_DT_F16) to round, so Wl = RNE16(w - Wh).  Orders (what the kernels load):
//   MODE_WS9 (conv_ws9.hip SW): [channel half mh][ky][hi, lo] 16x16x32 fragments, then [mh][j][hi, lo] 16x16x16
//   MODE_WS2 (conv_ws2.hip SPL): [channel group cg][hi | lo][step]
std::vector<float> split_weight_frags(const ConvKernelInfo& k, const std::vector<float>& pk) {
  std::vector<float> out(pk.size() * 2);
  size_t o = 0;
  auto put = [&](const float* f, size_t n, bool lo) {
    for (size_t i = 0; i < n; ++i) {
      const float hi = f16_to_f32(f32_to_f16_rne(f[i]));
      out[o++] = lo ? f[i] - hi : hi;
    }
  };
  if (k.mode == MODE_WS9) {
    const size_t fm = 64 * 8, fk = 64 * 4;  // elements per 16x16x32 / 16x16x16 fragment
    const float* k8 = pk.data() + 18 * fm;
    for (int mh = 0; mh < 2; ++mh) {
      for (int ky = 0; ky < 9; ++ky)
        for (int hl = 0; hl < 2; ++hl) put(pk.data() + (2 * ky + mh) * fm, fm, hl == 1);
      for (int j = 0; j < 3; ++j)
        for (int hl = 0; hl < 2; ++hl) put(k8 + (2 * j + mh) * fk, fk, hl == 1);
    }
  } else {  // MODE_WS2: [cg][step][lane][8] -> [cg][hl][step][lane][8]
    const size_t per_cg = pk.size() / (k.bn / 16);
    for (int cg = 0; cg < k.bn / 16; ++cg)
      for (int hl = 0; hl < 2; ++hl) put(pk.data() + cg * per_cg, per_cg, hl == 1);
  }
  return out;
}

// MODE_KYROT weight table (conv_out9.hip): [part p][block (kx, kc)][K half h][row 3*ky + c][4],
// element j of a row = input channel kc*16 + 8h + 4p + j (kc = 16-channel block of the padded
// input channels), c = model output channel 0..2.
// Split mode (NST_DT_F32S, kc = 8-channel block): element j of a row = input channel kc*8 + 4h + j, part 0 its
// Wh = RNE16(w) (exact fp32 value here) and part 1 w - Wh, which the fp16 upload rounds to Wl = RNE16(w - Wh).
std::vector<float> pack_kyrot_weights(const ConvKernelInfo& k, const LayerDef& d, const float* W) {
  const bool split = k.dtype == NST_DT_F32S;
  const int cpb = split ? 8 : 16, kc_n = (k.cinp_k ? k.cinp_k : k.cinp) / cpb, nblk = 9 * kc_n;
  std::vector<float> out((size_t)k.wbytes / 2, 0.f);
  for (int pp = 0; pp < 2; ++pp)
    for (int ky = 0; ky < 9; ++ky)
      for (int kx = 0; kx < 9; ++kx)
        for (int kc = 0; kc < kc_n; ++kc)
          for (int hh = 0; hh < 2; ++hh)
            for (int c = 0; c < 3; ++c)
              for (int j = 0; j < 4; ++j) {
                const int ci = split ? kc * 8 + 4 * hh + j : kc * 16 + 8 * hh + 4 * pp + j;
                if (ci >= d.cin) continue;
                const size_t row = (((size_t)pp * nblk + kx * kc_n + kc) * 2 + hh) * 27 + 3 * ky + c;
                const float w = W[(((size_t)c * d.cin + ci) * d.ks + ky) * d.ks + kx];
                const float hi = f16_to_f32(f32_to_f16_rne(w));
                out[row * 4 + j] = split ? (pp == 0 ? hi : w - hi) : w;
              }
  return out;
}

// MODE_WSTAT weight registers (conv_wstat.hip): [wave w][step s][lane][8 bf16].  Step s = 9 q + tap,
// part q = input channels 32q..32q+31, tap = 3 dy + dx; lane l holds MFMA row l & 15 = output
// channel 16 w + (l & 15), K elements = input channels 32 q + 8 (l >> 4) + i.
std::vector<float> pack_wstat_weights(const LayerDef& d, const float* W) {
  std::vector<float> out((size_t)8 * 36 * 64 * 8, 0.f);
  for (int w = 0; w < 8; ++w)
    for (int s = 0; s < 36; ++s)
      for (int l = 0; l < 64; ++l) {
        const int q = s / 9, t = s % 9, dy = t / 3, dx = t % 3;
        const int co = 16 * w + (l & 15);
        for (int i = 0; i < 8; ++i) {
          const int ci = 32 * q + 8 * (l >> 4) + i;
          if (co < d.cout && ci < d.cin)
            out[(((size_t)w * 36 + s) * 64 + l) * 8 + i] = W[(((size_t)co * d.cin + ci) * d.ks + dy) * d.ks + dx];
        }
      }
  return out;
}

// MODE_WSTAT on 32x32x16 MFMAs (conv_wst32.hip, ConvKernelInfo::tw == 32): [wave w][step s][lane][8 x 16 bit].
// Step s = 2 (9 q + tap) + kk: part q = input channels 32q..32q+31, tap = 3 dy + dx, K half kk; lane l holds
// MFMA row l & 31 = output channel 32 w + (l & 31), K elements = input channels 32 q + 16 kk + 8 (l >> 5) + i.
std::vector<float> pack_wst32_weights(const LayerDef& d, const float* W) {
  std::vector<float> out((size_t)4 * 72 * 64 * 8, 0.f);
  for (int w = 0; w < 4; ++w)
    for (int s = 0; s < 72; ++s)
      for (int l = 0; l < 64; ++l) {
        const int kk = s & 1, t = (s >> 1) % 9, q = (s >> 1) / 9, dy = t / 3, dx = t % 3;
        const int co = 32 * w + (l & 31);
        for (int i = 0; i < 8; ++i) {
          const int ci = 32 * q + 16 * kk + 8 * (l >> 5) + i;
          if (co < d.cout && ci < d.cin)
            out[(((size_t)w * 72 + s) * 64 + l) * 8 + i] = W[(((size_t)co * d.cin + ci) * d.ks + dy) * d.ks + dx];
        }
      }
  return out;
}

// MODE_WSTAT on 16x16x32 MFMAs (conv_wst16.hip, tw == 32, wn == 2): [wave w][step s][lane][8 x 16 bit].  Step
// s = 2 (9 q + tap) + b: part q = input channels 32q..32q+31, tap = 3 dy + dx, channel block b; lane l holds MFMA row
// l & 15 = output channel 32 w + 16 b + (l & 15), K elements = input channels 32 q + 8 (l >> 4) + i.
std::vector<float> pack_wst16_weights(const LayerDef& d, const float* W) {
  std::vector<float> out((size_t)4 * 72 * 64 * 8, 0.f);
  for (int w = 0; w < 4; ++w)
    for (int s = 0; s < 72; ++s)
      for (int l = 0; l < 64; ++l) {
        const int b = s & 1, t = (s >> 1) % 9, q = (s >> 1) / 9, dy = t / 3, dx = t % 3;
        const int co = 32 * w + 16 * b + (l & 15);
        for (int i = 0; i < 8; ++i) {
          const int ci = 32 * q + 8 * (l >> 4) + i;
          if (co < d.cout && ci < d.cin)
            out[(((size_t)w * 72 + s) * 64 + l) * 8 + i] = W[(((size_t)co * d.cin + ci) * d.ks + dy) * d.ks + dx];
        }
      }
  return out;
}

// MODE_WPHASE weight registers (conv_wphase.hip): [wave w][step s][subtile t][lane][8 bf16].  Wave w
// computes phase w & 3 for output channels half w >> 2; step s = 4 q + tap (part q = input channels
// 32q..32q+31, tap = 2 ty + tx); lane l holds MFMA row l & 15 = output channel
// (w >> 2) * coutp / 2 + 16 t + (l & 15), K elements = input channels 32 q + 8 (l >> 4) + i.
std::vector<float> pack_wphase_weights(const ConvKernelInfo& k, const LayerDef& d, const float* W) {
  const int bn = k.bn_k ? k.bn_k : k.bn;  // computed channels (the stored bn may be narrower)
  const int nstep = 4 * (k.cinp / 32), ns = bn / 32;
  std::vector<float> out((size_t)8 * nstep * ns * 64 * 8, 0.f);
  for (int w = 0; w < 8; ++w)
    for (int s = 0; s < nstep; ++s)
      for (int t = 0; t < ns; ++t)
        for (int l = 0; l < 64; ++l) {
          const int q = s / 4, tap = s % 4;
          const int co = (w >> 2) * (bn / 2) + 16 * t + (l & 15);
          for (int i = 0; i < 8; ++i) {
            const int ci = 32 * q + 8 * (l >> 4) + i;
            if (co < d.cout && ci < d.cin)
              out[((((size_t)w * nstep + s) * ns + t) * 64 + l) * 8 + i] = (float)phase_weight(d, W, co, ci, w & 3, tap);
          }
        }
  return out;
}

// MODE_WS2 weight registers (conv_ws2.hip): [channel group cg][step s][lane][8 bf16].  Step s = 9 q +
// tap, part q = input channels 32q..32q+31, tap = 3 dy + dx; lane l holds MFMA row l & 15 = output
// channel 16 cg + (l & 15), K elements = input channels 32 q + 8 (l >> 4) + i.
std::vector<float> pack_ws2_weights(const ConvKernelInfo& k, const LayerDef& d, const float* W) {
  const int ncg = k.bn / 16, nstep = 9 * ((k.cinp_k ? k.cinp_k : k.cinp) / 32);
  std::vector<float> out((size_t)ncg * nstep * 64 * 8, 0.f);
  for (int cg = 0; cg < ncg; ++cg)
    for (int s = 0; s < nstep; ++s)
      for (int l = 0; l < 64; ++l) {
        const int q = s / 9, t = s % 9, dy = t / 3, dx = t % 3;
        const int co = 16 * cg + (l & 15);
        for (int i = 0; i < 8; ++i) {
          const int ci = 32 * q + 8 * (l >> 4) + i;
          if (co < d.cout && ci < d.cin)
            out[(((size_t)cg * nstep + s) * 64 + l) * 8 + i] = W[(((size_t)co * d.cin + ci) * d.ks + dy) * d.ks + dx];
        }
      }
  return out;
}

// MODE_WS9 weight registers (conv_ws9.hip), the same in every wave.  Kernel columns 0..7: 18
// 16x16x32 fragments [ky][m][lane][8 bf16], lane l = output channel 16 m + (l & 15), K element
// i = tap kx = 2 (l >> 4) + (i >> 2), input channel i & 3.  Column 8 (k.korder == 1): 4 16x16x32
// fragments [j][m][lane][8 bf16], j = 0: kernel row 2 (l >> 4) + (i >> 2); j = 1: kernel row 8 in
// lane group 0, elements 0..3 only; input channel i & 3.  (k.korder == 0: 6 16x16x16 fragments
// [j][m][lane][4 bf16], kernel row 4 j + (l >> 4), input channel i.)
// 64-channel kernels (k.bn == 64, ReCoNet): one such 32-channel set per channel half, half h = channels 32 h ..
std::vector<float> pack_ws9_weights(const ConvKernelInfo& k, const LayerDef& d, const float* W) {
  const int bnk = k.bn_k ? k.bn_k : k.bn;  // computed channels (the stored bn may be narrower)
  if (bnk > 32) {
    std::vector<float> all;
    for (int h = 0; h < bnk / 32; ++h) {
      ConvKernelInfo kh = k;
      kh.bn = 32;
      kh.bn_k = 0;
      LayerDef dh = d;
      dh.cout = std::max(0, std::min(32, d.cout - 32 * h));
      const std::vector<float> part =
          dh.cout > 0 ? pack_ws9_weights(kh, dh, W + (size_t)32 * h * d.cin * 81) : pack_ws9_weights(kh, dh, W);
      all.insert(all.end(), part.begin(), part.end());
    }
    return all;
  }
  const bool pair = k.korder == 1;
  std::vector<float> out((size_t)18 * 64 * 8 + (pair ? 4 * 64 * 8 : 6 * 64 * 4), 0.f);
  auto w = [&](int co, int ci, int ky, int kx) -> float {
    return (co < d.cout && ci < d.cin && ky < 9) ? W[(((size_t)co * d.cin + ci) * 9 + ky) * 9 + kx] : 0.f;
  };
  for (int ky = 0; ky < 9; ++ky)
    for (int m = 0; m < 2; ++m)
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 8; ++i)
          out[(((size_t)ky * 2 + m) * 64 + l) * 8 + i] = w(16 * m + (l & 15), i & 3, ky, 2 * (l >> 4) + (i >> 2));
  float* k8 = out.data() + (size_t)18 * 64 * 8;
  if (pair) {
    for (int m = 0; m < 2; ++m)
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 8; ++i) {
          const int co = 16 * m + (l & 15);
          k8[(((size_t)0 * 2 + m) * 64 + l) * 8 + i] = w(co, i & 3, 2 * (l >> 4) + (i >> 2), 8);
          k8[(((size_t)1 * 2 + m) * 64 + l) * 8 + i] = ((l >> 4) == 0 && i < 4) ? w(co, i & 3, 8, 8) : 0.f;
        }
  } else {
    for (int j = 0; j < 3; ++j)
      for (int m = 0; m < 2; ++m)
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 4; ++i) k8[(((size_t)j * 2 + m) * 64 + l) * 4 + i] = w(16 * m + (l & 15), i, 4 * j + (l >> 4), 8);
  }
  return out;
}

// bias rows of an x-shift layer: row q = 3*s + c -> bias of output channel (perm) c
std::vector<float> xshift_bias(const float* b, bool reverse_channels) {
  std::vector<float> r(16, 0.f);
  for (int q = 0; q < 15; ++q) r[q] = b[reverse_channels ? 2 - q % 3 : q % 3];
  return r;
}

int upload(const void* host, size_t bytes, void** dev) {
  NST_HIP_CHECK(hipMalloc(dev, bytes));
  NST_HIP_CHECK(hipMemcpy(*dev, host, bytes, hipMemcpyHostToDevice));
  return NST_OK;
}
int upload_weights(int dtype, const std::vector<float>& pk, void** dst) {
  if (dtype == NST_DT_F32) return upload(pk.data(), pk.size() * 4, dst);
  if (dtype == NST_DT_F32S) {
    // generic fragments [frag][lane][4] fp32 -> [frag][2][lane][8] fp16: [Wh0..3, Wh0..3] and
    // [Wl0..3, 0 x 4] with Wh = RNE(w), Wl = RNE(w - Wh) (conv_impl.h F32Split)
    const size_t nfrag = pk.size() / 256;
    std::vector<uint16_t> pb(nfrag * 2 * 64 * 8, 0);
    for (size_t f = 0; f < nfrag; ++f)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 4; ++j) {
          const float w = pk[(f * 64 + lane) * 4 + j];
          const uint16_t hi = f32_to_f16_rne(w);
          const uint16_t lo = f32_to_f16_rne(w - f16_to_f32(hi));
          pb[((f * 2) * 64 + lane) * 8 + j] = hi;
          pb[((f * 2) * 64 + lane) * 8 + 4 + j] = hi;
          pb[((f * 2 + 1) * 64 + lane) * 8 + j] = lo;
        }
    return upload(pb.data(), pb.size() * 2, dst);
  }
  std::vector<uint16_t> pb(pk.size());
  for (size_t i = 0; i < pk.size(); ++i) pb[i] = dtype == NST_DT_F16 ? f32_to_f16_rne(pk[i]) : f32_to_bf16_rne(pk[i]);
  return upload(pb.data(), pb.size() * 2, dst);
}

struct DeviceGuard {
  int prev = -1;
  bool changed = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
      changed = hipSetDevice(dev) == hipSuccess;
    }
  }
  ~DeviceGuard() {
    if (changed) (void)hipSetDevice(prev);
  }
};

// conv output extent along one axis for an input extent L
int conv_out_dim(const LayerDef& d, int L) {
  switch (d.axis_mode) {
    case AX_REFLECT_UP2: return (2 * L + 2 * d.pad - d.ks) / d.stride + 1;
    case AX_ZERO_PREREFLECT: return (L + 2 * d.pre + 2 * d.pad - d.ks) / d.stride + 1;
    case AX_ZINSERT: return 2 * L;  // ConvTranspose2d(k3, s2, p1, output_padding 1)
    default: return (L + 2 * d.pad - d.ks) / d.stride + 1;
  }
}

// minimum input extent for which the reference's padding is legal
bool layer_input_ok(const LayerDef& d, int L) {
  if (d.axis_mode == AX_REFLECT) return L > d.pad;
  if (d.axis_mode == AX_REFLECT_UP2) return 2 * L > d.pad;
  if (d.axis_mode == AX_ZERO_PREREFLECT) return L > d.pre;
  return L >= 1;
}

struct Plan {
  bool ok = false;
  std::string err;
  // per op: input and output dims
  std::vector<int> ih, iw, oh, ow, ch, cw;  // ch/cw: conv extent (before crop)
  // per op: element bytes of its source, its output and the residual stream it joins / writes (0: none)
  std::vector<int> in_esz, out_esz, res_esz;
  size_t buf_bytes[NBUF] = {0, 0, 0, 0, 0, 0, 0};
  size_t partial_floats = 0;
  int out_h = 0, out_w = 0;
  size_t ws_bytes = 0;
  size_t seg_bytes = 0;
  size_t off_buf[NBUF], off_partial, off_seg, off_stats, off_pre = 0;
  size_t pre_bytes = 0;
};

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

// workgroup tiles of a conv launch: phase mode tiles the SOURCE grid (each source pixel -> 4 outputs)
void tile_grid(const ConvKernelInfo& k, int sh, int sw, int oh, int ow, int* tx, int* ty) {
  if (k.mode == MODE_PHASE || k.mode == MODE_WPHASE) {
    *tx = (sw + k.tw - 1) / k.tw;
    *ty = (sh + k.th - 1) / k.th;
  } else {
    *tx = (ow + k.tw - 1) / k.tw;
    *ty = (oh + k.th - 1) / k.th;
  }
}

Plan make_plan(const nst_handle* h, int n, int H, int W) {
  Plan P;
  int bh[NBUF], bw[NBUF], be[NBUF];  // extent and element bytes of what each buffer holds
  for (int b = 0; b < NBUF; ++b) be[b] = (int)act_elem_bytes(h->dtype);
  const size_t nops = h->prog.size();
  P.ih.resize(nops); P.iw.resize(nops); P.oh.resize(nops); P.ow.resize(nops); P.ch.resize(nops); P.cw.resize(nops);
  P.in_esz.assign(nops, 0); P.out_esz.assign(nops, 0); P.res_esz.assign(nops, 0);
  for (size_t i = 0; i < nops; ++i) {
    const Op& op = h->prog[i];
    const Layer& Ly = h->layers[op.layer];
    if (op.kind == OP_CONV) {
      const int sh = op.src == B_IMG ? H : bh[op.src];
      const int sw = op.src == B_IMG ? W : bw[op.src];
      if (!layer_input_ok(Ly.d, sh) || !layer_input_ok(Ly.d, sw)) {
        P.err = "input " + std::to_string(H) + "x" + std::to_string(W) + " too small for layer " + Ly.d.conv +
                " (padding must be smaller than its input " + std::to_string(sh) + "x" + std::to_string(sw) + ")";
        return P;
      }
      const int ch = conv_out_dim(Ly.d, sh), cw = conv_out_dim(Ly.d, sw);
      // the conv kernels address a frame (a launch's frames, for the weight-stationary ones) with
      // 32-bit buffer offsets, 0x80000000 and up reserved as the out-of-range offset: one frame's
      // activation must stay below 2^31 bytes (a 16-bit 128-channel map of 8.4 Gpx / 4)
      const int iesz = op.src == B_IMG ? 2 : be[op.src];
      if (op.src != B_IMG && iesz != Ly.in_esz) {
        P.err = "internal: layer " + Ly.d.conv + " reads " + std::to_string(iesz) + "-byte activations, its kernel " +
                std::to_string(Ly.in_esz);
        return P;
      }
      P.in_esz[i] = iesz;
      P.out_esz[i] = Ly.out_esz;
      const size_t fin = (size_t)sh * sw * (op.src == B_IMG ? 4 : Ly.cinp) * iesz;
      const size_t fout = (size_t)ch * cw * Ly.coutp * Ly.out_esz;
      if (std::max(fin, fout) >= (size_t)0x7FFFFF00u) {
        P.err = "input " + std::to_string(H) + "x" + std::to_string(W) + " too large: layer " + Ly.d.conv +
                " needs " + std::to_string(std::max(fin, fout)) + " bytes per frame (limit 2^31)";
        return P;
      }
      if (op.src == B_IMG && (Ly.prepad || Ly.k_u8fold)) {  // 16-bit x4 per pixel over the conv's padded input extent
        // + zeroed tail slack (prepad_slack_rows): the 9x9 kernel's last tile row reads up to 16 halo rows
        // (and a pixel of column wrap) from its tile origin, which may lie past the last frame's padded extent
        const int wpad = cw + Ly.d.ks - 1;
        const size_t pb = ((size_t)n * (ch + Ly.d.ks - 1) + prepad_slack_rows(wpad)) * wpad * 8;
        if (pb > P.pre_bytes) P.pre_bytes = pb;
      }
      if (op.res_buf >= 0) P.res_esz[i] = be[op.res_buf];
      if (op.res_out >= 0) {  // the joined residual stream: same geometry and format as the conv input
        bh[op.res_out] = sh; bw[op.res_out] = sw; be[op.res_out] = iesz;
        P.res_esz[i] = iesz;
        const size_t rb = (size_t)n * sh * sw * Ly.cinp * iesz;
        if (rb > P.buf_bytes[op.res_out]) P.buf_bytes[op.res_out] = rb;
      }
      P.ih[i] = sh; P.iw[i] = sw; P.ch[i] = ch; P.cw[i] = cw;
      if (op.dst == B_OUT) {
        if (h->arch == NST_ARCH_NST) {  // centre crop back to the input size (transformer_net_nst.py:121-125)
          P.oh[i] = H; P.ow[i] = W;
        } else {
          P.oh[i] = ch; P.ow[i] = cw;
        }
        P.out_h = P.oh[i]; P.out_w = P.ow[i];
      } else {
        P.oh[i] = ch; P.ow[i] = cw;
        bh[op.dst] = ch; bw[op.dst] = cw; be[op.dst] = Ly.out_esz;
        const size_t bytes = (size_t)n * ch * cw * Ly.coutp * Ly.out_esz;
        if (bytes > P.buf_bytes[op.dst]) P.buf_bytes[op.dst] = bytes;
        for (const ConvKernelInfo* kk : {Ly.k_main, Ly.k_u8fold}) {
          if (!kk) continue;
          int ttx, tty;
          tile_grid(*kk, sh, sw, ch, cw, &ttx, &tty);
          const size_t pf = (size_t)n * ttx * tty * kk->part_rows * Ly.coutp * 2;
          if (pf > P.partial_floats) P.partial_floats = pf;
        }
        const size_t sb = (size_t)n * IN_MAX_SEGMENTS * Ly.coutp * 16;
        if (sb > P.seg_bytes) P.seg_bytes = sb;
      }
    } else {
      P.ih[i] = P.oh[i] = bh[op.src];
      P.iw[i] = P.ow[i] = bw[op.src];
      P.in_esz[i] = be[op.src];
      P.res_esz[i] = be[op.r_buf];
      P.out_esz[i] = op.out_esz ? op.out_esz : be[op.src];
      be[op.dst] = P.out_esz[i];
      const size_t rb = (size_t)n * bh[op.src] * bw[op.src] * Ly.coutp * P.out_esz[i];
      if (rb > P.buf_bytes[op.dst]) P.buf_bytes[op.dst] = rb;
      bh[op.dst] = bh[op.src];
      bw[op.dst] = bw[op.src];
    }
  }
  size_t off = 0;
  for (int b = 0; b < NBUF; ++b) { P.off_buf[b] = off; off += align256(P.buf_bytes[b]); }
  P.off_partial = off;
  off += align256(P.partial_floats * 4);
  P.off_seg = off;
  off += align256(P.seg_bytes);
  P.off_pre = off;
  off += align256(P.pre_bytes);
  P.off_stats = off;
  for (const Layer& Ly : h->layers) off += align256((size_t)n * Ly.coutp * 8);
  P.ws_bytes = off;
  P.ok = true;
  return P;
}

struct PresetConsts {
  float ea[3], eb[3], ed[3];
  int eperm[3];
  float dp[3], dq[3], dr[3], ds[3];
  int dperm[3];
};

// fp32 constants exactly as the reference's torch expressions round them (pipeline.py:272-273, 1445-1486)
bool preset_consts(int preset, PresetConsts& c) {
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  const float caffe[3] = {103.939f, 116.779f, 123.68f};
  for (int i = 0; i < 3; ++i) {
    c.ea[i] = 1.f; c.eb[i] = 0.f; c.ed[i] = 1.f; c.eperm[i] = i;
    c.dp[i] = 0.f; c.dq[i] = 1.f; c.dr[i] = 1.f; c.ds[i] = 0.f; c.dperm[i] = i;
  }
  switch (preset) {
    case NST_PRESET_NONE: case NST_PRESET_RAW_01: return true;
    case NST_PRESET_TANH:
      for (int i = 0; i < 3; ++i) { c.ea[i] = 2.f; c.eb[i] = 1.f; c.dp[i] = 1.f; c.dq[i] = 0.5f; }
      return true;
    case NST_PRESET_IMAGENET_01:
      for (int i = 0; i < 3; ++i) { c.eb[i] = mean[i]; c.ed[i] = stdv[i]; c.dq[i] = stdv[i]; c.ds[i] = mean[i]; }
      return true;
    case NST_PRESET_IMAGENET_255:
      for (int i = 0; i < 3; ++i) {
        volatile float m = mean[i] * 255.0f, s = stdv[i] * 255.0f;
        c.ea[i] = 255.f; c.eb[i] = m; c.ed[i] = s; c.dr[i] = 255.f;
      }
      return true;
    case NST_PRESET_CAFFE_BGR:
      for (int i = 0; i < 3; ++i) {
        c.ea[i] = 255.f; c.eb[i] = caffe[i]; c.eperm[i] = 2 - i; c.dr[i] = 255.f; c.dperm[i] = 2 - i;
      }
      return true;
    case NST_PRESET_RAW_255:
      for (int i = 0; i < 3; ++i) { c.ea[i] = 255.f; c.dr[i] = 255.f; }
      return true;
    default: return false;
  }
}

// The first layer over uint8 frames with the io_preset encode folded into its weights: the reference feeds
// x_c = ((byte[perm c] / 255) * a_c - b_c) / d_c (pipeline.py:1445-1486) to the conv; the engine stages
// o_c = byte[perm c] / 256, exact in bf16 and fp16, so conv(W, x) = conv(W', o) + sum W b_c / d_c with
//   W'[.][c] = W[.][c] * 256 a_c / (255 d_c),   bias' = bias - sum_{c,ky,kx} W[.][c][ky][kx] b_c / d_c
// (fp64, then fp32; the reference's own fp32 rounding of x_c is ~2^-24 relative).  The operand then carries no
// rounding at all, which in the 16-bit modes was the largest single source of output error (tests/precision_study.py).
// The constant b_c / d_c survives reflection padding but not zero padding, so zero-padded first layers fold only
// presets with b = 0 (raw_01 / raw_255 / tanh's b = 1 does not).  false: no fold for this preset.
bool fold_first_layer(const LayerDef& d, const float* W, const float* b, int preset, std::vector<float>& Wf,
                      std::vector<float>& bf) {
  PresetConsts pc;
  if (preset == NST_PRESET_NONE || !preset_consts(preset, pc)) return false;
  if (d.axis_mode != AX_REFLECT)
    for (int c = 0; c < 3; ++c)
      if (pc.eb[c] != 0.f) return false;
  const int kk = d.ks * d.ks;
  Wf.assign(W, W + (size_t)d.cout * d.cin * kk);
  bf.assign(b, b + d.cout);
  for (int o = 0; o < d.cout; ++o) {
    double sb = b[o];
    for (int c = 0; c < d.cin; ++c) {
      const double sc = 256.0 * (double)pc.ea[c] / (255.0 * (double)pc.ed[c]), sh = (double)pc.eb[c] / (double)pc.ed[c];
      for (int t = 0; t < kk; ++t) {
        const size_t i = ((size_t)o * d.cin + c) * kk + t;
        Wf[i] = (float)((double)W[i] * sc);
        sb -= (double)W[i] * sh;
      }
    }
    bf[o] = (float)sb;
  }
  return true;
}

}  // namespace

namespace nst {
// pack a plain conv weight [cout][cin][ks][ks] (fp32, host) for a generic-kernel instantiation and
// upload it (bf16 or fp32 per the kernel); used by the VGG program (vgg_gatys.cpp)
int pack_upload_conv(const ConvKernelInfo& k, int cin, int cout, int ks, const float* W, int coutp, void** dev) {
  LayerDef d{"", "", cin, cout, ks, 1, AX_ZERO, ks / 2, 0, false};
  return upload_weights(k.dtype, pack_weights(k, d, W, coutp), dev);
}
int upload_floats(const float* host, size_t n, float** dev) { return upload(host, n * 4, (void**)dev); }
// the output decode constants of an io_preset (the region compositor's sources, region_api.cpp)
bool decode_consts_for_preset(int preset, DecodeConsts& d) {
  PresetConsts pc;
  if (!preset_consts(preset, pc)) return false;
  for (int c = 0; c < 3; ++c) {
    d.p[c] = pc.dp[c]; d.q[c] = pc.dq[c]; d.r[c] = pc.dr[c]; d.s[c] = pc.ds[c]; d.perm[c] = pc.dperm[c];
  }
  return true;
}
void tile_grid_of(const ConvKernelInfo& k, int sh, int sw, int oh, int ow, int* tx, int* ty) {
  tile_grid(k, sh, sw, oh, ow, tx, ty);
}
// ReCoNet(frn=True) (model.py:18-60 with frn.py:7-78): every FRN / TLU pair runs as the InstanceNorm
// / ReLU machinery with shifted activations.  TLU max(v, tau) = ReLU(v - tau) + tau, so the engine keeps
// z' = z - tau wherever the reference keeps a TLU output z:
//   * a ConvNormLayer with TLU: FRN shift beta - tau (the fill's ReLU then yields z');
//   * a ResLayer's join x' = ReLU(FRN(y) + x'_prev + tau_prev - tau_act): shift beta + tau_prev - tau_act
//     on the branch's second (activation-free) FRN;
//   * every conv reading a z' adds sum_{c,ky,kx} W[o][c][ky][kx] tau_c to its bias: with reflection
//     padding and nearest x2 upsampling a per-channel constant image stays constant, so
//     conv(z) = conv(z') + that sum everywhere.
// Layer indices: 0-2 encoder ConvNormLayers, 3 + 2r / 4 + 2r the branch of ResLayer r, 11 / 12 the
// decoder ConvNormLayers, 13 the ConvTanhLayer.
template <typename Get>
int frn_layer(Get& get, int li, const LayerDef& d, const float* W, const float* b, const float* bt,
              std::vector<float>& b_fold, std::vector<float>& bt_fold, float& eps) {
  auto act_tau = [](int l) -> std::string {  // TLU after layer l's FRN
    if (l <= 2) return "encoder.layers." + std::to_string(l) + ".layers.2.tau";
    if (l <= 10) return "encoder.layers." + std::to_string(3 + (l - 3) / 2) + ".branch.0.layers.2.tau";
    return l == 11 ? "decoder.layers.1.layers.2.tau" : "decoder.layers.3.layers.2.tau";
  };
  auto block_tau = [](int r) { return "encoder.layers." + std::to_string(3 + r) + ".activation.tau"; };
  auto stream_tau = [&](int r) { return r == 0 ? act_tau(2) : block_tau(r - 1); };  // the stream entering block r
  std::string in_tau;  // the TLU whose output this conv reads
  if (li == 1 || li == 2) in_tau = act_tau(li - 1);
  else if (li >= 3 && li <= 10) in_tau = (li - 3) % 2 == 0 ? stream_tau((li - 3) / 2) : act_tau(li - 1);
  else if (li == 11) in_tau = block_tau(3);
  else if (li >= 12) in_tau = act_tau(li - 1);
  const float* tin = nullptr;
  int rc = NST_OK;
  if (!in_tau.empty() && (rc = get(in_tau, d.cin, &tin)) != NST_OK) return rc;
  b_fold.assign(b, b + d.cout);
  if (tin) {
    const int kk = d.ks * d.ks;
    for (int o = 0; o < d.cout; ++o) {
      double s = b[o];
      for (int c = 0; c < d.cin; ++c) {
        double wsum = 0.0;
        for (int t = 0; t < kk; ++t) wsum += W[((size_t)o * d.cin + c) * kk + t];
        s += wsum * (double)tin[c];
      }
      b_fold[o] = (float)s;
    }
  }
  if (d.norm.empty()) return NST_OK;
  const float* e = nullptr;
  if ((rc = get(d.norm + ".eps", 1, &e)) != NST_OK) return rc;
  eps = std::fabs(e[0]);  // nu2 + eps.abs() (frn.py:74)
  bt_fold.assign(bt, bt + d.cout);
  const bool join = li >= 3 && li <= 10 && (li - 3) % 2 == 1;
  const float *t_own = nullptr, *t_prev = nullptr;
  if (join) {
    const int r = (li - 3) / 2;
    if ((rc = get(block_tau(r), d.cout, &t_own)) != NST_OK) return rc;
    if ((rc = get(stream_tau(r), d.cout, &t_prev)) != NST_OK) return rc;
  } else if ((rc = get(act_tau(li), d.cout, &t_own)) != NST_OK) {
    return rc;
  }
  for (int c = 0; c < d.cout; ++c)
    bt_fold[c] = (float)((double)bt[c] - (double)t_own[c] + (t_prev ? (double)t_prev[c] : 0.0));
  return NST_OK;
}

}  // namespace nst

extern "C" {

const char* nst_last_error(void) { return g_last_error.c_str(); }
const char* nst_version(void) { return "nst_hip 0.1.0 (gfx950)"; }

int nst_create(int arch, const nst_param* params, int n_params, int compute_dtype, int device,
               nst_handle** out) {
  return nst_create_ex(arch, params, n_params, compute_dtype, device, 0u, out);
}

int nst_create_ex(int arch, const nst_param* params, int n_params, int compute_dtype, int device,
                  unsigned flags, nst_handle** out) {
  if (!out || arch < 0 || arch > 3 || (compute_dtype != NST_DT_F32 && compute_dtype != NST_DT_BF16 && compute_dtype != NST_DT_F16 &&
                                           compute_dtype != NST_DT_F32S && compute_dtype != NST_DT_F16M) ||
      (flags & ~(unsigned)NST_KSEL_ALL) != 0) {
    set_error("nst_create: invalid arguments");
    return NST_E_INVALID;
  }
  const bool f16m = compute_dtype == NST_DT_F16M;
  // residual blocks on the split-operand kernel: the first (tests/precision_study.py: live max 0.958 LSB on the
  // bench frames; 1,114 frames/s), or the first two with NST_KSEL_F16M_TWO_BLOCKS (0.920 LSB; 1,014 frames/s)
  const int split_blocks = !f16m ? 0 : ((flags & NST_KSEL_F16M_TWO_BLOCKS) ? 2 : 1);
  if (f16m && (is_reconet(arch) || (flags & (NST_KSEL_UNFUSED_RESIDUAL | NST_KSEL_NO_WS9 | NST_KSEL_NO_WS2 | NST_KSEL_NO_PREPAD)))) {
    set_error("nst_create: NST_DT_F16M is built for the Johnson / NST nets with the default kernel selection");
    return NST_E_INVALID;
  }
  // per-layer arithmetic of NST_DT_F16M (tests/precision_study.py: these layers' roundings reach the frame most)
  auto layer_kdt = [&](size_t li) -> int {
    if (!f16m) return compute_dtype;
    if (li == 0) return NST_KDT_SW_O32;            // raw-byte operand x fp16 hi / lo weights, fp32 out
    if (li == 1 || li == 2) return NST_KDT_SPLIT_O32;  // split operand and weights, fp32 out
    if (li >= 3 && li < 3 + 2 * (size_t)split_blocks) return NST_KDT_SPLITO_O32;  // split residual blocks: split
                                                                                  // operand, fp16 weights, fp32
    return NST_DT_F16;
  };
  const bool no_pers = (flags & NST_KSEL_NO_PERSISTENT) != 0;
  *out = nullptr;
  std::map<std::string, const nst_param*> byname;
  for (int i = 0; i < n_params; ++i)
    if (params[i].name) byname[params[i].name] = &params[i];
  auto get = [&](const std::string& name, int64_t numel, const float** p) -> int {
    auto it = byname.find(name);
    if (it == byname.end()) { set_error("missing checkpoint tensor: " + name); return NST_E_PARAM; }
    if (it->second->numel != numel) {
      set_error("checkpoint tensor " + name + " has " + std::to_string(it->second->numel) +
                " elements, expected " + std::to_string(numel));
      return NST_E_PARAM;
    }
    *p = it->second->data;
    return NST_OK;
  };
  DeviceGuard guard(device);
  auto* h = new nst_handle();
  h->arch = arch; h->dtype = compute_dtype; h->device = device;
  std::vector<LayerDef> defs;
  const bool fuse_res = (flags & NST_KSEL_UNFUSED_RESIDUAL) == 0;
  build_program(arch, fuse_res, fuse_res, defs, h->prog, split_blocks);
  // layers whose fill joins the residual stream run the VAR_RES instantiation
  std::vector<int> res_layer(defs.size(), 0);
  for (const Op& op : h->prog)
    if (op.kind == OP_CONV && op.res_buf >= 0) res_layer[op.layer] = 1;
  // activation channel padding: fp32 chunks hold 4 channels (K step 16); bf16 chunks 8 (K step 32),
  // and bf16 tiles above 32 channels come in multiples of 64 (48->64, 96->128)
  auto pad_ch = [&](int c) {
    if (f32_storage(compute_dtype)) return round_up(c, 16);  // (NST_DT_F16M: 32 / 64 / 128 either way)
    return c <= 32 ? 32 : round_up(c, 64);
  };
  int rc = NST_OK;
  for (size_t li = 0; li < defs.size() && rc == NST_OK; ++li) {
    Layer Ly;
    Ly.d = defs[li];
    const LayerDef& d = Ly.d;
    const int kdt = layer_kdt(li);
    Ly.kdt = kdt;
    const bool image_in = li == 0;
    const bool final_layer = d.norm.empty();
    Ly.cinp = image_in ? 4 : pad_ch(d.cin);
    Ly.coutp = final_layer ? 16 : pad_ch(d.cout);
    // ReCoNet's decoder stream (decoder.layers.1 -> .3, 96 channels) stays unpadded in the 16-bit modes: 25 % fewer
    // MFMAs in both up-convs and 25 % fewer bytes of the 540p map than the 128-channel stride
    if (is_reconet(arch) && !f32_storage(compute_dtype) && !(flags & NST_KSEL_PAD_DECODER)) {
      if (li == 11) Ly.coutp = 96;
      if (li == 12) Ly.cinp = 96;
    }
    // the first layer's 48-channel output (encoder.layers.0 -> .1): the 9x9 kernel stores 48 of 64, the down-conv
    // stages zeros for the rest (with the unpadded 96-channel encoder map only)
    if (is_reconet(arch) && !f32_storage(compute_dtype) &&
        !(flags & (NST_KSEL_PAD_48 | NST_KSEL_PAD_ENCODER | NST_KSEL_NO_WS9 | NST_KSEL_NO_WS2 | NST_KSEL_NO_PREPAD))) {
      if (li == 0) Ly.coutp = 48;
      if (li == 1) Ly.cinp = 48;
    }
    // ... and its 48-channel output (decoder.layers.3 -> .4): the phase kernel stores 48 of its 64 computed channels,
    // the output conv stages zeros for the missing 16 (the three-part phase kernel and the row-streaming output conv
    // only: not with the padded 96-channel decoder stream or without those kernels)
    if (is_reconet(arch) && !f32_storage(compute_dtype) &&
        !(flags & (NST_KSEL_PAD_48 | NST_KSEL_PAD_DECODER | NST_KSEL_NO_WPHASE | NST_KSEL_NO_KYROT))) {
      if (li == 12) Ly.coutp = 48;
      if (li == 13) Ly.cinp = 48;
    }
    // ... and the encoder's (encoder.layers.1 -> .2): 96 output channels on 12-wave down-conv tiles, K of 96
    if (is_reconet(arch) && !f32_storage(compute_dtype) && !(flags & NST_KSEL_PAD_ENCODER)) {
      if (li == 1) Ly.coutp = 96;
      if (li == 2) Ly.cinp = 96;
    }
    const int ink = image_in ? IN_U8_NHWC : IN_ACT;
    const int outk = final_layer ? OUT_U8_NHWC : OUT_ACT;
    // preferred mapping: sub-pixel phases for x2 up-convs, x-shift rows for the 3-channel output
    // conv; the plain mapping is the fallback for shapes without a compiled variant
    const bool up = d.axis_mode == AX_REFLECT_UP2 || d.axis_mode == AX_ZINSERT;
    std::vector<int> modes;
    // x2 up-convs: weight-stationary phase kernel (conv_wphase.hip) where compiled; its fused join
    // has no ReLU after the sum (ReCoNet's has), so ReCoNet's residual consumers skip it
    if (up && !(res_layer[li] && is_reconet(arch)) && !(flags & NST_KSEL_NO_WPHASE))
      modes.push_back(MODE_WPHASE);
    if (up) modes.push_back(MODE_PHASE);
    if (final_layer && d.cout == 3) {
      if (!(flags & NST_KSEL_NO_KYROT)) modes.push_back(MODE_KYROT);
      modes.push_back(MODE_XSHIFT);
    }
    // residual-trunk convs (128 -> 128, 3x3): weight-stationary kernel (conv_wstat.hip); ReCoNet's
    // trunk is 192 channels and its join has a ReLU after the sum, so it never matches
    if (!up && !final_layer && !image_in && d.ks == 3 && d.stride == 1 && !is_reconet(arch) &&
        !(flags & NST_KSEL_NO_WSTAT))
      modes.push_back(MODE_WSTAT);
    // stride-2 down-convs: weight-stationary kernel (conv_ws2.hip) where compiled
    if (!up && !final_layer && !image_in && d.ks == 3 && d.stride == 2 && !(flags & NST_KSEL_NO_WS2))
      modes.push_back(MODE_WS2);
    if (kdt == NST_KDT_SPLITO_O32) modes.insert(modes.begin(), MODE_WS1S);
    modes.push_back(MODE_STD);
    // image layer: prefer the conv over the pre-padded encoded input (one streaming pre-pass, plain
    // 16-byte fill loads) when it is compiled for this shape; it serves u8 and f32 inputs alike
    if (image_in && !(flags & NST_KSEL_NO_PREPAD)) {
      // weight-stationary 9x9 kernel (conv_ws9.hip) where compiled, else the generic one
      Ly.k_main = (flags & NST_KSEL_NO_WS9)
                      ? nullptr
                      : find_conv_kernel(kdt, MODE_WS9, d.ks, d.stride, Ly.cinp, Ly.coutp, IN_ACT, outk, 0, no_pers);
      if (Ly.k_main) Ly.mode = MODE_WS9;
      else Ly.k_main = find_conv_kernel(kdt, MODE_STD, d.ks, d.stride, Ly.cinp, Ly.coutp, IN_ACT, outk, 0, no_pers);
      if (Ly.k_main && d.stride == 1) { Ly.prepad = true; Ly.k_alt = Ly.k_main; modes.clear(); }
      else Ly.k_main = nullptr;
    }
    for (int mode : modes) {
      Ly.k_main = find_conv_kernel(kdt, mode, d.ks, d.stride, Ly.cinp, Ly.coutp, ink, outk, res_layer[li], no_pers);
      Ly.k_alt = nullptr;
      if (image_in) Ly.k_alt = find_conv_kernel(kdt, mode, d.ks, d.stride, Ly.cinp, Ly.coutp, IN_F32_NCHW, outk, 0, no_pers);
      if (final_layer) Ly.k_alt = find_conv_kernel(kdt, mode, d.ks, d.stride, Ly.cinp, Ly.coutp, ink, OUT_F32_NCHW, 0, no_pers);
      const bool tanh_ok = mode != MODE_KYROT || !Ly.k_main ||
                           (Ly.k_main->tanh_out == (is_reconet(arch) ? 1 : 0) && Ly.k_alt &&
                            Ly.k_alt->tanh_out == Ly.k_main->tanh_out);
      if (Ly.k_main && tanh_ok && (!(image_in || final_layer) || Ly.k_alt)) { Ly.mode = mode; break; }
      Ly.k_main = nullptr;
    }
    if (!Ly.k_main || ((image_in || final_layer) && !Ly.k_alt)) {
      set_error("no compiled conv kernel for layer " + d.conv + " (ks " + std::to_string(d.ks) + " stride " +
                std::to_string(d.stride) + " cin " + std::to_string(Ly.cinp) + " cout " + std::to_string(Ly.coutp) + ")");
      rc = NST_E_SHAPE;
      break;
    }
    const float *W = nullptr, *b = nullptr, *gm = nullptr, *bt = nullptr;
    const int64_t wn = (int64_t)d.cout * d.cin * d.ks * d.ks;
    if ((rc = get(d.conv + ".weight", wn, &W)) != NST_OK) break;
    if ((rc = get(d.conv + ".bias", d.cout, &b)) != NST_OK) break;
    if (!final_layer) {
      if ((rc = get(d.norm + ".weight", d.cout, &gm)) != NST_OK) break;
      if ((rc = get(d.norm + ".bias", d.cout, &bt)) != NST_OK) break;
    }
    std::vector<float> b_fold, bt_fold;
    if (arch == NST_ARCH_RECONET_FRN) {
      if ((rc = frn_layer(get, (int)li, d, W, b, bt, b_fold, bt_fold, Ly.eps)) != NST_OK) break;
      b = b_fold.data();
      if (!final_layer) bt = bt_fold.data();
      Ly.frn = final_layer ? 0 : 1;
    }
    auto upload_packed = [&](const std::vector<float>& pk, void** dst) -> int {
      if (Ly.k_main->split_w) return upload_weights(NST_DT_F16, split_weight_frags(*Ly.k_main, pk), dst);
      // the split-operand kernels (NST_KDT_*) take plain fp16 weights
      return upload_weights(kdt >= NST_KDT_SW_O32 ? NST_DT_F16 : kdt, pk, dst);
    };
    Ly.in_esz = Ly.k_main->in_esz ? Ly.k_main->in_esz : (int)act_elem_bytes(kdt);
    Ly.out_esz = Ly.k_main->out_esz ? Ly.k_main->out_esz : (int)act_elem_bytes(kdt);
    if (Ly.mode == MODE_KYROT) {
      const std::vector<float> pk = pack_kyrot_weights(*Ly.k_main, d, W);
      // the split table holds its Wh / Wl parts itself: plain fp16 upload
      if ((rc = Ly.k_main->dtype == NST_DT_F32S ? upload_weights(NST_DT_F16, pk, &Ly.wpk) : upload_packed(pk, &Ly.wpk)) != NST_OK)
        break;
    } else if (Ly.mode == MODE_WSTAT) {
      if ((rc = upload_packed(Ly.k_main->tw != 32 ? pack_wstat_weights(d, W)
                                                   : Ly.k_main->wn == 2 ? pack_wst16_weights(d, W) : pack_wst32_weights(d, W),
                              &Ly.wpk)) != NST_OK)
        break;
    } else if (Ly.mode == MODE_WPHASE) {
      if ((rc = upload_packed(pack_wphase_weights(*Ly.k_main, d, W), &Ly.wpk)) != NST_OK) break;
    } else if (Ly.mode == MODE_WS2 || Ly.mode == MODE_WS1S) {  // [channel group][step][lane][8]: the same order
      if ((rc = upload_packed(pack_ws2_weights(*Ly.k_main, d, W), &Ly.wpk)) != NST_OK) break;
    } else if (Ly.mode == MODE_WS9) {
      if ((rc = upload_packed(pack_ws9_weights(*Ly.k_main, d, W), &Ly.wpk)) != NST_OK) break;
    } else if ((rc = upload_packed(pack_weights(*Ly.k_main, d, W, Ly.coutp), &Ly.wpk)) != NST_OK) {
      break;
    }
    if (Ly.prepad && !f32_storage(compute_dtype) && !(flags & NST_KSEL_NO_FOLD)) {
      for (int pr = 1; pr < 8 && rc == NST_OK; ++pr) {
        std::vector<float> Wf, bfo;
        if (!fold_first_layer(d, W, b, pr, Wf, bfo)) continue;
        std::vector<float> pk = Ly.mode == MODE_WS9 ? pack_ws9_weights(*Ly.k_main, d, Wf.data())
                                                    : pack_weights(*Ly.k_main, d, Wf.data(), Ly.coutp);
        std::vector<float> bpad(Ly.coutp, 0.f);
        std::copy(bfo.begin(), bfo.end(), bpad.begin());
        if ((rc = upload_packed(pk, &Ly.wpk_fold[pr])) != NST_OK) break;
        rc = upload(bpad.data(), bpad.size() * 4, (void**)&Ly.bias_fold[pr]);
      }
      if (rc != NST_OK) break;
    }
    // NST_DT_F32S over uint8 frames: raw byte / 256 is exact in fp16, so NST_DT_F16M's split-weight 9x9 kernel (fp16
    // hi / lo weight pairs, fp32 accumulate and output) over the folded encode computes what the split-operand
    // generic kernel computes for those frames (its lo operand half is zero) at conv_ws9.hip's rate
    if (image_in && compute_dtype == NST_DT_F32S && d.stride == 1 &&
        !(flags & (NST_KSEL_NO_FOLD | NST_KSEL_NO_WS9 | NST_KSEL_NO_PREPAD))) {
      const ConvKernelInfo* kf = find_conv_kernel(NST_KDT_SW_O32, MODE_WS9, d.ks, d.stride, 4, Ly.coutp, IN_ACT, OUT_ACT, 0, no_pers);
      if (kf && kf->out_esz == Ly.out_esz && kf->bn == Ly.coutp) {
        for (int pr = 1; pr < 8 && rc == NST_OK; ++pr) {
          std::vector<float> Wf, bfo;
          if (!fold_first_layer(d, W, b, pr, Wf, bfo)) continue;
          if ((rc = upload_weights(NST_DT_F16, split_weight_frags(*kf, pack_ws9_weights(*kf, d, Wf.data())), &Ly.wpk_fold[pr])) != NST_OK)
            break;
          std::vector<float> bpad(Ly.coutp, 0.f);
          std::copy(bfo.begin(), bfo.end(), bpad.begin());
          rc = upload(bpad.data(), bpad.size() * 4, (void**)&Ly.bias_fold[pr]);
        }
        if (rc != NST_OK) break;
        Ly.k_u8fold = kf;
      }
    }
    std::vector<float> bp(Ly.coutp, 0.f), gp(Ly.coutp, 0.f), btp(Ly.coutp, 0.f);
    for (int c = 0; c < d.cout; ++c) {
      bp[c] = b[c];
      if (gm) { gp[c] = gm[c]; btp[c] = bt[c]; }
    }
    if (Ly.mode == MODE_XSHIFT) {
      // rows carry (shift, channel); a second, channel-reversed packing serves caffe_bgr's BGR decode
      bp = xshift_bias(b, false);
      std::vector<float> br = xshift_bias(b, true);
      if ((rc = upload_packed(pack_weights(*Ly.k_main, d, W, Ly.coutp, true), &Ly.wpk_rev)) != NST_OK) break;
      if ((rc = upload(br.data(), br.size() * 4, (void**)&Ly.bias_rev)) != NST_OK) break;
    }
    if ((rc = upload(bp.data(), bp.size() * 4, (void**)&Ly.bias)) != NST_OK) break;
    if (!final_layer) {
      if ((rc = upload(gp.data(), gp.size() * 4, (void**)&Ly.gamma)) != NST_OK) break;
      if ((rc = upload(btp.data(), btp.size() * 4, (void**)&Ly.beta)) != NST_OK) break;
    }
    h->layers.push_back(Ly);
  }
  if (rc != NST_OK) {
    nst_destroy(h);
    return rc;
  }
  // x_0 export needs block 1's conv1 on the weight-stationary kernel; otherwise block 2's join
  // normalises conv3's output itself (the same layers and residual layers either way)
  // x_0 export: the weight-stationary trunk kernel and the generic stride-1 kernel write it from their fill
  if (fuse_res && !f16m && h->layers[3].mode != MODE_WSTAT && h->layers[3].mode != MODE_STD)
    build_program(arch, true, false, defs, h->prog);
  // ReCoNet's 16-bit programs (generic kernels with launch tails) run a batch as 2 sub-batches on 2 streams: 10.66-10.75
  // -> 10.38-10.45 ms per 8 1080p frames (4 sub-batches: 11.1, more streams than the 4 hardware queues;
  // tools/stream_split_bench.py, profiles/r05_x_stream_split.txt); the Johnson / NST programs (persistent kernels
  // filling every CU) measured slower split (5.17 -> 5.27 / 5.44 ms), fp16m neutral
  // The split-fp16 mode's generic kernels gain too: Johnson fp32s 478 -> 485 frames/s with 2 (profiles/r05_ag_*)
  h->split = (is_reconet(arch) && !f32_storage(compute_dtype)) || compute_dtype == NST_DT_F32S ? 2 : 1;
  *out = h;
  return NST_OK;
}

void nst_destroy(nst_handle* h) {
  if (!h) return;
  DeviceGuard guard(h->device);
  for (int i = 0; i < NST_MAX_STREAM_SPLIT; ++i) {
    if (h->sub[i]) (void)hipStreamDestroy(h->sub[i]);
    if (h->join[i]) (void)hipEventDestroy(h->join[i]);
  }
  if (h->fork) (void)hipEventDestroy(h->fork);
  if (h->range_flag) (void)hipFree(h->range_flag);
  for (Layer& Ly : h->layers) {
    if (Ly.wpk) (void)hipFree(Ly.wpk);
    if (Ly.wpk_rev) (void)hipFree(Ly.wpk_rev);
    if (Ly.bias_rev) (void)hipFree(Ly.bias_rev);
    if (Ly.bias) (void)hipFree(Ly.bias);
    if (Ly.gamma) (void)hipFree(Ly.gamma);
    if (Ly.beta) (void)hipFree(Ly.beta);
    for (int pr = 0; pr < 8; ++pr) {
      if (Ly.wpk_fold[pr]) (void)hipFree(Ly.wpk_fold[pr]);
      if (Ly.bias_fold[pr]) (void)hipFree(Ly.bias_fold[pr]);
    }
  }
  delete h;
}

int nst_output_hw(const nst_handle* h, int in_h, int in_w, int* out_h, int* out_w) {
  if (!h || !out_h || !out_w || in_h <= 0 || in_w <= 0) { set_error("nst_output_hw: invalid arguments"); return NST_E_INVALID; }
  Plan P = make_plan(h, 1, in_h, in_w);
  if (!P.ok) { set_error(P.err); return NST_E_SHAPE; }
  *out_h = P.out_h;
  *out_w = P.out_w;
  return NST_OK;
}

int nst_input_exact(const nst_handle* h, int x_fmt, int preset, int* exact) {
  if (!h || !exact || (x_fmt != NST_IO_U8_NHWC && x_fmt != NST_IO_F32_NCHW) || preset < 0 || preset >= 8) {
    set_error("nst_input_exact: invalid arguments");
    return NST_E_INVALID;
  }
  if (f32_storage(h->dtype)) { *exact = 1; return NST_OK; }  // the operand keeps the encoded fp32 value
  *exact = 0;
  for (const Layer& Ly : h->layers)
    if (Ly.prepad) *exact = (x_fmt == NST_IO_U8_NHWC && Ly.wpk_fold[preset] != nullptr) ? 1 : 0;
  return NST_OK;
}

int nst_workspace_bytes(const nst_handle* h, int n, int in_h, int in_w, size_t* out) {
  if (!h || !out || n <= 0 || in_h <= 0 || in_w <= 0) { set_error("nst_workspace_bytes: invalid arguments"); return NST_E_INVALID; }
  Plan P = make_plan(h, n, in_h, in_w);
  if (!P.ok) { set_error(P.err); return NST_E_SHAPE; }
  // a split batch takes one workspace slice per sub-batch; enough for the unsplit run too (profiling, range check)
  const int k = std::min(h->split, n);
  size_t bytes = P.ws_bytes;
  if (k > 1) {
    const int nb = (n + k - 1) / k;
    const Plan Q = make_plan(h, nb, in_h, in_w);
    if (!Q.ok) { set_error(Q.err); return NST_E_SHAPE; }
    bytes = std::max(bytes, (size_t)((n + nb - 1) / nb) * align256(Q.ws_bytes));
  }
  *out = bytes;
  return NST_OK;
}

int nst_set_stream_split(nst_handle* h, int k) {
  if (!h || k < 1 || k > NST_MAX_STREAM_SPLIT) { set_error("nst_set_stream_split: invalid arguments"); return NST_E_INVALID; }
  h->split = k;
  return NST_OK;
}

}  // extern "C"

namespace {

// per-op device copies of what an op produced (nst_forward_capture)
struct Capture {
  void* const* act;
  void* const* res;
  void* const* stats;
};

int forward_impl(nst_handle* h, const void* x, int x_fmt, int n, int in_h, int in_w, int preset, void* y, int y_fmt,
                 void* workspace, size_t workspace_bytes, void* stream, const Capture* cap) {
  if (!h || !x || !y || n <= 0 || in_h <= 0 || in_w <= 0 ||
      (x_fmt != NST_IO_F32_NCHW && x_fmt != NST_IO_U8_NHWC) || (y_fmt != NST_IO_F32_NCHW && y_fmt != NST_IO_U8_NHWC)) {
    set_error("nst_forward: invalid arguments");
    return NST_E_INVALID;
  }
  PresetConsts pc;
  if (!preset_consts(preset, pc)) { set_error("nst_forward: unknown preset " + std::to_string(preset)); return NST_E_INVALID; }
  if (preset == NST_PRESET_NONE && (x_fmt == NST_IO_U8_NHWC || y_fmt == NST_IO_U8_NHWC)) {
    set_error("nst_forward: uint8 frames need an io_preset");
    return NST_E_INVALID;
  }
  Plan P = make_plan(h, n, in_h, in_w);
  if (!P.ok) { set_error(P.err); return NST_E_SHAPE; }
  if (y_fmt == NST_IO_U8_NHWC && (P.out_h != in_h || P.out_w != in_w)) {
    set_error("nst_forward: model output " + std::to_string(P.out_h) + "x" + std::to_string(P.out_w) +
              " differs from the input; request F32 output and use nst_decode_resize_u8");
    return NST_E_SHAPE;
  }
  if (!workspace || workspace_bytes < P.ws_bytes) {
    set_error("nst_forward: workspace too small (" + std::to_string(workspace_bytes) + " < " + std::to_string(P.ws_bytes) + ")");
    return NST_E_WORKSPACE;
  }
  DeviceGuard guard(h->device);
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  void* bufs[NBUF];
  for (int b = 0; b < NBUF; ++b) bufs[b] = ws + P.off_buf[b];
  float* partial = (float*)(ws + P.off_partial);
  std::vector<float2*> stats(h->layers.size());
  {
    size_t off = P.off_stats;
    for (size_t li = 0; li < h->layers.size(); ++li) {
      stats[li] = (float2*)(ws + off);
      off += align256((size_t)n * h->layers[li].coutp * 8);
    }
  }
  // run op i over the batch (every activation buffer holds its frames contiguously at the op's shape, every IN
  // table is [frame][channel])
  auto run_op = [&](size_t i) -> int {
    const Op& op = h->prog[i];
    const Layer& Ly = h->layers[op.layer];
    auto tab = [&](int layer) { return layer >= 0 ? stats[layer] : nullptr; };
    if (op.kind == OP_RESADD) {
      const int hw = P.oh[i] * P.ow[i];
      // element formats of y / r / out: all the handle's, all fp32 (NST_DT_F16M's first join), or fp32 -> fp16
      const int rdt = P.out_esz[i] == 4 ? NST_DT_F32 : h->dtype;
      hipError_t e = (P.in_esz[i] == 4 && P.res_esz[i] == 4 && P.out_esz[i] == 2)
                         ? launch_residual_f32_to_f16(bufs[op.src], tab(op.layer), bufs[op.r_buf], tab(op.r_norm),
                                                      op.r_relu, op.relu_out, bufs[op.dst], n, hw, Ly.coutp, st)
                         : launch_residual(rdt, bufs[op.src], tab(op.layer), bufs[op.r_buf], tab(op.r_norm), op.r_relu,
                                           op.relu_out, bufs[op.dst], n, hw, Ly.coutp, st);
      if (e != hipSuccess) { set_error(std::string("residual launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
      if (cap && cap->act && cap->act[i])
        NST_HIP_CHECK(hipMemcpyAsync(cap->act[i], bufs[op.dst], (size_t)n * hw * Ly.coutp * P.out_esz[i],
                                     hipMemcpyDeviceToDevice, st));
      return NST_OK;
    }
    const bool image_in = op.src == B_IMG, final_out = op.dst == B_OUT;
    const ConvKernelInfo* k = Ly.k_main;
    if (image_in && x_fmt == NST_IO_F32_NCHW) k = Ly.k_alt;
    if (final_out && y_fmt == NST_IO_F32_NCHW) k = Ly.k_alt;
    // uint8 frames through a first layer with this preset folded in: stage the raw bytes (exact operand)
    const bool fold = image_in && x_fmt == NST_IO_U8_NHWC && preset >= 0 && preset < 8 && Ly.wpk_fold[preset] != nullptr &&
                      (Ly.prepad || Ly.k_u8fold);
    if (fold && Ly.k_u8fold) k = Ly.k_u8fold;
    const bool prepad = Ly.prepad || (fold && Ly.k_u8fold);
    const int mode = fold && Ly.k_u8fold ? MODE_WS9 : Ly.mode;
    const int kdt = fold && Ly.k_u8fold ? NST_KDT_SW_O32 : Ly.kdt;
    ConvParams p;
    std::memset(&p, 0, sizeof(p));
    p.in = image_in ? x : bufs[op.src];
    p.hs = P.ih[i];
    p.ws = P.iw[i];
    p.cs = image_in ? 3 : Ly.cinp;
    p.axis_mode = Ly.d.axis_mode;
    p.pad = Ly.d.axis_mode == AX_ZINSERT ? 1 : Ly.d.pad;
    if (mode == MODE_PHASE || mode == MODE_WPHASE) {
      // source-grid halo of one pixel; nearest-x2 reflect(1) == clamp on the source grid,
      // ConvTranspose reads zeros past the edge
      p.axis_mode = Ly.d.axis_mode == AX_ZINSERT ? AX_ZERO : AX_CLAMP;
      p.pad = 1;
      p.ph_off[0] = Ly.d.axis_mode == AX_ZINSERT ? 1 : 0;
      p.ph_off[1] = 1;
    }
    p.pre = Ly.d.pre;
    p.in_norm = tab(op.in_norm);
    p.in_relu = op.in_norm >= 0 && op.res_buf < 0 ? 1 : 0;
    if (op.res_buf >= 0) {
      p.res_r = bufs[op.res_buf];
      p.res_rnorm = tab(op.r_norm);
      p.res_relu = op.relu_out;
    }
    p.res_out = op.res_out >= 0 ? bufs[op.res_out] : nullptr;
    for (int c = 0; c < 3; ++c) {
      p.enc_a[c] = pc.ea[c]; p.enc_b[c] = pc.eb[c]; p.enc_d[c] = pc.ed[c]; p.enc_perm[c] = pc.eperm[c];
      p.dec_p[c] = pc.dp[c]; p.dec_q[c] = pc.dq[c]; p.dec_r[c] = pc.dr[c]; p.dec_s[c] = pc.ds[c]; p.dec_perm[c] = pc.dperm[c];
    }
    if (image_in && x_fmt == NST_IO_F32_NCHW && preset == NST_PRESET_NONE) {
      for (int c = 0; c < 3; ++c) { p.enc_a[c] = 1.f; p.enc_b[c] = 0.f; p.enc_d[c] = 1.f; p.enc_perm[c] = c; }
    }
    p.enc_raw = fold ? 1 : 0;
    if (image_in && prepad) {
      // resolve padding + encode once into the workspace, then run the conv over it with an
      // identity coordinate map (pad 0, no reflection)
      const int hp = P.ch[i] + Ly.d.ks - 1, wp = P.cw[i] + Ly.d.ks - 1;
      void* pre = ws + P.off_pre;
      // the staged operand's format: bf16, or fp16 (the fp16 mode and NST_DT_F16M's split-weight first layer)
      const int pdt = (kdt == NST_DT_F16 || kdt == NST_KDT_SW_O32 || kdt == NST_KDT_SW_O16) ? NST_DT_F16 : NST_DT_BF16;
      hipError_t e = launch_prepad_encode(pdt, p, x_fmt == NST_IO_U8_NHWC ? IN_U8_NHWC : IN_F32_NCHW, n, hp, wp, pre, st);
      if (e != hipSuccess) { set_error(std::string("prepad launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
      p.in = pre;
      p.hs = hp;
      p.ws = wp;
      p.cs = 4;
      p.axis_mode = AX_ZERO;
      p.pad = 0;
      p.pre = 0;
    }
    p.dec_tanh = (is_reconet(h->arch) && final_out) ? 1 : 0;
    p.wpk = fold ? Ly.wpk_fold[preset] : Ly.wpk;
    p.bias = fold ? Ly.bias_fold[preset] : Ly.bias;
    if (mode == MODE_XSHIFT && final_out && y_fmt == NST_IO_U8_NHWC && pc.dperm[0] == 2) {
      p.wpk = Ly.wpk_rev;  // decode channel c from model channel 2-c (caffe_bgr)
      p.bias = Ly.bias_rev;
    }
    p.hconv = P.ch[i];
    p.wconv = P.cw[i];
    p.oh = P.oh[i];
    p.ow = P.ow[i];
    p.crop_y = (P.ch[i] - P.oh[i]) / 2;
    p.crop_x = (P.cw[i] - P.ow[i]) / 2;
    p.out = final_out ? y : bufs[op.dst];
    p.cout_real = Ly.d.cout;
    p.cout_stride = Ly.coutp;
    tile_grid(*k, p.hs, p.ws, p.oh, p.ow, &p.tiles_x, &p.tiles_y);
    p.n_cblk = Ly.coutp / k->bn;
    if (p.res_out != nullptr && p.res_r == nullptr &&
        ((mode != MODE_WSTAT && mode != MODE_STD) || p.in_norm == nullptr || Ly.d.stride != 1)) {
      set_error("conv " + Ly.d.conv + ": only the trunk kernels (weight-stationary / generic stride-1) write their "
                "normalised input");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WSTAT && p.res_r != nullptr && (p.in_norm == nullptr || p.res_out == nullptr || p.res_relu)) {
      set_error("conv " + Ly.d.conv + ": weight-stationary kernel joins IN(y) + r into a residual-stream buffer");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WS2 && k->cinp_k && (p.axis_mode != AX_REFLECT)) {
      set_error("conv " + Ly.d.conv + ": the narrow-input down-conv is built for reflection padding");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WS2 && (p.in_norm == nullptr || p.res_r != nullptr || p.crop_x || p.crop_y)) {
      set_error("conv " + Ly.d.conv + ": weight-stationary down-conv reads a normalized activation, uncropped");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WS9 && (!prepad || p.in_norm != nullptr || p.res_r != nullptr || p.crop_x || p.crop_y || final_out)) {
      set_error("conv " + Ly.d.conv + ": weight-stationary 9x9 kernel reads the pre-padded frame, uncropped");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WS1S && (p.res_r != nullptr || p.res_out != nullptr || p.crop_x || p.crop_y)) {
      set_error("conv " + Ly.d.conv + ": split-operand trunk kernel runs plain convs, uncropped");
      return NST_E_SHAPE;
    }
    if ((mode == MODE_WPHASE || mode == MODE_WSTAT || mode == MODE_WS2 || mode == MODE_WS9 ||
         mode == MODE_WS1S) && p.cout_stride != k->bn) {
      set_error("conv " + Ly.d.conv + ": weight-stationary kernels store whole pixels of bn channels");
      return NST_E_SHAPE;
    }
    if (mode == MODE_WPHASE && p.res_r != nullptr &&
        (p.in_norm == nullptr || p.res_out != nullptr || p.res_relu || p.res_rnorm != nullptr)) {
      set_error("conv " + Ly.d.conv + ": weight-stationary phase kernel joins IN(y) + r without writing the stream");
      return NST_E_SHAPE;
    }
    if (k->persistent && p.n_cblk != 1) { set_error("conv " + Ly.d.conv + ": persistent kernel needs one channel block"); return NST_E_SHAPE; }
    p.partial = final_out ? nullptr : partial;
    dim3 grid(p.tiles_x * p.tiles_y, n * p.n_cblk);
    nst_handle::Rec rec{op.layer, nullptr, nullptr};
    if (h->profiling) {
      NST_HIP_CHECK(hipEventCreate(&rec.a));
      NST_HIP_CHECK(hipEventCreate(&rec.b));
      NST_HIP_CHECK(hipEventRecord(rec.a, st));
    }
    k->launch(p, grid, st);
    hipError_t e = hipGetLastError();
    if (h->profiling && e == hipSuccess) {
      NST_HIP_CHECK(hipEventRecord(rec.b, st));
      h->recs.push_back(rec);
    }
    if (e != hipSuccess) { set_error("conv " + Ly.d.conv + " launch: " + hipGetErrorString(e)); return NST_E_HIP; }
    if (!final_out) {
      e = launch_in_finalize(partial, n, p.tiles_x * p.tiles_y * k->part_rows, Ly.coutp, (double)p.hconv * (double)p.wconv,
                             Ly.gamma, Ly.beta, Ly.eps, Ly.frn, tab(op.layer), ws + P.off_seg, st);
      if (e == hipSuccess && h->range_flag)
        e = launch_check_finite((const float*)tab(op.layer), (size_t)n * Ly.coutp * 2, h->range_flag, st);
      if (e != hipSuccess) { set_error(std::string("finalize launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
    }
    if (cap && !final_out) {
      if (cap->act && cap->act[i])
        NST_HIP_CHECK(hipMemcpyAsync(cap->act[i], bufs[op.dst], (size_t)n * P.oh[i] * P.ow[i] * Ly.coutp * P.out_esz[i],
                                     hipMemcpyDeviceToDevice, st));
      if (cap->res && cap->res[i] && op.res_out >= 0)
        NST_HIP_CHECK(hipMemcpyAsync(cap->res[i], bufs[op.res_out], (size_t)n * P.ih[i] * P.iw[i] * Ly.cinp * P.res_esz[i],
                                     hipMemcpyDeviceToDevice, st));
      if (cap->stats && cap->stats[i])
        NST_HIP_CHECK(hipMemcpyAsync(cap->stats[i], stats[op.layer], (size_t)n * Ly.coutp * 8, hipMemcpyDeviceToDevice, st));
    }
    return NST_OK;
  };
  if (h->range_flag) NST_HIP_CHECK(hipMemsetAsync(h->range_flag, 0, sizeof(int), st));
  for (size_t i = 0; i < h->prog.size(); ++i) {
    const int rc = run_op(i);
    if (rc != NST_OK) return rc;
  }
  if (h->range_flag) {  // synchronous: the caller asked for the verdict of this forward
    if (y_fmt == NST_IO_F32_NCHW)
      NST_HIP_CHECK(launch_check_finite((const float*)y, (size_t)n * 3 * P.out_h * P.out_w, h->range_flag, st));
    int bad = 0;
    NST_HIP_CHECK(hipMemcpyAsync(&bad, h->range_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    NST_HIP_CHECK(hipStreamSynchronize(st));
    if (bad) {
      set_error("nst_forward: a non-finite InstanceNorm statistic or output value (an activation left the range of "
                "the compute dtype: fp16 / split-fp16 operands hold |v| <= 65504)");
      return NST_E_RANGE;
    }
  }
  return NST_OK;
}

}  // namespace

extern "C" {

int nst_forward(nst_handle* h, const void* x, int x_fmt, int n, int in_h, int in_w, int preset, void* y,
                int y_fmt, void* workspace, size_t workspace_bytes, void* stream) {
  // one stream: profiling (per-layer event pairs) and the range check (a synchronous verdict) keep the batch whole
  const int k = (!h || h->profiling || h->range_flag || n <= 1) ? 1 : std::min(h->split, n);
  if (k == 1 || !x || !y || in_h <= 0 || in_w <= 0 || (x_fmt != NST_IO_F32_NCHW && x_fmt != NST_IO_U8_NHWC) ||
      (y_fmt != NST_IO_F32_NCHW && y_fmt != NST_IO_U8_NHWC))
    return forward_impl(h, x, x_fmt, n, in_h, in_w, preset, y, y_fmt, workspace, workspace_bytes, stream, nullptr);
  const int nb = (n + k - 1) / k, parts = (n + nb - 1) / nb;
  const Plan Q = make_plan(h, nb, in_h, in_w);
  if (!Q.ok) { set_error(Q.err); return NST_E_SHAPE; }
  const size_t per = align256(Q.ws_bytes);
  // the size nst_workspace_bytes reports (the split slices, or the whole batch's plan if larger): one contract
  const Plan Pn = make_plan(h, n, in_h, in_w);
  if (!Pn.ok) { set_error(Pn.err); return NST_E_SHAPE; }
  const size_t need = std::max(Pn.ws_bytes, per * parts);
  if (!workspace || workspace_bytes < need) {
    set_error("nst_forward: workspace too small (" + std::to_string(workspace_bytes) + " < " + std::to_string(need) + ")");
    return NST_E_WORKSPACE;
  }
  DeviceGuard guard(h->device);
  if (!h->fork) NST_HIP_CHECK(hipEventCreateWithFlags(&h->fork, hipEventDisableTiming));
  for (int i = 0; i < parts; ++i) {
    if (!h->sub[i]) NST_HIP_CHECK(hipStreamCreateWithFlags(&h->sub[i], hipStreamNonBlocking));
    if (!h->join[i]) NST_HIP_CHECK(hipEventCreateWithFlags(&h->join[i], hipEventDisableTiming));
  }
  const hipStream_t st = (hipStream_t)stream;
  const size_t fx = x_fmt == NST_IO_U8_NHWC ? (size_t)in_h * in_w * 3 : (size_t)3 * in_h * in_w * 4;
  const size_t fy = y_fmt == NST_IO_U8_NHWC ? (size_t)Q.out_h * Q.out_w * 3 : (size_t)3 * Q.out_h * Q.out_w * 4;
  NST_HIP_CHECK(hipEventRecord(h->fork, st));
  int rc = NST_OK;
  for (int i = 0; i < parts; ++i) {
    NST_HIP_CHECK(hipStreamWaitEvent(h->sub[i], h->fork, 0));
    const int f0 = i * nb, m = std::min(nb, n - f0);
    if (rc == NST_OK)
      rc = forward_impl(h, (const char*)x + f0 * fx, x_fmt, m, in_h, in_w, preset, (char*)y + f0 * fy, y_fmt,
                        (char*)workspace + i * per, per, h->sub[i], nullptr);
    // joined even after a failed launch: nothing queued on a sub-stream outlives the caller's stream order
    NST_HIP_CHECK(hipEventRecord(h->join[i], h->sub[i]));
    NST_HIP_CHECK(hipStreamWaitEvent(st, h->join[i], 0));
  }
  return rc;
}

int nst_forward_capture(nst_handle* h, const void* x, int x_fmt, int n, int in_h, int in_w, int preset, void* y,
                        int y_fmt, void* workspace, size_t workspace_bytes, void* const* act, void* const* res,
                        void* const* stats, void* stream) {
  const Capture cap{act, res, stats};
  return forward_impl(h, x, x_fmt, n, in_h, in_w, preset, y, y_fmt, workspace, workspace_bytes, stream, &cap);
}

int nst_set_range_check(nst_handle* h, int enable) {
  if (!h) { set_error("nst_set_range_check: null handle"); return NST_E_INVALID; }
  DeviceGuard guard(h->device);
  if (enable && !h->range_flag) {
    if (hipMalloc(&h->range_flag, sizeof(int)) != hipSuccess) {
      h->range_flag = nullptr;
      set_error("nst_set_range_check: hipMalloc failed");
      return NST_E_HIP;
    }
  } else if (!enable && h->range_flag) {
    (void)hipFree(h->range_flag);
    h->range_flag = nullptr;
  }
  return NST_OK;
}

int nst_num_ops(const nst_handle* h) { return h ? (int)h->prog.size() : 0; }

int nst_op_describe(const nst_handle* h, int n, int in_h, int in_w, int op_index, nst_op_desc* out) {
  if (!h || !out || n <= 0 || in_h <= 0 || in_w <= 0 || op_index < 0 || op_index >= (int)h->prog.size()) {
    set_error("nst_op_describe: invalid arguments");
    return NST_E_INVALID;
  }
  Plan P = make_plan(h, n, in_h, in_w);
  if (!P.ok) { set_error(P.err); return NST_E_SHAPE; }
  const Op& op = h->prog[op_index];
  const Layer& Ly = h->layers[op.layer];
  std::memset(out, 0, sizeof(*out));
  out->kind = op.kind;
  out->layer = op.layer;
  out->src = op.src;
  out->dst = op.dst;
  if (op.kind == OP_CONV) {
    out->in_norm = op.in_norm;
    out->in_relu = op.in_norm >= 0 && op.res_buf < 0 ? 1 : 0;
    out->res_buf = op.res_buf;
    out->res_norm = op.res_buf >= 0 ? op.r_norm : -1;
    out->res_out = op.res_out;
    out->relu_out = op.res_buf >= 0 ? op.relu_out : 0;
  } else {
    out->in_norm = op.layer;  // out = IN_layer(src) + r
    out->in_relu = 0;
    out->res_buf = op.r_buf;
    out->res_norm = op.r_norm;
    out->res_out = -1;
    out->relu_out = op.relu_out;
  }
  out->in_h = P.ih[op_index];
  out->in_w = P.iw[op_index];
  out->out_h = P.oh[op_index];
  out->out_w = P.ow[op_index];
  out->conv_h = P.ch[op_index];
  out->conv_w = P.cw[op_index];
  out->cin_stride = op.src == B_IMG ? 3 : Ly.cinp;
  out->cout_stride = Ly.coutp;
  out->kernel_mode = Ly.mode;
  out->elem_bytes = P.out_esz[op_index];
  out->in_elem_bytes = P.in_esz[op_index];
  out->res_elem_bytes = P.res_esz[op_index];
  out->kernel_dtype = op.kind == OP_CONV ? Ly.kdt : h->dtype;
  return NST_OK;
}

int nst_profile_begin(nst_handle* h) {
  if (!h) { set_error("nst_profile_begin: null handle"); return NST_E_INVALID; }
  h->profiling = true;
  return NST_OK;
}

int nst_profile_end(nst_handle* h, int n_layers, float* total_ms, int* launches) {
  if (!h || n_layers < 0 || (n_layers > 0 && (!total_ms || !launches))) {
    set_error("nst_profile_end: invalid arguments");
    return NST_E_INVALID;
  }
  DeviceGuard guard(h->device);
  for (int i = 0; i < n_layers; ++i) { total_ms[i] = 0.f; launches[i] = 0; }
  int rc = NST_OK;
  for (auto& r : h->recs) {
    float ms = 0.f;
    hipError_t e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess && rc == NST_OK) {
      set_error(std::string("hipEventElapsedTime: ") + hipGetErrorString(e));
      rc = NST_E_HIP;
    }
    if (r.layer < n_layers) { total_ms[r.layer] += ms; launches[r.layer] += 1; }
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  h->recs.clear();
  h->profiling = false;
  return rc;
}

int nst_num_layers(const nst_handle* h) { return h ? (int)h->layers.size() : 0; }

const char* nst_layer_name(const nst_handle* h, int layer) {
  if (!h || layer < 0 || layer >= (int)h->layers.size()) return "";
  return h->layers[layer].d.conv.c_str();
}

int nst_decode_resize_u8(const float* y, int n, int h, int w, int preset, uint8_t* out, int out_h, int out_w,
                         void* stream) {
  PresetConsts pc;
  if (!y || !out || n <= 0 || h <= 0 || w <= 0 || out_h <= 0 || out_w <= 0 || !preset_consts(preset, pc)) {
    set_error("nst_decode_resize_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_decode_resize_u8(y, n, h, w, pc.dp, pc.dq, pc.dr, pc.ds, pc.dperm, out, out_h, out_w,
                                         (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("decode_resize launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_blend_models_u8(const float* const* ys, const int* presets, const float* weights, int m, int n, int h,
                        int w, uint8_t* out, int out_h, int out_w, void* stream) {
  if (!ys || !presets || !weights || !out || m <= 0 || m > NST_MAX_MODELS || n <= 0 || h <= 0 || w <= 0 ||
      out_h <= 0 || out_w <= 0) {
    set_error("nst_blend_models_u8: invalid arguments");
    return NST_E_INVALID;
  }
  float dp[NST_MAX_MODELS][3], dq[NST_MAX_MODELS][3], dr[NST_MAX_MODELS][3], ds[NST_MAX_MODELS][3];
  int perm[NST_MAX_MODELS][3];
  for (int k = 0; k < m; ++k) {
    PresetConsts pc;
    if (!ys[k] || !preset_consts(presets[k], pc)) {
      set_error("nst_blend_models_u8: bad model output or preset for slot " + std::to_string(k));
      return NST_E_INVALID;
    }
    for (int c = 0; c < 3; ++c) {
      dp[k][c] = pc.dp[c]; dq[k][c] = pc.dq[c]; dr[k][c] = pc.dr[c]; ds[k][c] = pc.ds[c]; perm[k][c] = pc.dperm[c];
    }
  }
  hipError_t e = launch_blend_models_u8(ys, dp, dq, dr, ds, perm, weights, m, n, h, w, out, out_h, out_w,
                                        (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("blend_models launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_lab_create(const uint8_t* rgb2lab, const uint8_t* lab2rgb, int device, nst_lab** out) {
  if (!rgb2lab || !lab2rgb || !out) { set_error("nst_lab_create: invalid arguments"); return NST_E_INVALID; }
  DeviceGuard guard(device);
  auto* l = new nst_lab();
  l->device = device;
  // widen the 3-byte entries to one dword each (a lookup is one aligned 4-byte load on the device)
  const size_t entries = (size_t)1 << 24;
  std::vector<uint32_t> wide(entries);
  auto widen = [&](const uint8_t* t) {
    for (size_t i = 0; i < entries; ++i)
      wide[i] = (uint32_t)t[3 * i] | ((uint32_t)t[3 * i + 1] << 8) | ((uint32_t)t[3 * i + 2] << 16);
  };
  widen(rgb2lab);
  int rc = upload(wide.data(), entries * 4, (void**)&l->rgb2lab);
  if (rc == NST_OK) {
    widen(lab2rgb);
    rc = upload(wide.data(), entries * 4, (void**)&l->lab2rgb);
  }
  if (rc != NST_OK) { nst_lab_destroy(l); return rc; }
  *out = l;
  return NST_OK;
}

void nst_lab_destroy(nst_lab* l) {
  if (!l) return;
  DeviceGuard guard(l->device);
  if (l->rgb2lab) (void)hipFree(l->rgb2lab);
  if (l->lab2rgb) (void)hipFree(l->lab2rgb);
  delete l;
}

int nst_lab_ema_u8(const nst_lab* lab, const uint8_t* rgb_in, uint8_t* rgb_out, int n, int h, int w,
                   int smooth_lightness, float alpha, float one_minus_alpha, int smooth_chroma, float chroma_alpha,
                   float one_minus_chroma_alpha, float* state, int first, void* stream) {
  if (!lab || !rgb_in || !rgb_out || !state || n <= 0 || h <= 0 || w <= 0) {
    set_error("nst_lab_ema_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_lab_ema(lab->rgb2lab, lab->lab2rgb, rgb_in, rgb_out, n, h * w, smooth_lightness, alpha,
                                one_minus_alpha, smooth_chroma, chroma_alpha, one_minus_chroma_alpha, state, first,
                                (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("lab_ema launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_lab_planes_u8(const nst_lab* lab, const uint8_t* rgb_in, int n, int h, int w, int smooth_lightness,
                      int smooth_chroma, uint8_t* planes, void* stream) {
  const int sl = smooth_lightness ? 1 : 0, sc = smooth_chroma ? 1 : 0;
  if (!lab || !rgb_in || !planes || n <= 0 || h <= 0 || w <= 0 || !(sl || sc)) {
    set_error("nst_lab_planes_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_lab_planes(lab->rgb2lab, rgb_in, planes, n, h * w, sl, sc, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("lab_planes launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_lab_ema_planes(const uint8_t* planes_in, uint8_t* planes_out, int n, int h, int w, int smooth_lightness,
                       float alpha, float one_minus_alpha, int smooth_chroma, float chroma_alpha,
                       float one_minus_chroma_alpha, float* state, int first, void* stream) {
  const int sl = smooth_lightness ? 1 : 0, sc = smooth_chroma ? 1 : 0;
  if (!planes_in || !planes_out || !state || n <= 0 || h <= 0 || w <= 0 || !(sl || sc)) {
    set_error("nst_lab_ema_planes: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_lab_ema_planes(planes_in, planes_out, n, h * w, sl, alpha, one_minus_alpha, sc, chroma_alpha,
                                       one_minus_chroma_alpha, state, first, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("lab_ema_planes launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_lab_merge_u8(const nst_lab* lab, const uint8_t* rgb_in, const uint8_t* planes, int n, int h, int w,
                     int smooth_lightness, int smooth_chroma, uint8_t* rgb_out, void* stream) {
  const int sl = smooth_lightness ? 1 : 0, sc = smooth_chroma ? 1 : 0;
  if (!lab || !rgb_in || !planes || !rgb_out || n <= 0 || h <= 0 || w <= 0 || !(sl || sc)) {
    set_error("nst_lab_merge_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_lab_merge(lab->rgb2lab, lab->lab2rgb, rgb_in, planes, rgb_out, n, h * w, sl, sc,
                                  (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("lab_merge launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_blend_models_lab_u8(const nst_lab* lab, const uint8_t* const* frames, int m, const float* weights_rest,
                            int n_rest, float w_l, float w_ab, int n, int h, int w, uint8_t* out, void* stream) {
  if (!lab || !frames || !out || m < 1 || m > NST_MAX_MODELS || n_rest < 0 || (n_rest > 0 && !weights_rest) ||
      n <= 0 || h <= 0 || w <= 0) {
    set_error("nst_blend_models_lab_u8: invalid arguments");
    return NST_E_INVALID;
  }
  for (int i = 0; i < m; ++i)
    if (!frames[i]) { set_error("nst_blend_models_lab_u8: null frame pointer"); return NST_E_INVALID; }
  const int nrest = std::min(m - 1, n_rest);  // zip(outputs[1:], weights_rest)
  hipError_t e = launch_lab_blend(lab->rgb2lab, lab->lab2rgb, frames, weights_rest, nrest, w_l, w_ab,
                                  (size_t)n * h * w, out, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("lab_blend launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_mask_feather(const uint8_t* mask, int n, int h, int w, float sigma, float* scratch, float* alpha,
                     void* stream) {
  if (!mask || !scratch || !alpha || n <= 0 || h <= 0 || w <= 0 || !(sigma > 0.f)) {
    set_error("nst_mask_feather: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_mask_feather(mask, n, h, w, sigma, scratch, alpha, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("mask_feather launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_blend_u8(const uint8_t* styled, const uint8_t* orig, const float* mask, int composite_mode, float blend,
                 float one_minus_blend, uint8_t* out, int n, int h, int w, void* stream) {
  if (!styled || !orig || !out || n <= 0 || h <= 0 || w <= 0 || composite_mode < 0 || composite_mode > 1) {
    set_error("nst_blend_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_blend(styled, orig, mask, composite_mode, blend, one_minus_blend, out, n, h * w,
                              (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("blend launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_blend_mask8_u8(const uint8_t* styled, const uint8_t* orig, const uint8_t* mask, int composite_mode, float blend,
                       float one_minus_blend, uint8_t* out, int n, int h, int w, void* stream) {
  if (!styled || !orig || !mask || !out || n <= 0 || h <= 0 || w <= 0 || composite_mode < 0 || composite_mode > 1) {
    set_error("nst_blend_mask8_u8: invalid arguments");
    return NST_E_INVALID;
  }
  hipError_t e = launch_blend(styled, orig, nullptr, composite_mode, blend, one_minus_blend, out, n, h * w,
                              (hipStream_t)stream, mask);
  if (e != hipSuccess) { set_error(std::string("blend launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

int nst_gram_workspace_bytes(int n, int c, int hw, size_t* out) {
  if (n <= 0 || c <= 0 || hw <= 0 || !out) { set_error("nst_gram_workspace_bytes: invalid arguments"); return NST_E_INVALID; }
  *out = gram_workspace_bytes(n, c, hw);
  return NST_OK;
}

int nst_gram(const void* F, int dtype, int layout, int n, int c, int hw, float* G, void* workspace,
             size_t workspace_bytes, void* stream) {
  if (!F || !G || n <= 0 || c <= 0 || hw <= 0 || (dtype != NST_DT_F32 && dtype != NST_DT_BF16) ||
      (layout != NST_GRAM_CHW && layout != NST_GRAM_HWC)) {
    set_error("nst_gram: invalid arguments");
    return NST_E_INVALID;
  }
  const int vec = dtype == NST_DT_BF16 ? 8 : 4;
  const int minor = layout == NST_GRAM_CHW ? hw : c;  // the contiguous axis of F's 16-byte loads
  if (minor % vec != 0 || ((uintptr_t)F % 16) != 0) {
    set_error("nst_gram: the contiguous axis (" + std::string(layout == NST_GRAM_CHW ? "h*w" : "c") +
              ") must be a multiple of " + std::to_string(vec) + " and F 16-byte aligned");
    return NST_E_SHAPE;
  }
  const size_t need = gram_workspace_bytes(n, c, hw);
  if (need > 0 && (!workspace || workspace_bytes < need)) {
    set_error("nst_gram: workspace too small (" + std::to_string(workspace_bytes) + " < " + std::to_string(need) + ")");
    return NST_E_WORKSPACE;
  }
  hipError_t e = launch_gram(F, dtype, layout == NST_GRAM_HWC, n, c, hw, G, workspace, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(std::string("gram launch: ") + hipGetErrorString(e)); return NST_E_HIP; }
  return NST_OK;
}

}  // extern "C"
