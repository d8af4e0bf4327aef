// conv_tab32.h — the generic conv_kernel instantiations of the 4-byte activation formats: fp32 (the
// parity mode, conv_f32.hip) and the split-fp16 mode (NST_DT_F32S, conv_f32s.hip).  Smaller tiles
// than the 16-bit tables: an fp32 LDS entry is twice as wide.
#pragma once
#include "conv_impl.h"

// Tile shapes (TH, TW, WM, WN) of the Johnson/NST layers; overridable at build time for tile sweeps.
// Trunk 8x16 tiles on 8 waves (2x4) and 8-row up-conv / output tiles: r03 sweep of the split-fp16 mode
// (tools/mode_profile.py), 221 -> 297 frames/s over the 4x16-tile shapes the fp32 mode started with
// r04: the down-convs and the trunk on waves of 16 output channels over the whole tile (WM = 1; the Gatys VGG
// finding): split-fp16 conv2 2.37 -> 1.01 ms, conv3 1.15 -> 0.72, trunk 1.05 -> 1.02 per batch of 8
#ifndef NST_T32_C1
#define NST_T32_C1 8, 32, 4, 1
#endif
#ifndef NST_T32_C2
#define NST_T32_C2 4, 16, 1, 4
#endif
#ifndef NST_T32_C3
#define NST_T32_C3 8, 16, 1, 8
#endif
#ifndef NST_T32_RES
#define NST_T32_RES 8, 16, 1, 8
#endif
#ifndef NST_T32_D1
#define NST_T32_D1 8, 16, 1, 4
#endif
#ifndef NST_T32_D2
#define NST_T32_D2 8, 16, 1, 4
#endif
#ifndef NST_T32_OUT
#define NST_T32_OUT 8, 32, 4, 1
#endif
// the 3-channel output conv as x-shift rows (5 shifts x 3 channels per 16-row MFMA block instead of 3 of 16 rows):
// fp32 parity mode 162.5 -> 186.7 frames/s (output conv 11.9 -> 5.5 ms per batch of 8), split-fp16 297.5 -> 312.2
// (6.1 -> 4.8 ms); 8-row or 8-wave x-shift tiles exceed the LDS budget for 4-byte entries
#ifndef NST_T32_XS
#define NST_T32_XS 4, 80, 4, 1
#endif

namespace nst {
template <typename F>
const ConvKernelInfo* conv_table_32(int* count) {
#define E(...) ConvInst<__VA_ARGS__>::info()
  constexpr int SD = MODE_STD, PH = MODE_PHASE, XS = MODE_XSHIFT;
  (void)XS;
  static const ConvKernelInfo table[] = {
      //  T  MODE KS S CINP BN TH TW WM WN  IN           OUT
      E(F, SD, 9, 1, 4, 32, NST_T32_C1, IN_U8_NHWC, OUT_ACT),
      E(F, SD, 9, 1, 4, 32, NST_T32_C1, IN_F32_NCHW, OUT_ACT),
      E(F, SD, 3, 2, 32, 64, NST_T32_C2, IN_ACT, OUT_ACT),
      E(F, SD, 3, 2, 64, 128, NST_T32_C3, IN_ACT, OUT_ACT),
      E(F, SD, 3, 1, 128, 128, NST_T32_RES, IN_ACT, OUT_ACT),
      E(F, PH, 3, 1, 128, 64, NST_T32_D1, IN_ACT, OUT_ACT),
      E(F, PH, 3, 1, 64, 32, NST_T32_D2, IN_ACT, OUT_ACT),
      E(F, SD, 9, 1, 32, 16, NST_T32_OUT, IN_ACT, OUT_U8_NHWC),
      E(F, SD, 9, 1, 32, 16, NST_T32_OUT, IN_ACT, OUT_F32_NCHW),
#ifdef NST_T32_XS
      E(F, XS, 9, 1, 32, 16, NST_T32_XS, IN_ACT, OUT_U8_NHWC),   // output conv, 5 x-shifts x 3 channels per MFMA row block
      E(F, XS, 9, 1, 32, 16, NST_T32_XS, IN_ACT, OUT_F32_NCHW),
#endif
      // ReCoNet (48/96/192 channels: multiples of 16, no padding in fp32)
      E(F, SD, 9, 1, 4, 48, 8, 32, 4, 1, IN_U8_NHWC, OUT_ACT),
      E(F, SD, 9, 1, 4, 48, 8, 32, 4, 1, IN_F32_NCHW, OUT_ACT),
      E(F, SD, 3, 2, 48, 96, 4, 16, 2, 2, IN_ACT, OUT_ACT),
      E(F, SD, 3, 2, 96, 192, 2, 16, 2, 2, IN_ACT, OUT_ACT),
      E(F, SD, 3, 1, 192, 192, 4, 16, 2, 2, IN_ACT, OUT_ACT),
      E(F, PH, 3, 1, 192, 96, 2, 16, 1, 4, IN_ACT, OUT_ACT),
      E(F, PH, 3, 1, 96, 48, 4, 16, 1, 4, IN_ACT, OUT_ACT),
      // consumers of the residual stream (residual join fused into the fill)
      E(F, SD, 3, 1, 128, 128, NST_T32_RES, IN_ACT, OUT_ACT, VAR_RES),
      E(F, PH, 3, 1, 128, 64, NST_T32_D1, IN_ACT, OUT_ACT, VAR_RES),
      E(F, SD, 3, 1, 192, 192, 4, 16, 2, 2, IN_ACT, OUT_ACT, VAR_RES),
      E(F, PH, 3, 1, 192, 96, 2, 16, 1, 4, IN_ACT, OUT_ACT, VAR_RES),
      E(F, SD, 9, 1, 48, 16, 2, 32, 4, 1, IN_ACT, OUT_U8_NHWC),
      E(F, SD, 9, 1, 48, 16, 2, 32, 4, 1, IN_ACT, OUT_F32_NCHW),
  };
#undef E
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
}  // namespace nst
