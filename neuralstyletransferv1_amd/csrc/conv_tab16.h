// conv_tab16.h — the generic conv_kernel instantiations of the 16-bit modes (bf16: conv_bf16.hip,
// fp16: conv_f16.hip; one table per translation unit).  Tile choices per layer shape: see DESIGN.md
// "Kernels".
#pragma once
#include "conv_impl.h"

// Tile shapes (TH, TW, WM, WN) of the Johnson/NST layers; overridable at build time for tile sweeps
// tile shapes (TH, TW, WM, WN) of the generic instantiations
#define NST_C1_TILE 8, 32, 4, 1
#define NST_C2_TILE 4, 16, 2, 2
#define NST_C3_TILE 4, 16, 2, 2
#define NST_D1_TILE 4, 16, 1, 4
#define NST_D2_TILE 4, 16, 1, 4
#ifndef NST_R_UP1_TILE
#define NST_R_UP1_TILE 8, 16, 1, 4  // ReCoNet 192 -> 96 up-conv (phases): 8 x 16 tiles 1 % ahead of 4 x 32 after the keep-live change (r04); 2.24 -> 1.61 ms per batch of 8 vs 2 x 16 (r03)
#endif
#ifndef NST_R_TRUNK_TILE
#define NST_R_TRUNK_TILE 16, 16, 2, 4  // ReCoNet 192-channel trunk: 8 waves (2 x 4: 8 x 3 accumulator sub-tiles each,
                                       // two waves per SIMD): 0.968 -> 0.735 ms per conv and batch of 8 (r04 sweep;
                                       // 2 x 2 waves 0.968, 4 x 2 0.792, 4 x 1 0.978; r03: 8 x 16 tiles 1.12)
#endif
#ifndef NST_R_TRUNK_RES_TILE
#define NST_R_TRUNK_RES_TILE NST_R_TRUNK_TILE  // ... its joined form (the residual join in the fill)
#endif
#ifndef NST_R_DOWN2_96_TILE
#define NST_R_DOWN2_96_TILE NST_R_DOWN2_TILE  // ... with its input unpadded (96 channels)
#endif
#ifndef NST_R_C1_TILE
#define NST_R_C1_TILE 16, 16, 4, 2  // ReCoNet 9x9 first layer (48 -> 64 channels): 8 waves on 16 x 16 tiles, 1.064 ->
                                    // 0.93 ms (r04 sweeps: 16 x 32 1.008, 8 x 64 1.345)
#endif
#ifndef NST_R_DOWN2_TILE
#define NST_R_DOWN2_TILE 8, 16, 2, 4  // ReCoNet 96 -> 192 stride-2 conv: 8 waves, 1.248 -> 0.774 ms (r04; r03: 4 x 32 tiles
                                      // 1.27 -> 1.01 ms, but the fp16 ReCoNet golden then had one value 3 LSB off)
#endif

namespace nst {
#define E(...) ConvInst<__VA_ARGS__>::info()
template <typename B>
const ConvKernelInfo* conv_table_16(int* count) {
  constexpr int SD = MODE_STD, PH = MODE_PHASE, XS = MODE_XSHIFT;
  static const ConvKernelInfo table[] = {
      //  T  MODE KS S CINP BN TH TW WM WN  IN           OUT
      E(B, SD, 9, 1, 4, 32, NST_C1_TILE, IN_ACT, OUT_ACT),        // Johnson/NST conv1 over the pre-padded encoded input (conv_prep.hip)
      E(B, SD, 9, 1, 4, 32, NST_C1_TILE, IN_U8_NHWC, OUT_ACT),    // Johnson/NST conv1 (frames)
      E(B, SD, 9, 1, 4, 32, NST_C1_TILE, IN_F32_NCHW, OUT_ACT),   // Johnson/NST conv1 (tensor API)
      E(B, SD, 3, 2, 32, 64, NST_C2_TILE, IN_ACT, OUT_ACT),       // conv2 / down2
      E(B, SD, 3, 2, 64, 128, NST_C3_TILE, IN_ACT, OUT_ACT),      // conv3 / down3 / ReCoNet enc1
      E(B, SD, 3, 1, 128, 128, 8, 16, 2, 2, IN_ACT, OUT_ACT),     // residual trunk (register-streamed; see conv_bf16_wl.hip)
      E(B, PH, 3, 1, 128, 64, NST_D1_TILE, IN_ACT, OUT_ACT),      // deconv1 / up1 / ReCoNet dec2 (phases)
      E(B, PH, 3, 1, 64, 32, NST_D2_TILE, IN_ACT, OUT_ACT),       // deconv2 / up2 (phases)
      E(B, XS, 9, 1, 32, 16, 8, 80, 8, 1, IN_ACT, OUT_U8_NHWC),   // deconv3 / final (frames, x-shift, 8 waves)
      E(B, XS, 9, 1, 32, 16, 8, 80, 8, 1, IN_ACT, OUT_F32_NCHW),  // deconv3 / final (tensor API)
      // ReCoNet (48/96/192 channels, padded to 64/128/192)
      E(B, SD, 9, 1, 4, 64, NST_R_C1_TILE, IN_ACT, OUT_ACT),
      E(B, SD, 9, 1, 4, 64, NST_R_C1_TILE, IN_U8_NHWC, OUT_ACT),
      E(B, SD, 9, 1, 4, 64, NST_R_C1_TILE, IN_F32_NCHW, OUT_ACT),
      E(B, SD, 3, 2, 128, 192, NST_R_DOWN2_TILE, IN_ACT, OUT_ACT),
      // the encoder's 96-channel map unpadded (nst_api.cpp: ReCoNet layers 1 / 2)
      E(B, SD, 3, 2, 64, 96, NST_C3_TILE, IN_ACT, OUT_ACT),
      E(B, SD, 3, 2, 96, 192, NST_R_DOWN2_96_TILE, IN_ACT, OUT_ACT),
      E(B, SD, 3, 1, 192, 192, NST_R_TRUNK_TILE, IN_ACT, OUT_ACT),
      E(B, PH, 3, 1, 192, 128, NST_R_UP1_TILE, IN_ACT, OUT_ACT),
      // consumers of the residual stream (residual join fused into the fill)
      E(B, SD, 3, 1, 128, 128, 8, 16, 2, 2, IN_ACT, OUT_ACT, VAR_RES),
      E(B, PH, 3, 1, 128, 64, NST_D1_TILE, IN_ACT, OUT_ACT, VAR_RES),
      E(B, SD, 3, 1, 192, 192, NST_R_TRUNK_RES_TILE, IN_ACT, OUT_ACT, VAR_RES),
      E(B, PH, 3, 1, 192, 128, NST_R_UP1_TILE, IN_ACT, OUT_ACT, VAR_RES),
      // the decoder's 96-channel stream unpadded (nst_api.cpp: ReCoNet layers 11 / 12)
      E(B, PH, 3, 1, 192, 96, NST_R_UP1_TILE, IN_ACT, OUT_ACT),
      E(B, PH, 3, 1, 192, 96, NST_R_UP1_TILE, IN_ACT, OUT_ACT, VAR_RES),
      E(B, PH, 3, 1, 96, 64, NST_D1_TILE, IN_ACT, OUT_ACT),
      E(B, SD, 9, 1, 64, 16, 8, 32, 4, 1, IN_ACT, OUT_U8_NHWC),
      E(B, SD, 9, 1, 64, 16, 8, 32, 4, 1, IN_ACT, OUT_F32_NCHW),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E
}  // namespace nst
