// conv_bf16_wl.hip — bf16 (and fp16, ReCoNet) instantiations of the persistent / LDS-weight-ring conv kernels.
// Own translation unit: these fully unroll a long K loop and are built with a raised
// pragma-unroll cap (Makefile), which the register-streamed kernels must not inherit.
#include "conv_impl.h"

namespace nst {
typedef __bf16 B;
typedef _Float16 H;
#define E(...) ConvInst<__VA_ARGS__>::info()
constexpr int SD = MODE_STD;
constexpr int WLP = VAR_WL | VAR_PERS;
const ConvKernelInfo* conv_table_bf16_wl(int* count) {
  static const ConvKernelInfo table[] = {
      //  T  MODE KS S CINP BN TH TW WM WN  IN      OUT      VAR
      E(B, SD, 3, 1, 128, 128, 16, 16, 4, 2, IN_ACT, OUT_ACT, WLP),            // residual trunk
      E(B, SD, 3, 1, 128, 128, 16, 16, 4, 2, IN_ACT, OUT_ACT, WLP | VAR_RES),  // + residual join
      // ReCoNet's 192-channel trunk (model.py:43-60): 8x16 tiles, 8 waves; halo 75 KB + a 3 x 24 KiB weight ring
      E(B, SD, 3, 1, 192, 192, 8, 16, 2, 4, IN_ACT, OUT_ACT, WLP),
      E(B, SD, 3, 1, 192, 192, 8, 16, 2, 4, IN_ACT, OUT_ACT, WLP | VAR_RES),
      E(H, SD, 3, 1, 192, 192, 8, 16, 2, 4, IN_ACT, OUT_ACT, WLP),
      E(H, SD, 3, 1, 192, 192, 8, 16, 2, 4, IN_ACT, OUT_ACT, WLP | VAR_RES),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
}  // namespace nst
