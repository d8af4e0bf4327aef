// conv_bf16_wl.hip — bf16 instantiations of the persistent / LDS-weight-ring conv kernels.
// Own translation unit: these fully unroll a long K loop and are built with a raised
// pragma-unroll cap (Makefile), which the register-streamed kernels must not inherit.
#include "conv_impl.h"

namespace nst {
typedef __bf16 B;
#define E(...) ConvInst<__VA_ARGS__>::info()
constexpr int SD = MODE_STD;
constexpr int WLP = VAR_WL | VAR_PERS;
const ConvKernelInfo* conv_table_bf16_wl(int* count) {
  static const ConvKernelInfo table[] = {
      //  T  MODE KS S CINP BN TH TW WM WN  IN      OUT      VAR
      E(B, SD, 3, 1, 128, 128, 16, 16, 4, 2, IN_ACT, OUT_ACT, WLP),            // residual trunk
      E(B, SD, 3, 1, 128, 128, 16, 16, 4, 2, IN_ACT, OUT_ACT, WLP | VAR_RES),  // + residual join
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
}  // namespace nst
