// conv_f32.hip — fp32 (parity mode, exact-f32 MFMA) instantiations of conv_kernel (conv_tab32.h).
#include "conv_tab32.h"

namespace nst {
const ConvKernelInfo* conv_table_f32(int* count) { return conv_table_32<float>(count); }
}  // namespace nst
