// conv_f32s.hip — split-fp16 mode (NST_DT_F32S: fp32 activations, fp16 hi/lo operand pairs on
// v_mfma_f32_16x16x32_f16) instantiations of conv_kernel (conv_tab32.h).
#include "conv_tab32.h"

namespace nst {
const ConvKernelInfo* conv_table_f32s(int* count) { return conv_table_32<F32Split>(count); }
}  // namespace nst
