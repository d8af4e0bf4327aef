// conv_bf16.hip — bf16 (throughput mode) instantiations of the generic conv_kernel (conv_tab16.h).
#include "conv_tab16.h"

namespace nst {
const ConvKernelInfo* conv_table_bf16(int* count) { return conv_table_16<__bf16>(count); }
}  // namespace nst
