// conv_f16.hip — fp16 (NST_DT_F16) instantiations of the generic conv_kernel (conv_tab16.h): the layers
// without a weight-stationary kernel (ReCoNet's 192-channel trunk, the NST_KSEL_NO_* fallbacks).
#include "conv_tab16.h"

namespace nst {
const ConvKernelInfo* conv_table_f16(int* count) { return conv_table_16<_Float16>(count); }
}  // namespace nst
