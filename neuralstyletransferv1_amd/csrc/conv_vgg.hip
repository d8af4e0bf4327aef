// conv_vgg.hip — bf16 instantiations of the generic implicit-GEMM conv (conv_impl.h) for the
// VGG-19 feature extractor of the Gatys loop (configs[2]; vgg_gatys.cpp): 3x3, stride 1, zero
// padding 1.  Forward: the image layer reads the fp32 NCHW image with the ImageNet normalisation
// (utils.py:93-96 preprocess_for_vgg) as the fill's encode; every other layer reads the stored
// pre-activation of its producer with the ReLU applied in the fill (unit InstanceNorm table) or the
// already-rectified pooled map.  Backward (input gradients only: the image is the variable): the
// same kernel over the masked output gradient with the flipped, transposed weights; the image
// layer's gradient leaves as fp32 NCHW.
#include "conv_impl.h"

#ifndef NST_VGG_T12
#define NST_VGG_T12 8, 16, 2, 2  // conv1_2 forward (64 -> 64 @ the full image)
#endif
#ifndef NST_VGG_T11
#define NST_VGG_T11 8, 32, 4, 1  // conv1_1 forward (the normalised image)
#endif
#ifndef NST_VGG_TB1
#define NST_VGG_TB1 8, 32, 4, 1  // conv1_1 backward (-> the image gradient)
#endif

#ifndef NST_VGG_T21
#define NST_VGG_T21 8, 16, 2, 2  // conv2_1 forward (64 -> 128)
#endif
#ifndef NST_VGG_T22
#define NST_VGG_T22 8, 16, 2, 4  // 128 -> 128 (8 waves: 0.995 vs 1.005 ms per step)
#endif
#ifndef NST_VGG_T3
#define NST_VGG_T3 8, 16, 1, 8  // 256 input channels (8 waves of 16 output channels: 0.875 vs 1.002 ms per step for 2 x 2)
#endif
#ifndef NST_VGG_T4
#define NST_VGG_T4 4, 16, 1, 8  // 512 input channels (8 waves of 16 output channels: 0.835 vs 0.89)
#endif
#ifndef NST_VGG_TB2
#define NST_VGG_TB2 8, 16, 2, 2  // conv2_1 backward (128 -> 64)
#endif

namespace nst {
typedef __bf16 B;
#define E(...) ConvInst<__VA_ARGS__>::info()
constexpr int SD = MODE_STD;
const ConvKernelInfo* conv_table_vgg(int* count) {
  static const ConvKernelInfo table[] = {
      //  T  MODE KS S CINP BN TH TW WM WN  IN           OUT
      // forward
      E(B, SD, 3, 1, 4, 64, NST_VGG_T11, IN_F32_NCHW, OUT_ACT),   // conv1_1 (normalised image)
      E(B, SD, 3, 1, 64, 64, NST_VGG_T12, IN_ACT, OUT_ACT),       // conv1_2
      E(B, SD, 3, 1, 64, 128, NST_VGG_T21, IN_ACT, OUT_ACT),      // conv2_1
      E(B, SD, 3, 1, 128, 128, NST_VGG_T22, IN_ACT, OUT_ACT),     // conv2_2, conv3_1 (2 channel blocks); backward 2_2
      E(B, SD, 3, 1, 256, 128, NST_VGG_T3, IN_ACT, OUT_ACT),     // conv3_2..3_4, conv4_1; backward 3_1..3_4
      E(B, SD, 3, 1, 512, 128, NST_VGG_T4, IN_ACT, OUT_ACT),     // conv4_2..5_1; backward 4_1..5_1
      // backward
      E(B, SD, 3, 1, 128, 64, NST_VGG_TB2, IN_ACT, OUT_ACT),      // conv2_1 -> 64 input channels
      E(B, SD, 3, 1, 64, 16, NST_VGG_TB1, IN_ACT, OUT_F32_NCHW),  // conv1_1 -> the image gradient (3 of 16)
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
}  // namespace nst
