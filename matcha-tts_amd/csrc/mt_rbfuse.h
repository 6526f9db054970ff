#pragma once
#include "mt_common.h"

namespace mt {

struct RBConv {
  const void* w;       // packed [C][k][C] (GEMM rows = output channels)
  const float* bias;   // [C]
};

// One fused HiFi-GAN ResBlock1 stage: y = (sum_j rb_j(x)) / div  (see mt_rbfuse.hip)
struct RBArgs {
  const void* x;
  void* y;
  int B, L, nk, npair, hmax;
  int k[3];
  int dil[3][3];
  RBConv c1[3][3], c2[3][3];   // [resblock][pair]
  int r1a[3][3], r1b[3][3];    // local output row range of each conv (rows of the tile + halo)
  int r2a[3][3], r2b[3][3];
  float slope, div;
};

bool rbfuse_supported(int dtype, int C);
int rbfuse_tile_n(int C);
int launch_rbfuse(int dtype, int C, const RBArgs& a, hipStream_t st);

}  // namespace mt
