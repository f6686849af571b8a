// Internal interface of the halo-tiled weight gradient (wgrad_halo.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace umamd {

// number of partial slabs the halo kernel writes for this bf16 conv, or 0 if
// the shape is not covered (then the generic implicit-GEMM kernel runs)
int hwgrad_splits(int N, int H, int W, int C, int ldx, int K, int R, int stride, int pad,
                  int reflect, int P, int Q, int ldy);
// slabs: [splits][K][R*R*C] f32, splits as returned above; UM_OK or error
int hwgrad_run(const void* x, int N, int H, int W, int C, int ldx, int K, int R, int stride,
               int pad, int reflect, int P, int Q, const void* dy, int ldy, float* slabs,
               int splits, hipStream_t st);

}  // namespace umamd
