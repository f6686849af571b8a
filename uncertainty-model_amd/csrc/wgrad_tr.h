// Internal interface of the transposed-read implicit-GEMM weight gradient
// (wgrad_tr.hip), bf16.
#pragma once

#include <hip/hip_runtime.h>

namespace umamd {

int wgrad_tr_bm(int K);  // output-channel tile (64 or 128)
int wgrad_tr_blocks_per_cu(int K);  // resident workgroups per CU of that instance
// slabs [splits][K][R*R*C] f32
int wgrad_tr_run(const void* x, int N, int H, int W, int C, int ldx, int K, int R, int stride,
                 int pad, int reflect, int P, int Q, const void* dy, int ldy, float* slabs,
                 int splits, hipStream_t st);

}  // namespace umamd
