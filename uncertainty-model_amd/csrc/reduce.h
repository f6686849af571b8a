// Internal interface of the one-launch column reductions (reduce.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace umamd {

enum { COLRED_SUMS = 0, COLRED_BN_FWD = 1, COLRED_BN_BWD = 2, COLRED_ROWS = 3, COLRED_NMODES = 4 };

struct ColRed {
  const float* parts;  // [nparts] rows, channel c value v at row*rowstride + c*NV + v
  int nparts, C;
  long rowstride;
  double* ws;  // [blocks][C][NV] f64 slab rows (caller-owned, um_colred_ws bytes)
  int rows_per_block;
  int mode;
  // COLRED_SUMS
  double* st;
  // BN forward / backward
  double count;
  const float *gamma, *beta;
  float eps, momentum;
  float *running_mean, *running_var;
  long long* nbt;
  float *mean, *invstd, *scale, *shift;
  const float* invstd_in;
  float *dgamma, *dbeta, *dbias, *k1, *k2, *k3;
  // COLRED_ROWS
  float* out;
  int accumulate;
};

int colred_blocks(int nparts, int C, int NV);
long colred_ws_bytes(int nparts, int C, int NV);
int colred_run(ColRed a, int NV, hipStream_t st);

}  // namespace umamd
