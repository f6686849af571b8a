// Fused multi-tensor Adam (torch.optim.Adam semantics, no amsgrad), replacing
// the optimiser step of reference train/train.py:228-229 (Adam(params, lr)).
//   m = b1*m + (1-b1)*g ; v = b2*v + (1-b2)*g^2
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)      (+ L2 weight decay on g)
// One launch updates every parameter: the host passes a device table of
// {param, grad, exp_avg, exp_avg_sq, numel} and a chunk table.
#include "common.h"

namespace {

struct AdamEntry {
  float* p;
  const float* g;
  float* m;
  float* v;
  long long n;
};

constexpr int CHUNK = 4096;

__global__ void adam_kernel(const AdamEntry* __restrict__ tab, const int2* __restrict__ chunks,
                            int nchunks, float lr_bc1, float b1, float b2, float inv_sqrt_bc2,
                            float eps, float wd, const int* __restrict__ dstep,
                            const float* __restrict__ dlr) {
  if (dstep != nullptr) {  // graph-replayable: step count (and lr) live on the device
    const int step = *dstep;
    const float lr = dlr ? *dlr : lr_bc1;
    lr_bc1 = (float)(lr / (1.0 - pow((double)b1, step)));
    inv_sqrt_bc2 = (float)(1.0 / sqrt(1.0 - pow((double)b2, step)));
  }
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const int2 ch = chunks[ci];  // (entry, chunk index within entry)
    const AdamEntry e = tab[ch.x];
    const long long s0 = (long long)ch.y * CHUNK;
    const long long s1 = min(e.n, s0 + CHUNK);
    for (long long i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
      float g = e.g ? e.g[i] : 0.f;
      float p = e.p[i];
      if (wd != 0.f) g += wd * p;
      const float m = b1 * e.m[i] + (1.f - b1) * g;
      const float v = b2 * e.v[i] + (1.f - b2) * g * g;
      e.m[i] = m;
      e.v[i] = v;
      p -= lr_bc1 * m / (sqrtf(v) * inv_sqrt_bc2 + eps);
      e.p[i] = p;
    }
  }
}

__global__ void inc_kernel(int* step) { *step += 1; }

}  // namespace

extern "C" {

int um_adam_chunk(void) { return CHUNK; }

// table: device array of n_entries x {p, g, m, v, numel} (5 x 8 bytes each)
// chunks: device int2 array (entry, chunk)
int um_adam_step(const void* table, const void* chunks, int nchunks, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int step, hipStream_t st) {
  UM_CHECK_ARG(step >= 1, "um_adam_step: step %d", step);
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const int blocks = nchunks < 8192 ? nchunks : 8192;
  if (blocks == 0) return UM_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, (const AdamEntry*)table,
                     (const int2*)chunks, nchunks, (float)(lr / bc1), beta1, beta2,
                     (float)(1.0 / sqrt(bc2)), eps, weight_decay, nullptr, nullptr);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// Graph-replayable variant: increments the device step counter, then updates
// with bias corrections computed from it; lr read from dlr (device) if given.
int um_adam_step_dev(const void* table, const void* chunks, int nchunks, float lr,
                     const float* dlr, float beta1, float beta2, float eps, float weight_decay,
                     int* dstep, hipStream_t st) {
  UM_CHECK_ARG(dstep != nullptr, "um_adam_step_dev: step counter");
  hipLaunchKernelGGL(inc_kernel, dim3(1), dim3(1), 0, st, dstep);
  const int blocks = nchunks < 8192 ? nchunks : 8192;
  if (blocks == 0) return UM_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, (const AdamEntry*)table,
                     (const int2*)chunks, nchunks, lr, beta1, beta2, 1.f, eps, weight_decay,
                     dstep, dlr);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
