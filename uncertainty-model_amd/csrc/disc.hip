// Adversarial path helpers (reference model/discriminator.py:13-86,
// train/loss.py:267-337, train/utils.py:248-273).  The discriminator's
// EncoderStages run on the encoder kernels; these are the pieces around
// them:
//
//   um_nhwc_to_image    NHWC (T) -> NCHW f32 of the first C channels: the
//                       adjoint of um_image_to_nhwc (the recon pyramid fed to
//                       the discriminator carries gradient to the disparities)
//   um_disc_head_fwd    sigmoid(Linear(flatten(x))) of the last feature map:
//                       flatten is the reference's NCHW view (:82), so the
//                       weight index of NHWC element (p, c) is c*HW + p
//   um_disc_head_bwd    its gradient w.r.t. x, the weight and the bias
//   um_l1_mean          mean |a - b| of two NHWC feature maps (PerceptualLoss
//                       via train/utils.py l1_loss), last-workgroup f64 finish
//   um_l1_mean_bwd      d/da = -d/db = g * sign(a - b) / n
#include "common.h"

namespace {

template <typename T>
__global__ void nhwc_to_image_kernel(const T* __restrict__ x, int N, int C, int H, int W, int ld,
                                     float* __restrict__ out) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i % ((long)H * W);
    const long nc = i / ((long)H * W);
    const int c = nc % C, n = nc / C;
    out[i] = to_f32(x[((long)n * H * W + p) * ld + c]);
  }
}

// one workgroup per image: logit = b + sum_{p,c} w[c*HW + p] * x[n][p][c]
template <typename T>
__global__ void __launch_bounds__(256) head_fwd_kernel(const T* __restrict__ x, int HW, int C,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ prob) {
  __shared__ float red[4];
  const int n = blockIdx.x;
  const T* xn = x + (long)n * HW * C;
  float acc = 0.f;
  for (long i = threadIdx.x; i < (long)HW * C; i += 256) {
    const int p = i / C, c = i - (i / C) * C;
    acc += w[(long)c * HW + p] * to_f32(xn[i]);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float z = (red[0] + red[1]) + (red[2] + red[3]) + bias[0];
    prob[n] = 1.f / (1.f + expf(-z));
  }
}

// dlogit[n] = dprob[n] * p (1 - p); dx = dlogit * w; dw[j] = sum_n dlogit[n] x[n][j]
template <typename T>
__global__ void head_bwd_kernel(const T* __restrict__ x, int N, int HW, int C,
                                const float* __restrict__ w, const float* __restrict__ prob,
                                const float* __restrict__ dprob, T* __restrict__ dx,
                                float* __restrict__ dw, float* __restrict__ db) {
  const long M = (long)HW * C;
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < M;
       j += (long)gridDim.x * blockDim.x) {
    const int p = j / C, c = j - (j / C) * C;
    const long wi = (long)c * HW + p;
    const float wv = w[wi];
    float g = 0.f;
    for (int n = 0; n < N; ++n) {
      const float dl = dprob[n] * prob[n] * (1.f - prob[n]);
      if (dx) dx[(long)n * M + j] = from_f32<T>(dl * wv);
      g += dl * to_f32(x[(long)n * M + j]);
    }
    if (dw) dw[wi] = g;
  }
  if (db != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dprob[n] * prob[n] * (1.f - prob[n]);
    db[0] = s;
  }
}

__device__ unsigned int g_l1_ticket;

template <typename T>
__global__ void __launch_bounds__(256) l1_mean_kernel(const T* __restrict__ a,
                                                      const T* __restrict__ b, long n,
                                                      double* __restrict__ parts,
                                                      float* __restrict__ out) {
  __shared__ double red[4];
  __shared__ int last;
  float acc = 0.f;
  for (long i = blockIdx.x * 256l + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    acc += fabsf(to_f32(a[i]) - to_f32(b[i]));
  double d = acc;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) parts[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&g_l1_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1);
    if (last) {
      __hip_atomic_store(&g_l1_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  double s = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) s += parts[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)(((red[0] + red[1]) + (red[2] + red[3])) / (double)n);
}

template <typename T>
__global__ void l1_mean_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b, long n,
                                   const float* __restrict__ g, T* __restrict__ da,
                                   T* __restrict__ db) {
  const float k = g[0] / (float)n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float d = to_f32(a[i]) - to_f32(b[i]);
    const float s = ((d > 0.f) - (d < 0.f)) * k;
    if (da) da[i] = from_f32<T>(s);
    if (db) db[i] = from_f32<T>(-s);
  }
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

constexpr int L1_BLOCKS = 1024;

}  // namespace

extern "C" {

int um_nhwc_to_image(int dtype, const void* x, int N, int C, int H, int W, int ld, float* out,
                     hipStream_t st) {
  UM_CHECK_ARG(C <= ld, "um_nhwc_to_image: C %d > ld %d", C, ld);
  const int g = grid_for((long)N * C * H * W);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(nhwc_to_image_kernel<bf16_t>, dim3(g), dim3(256), 0, st,
                       (const bf16_t*)x, N, C, H, W, ld, out);
  else
    hipLaunchKernelGGL(nhwc_to_image_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x,
                       N, C, H, W, ld, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_disc_head_fwd(int dtype, const void* x, int N, int HW, int C, const float* w,
                     const float* bias, float* prob, hipStream_t st) {
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, dim3(N), dim3(256), 0, st, (const bf16_t*)x, HW,
                       C, w, bias, prob);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(N), dim3(256), 0, st, (const float*)x, HW, C,
                       w, bias, prob);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_disc_head_bwd(int dtype, const void* x, int N, int HW, int C, const float* w,
                     const float* prob, const float* dprob, void* dx, float* dw, float* db,
                     hipStream_t st) {
  const int g = grid_for((long)HW * C);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(head_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, N,
                       HW, C, w, prob, dprob, (bf16_t*)dx, dw, db);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, N, HW,
                       C, w, prob, dprob, (float*)dx, dw, db);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

long um_l1_mean_ws(void) { return L1_BLOCKS * sizeof(double); }

int um_l1_mean(int dtype, const void* a, const void* b, long n, double* ws, float* out,
               hipStream_t st) {
  UM_CHECK_ARG(n > 0, "um_l1_mean: empty");
  const int g = (int)std::min<long>(L1_BLOCKS, (n + 255) / 256);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(l1_mean_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)a,
                       (const bf16_t*)b, n, ws, out);
  else
    hipLaunchKernelGGL(l1_mean_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)a,
                       (const float*)b, n, ws, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_l1_mean_bwd(int dtype, const void* a, const void* b, long n, const float* g, void* da,
                   void* db, hipStream_t st) {
  const int gr = grid_for(n);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(l1_mean_bwd_kernel<bf16_t>, dim3(gr), dim3(256), 0, st, (const bf16_t*)a,
                       (const bf16_t*)b, n, g, (bf16_t*)da, (bf16_t*)db);
  else
    hipLaunchKernelGGL(l1_mean_bwd_kernel<float>, dim3(gr), dim3(256), 0, st, (const float*)a,
                       (const float*)b, n, g, (float*)da, (float*)db);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
