// Evaluation metrics (reference train/evaluate.py:66-196 and
// train/sparsification.py:8-61), off the training hot path:
//
//   um_ssim_gauss       torchmetrics structural_similarity_index_measure as the
//                       reference calls it (gaussian window, sigma 1.5 -> 11
//                       taps, data_range 1, k1 0.01, k2 0.03): per-image mean
//                       of the SSIM map over the interior (the torchmetrics
//                       crop of its reflect padding = every full window).
//   um_avgpool_valid    nn.AvgPool2d(k, stride=1) (no padding)
//   um_spars_sort       per (image, view) segment: sort the predicted error
//                       descending and carry the oracle error along
//                       (argsort + gather, sparsification.py:18-19), hipCUB
//                       segmented radix sort
//   um_spars_curve      the 100-step sparsification curve: mean of the
//                       oracle error left after removing the first
//                       int(step/steps * L) sorted pixels, over its full mean,
//                       averaged over the segments (sparsification.py:21-36)
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

// -------------------------------------------------------- gaussian SSIM ----
constexpr int SK = 11, SR = 5;           // 11-tap window (sigma 1.5)
constexpr int STY = 16, STX = 64;        // output tile
constexpr int SRY = STY + 2 * SR, SRX = STX + 2 * SR;

struct SsimArgs {
  const float* x;  // preds  [N][C][H][W]
  const float* y;  // target
  int N, C, H, W;
  float c1, c2;
  float g[SK];      // normalised 1-D gaussian
  double* parts;    // [N][tiles] partial sums of the SSIM map
  int tiles_x, tiles_y;
};

__global__ void __launch_bounds__(256) ssim_gauss_kernel(SsimArgs a) {
  __shared__ float sx[SRY][SRX], sy[SRY][SRX];
  __shared__ float hq[5][SRY][STX];  // horizontal pass of x, y, xx, yy, xy
  __shared__ double red[4];
  const int tid = threadIdx.x;
  const int per = a.tiles_x * a.tiles_y;
  const int n = blockIdx.x / per, t = blockIdx.x - n * per;
  // output coordinates are in the valid region: pixel (oy, ox) is the window
  // centred at image (oy + SR, ox + SR)
  const int oy0 = (t / a.tiles_x) * STY, ox0 = (t % a.tiles_x) * STX;
  const int OH = a.H - 2 * SR, OW = a.W - 2 * SR;
  double acc = 0.0;
  for (int c = 0; c < a.C; ++c) {
    const float* X = a.x + ((long)n * a.C + c) * a.H * a.W;
    const float* Y = a.y + ((long)n * a.C + c) * a.H * a.W;
    for (int i = tid; i < SRY * SRX; i += 256) {
      const int r = i / SRX, q = i % SRX;
      const int yy = min(oy0 + r, a.H - 1), xx = min(ox0 + q, a.W - 1);
      sx[r][q] = X[(long)yy * a.W + xx];
      sy[r][q] = Y[(long)yy * a.W + xx];
    }
    __syncthreads();
    for (int i = tid; i < SRY * STX; i += 256) {
      const int r = i / STX, q = i % STX;
      float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < SK; ++k) {
        const float xv = sx[r][q + k], yv = sy[r][q + k], w = a.g[k];
        v[0] += w * xv;
        v[1] += w * yv;
        v[2] += w * xv * xv;
        v[3] += w * yv * yv;
        v[4] += w * xv * yv;
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) hq[k][r][q] = v[k];
    }
    __syncthreads();
    for (int i = tid; i < STY * STX; i += 256) {
      const int r = i / STX, q = i % STX;
      if (oy0 + r >= OH || ox0 + q >= OW) continue;
      float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < SK; ++k)
#pragma unroll
        for (int j = 0; j < 5; ++j) v[j] += a.g[k] * hq[j][r + k][q];
      const float mx2 = v[0] * v[0], my2 = v[1] * v[1], mxy = v[0] * v[1];
      const float sxx = v[2] - mx2, syy = v[3] - my2, sxy = v[4] - mxy;
      acc += (double)(((2.f * mxy + a.c1) * (2.f * sxy + a.c2)) /
                      ((mx2 + my2 + a.c1) * (sxx + syy + a.c2)));
    }
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) a.parts[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[n] = sum of the image's tile partials / (C * OH * OW)
__global__ void ssim_finish_kernel(const double* parts, int N, int tiles, double count,
                                   float* out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int t = 0; t < tiles; ++t) s += parts[(long)n * tiles + t];
  out[n] = (float)(s / count);
}

// ------------------------------------------------------- average pooling ---
__global__ void avgpool_valid_kernel(const float* __restrict__ x, int NC, int H, int W, int k,
                                     float* __restrict__ out) {
  const int OH = H - k + 1, OW = W - k + 1;
  const long total = (long)NC * OH * OW;
  const float inv = 1.f / (float)(k * k);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ox = i % OW;
    const int oy = (i / OW) % OH;
    const long pl = i / ((long)OW * OH);
    const float* p = x + pl * H * W + (long)oy * W + ox;
    float s = 0.f;
    for (int u = 0; u < k; ++u)
      for (int v = 0; v < k; ++v) s += p[(long)u * W + v];
    out[i] = s * inv;
  }
}

// -------------------------------------------------- sparsification curve --
__global__ void seg_offsets_kernel(int* offs, int nseg, int L) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= nseg) offs[i] = i * L;
}

// one workgroup per segment: normalised[seg][k] = mean(sorted[cut_k:]) / mean(all)
__global__ void __launch_bounds__(256) spars_curve_kernel(const float* __restrict__ sorted, int L,
                                                          int steps, double* __restrict__ norm) {
  extern __shared__ double isum[];  // [steps]
  const float* v = sorted + (long)blockIdx.x * L;
  auto cut = [&](int k) { return (int)((double)k / (double)steps * (double)L); };
  for (int k = threadIdx.x; k < steps; k += blockDim.x) {
    const int c0 = cut(k), c1 = k + 1 < steps ? cut(k + 1) : L;
    double s = 0.0;
    for (int i = c0; i < c1; ++i) s += (double)v[i];
    isum[k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double suffix = 0.0;
    for (int k = steps - 1; k >= 0; --k) {
      suffix += isum[k];
      isum[k] = suffix;
    }
    const double mean = isum[0] / (double)L;
    for (int k = 0; k < steps; ++k)
      norm[(long)blockIdx.x * steps + k] = (isum[k] / (double)(L - cut(k))) / mean;
  }
}

__global__ void spars_mean_kernel(const double* norm, int nseg, int steps, float* curve) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= steps) return;
  double s = 0.0;
  for (int g = 0; g < nseg; ++g) s += norm[(long)g * steps + k];
  curve[k] = (float)(s / (double)nseg);
}

}  // namespace

extern "C" {

long um_ssim_ws(int N, int H, int W) {
  const int OH = H - 2 * SR, OW = W - 2 * SR;
  if (OH <= 0 || OW <= 0) return 0;
  return (long)N * ceil_div(OH, STY) * ceil_div(OW, STX) * sizeof(double);
}

int um_ssim_gauss(const float* x, const float* y, int N, int C, int H, int W, float data_range,
                  float sigma, double* ws, float* out, hipStream_t st) {
  UM_CHECK_ARG((int)(3.5f * sigma + 0.5f) * 2 + 1 == SK,
               "um_ssim_gauss: sigma %g gives a window other than %d taps", sigma, SK);
  UM_CHECK_ARG(H > 2 * SR && W > 2 * SR, "um_ssim_gauss: image %dx%d smaller than the window",
               H, W);
  SsimArgs a{};
  a.x = x; a.y = y; a.N = N; a.C = C; a.H = H; a.W = W;
  a.c1 = (0.01f * data_range) * (0.01f * data_range);
  a.c2 = (0.03f * data_range) * (0.03f * data_range);
  // torchmetrics _gaussian: arange((1-k)/2, (1+k)/2) in f32, exp(-(d/s)^2/2), / sum
  float gs = 0.f;
  for (int k = 0; k < SK; ++k) {
    const float d = (float)(k - SR) / sigma;
    a.g[k] = expf(-(d * d) / 2.f);
    gs += a.g[k];
  }
  for (int k = 0; k < SK; ++k) a.g[k] /= gs;
  a.tiles_y = ceil_div(H - 2 * SR, STY);
  a.tiles_x = ceil_div(W - 2 * SR, STX);
  a.parts = ws;
  const int tiles = a.tiles_x * a.tiles_y;
  hipLaunchKernelGGL(ssim_gauss_kernel, dim3(N * tiles), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ssim_finish_kernel, dim3(ceil_div(N, 64)), dim3(64), 0, st, ws, N, tiles,
                     (double)C * (H - 2 * SR) * (W - 2 * SR), out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_avgpool_valid(const float* x, int NC, int H, int W, int k, float* out, hipStream_t st) {
  UM_CHECK_ARG(k >= 1 && k <= H && k <= W, "um_avgpool_valid: window %d vs %dx%d", k, H, W);
  const long total = (long)NC * (H - k + 1) * (W - k + 1);
  long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(avgpool_valid_kernel, dim3((int)std::max(b, 1l)), dim3(256), 0, st, x, NC, H,
                     W, k, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// scratch bytes of um_spars_sort (segment offsets + hipCUB temporary storage)
long um_spars_sort_ws(int nseg, int L) {
  size_t bytes = 0;
  hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
      nullptr, bytes, (const float*)nullptr, (float*)nullptr, (const float*)nullptr,
      (float*)nullptr, nseg * L, nseg, (const int*)nullptr, (const int*)nullptr);
  return (long)bytes + (long)(nseg + 1) * sizeof(int) + 256;
}

int um_spars_sort(const float* keys, const float* vals, int nseg, int L, float* keys_out,
                  float* vals_out, void* ws, long ws_bytes, hipStream_t st) {
  int* offs = reinterpret_cast<int*>(ws);
  char* tmp = reinterpret_cast<char*>(ws) + (((nseg + 1) * sizeof(int) + 255) / 256) * 256;
  size_t bytes = (size_t)(ws_bytes - (tmp - reinterpret_cast<char*>(ws)));
  hipLaunchKernelGGL(seg_offsets_kernel, dim3(ceil_div(nseg + 1, 256)), dim3(256), 0, st, offs,
                     nseg, L);
  const hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
      tmp, bytes, keys, keys_out, vals, vals_out, nseg * L, nseg, offs, offs + 1, 0,
      sizeof(float) * 8, st);
  UM_CHECK_ARG(e == hipSuccess, "um_spars_sort: hipcub %s", hipGetErrorString(e));
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_spars_curve(const float* sorted_vals, int nseg, int L, int steps, double* ws,
                   float* curve, hipStream_t st) {
  UM_CHECK_ARG(steps >= 1 && steps <= 4096 && L >= 1, "um_spars_curve: steps %d, L %d", steps, L);
  hipLaunchKernelGGL(spars_curve_kernel, dim3(nseg), dim3(256), steps * sizeof(double), st,
                     sorted_vals, L, steps, ws);
  hipLaunchKernelGGL(spars_mean_kernel, dim3(ceil_div(steps, 128)), dim3(128), 0, st, ws, nseg,
                     steps, curve);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
