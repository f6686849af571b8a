// Input pipeline on the device: the reference's per-sample transforms
// (train/transforms.py:15-129, composed in main.py:78-89 /
// parallel_main.py:111-124):
//
//   ResizeImage((256, 512))  torchvision Resize -> PIL Image.resize(BILINEAR)
//   RandomFlip(0.5)          mirror of the resized PIL image (both views)
//   ToTensor()               uint8 HWC -> f32 CHW / 255
//   RandomAugment(0.5, ...)  clamp((x ** g) * b * colour[c], 0, 1)
//
// The host draws the flip / augment decisions and values with numpy in the
// reference's order (umamd/imageprep.py) and passes them per sample; these
// kernels do the arithmetic for a whole batch of both views in two launches.
//
// Resize is Pillow's two-pass 8-bit resampler (libImaging/Resample.c,
// Pillow 12.2): a separable triangle filter whose support scales with the
// downscale factor (antialias), coefficients normalised per output pixel and
// quantised to 22-bit fixed point on the host (precompute_coeffs +
// normalize_coeffs_8bpc), the horizontal pass first into an 8-bit
// intermediate (round half up, clip to [0, 255]), then the vertical pass.
// Integer arithmetic throughout, so the result is bit-identical to PIL's.
#include "common.h"

namespace {

constexpr int PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ uint32_t clip8(int ss) {
  int v = ss >> PREC;
  return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pass 1: src [view][N][Hs][Ws][3] u8 -> tmp [view][N][Hs][Wd][3] u8
// one thread per (view, n, y, xx) output pixel of the horizontal pass
__global__ void resample_h_kernel(const uint8_t* __restrict__ left,
                                  const uint8_t* __restrict__ right, int N, int Hs, int Ws,
                                  int Wd, const int* __restrict__ bounds,
                                  const int* __restrict__ kk, int ks, uint8_t* __restrict__ tmp) {
  const long total = 2L * N * Hs * Wd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % Wd);
    const long row = i / Wd;          // (view, n, y)
    const int view = (int)(row / ((long)N * Hs));
    const long vrow = row - (long)view * N * Hs;  // n * Hs + y
    const uint8_t* src = (view == 0 ? left : right) + vrow * Ws * 3;
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int* k = kk + (long)xx * ks;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
      const uint8_t* p = src + (xmin + x) * 3;
      const int w = k[x];
      s0 += (int)p[0] * w;
      s1 += (int)p[1] * w;
      s2 += (int)p[2] * w;
    }
    uint8_t* o = tmp + i * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
  }
}

// pass 2: tmp -> out_view [N][3][Hd][Wd] f32 with ToTensor, flip, augment;
// one thread per (view, n, yy, x) output pixel, all 3 channels
__global__ void resample_v_kernel(const uint8_t* __restrict__ tmp, int N, int Hs, int Hd,
                                  int Wd, const int* __restrict__ bounds,
                                  const int* __restrict__ kk, int ks,
                                  const float* __restrict__ params, float* __restrict__ out_l,
                                  float* __restrict__ out_r) {
  const long total = 2L * N * Hd * Wd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % Wd);
    const long r = i / Wd;
    const int yy = (int)(r % Hd);
    const long vn = r / Hd;          // view * N + n
    const int view = (int)(vn / N);
    const int n = (int)(vn - (long)view * N);
    const float* pr = params + n * 8;  // flip, augment, gamma, brightness, colour[3], pad
    // RandomFlip mirrors the resized image: output column x reads column Wd-1-x
    const int xs = pr[0] != 0.f ? Wd - 1 - x : x;
    const uint8_t* col = tmp + (vn * Hs * Wd + xs) * 3;
    const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
    const int* k = kk + (long)yy * ks;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* p = col + (long)(ymin + y) * Wd * 3;
      const int w = k[y];
      s0 += (int)p[0] * w;
      s1 += (int)p[1] * w;
      s2 += (int)p[2] * w;
    }
    // ToTensor: float(u8) / 255 (IEEE division, as torch's div)
    float v[3] = {(float)clip8(s0) / 255.0f, (float)clip8(s1) / 255.0f,
                  (float)clip8(s2) / 255.0f};
    if (pr[1] != 0.f) {  // RandomAugment.transform: gamma, brightness, colour, clamp
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float t = powf(v[c], pr[2]);
        t = t * pr[3];
        t = t * pr[4 + c];
        v[c] = fminf(fmaxf(t, 0.f), 1.f);
      }
    }
    float* o = (view == 0 ? out_l : out_r) + (long)n * 3 * Hd * Wd + (long)yy * Wd + x;
    const long plane = (long)Hd * Wd;
    o[0] = v[0];
    o[plane] = v[1];
    o[2 * plane] = v[2];
  }
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

long um_stereo_prep_ws(int N, int Hs, int Wd) { return 2L * N * Hs * Wd * 3; }

int um_stereo_prep(int N, int Hs, int Ws, const unsigned char* left, const unsigned char* right,
                   int Hd, int Wd, const int* bounds_h, const int* kk_h, int ks_h,
                   const int* bounds_v, const int* kk_v, int ks_v, const float* params,
                   unsigned char* tmp, float* out_left, float* out_right, hipStream_t st) {
  UM_CHECK_ARG(N > 0 && Hs > 0 && Ws > 0 && Hd > 0 && Wd > 0 && ks_h > 0 && ks_v > 0,
               "um_stereo_prep: bad sizes N=%d Hs=%d Ws=%d Hd=%d Wd=%d", N, Hs, Ws, Hd, Wd);
  UM_CHECK_ARG(left && right && bounds_h && kk_h && bounds_v && kk_v && params && tmp &&
                   out_left && out_right,
               "um_stereo_prep: null pointer");
  hipLaunchKernelGGL(resample_h_kernel, dim3(grid_for(2L * N * Hs * Wd)), dim3(256), 0, st,
                     left, right, N, Hs, Ws, Wd, bounds_h, kk_h, ks_h, tmp);
  UM_LAUNCH_CHECK();
  hipLaunchKernelGGL(resample_v_kernel, dim3(grid_for(2L * N * Hd * Wd)), dim3(256), 0, st, tmp,
                     N, Hs, Hd, Wd, bounds_v, kk_v, ks_v, params, out_left, out_right);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
