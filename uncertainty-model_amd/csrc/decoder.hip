// Decoder-stage data movement, reference model/layers/decoder.py:210-249:
//   skip = F.interpolate(skip, x2, bilinear, align_corners=True)      :230
//   cat((feature_map, skip))                                           :233
//   PixelShuffle(2) of the upsample conv output                        :191,235
//   cat((x_up, skip_out[, interpolate(disp, x2)]))                     :236-242
//   SELayer squeeze (AdaptiveAvgPool2d(1)) / excite MLP / x * s        :90-136
// A concat is materialised once by um_concat_build from up to 8 sources, each
// COPY / UP2 (bilinear x2, align_corners=True) / PSHUF (pixel shuffle x2),
// optionally scaled per (n, c) (the SE gate is applied here instead of
// materialising x * s).  Backward: one launch per source with per-(n,c)
// gate gradients reduced in-block then atomically added.
#include <algorithm>

#include "common.h"

namespace {

constexpr int MAX_SRC = 8;

struct CatSrc {
  const void* ptr;
  const float* scale;  // [N][C] or null
  int C, ld, op, coff, dtype, h, w;
};
struct CatArgs {
  CatSrc s[MAX_SRC];
  int nsrc;
};

// torch upsample_bilinear2d(align_corners=True) source index for output i
__device__ __forceinline__ void up_index(int i, int in, int out, int& i0, int& i1, float& l1) {
  const float sc = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float src = sc * (float)i;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = src - (float)i0;
}

__device__ __forceinline__ float ld_any(const void* p, long off, int dt) {
  return dt == UM_BF16 ? __bfloat162float(reinterpret_cast<const bf16_t*>(p)[off])
                       : reinterpret_cast<const float*>(p)[off];
}
__device__ __forceinline__ void st_any(void* p, long off, int dt, float v, int acc) {
  if (dt == UM_BF16) {
    bf16_t* q = reinterpret_cast<bf16_t*>(p) + off;
    *q = __float2bfloat16(acc ? __bfloat162float(*q) + v : v);
  } else {
    float* q = reinterpret_cast<float*>(p) + off;
    *q = acc ? *q + v : v;
  }
}

template <typename T>
__global__ void concat_build_kernel(CatArgs a, int N, int H, int W, int Ctot, T* __restrict__ dst,
                                    int ld) {
  const long total = (long)N * H * W * Ctot;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = i % Ctot;
    const long pix = i / Ctot;
    const int x = pix % W;
    const int y = (pix / W) % H;
    const int n = pix / ((long)W * H);
    float v = 0.f;
    for (int k = 0; k < a.nsrc; ++k) {
      const CatSrc& s = a.s[k];
      const int cc = c - s.coff;
      if (cc < 0 || cc >= s.C) continue;
      if (s.op == UM_CAT_COPY) {
        v = ld_any(s.ptr, ((long)(n * H + y) * W + x) * s.ld + cc, s.dtype);
      } else if (s.op == UM_CAT_UP2) {
        int y0, y1, x0, x1;
        float ly, lx;
        up_index(y, s.h, H, y0, y1, ly);
        up_index(x, s.w, W, x0, x1, lx);
        const long b = (long)n * s.h;
        const float v00 = ld_any(s.ptr, ((b + y0) * s.w + x0) * s.ld + cc, s.dtype);
        const float v01 = ld_any(s.ptr, ((b + y0) * s.w + x1) * s.ld + cc, s.dtype);
        const float v10 = ld_any(s.ptr, ((b + y1) * s.w + x0) * s.ld + cc, s.dtype);
        const float v11 = ld_any(s.ptr, ((b + y1) * s.w + x1) * s.ld + cc, s.dtype);
        v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
      } else {  // PSHUF: src [N][H/2][W/2][4C], channel cc*4 + (y&1)*2 + (x&1)
        v = ld_any(s.ptr, ((long)(n * s.h + (y >> 1)) * s.w + (x >> 1)) * s.ld + cc * 4 +
                              (y & 1) * 2 + (x & 1),
                   s.dtype);
      }
      if (s.scale) v *= s.scale[n * s.C + cc];
      break;
    }
    dst[pix * ld + c] = from_f32<T>(v);
  }
}

// ---- backward: block = 64 channels x 4 pixel lanes; grid (pixel chunks, C/64, N)
constexpr int BWD_CHUNK = 256;  // source pixels per block

template <typename T>
__global__ void cat_bwd_copy_kernel(const T* __restrict__ g, int ldg, int coff, int H, int W,
                                    CatSrc s, void* dsrc, int ldd, int dsd, int acc,
                                    float* __restrict__ dscale) {
  const int n = blockIdx.z;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int pl = threadIdx.x >> 6;
  const long P = (long)H * W;
  const long p0 = (long)blockIdx.x * BWD_CHUNK, p1 = min(P, p0 + BWD_CHUNK);
  float ds = 0.f;
  if (c < s.C) {
    const float sc = s.scale ? s.scale[n * s.C + c] : 1.f;
    for (long p = p0 + pl; p < p1; p += 4) {
      const long pix = (long)n * P + p;
      const float gv = to_f32(g[pix * ldg + coff + c]);
      if (dsrc) st_any(dsrc, pix * ldd + c, dsd, gv * sc, acc);
      if (dscale) ds += gv * ld_any(s.ptr, pix * s.ld + c, s.dtype);
    }
  }
  if (dscale) {
    __shared__ float red[4][64];
    red[pl][threadIdx.x & 63] = ds;
    __syncthreads();
    if (pl == 0 && c < s.C)
      atomicAdd(&dscale[n * s.C + c], red[0][c & 63] + red[1][c & 63] + red[2][c & 63] +
                                          red[3][c & 63]);
  }
}

// UP2 adjoint: low-res pixel (py, px) gathers from the high-res pixels whose
// bilinear taps hit it (recomputing the forward's indices/weights exactly).
__device__ __forceinline__ int up_adj(int j, int in, int out, int* idx, float* wt) {
  // candidates i with i0(i)==j or i1(i)==j ; scale ~ in/out
  int cnt = 0;
  const float sc = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  int lo = sc > 0.f ? (int)floorf((j - 1) / sc) - 1 : 0;
  int hi = sc > 0.f ? (int)ceilf((j + 1) / sc) + 1 : out - 1;
  if (lo < 0) lo = 0;
  if (hi > out - 1) hi = out - 1;
  for (int i = lo; i <= hi && cnt < 8; ++i) {
    int i0, i1;
    float l1;
    up_index(i, in, out, i0, i1, l1);
    float w = 0.f;
    if (i0 == j) w += 1.f - l1;
    if (i1 == j) w += l1;
    if (w != 0.f || i0 == j || i1 == j) {
      idx[cnt] = i;
      wt[cnt] = w;
      ++cnt;
    }
  }
  return cnt;
}

template <typename T>
__global__ void cat_bwd_up2_kernel(const T* __restrict__ g, int ldg, int coff, int H, int W,
                                   CatSrc s, void* dsrc, int ldd, int dsd, int acc,
                                   float* __restrict__ dscale) {
  const int n = blockIdx.z;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int pl = threadIdx.x >> 6;
  const long P = (long)s.h * s.w;
  const long p0 = (long)blockIdx.x * BWD_CHUNK, p1 = min(P, p0 + BWD_CHUNK);
  float ds = 0.f;
  if (c < s.C) {
    const float sc = s.scale ? s.scale[n * s.C + c] : 1.f;
    for (long p = p0 + pl; p < p1; p += 4) {
      const int py = p / s.w, px = p % s.w;
      int yi[8], xi[8];
      float yw[8], xw[8];
      const int ny = up_adj(py, s.h, H, yi, yw);
      const int nx = up_adj(px, s.w, W, xi, xw);
      float gv = 0.f;
      for (int a = 0; a < ny; ++a)
        for (int b = 0; b < nx; ++b)
          gv += yw[a] * xw[b] * to_f32(g[((long)(n * H + yi[a]) * W + xi[b]) * ldg + coff + c]);
      const long sp = (long)n * P + p;
      if (dsrc) st_any(dsrc, sp * ldd + c, dsd, gv * sc, acc);
      if (dscale) ds += gv * ld_any(s.ptr, sp * s.ld + c, s.dtype);
    }
  }
  if (dscale) {
    __shared__ float red[4][64];
    red[pl][threadIdx.x & 63] = ds;
    __syncthreads();
    if (pl == 0 && c < s.C)
      atomicAdd(&dscale[n * s.C + c], red[0][c & 63] + red[1][c & 63] + red[2][c & 63] +
                                          red[3][c & 63]);
  }
}

template <typename T>
__global__ void cat_bwd_pshuf_kernel(const T* __restrict__ g, int ldg, int coff, int H, int W,
                                     CatSrc s, void* dsrc, int ldd, int dsd, int acc) {
  // thread per source element (n, p, q, cs), cs in [0, 4C)
  const long total = (long)gridDim.z * s.h * s.w * 4 * s.C;
  (void)total;
  const int n = blockIdx.z;
  const int C4 = 4 * s.C;
  const long P = (long)s.h * s.w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P * C4;
       i += (long)gridDim.x * blockDim.x) {
    const int cs = i % C4;
    const long p = i / C4;
    const int py = p / s.w, px = p % s.w;
    const int c = cs >> 2, yy = 2 * py + ((cs >> 1) & 1), xx = 2 * px + (cs & 1);
    const float gv = to_f32(g[((long)(n * H + yy) * W + xx) * ldg + coff + c]);
    st_any(dsrc, ((long)n * P + p) * ldd + cs, dsd, gv, acc);
  }
}

// ---- SE
template <typename T>
__global__ void channel_mean_kernel(const T* __restrict__ x, int ld, long S, int C,
                                    float* __restrict__ out) {
  const int n = blockIdx.z;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int pl = threadIdx.x >> 6;
  const long p0 = (long)blockIdx.x * 1024, p1 = min(S, p0 + 1024);
  float t = 0.f;
  if (c < C)
    for (long p = p0 + pl; p < p1; p += 4) t += to_f32(x[((long)n * S + p) * ld + c]);
  __shared__ float red[4][64];
  red[pl][threadIdx.x & 63] = t;
  __syncthreads();
  if (pl == 0 && c < C)
    atomicAdd(&out[n * C + c],
              (red[0][c & 63] + red[1][c & 63] + red[2][c & 63] + red[3][c & 63]) / (float)S);
}

__global__ void se_mlp_fwd_kernel(const float* __restrict__ pooled, const float* __restrict__ w1,
                                  const float* __restrict__ w2, int C, int R,
                                  float* __restrict__ z1, float* __restrict__ s) {
  extern __shared__ float sh[];
  const int n = blockIdx.x;
  float* p = sh;       // [C]
  float* z = sh + C;   // [R]
  for (int c = threadIdx.x; c < C; c += blockDim.x) p[c] = pooled[n * C + c];
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    float t = 0.f;
    for (int c = 0; c < C; ++c) t += w1[r * C + c] * p[c];
    t = fmaxf(t, 0.f);
    z[r] = t;
    z1[n * R + r] = t;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float t = 0.f;
    for (int r = 0; r < R; ++r) t += w2[c * R + r] * z[r];
    s[n * C + c] = sigmoidf_(t);
  }
}

// single block; dw1 [R][C], dw2 [C][R] accumulated; dpool_scaled[n][c] = dpool / S
__global__ void se_mlp_bwd_kernel(int N, int C, int R, const float* __restrict__ ds,
                                  const float* __restrict__ s, const float* __restrict__ z1,
                                  const float* __restrict__ pooled, const float* __restrict__ w1,
                                  const float* __restrict__ w2, float* __restrict__ dw1,
                                  float* __restrict__ dw2, float* __restrict__ dpool,
                                  float inv_S) {
  extern __shared__ float sh[];
  float* dl2 = sh;            // [N][C]
  float* dz = sh + N * C;     // [N][R]
  for (int i = threadIdx.x; i < N * C; i += blockDim.x) {
    const float sv = s[i];
    dl2[i] = ds[i] * sv * (1.f - sv);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N * R; i += blockDim.x) {
    const int n = i / R, r = i % R;
    float t = 0.f;
    for (int c = 0; c < C; ++c) t += w2[c * R + r] * dl2[n * C + c];
    dz[i] = z1[i] > 0.f ? t : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * R; i += blockDim.x) {
    const int c = i / R, r = i % R;  // dw2[c][r]
    float t = 0.f;
    for (int n = 0; n < N; ++n) t += dl2[n * C + c] * z1[n * R + r];
    dw2[i] += t;
  }
  for (int i = threadIdx.x; i < R * C; i += blockDim.x) {
    const int r = i / C, c = i % C;  // dw1[r][c]
    float t = 0.f;
    for (int n = 0; n < N; ++n) t += dz[n * R + r] * pooled[n * C + c];
    dw1[i] += t;
  }
  for (int i = threadIdx.x; i < N * C; i += blockDim.x) {
    const int n = i / C, c = i % C;
    float t = 0.f;
    for (int r = 0; r < R; ++r) t += w1[r * C + c] * dz[n * R + r];
    dpool[i] = t * inv_S;
  }
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

int um_concat_build(int dtype, int N, int H, int W, void* dst, int ld, int Ctot, int nsrc,
                    const um_cat_src* srcs, hipStream_t st) {
  UM_CHECK_ARG(nsrc >= 1 && nsrc <= MAX_SRC, "um_concat_build: nsrc %d", nsrc);
  CatArgs a{};
  a.nsrc = nsrc;
  for (int i = 0; i < nsrc; ++i) {
    const um_cat_src& s = srcs[i];
    a.s[i] = CatSrc{s.ptr, s.scale, s.C, s.ld, s.op, s.coff, s.dtype, s.h, s.w};
    UM_CHECK_ARG(s.coff + s.C <= Ctot, "um_concat_build: source %d exceeds Ctot", i);
    UM_CHECK_ARG(s.op != UM_CAT_COPY || (s.h == H && s.w == W), "um_concat_build: copy size");
    UM_CHECK_ARG(s.op == UM_CAT_COPY || (2 * s.h == H && 2 * s.w == W), "um_concat_build: x2 size");
  }
  const long total = (long)N * H * W * Ctot;
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(concat_build_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, a, N,
                       H, W, Ctot, (bf16_t*)dst, ld);
  else
    hipLaunchKernelGGL(concat_build_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, a, N,
                       H, W, Ctot, (float*)dst, ld);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_concat_bwd_src(int dtype, int N, int H, int W, const void* g, int ldg,
                      const um_cat_src* src, void* dsrc, int ldd, int dsrc_dtype, int accumulate,
                      float* dscale, hipStream_t st) {
  const um_cat_src& s0 = *src;
  CatSrc s{s0.ptr, s0.scale, s0.C, s0.ld, s0.op, s0.coff, s0.dtype, s0.h, s0.w};
  if (s.op == UM_CAT_PSHUF) {
    UM_CHECK_ARG(dsrc != nullptr && dscale == nullptr, "um_concat_bwd_src: pshuf args");
    const long per_n = (long)s.h * s.w * 4 * s.C;
    dim3 grid((unsigned)std::min<long>((per_n + 255) / 256, 2048), 1, N);
    if (dtype == UM_BF16)
      hipLaunchKernelGGL(cat_bwd_pshuf_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)g,
                         ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate);
    else
      hipLaunchKernelGGL(cat_bwd_pshuf_kernel<float>, grid, dim3(256), 0, st, (const float*)g, ldg,
                         s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate);
  } else {
    const long P = (long)s.h * s.w;
    dim3 grid(ceil_div(P, BWD_CHUNK), ceil_div(s.C, 64), N);
    if (s.op == UM_CAT_COPY) {
      if (dtype == UM_BF16)
        hipLaunchKernelGGL(cat_bwd_copy_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)g,
                           ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, dscale);
      else
        hipLaunchKernelGGL(cat_bwd_copy_kernel<float>, grid, dim3(256), 0, st, (const float*)g,
                           ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, dscale);
    } else {
      if (dtype == UM_BF16)
        hipLaunchKernelGGL(cat_bwd_up2_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)g,
                           ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, dscale);
      else
        hipLaunchKernelGGL(cat_bwd_up2_kernel<float>, grid, dim3(256), 0, st, (const float*)g,
                           ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, dscale);
    }
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_channel_mean(int dtype, int N, long S, int C, const void* x, int ld, float* out,
                    hipStream_t st) {
  dim3 grid(ceil_div(S, 1024), ceil_div(C, 64), N);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(channel_mean_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, ld,
                       S, C, out);
  else
    hipLaunchKernelGGL(channel_mean_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ld, S,
                       C, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_se_mlp_fwd(int N, int C, int R, const float* pooled, const float* w1, const float* w2,
                  float* z1, float* s, hipStream_t st) {
  hipLaunchKernelGGL(se_mlp_fwd_kernel, dim3(N), dim3(256), (C + R) * sizeof(float), st, pooled,
                     w1, w2, C, R, z1, s);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_se_mlp_bwd(int N, int C, int R, const float* ds, const float* s, const float* z1,
                  const float* pooled, const float* w1, const float* w2, float* dw1, float* dw2,
                  float* dpool_scaled, float inv_S, hipStream_t st) {
  const size_t shm = ((size_t)N * C + (size_t)N * R) * sizeof(float);
  UM_CHECK_ARG(shm <= 64 * 1024, "um_se_mlp_bwd: N*C too large (%d x %d)", N, C);
  hipLaunchKernelGGL(se_mlp_bwd_kernel, dim3(1), dim3(256), shm, st, N, C, R, ds, s, z1, pooled,
                     w1, w2, dw1, dw2, dpool_scaled, inv_S);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
