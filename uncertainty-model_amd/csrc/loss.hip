// Monodepth-style loss stack with uncertainty: image pyramid, bilinear
// reconstruction and the fused 4-scale loss, forward + analytic backward.
// Reference: train/utils.py:27-135 (pyramid, bilinear warp) and
// train/loss.py:15-264,340-434,512-568 (WSSIM, L-R consistency, edge-aware
// smoothness, reprojection-error NLL, Tukra total).
//
// Images are NCHW f32 [N][6][h][w] (left = channels 0-2, right = 3-5).
// Predictions are the disp head's NHWC f32 [N][h][w][4]: channel 0/1 =
// left/right disparity, 2/3 = left/right uncertainty.
//
// Warp (F6): sample x = ((2*(lin(j)+shift) - 1) + 1) * W/2 - 0.5 with
// lin = torch.linspace(0,1,W) in f32, y likewise with shift 0; bilinear,
// zero padding (grid_sample align_corners=False).
//
// Launch structure (one step, all scales):
//   um_pyramid         ONE launch, every level (level 0 = exact copy)
//   um_recon_pyramid   ONE launch, every level and both views
//   um_loss_fwd        every scale, both views, the six loss terms as f64
//                      per-tile sums, then a one-workgroup launch that
//                      reduces them in a fixed order.  With gpart (a step that
//                      will differentiate the loss) the tile launch is
//                      loss_grad_kernel<true>: the terms AND the gradient per
//                      unit gout from one pass over the tiles.
//   um_loss_bwd        with gpart: ONE launch (the consistency scatter, which
//                      scales and completes the partials); without: the
//                      scatter, then loss_grad_kernel<false>.
// The loss kernels do not read the reconstruction: each tile re-warps the
// opposite view itself (the recon of a pixel is 12 L2-resident taps), so
// the WSSIM term's gradient through the warp is computed in place.  The
// consistency terms' gradient w.r.t. the warped (opposite) disparity is a
// data-dependent scatter along the row; the warp moves rows by < 1, so a
// workgroup that owns a strip of rows takes the scatter of the source rows
// one above and one below it as well and accumulates in LDS: no atomics to
// global memory, every gradient element is stored exactly once.
#include "common.h"
#include "igemm.h"

namespace {

constexpr int MAXS = 6;  // pyramid levels handled by one launch

// arr[i] for a wave-uniform i without dynamically indexing a by-value kernel
// argument (which would copy the array to scratch): unrolled selects
template <typename T>
__device__ __forceinline__ T pick(const T* arr, int i) {
  T v = arr[0];
#pragma unroll
  for (int k = 1; k < MAXS; ++k)
    if (k == i) v = arr[k];
  return v;
}
template <typename T>
__device__ __forceinline__ T pick1(const T* arr, int i) {  // arrays of MAXS + 1
  T v = arr[0];
#pragma unroll
  for (int k = 1; k <= MAXS; ++k)
    if (k == i) v = arr[k];
  return v;
}

__device__ __forceinline__ float lin01(int i, int n) {
  // torch.linspace(0, 1, n) (CPU kernel: symmetric halves)
  if (n <= 1) return 0.f;
  const float step = 1.f / (float)(n - 1);
  return (i < n / 2) ? step * (float)i : 1.f - step * (float)(n - 1 - i);
}

struct Samp {
  int x0, y0;
  float w, e, n, s;  // torch naming: w = x - x0, e = 1 - w, n = y - y0, s = 1 - n
};

__device__ __forceinline__ Samp warp_at(int x, int y, float shift, int W, int H) {
  const float gx = 2.f * (lin01(x, W) + shift) - 1.f;
  const float gy = 2.f * lin01(y, H) - 1.f;
  const float ix = (gx + 1.f) * ((float)W * 0.5f) - 0.5f;
  const float iy = (gy + 1.f) * ((float)H * 0.5f) - 0.5f;
  Samp t;
  const float fx = floorf(ix), fy = floorf(iy);
  t.x0 = (int)fx;
  t.y0 = (int)fy;
  t.w = ix - fx;
  t.e = 1.f - t.w;
  t.n = iy - fy;
  t.s = 1.f - t.n;
  return t;
}

// value of plane at (y, x) with zero padding; plane element (y,x) at p[(y*W + x) * st]
__device__ __forceinline__ float pv(const float* p, int y, int x, int H, int W, long st) {
  return (x >= 0 && x < W && y >= 0 && y < H) ? p[((long)y * W + x) * st] : 0.f;
}

// sample value and d(value)/d(ix)
__device__ __forceinline__ float sample(const float* p, const Samp& t, int H, int W, long st,
                                        float* dix) {
  const float nw = pv(p, t.y0, t.x0, H, W, st), ne = pv(p, t.y0, t.x0 + 1, H, W, st);
  const float sw = pv(p, t.y0 + 1, t.x0, H, W, st), se = pv(p, t.y0 + 1, t.x0 + 1, H, W, st);
  if (dix) *dix = t.s * (ne - nw) + t.n * (se - sw);
  return nw * (t.s * t.e) + ne * (t.s * t.w) + sw * (t.n * t.e) + se * (t.n * t.w);
}

__device__ __forceinline__ void up_index(int i, int in, int out, int& i0, int& i1, float& l1) {
  const float sc = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float src = sc * (float)i;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = src - (float)i0;
}

// adjoint of ones under the 1D align_corners upsample in -> out, at index j
__device__ float up_adj_sum(int j, int in, int out) {
  const float sc = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  int lo = sc > 0.f ? (int)floorf((j - 1) / sc) - 1 : 0;
  int hi = sc > 0.f ? (int)ceilf((j + 1) / sc) + 1 : out - 1;
  lo = max(lo, 0);
  hi = min(hi, out - 1);
  float u = 0.f;
  for (int i = lo; i <= hi; ++i) {
    int i0, i1;
    float l1;
    up_index(i, in, out, i0, i1, l1);
    if (i0 == j) u += 1.f - l1;
    if (i1 == j) u += l1;
  }
  return u;
}

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) - (x < 0.f); }

// The same warp with the per-image constants hoisted: lin01 with a
// precomputed step, the row part (which does not depend on the shift) from a
// per-row table.  Bit-identical to warp_at.
struct RowW {
  int y0;
  float n;  // iy - y0
};
__device__ __forceinline__ float lin01s(int i, int n, int half, float step) {
  return n <= 1 ? 0.f : (i < half) ? step * (float)i : 1.f - step * (float)(n - 1 - i);
}
__device__ __forceinline__ RowW row_w(int y, int H) {
  const float gy = 2.f * lin01(y, H) - 1.f;
  const float iy = (gy + 1.f) * ((float)H * 0.5f) - 0.5f;
  const float fy = floorf(iy);
  RowW r;
  r.y0 = (int)fy;
  r.n = iy - fy;
  return r;
}
__device__ __forceinline__ Samp warp_tab(float linx, const RowW& rw, float shift, float Wh) {
  const float gx = 2.f * (linx + shift) - 1.f;
  const float ix = (gx + 1.f) * Wh - 0.5f;
  Samp t;
  const float fx = floorf(ix);
  t.x0 = (int)fx;
  t.y0 = rw.y0;
  t.w = ix - fx;
  t.e = 1.f - t.w;
  t.n = rw.n;
  t.s = 1.f - rw.n;
  return t;
}

constexpr float C1 = 0.01f * 0.01f;
constexpr float C2 = 0.03f * 0.03f;

// SSIM of one channel over the 3x3 window whose top-left is (r, q) of the
// staged tiles (reference train/loss.py:43-74: valid 3x3 average pools)
struct Stats {
  float mx, my, vx, vy, vxy;
};
template <int RX>
__device__ __forceinline__ Stats win_stats(const float (*I)[RX], const float (*R)[RX], int r,
                                           int q) {
  float sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float xv = I[r + u][q + w], yv = R[r + u][q + w];
      sx += xv; sy += yv; sxx += xv * xv; syy += yv * yv; sxy += xv * yv;
    }
  // the 3x3 mean as a multiply by 1/9 (within an ulp of the reference's
  // avg_pool division; an IEEE division here is ~10 instructions)
  constexpr float k9 = 1.f / 9.f;
  Stats st;
  st.mx = sx * k9;
  st.my = sy * k9;
  st.vx = sxx * k9 - st.mx * st.mx;
  st.vy = syy * k9 - st.my * st.my;
  st.vxy = sxy * k9 - st.mx * st.my;
  return st;
}
__device__ __forceinline__ float ssim_of(const Stats& t) {
  return ((2 * t.mx * t.my + C1) * (2 * t.vxy + C2)) /
         ((t.mx * t.mx + t.my * t.my + C1) * (t.vx + t.vy + C2));
}

// ----------------------------------------------------------------- pyramid --
struct PyrArgs {
  const float* x;
  float* out[MAXS];
  long off[MAXS + 1];  // work-item offsets: level 0 in float4 items, others per element
  int NC, H, W, nlev;
};

__global__ void pyramid_kernel(PyrArgs a) {
  const long total = pick1(a.off, a.nlev);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    if (i < a.off[1]) {  // level 0: interpolate to the same size = exact copy
      reinterpret_cast<float4*>(a.out[0])[i] = reinterpret_cast<const float4*>(a.x)[i];
      continue;
    }
    int l = 1;
#pragma unroll
    for (int k = 2; k < MAXS; ++k)
      if (k < a.nlev && i >= a.off[k]) l = k;
    const long j = i - pick1(a.off, l);
    const int h = a.H >> l, w = a.W >> l;
    const int xo = j % w;
    const int yo = (j / w) % h;
    const long pl = j / ((long)w * h);
    const float* p = a.x + pl * a.H * a.W;
    int y0, y1, x0, x1;
    float ly, lx;
    up_index(yo, a.H, h, y0, y1, ly);
    up_index(xo, a.W, w, x0, x1, lx);
    const long W = a.W;
    pick(a.out, l)[j] = (1.f - ly) * ((1.f - lx) * p[y0 * W + x0] + lx * p[y0 * W + x1]) +
                  ly * ((1.f - lx) * p[y1 * W + x0] + lx * p[y1 * W + x1]);
  }
}

// ------------------------------------------------------------------- warp --
// out[n][c][y][x] = sample(img[n][c], shift = sign * disp[n][y][x])
__global__ void warp_kernel(const float* __restrict__ img, int N, int C, int H, int W,
                            const float* __restrict__ disp, long dsn, long dsp, float sign,
                            float* __restrict__ out) {
  const long total = (long)N * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = i % W;
    const int y = (i / W) % H;
    const int n = i / ((long)W * H);
    const float d = disp[n * dsn + ((long)y * W + x) * dsp];
    const Samp t = warp_at(x, y, sign * d, W, H);
    for (int c = 0; c < C; ++c) {
      const float* p = img + ((long)n * C + c) * H * W;
      out[(((long)n * C + c) * H + y) * W + x] = sample(p, t, H, W, 1, nullptr);
    }
  }
}

// d(sum_c gout * warp)/d(disp) at each pixel: gdisp = sum_c gout_c * dix_c * sign * W
// (the image operand is data: no gradient)
__global__ void warp_bwd_kernel(const float* __restrict__ img, int N, int C, int H, int W,
                                const float* __restrict__ disp, long dsn, long dsp, float sign,
                                const float* __restrict__ gout, float* __restrict__ gdisp,
                                long gsn, long gsp) {
  const long total = (long)N * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = i % W;
    const int y = (i / W) % H;
    const int n = i / ((long)W * H);
    const float d = disp[n * dsn + ((long)y * W + x) * dsp];
    const Samp t = warp_at(x, y, sign * d, W, H);
    float g = 0.f;
    for (int c = 0; c < C; ++c) {
      const float* p = img + ((long)n * C + c) * H * W;
      float dix;
      sample(p, t, H, W, 1, &dix);
      g += gout[(((long)n * C + c) * H + y) * W + x] * dix;
    }
    gdisp[n * gsn + ((long)y * W + x) * gsp] = g * sign * (float)W;
  }
}

// reconstruct_pyramid: every level, both views.  out[l][n][0..2] = left
// recon = warp(right image, -d_L), out[l][n][3..5] = right recon = warp(left
// image, +d_R) (reference train/utils.py:112-135)
struct ReconArgs {
  const float* img[MAXS];
  const float* pred[MAXS];
  float* out[MAXS];
  long psn[MAXS], psc[MAXS], psp[MAXS];  // prediction strides (image, channel, pixel)
  long off[MAXS + 1];
  int N, H, W, nlev;
};

__global__ void recon_kernel(ReconArgs a) {
  const long total = pick1(a.off, a.nlev);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int l = 0;
#pragma unroll
    for (int k = 1; k < MAXS; ++k)
      if (k < a.nlev && i >= a.off[k]) l = k;
    const long j = i - pick1(a.off, l);
    const int H = a.H >> l, W = a.W >> l;
    const long HW = (long)H * W;
    const int x = j % W;
    const int y = (j / W) % H;
    const int n = j / HW;
    const float* pp = pick(a.pred, l) + n * pick(a.psn, l) + ((long)y * W + x) * pick(a.psp, l);
    const float* im = pick(a.img, l) + (long)n * 6 * HW;
    float* o = pick(a.out, l) + (long)n * 6 * HW + (long)y * W + x;
    const long psc = pick(a.psc, l);
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const float d = pp[v * psc];
      const Samp t = warp_at(x, y, v == 0 ? -d : d, W, H);
      const float* op = im + (long)(1 - v) * 3 * HW;
#pragma unroll
      for (int c = 0; c < 3; ++c) o[(v * 3 + c) * HW] = sample(op + c * HW, t, H, W, 1, nullptr);
    }
  }
}

// --------------------------------------------------------- fused loss ------
struct LScale {
  const float* img;   // [N][6][h][w]
  const float* pred;  // NHWC [N][h][w][4]
  float* dpred;       // bwd output NHWC [N][h][w][4]
  float* gpart;       // gradient partials per unit gout (see loss_grad_kernel<true>)
  int h, w, tiles_x, tiles_y, block0;
};

// per-scale geometry as separate arrays (struct of arrays): a workgroup picks
// its scale's fields with uniform selects
struct LArgs {
  const float* img[MAXS];
  const float* pred[MAXS];
  float* dpred[MAXS];
  float* gpart[MAXS];  // fused forward: per-unit-gout gradient partials NHWC [N][h][w][4]
  int h[MAXS], w[MAXS], tiles_x[MAXS], tiles_y[MAXS], block0[MAXS];
  int nscales, N, nblocks;
  float alpha;
  int loss_type;   // 0 l1, 1 bayesian, 2 log_bayesian
  float esw, ecw;  // error-loss smoothness / consistency weights
  float w_wssim, w_cons, w_smooth, w_err;
  double* parts;      // fwd: [nblocks][8] f64 partial terms
  float* emap;        // fwd: error map of the last scale [N][2][h][w] (or null)
  float* rec[MAXS];   // fwd (optional): the reconstruction [N][6][h][w] as a side output
  float* out;         // fwd: [6] disp_loss, error_loss, wssim, consistency, smoothness, error
  float* disp_loss;    // fwd (optional): out[0] again
  float* error_loss;   // fwd (optional): out[1] again
  const float* gout_d;  // bwd: d total / d disp_loss (a device scalar; null = 0)
  const float* gout_e;  // bwd: d total / d error_loss (null = 0)
};

__device__ __forceinline__ float gval(const float* p) { return p != nullptr ? *p : 0.f; }

__device__ __forceinline__ int scale_of(const LArgs& a, int b) {
  int s = 0;
#pragma unroll
  for (int k = 1; k < MAXS; ++k)
    if (k < a.nscales && b >= a.block0[k]) s = k;
  return s;
}
__device__ __forceinline__ LScale scale_desc(const LArgs& a, int s) {
  LScale S;
  S.img = pick(a.img, s);
  S.pred = pick(a.pred, s);
  S.dpred = pick(a.dpred, s);
  S.gpart = pick(a.gpart, s);
  S.h = pick(a.h, s);
  S.w = pick(a.w, s);
  S.tiles_x = pick(a.tiles_x, s);
  S.tiles_y = pick(a.tiles_y, s);
  S.block0 = pick(a.block0, s);
  return S;
}


// ---------------------------------------------------------- tile staging --
// A tile of TY x TX pixels of one image, scale and view.  Staged region =
// rows [ty0-2, ty0+TY+3), cols [tx0-2, tx0+TX+3): the pixels, the SSIM
// windows of the DSSIM grid points the tile's upsample reads (grid rows
// [ty0-2, ty0+TY]) and the smoothness neighbours.  Out-of-image positions
// hold zeros.  Loads are issued in groups of G independent positions
// (branch-free: clamped addresses, selects), so each thread keeps ~G*15
// loads in flight instead of one dependent chain at a time.
template <int TY, int TX>
struct Tile {
  static constexpr int RY = TY + 5, RX = TX + 5;  // staged region
  static constexpr int GY = TY + 3, GX = TX + 3;  // grid points
  static constexpr int NP = RY * RX;
};

__device__ __forceinline__ float ldc(const float* p, int y, int x, int H, int W, int st) {
  // plane value at (y, x), zero outside (address clamped: no branch)
  const bool in = x >= 0 && x < W && y >= 0 && y < H;
  const int yy = min(max(y, 0), H - 1), xx = min(max(x, 0), W - 1);
  const float v = p[(yy * W + xx) * st];
  return in ? v : 0.f;
}

// the two horizontal taps (y, x) and (y, x + 1) of a plane, zero outside,
// as one dword-aligned 8-byte load (W >= 2; address clamped: no branch)
__device__ __forceinline__ void ldc2(const float* p, int y, int x, int H, int W, float& lo,
                                     float& hi) {
  const bool yin = y >= 0 && y < H;
  const int yy = min(max(y, 0), H - 1), xs = min(max(x, 0), W - 2);
  float2 v;
  __builtin_memcpy(&v, p + yy * W + xs, sizeof(v));
  const bool mid = x >= 0 && x <= W - 2;
  lo = yin && mid ? v.x : (yin && x == W - 1 ? v.y : 0.f);
  hi = yin && mid ? v.y : (yin && x == -1 ? v.x : 0.f);
}

// per-tile coordinate tables (LDS): lin01 of the staged columns, the warp's
// row part of the staged rows, and the DSSIM upsample taps of the pixel rows
// and columns (relative to the grid tile origin ty0-2 / tx0-2)
struct UpTap {
  int i0, i1;
  float l1;
};
template <int TY, int TX>
struct Tabs {
  float lin[Tile<TY, TX>::RX];
  RowW row[Tile<TY, TX>::RY];
  UpTap uy[TY], ux[TX];
};
template <int TY, int TX>
__device__ __forceinline__ void init_tabs(Tabs<TY, TX>& tb, int H, int W, int ty0, int tx0) {
  using T = Tile<TY, TX>;
  for (int i = threadIdx.x; i < T::RX + T::RY + TY + TX; i += blockDim.x) {
    if (i < T::RX) {
      tb.lin[i] = lin01(tx0 - 2 + i, W);
    } else if (i < T::RX + T::RY) {
      const int r = i - T::RX;
      tb.row[r] = row_w(ty0 - 2 + r, H);
    } else if (i < T::RX + T::RY + TY) {
      const int r = i - T::RX - T::RY;
      UpTap u;
      up_index(min(ty0 + r, H - 1), H - 2, H, u.i0, u.i1, u.l1);
      u.i0 -= ty0 - 2;
      u.i1 -= ty0 - 2;
      tb.uy[r] = u;
    } else {
      const int q = i - T::RX - T::RY - TY;
      UpTap u;
      up_index(min(tx0 + q, W - 1), W - 2, W, u.i0, u.i1, u.l1);
      u.i0 -= tx0 - 2;
      u.i1 -= tx0 - 2;
      tb.ux[q] = u;
    }
  }
}

// predictions of the staged region, float4 per pixel (d_L, d_R, s_L, s_R)
template <int TY, int TX, int NT = 256>
__device__ __forceinline__ void stage_pred(const float* pp, int H, int W, int ty0, int tx0,
                                           float4 (*sP)[Tile<TY, TX>::RX]) {
  using T = Tile<TY, TX>;
  constexpr int K = (T::NP + NT - 1) / NT;
  float4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = min((int)threadIdx.x + k * NT, T::NP - 1);
    const int r = i / T::RX, q = i - (i / T::RX) * T::RX;
    const int y = ty0 - 2 + r, x = tx0 - 2 + q;
    const bool in = x >= 0 && x < W && y >= 0 && y < H;
    const int yy = min(max(y, 0), H - 1), xx = min(max(x, 0), W - 1);
    v[k] = *reinterpret_cast<const float4*>(pp + ((long)yy * W + xx) * 4);
    if (!in) v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < T::NP) sP[i / T::RX][i % T::RX] = v[k];
  }
}

__device__ __forceinline__ float comp(const float4& v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// image of view v and its reconstruction (warp of the opposite view by
// sign * d_v); with DIX also d(recon_c)/d(ix) at the TY x TX pixels
template <int TY, int TX, bool DIX, int NT = 256>
__device__ __forceinline__ void stage_view(const float* Iv, const float* Io, int H, int W, int HW,
                                           int ty0, int tx0, int v, const Tabs<TY, TX>& tb,
                                           const float4 (*sP)[Tile<TY, TX>::RX],
                                           float (*sI)[Tile<TY, TX>::RY][Tile<TY, TX>::RX],
                                           float (*sR)[Tile<TY, TX>::RY][Tile<TY, TX>::RX],
                                           float (*sX)[TY][TX]) {
  using T = Tile<TY, TX>;
  constexpr int K = (T::NP + NT - 1) / NT;
  constexpr int G = 2;
  const float sign = v == 0 ? -1.f : 1.f;
  const float Wh = (float)W * 0.5f;
#pragma unroll 1
  for (int k0 = 0; k0 < K; k0 += G) {
    int r[G], q[G];
    bool in[G];
    Samp t[G];
    int own[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int i = min((int)threadIdx.x + (k0 + g) * NT, T::NP - 1);
      r[g] = i / T::RX;
      q[g] = i - r[g] * T::RX;
      const int y = ty0 - 2 + r[g], x = tx0 - 2 + q[g];
      in[g] = x >= 0 && x < W && y >= 0 && y < H;
      own[g] = min(max(y, 0), H - 1) * W + min(max(x, 0), W - 1);
      t[g] = warp_tab(tb.lin[q[g]], tb.row[r[g]], sign * comp(sP[r[g]][q[g]], v), Wh);
    }
    float iv[G][3], tp[G][3][4];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        iv[g][c] = Iv[c * HW + own[g]];
        const float* op = Io + c * HW;
        ldc2(op, t[g].y0, t[g].x0, H, W, tp[g][c][0], tp[g][c][1]);
        ldc2(op, t[g].y0 + 1, t[g].x0, H, W, tp[g][c][2], tp[g][c][3]);
      }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int i = threadIdx.x + (k0 + g) * NT;
      if (k0 + g >= K || i >= T::NP) continue;
      const Samp& u = t[g];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float nw = tp[g][c][0], ne = tp[g][c][1], sw = tp[g][c][2], se = tp[g][c][3];
        const float rv = nw * (u.s * u.e) + ne * (u.s * u.w) + sw * (u.n * u.e) + se * (u.n * u.w);
        sI[c][r[g]][q[g]] = in[g] ? iv[g][c] : 0.f;
        sR[c][r[g]][q[g]] = in[g] ? rv : 0.f;
        if (DIX) {
          const int ly = r[g] - 2, lx = q[g] - 2;
          if (ly >= 0 && ly < TY && lx >= 0 && lx < TX)
            sX[c][ly][lx] = u.s * (ne - nw) + u.n * (se - sw);
        }
      }
    }
  }
}

// opposite-disparity samples for the consistency terms of NPX pixels:
// value and d/d(ix) of the bilinear sample of plane opp (pixel stride 4)
template <int NPX>
__device__ __forceinline__ void cons_samples(const float* opp, int H, int W, const Samp* t,
                                             float* wv, float* dix) {
  float tp[NPX][4];
#pragma unroll
  for (int k = 0; k < NPX; ++k) {
    tp[k][0] = ldc(opp, t[k].y0, t[k].x0, H, W, 4);
    tp[k][1] = ldc(opp, t[k].y0, t[k].x0 + 1, H, W, 4);
    tp[k][2] = ldc(opp, t[k].y0 + 1, t[k].x0, H, W, 4);
    tp[k][3] = ldc(opp, t[k].y0 + 1, t[k].x0 + 1, H, W, 4);
  }
#pragma unroll
  for (int k = 0; k < NPX; ++k) {
    const Samp& u = t[k];
    wv[k] = tp[k][0] * (u.s * u.e) + tp[k][1] * (u.s * u.w) + tp[k][2] * (u.n * u.e) +
            tp[k][3] * (u.n * u.w);
    if (dix) dix[k] = u.s * (tp[k][1] - tp[k][0]) + u.n * (tp[k][3] - tp[k][2]);
  }
}

// DSSIM upsampled to pixel (ly, lx) of the tile from the grid tile
template <int GX>
__device__ __forceinline__ float dssim_up(const float (*sD)[GX], const UpTap& uy,
                                          const UpTap& ux) {
  return (1.f - uy.l1) * ((1.f - ux.l1) * sD[uy.i0][ux.i0] + ux.l1 * sD[uy.i0][ux.i1]) +
         uy.l1 * ((1.f - ux.l1) * sD[uy.i1][ux.i0] + ux.l1 * sD[uy.i1][ux.i1]);
}

// Block sums of the six loss terms (f64) into parts[blockIdx.x][0..5]; a
// separate one-workgroup launch (loss_reduce_kernel) scales them per pyramid
// level and sums them in a fixed order (deterministic).  An in-kernel
// "last workgroup" ticket measured slower: every workgroup then waits for its
// partials to land and (on gfx950) writes back its XCD's dirty L2 lines.
template <int NT>
__device__ __forceinline__ void loss_partials(const LArgs& a, const float (&acc)[6],
                                              double (*red)[NT / 64]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const float tsum = wave_sum(acc[k]);
    if ((tid & 63) == 0) red[k][tid >> 6] = (double)tsum;
  }
  __syncthreads();
  if (tid < 6) {
    double r = 0.0;
    for (int w = 0; w < NT / 64; ++w) r += red[tid][w];
    a.parts[(long)blockIdx.x * 8 + tid] = r;
  }
}

constexpr int RNT = 1024;

// out[6] from the block sums: per level s the pixel means (the smoothness
// term also / 2^s, the NLL / 2 and for log_bayesian / 2 again), summed over
// every block in a fixed order, then the weighted totals
__global__ void __launch_bounds__(RNT) loss_reduce_kernel(LArgs a) {
  __shared__ double red[6][RNT / 64];
  __shared__ double fac[MAXS][6];
  const int tid = threadIdx.x;
  if (tid < a.nscales * 6) {
    const int s = tid / 6, k = tid - s * 6;
    const double np = (double)a.N * pick(a.h, s) * pick(a.w, s);
    double f = 1.0 / np;
    if (k == 2) f /= (double)(1 << s);
    if (k == 3) f *= a.loss_type == 2 ? 0.25 : 0.5;
    fac[s][k] = f;
  }
  __syncthreads();
  double q[6] = {0, 0, 0, 0, 0, 0};
  constexpr int U = 4;  // rows in flight per thread (the partials come from other XCDs' L2s)
  for (int b0 = tid; b0 < a.nblocks; b0 += U * RNT) {
    double2 v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = min(b0 + u * RNT, a.nblocks - 1);
      const double2* p = reinterpret_cast<const double2*>(a.parts + (long)b * 8);
      v[u][0] = p[0];
      v[u][1] = p[1];
      v[u][2] = p[2];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + u * RNT;
      if (b >= a.nblocks) break;
      const int s = scale_of(a, b);
      q[0] += v[u][0].x * fac[s][0];
      q[1] += v[u][0].y * fac[s][1];
      q[2] += v[u][1].x * fac[s][2];
      q[3] += v[u][1].y * fac[s][3];
      q[4] += v[u][2].x * fac[s][4];
      q[5] += v[u][2].y * fac[s][5];
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q[k] += __shfl_xor(q[k], o, 64);
  }
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) red[k][tid >> 6] = q[k];
  __syncthreads();
  double f[6];
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      f[k] = 0.0;
      for (int w = 0; w < RNT / 64; ++w) f[k] += red[k][w];
    }
  }
  if (tid == 0) {
    const double ws = f[0], cs = f[1], sm = f[2];
    const double er = f[3] + (double)a.esw * f[5] + (double)a.ecw * f[4];
    a.out[0] = (float)(ws * a.w_wssim + cs * a.w_cons + sm * a.w_smooth);
    a.out[1] = (float)(er * a.w_err);
    if (a.disp_loss != nullptr) *a.disp_loss = a.out[0];
    if (a.error_loss != nullptr) *a.error_loss = a.out[1];
    a.out[2] = (float)ws;
    a.out[3] = (float)cs;
    a.out[4] = (float)sm;
    a.out[5] = (float)er;
  }
}

// ------------------------------------------------------------ forward ------
constexpr int FTY = 16, FTX = 64, FNT = 512;
using FT = Tile<FTY, FTX>;

__device__ __forceinline__ float fdiv(float a, float b) { return __fdividef(a, b); }

__global__ void __launch_bounds__(FNT, 2) loss_fwd_kernel(LArgs a) {
  __shared__ float4 sP[FT::RY][FT::RX];
  __shared__ float sI[3][FT::RY][FT::RX], sR[3][FT::RY][FT::RX];
  __shared__ float sD[FT::GY][FT::GX];
  __shared__ Tabs<FTY, FTX> tb;
  __shared__ double red[6][FNT / 64];
  const int tid = threadIdx.x;
  const int s = scale_of(a, blockIdx.x);
  const LScale S = scale_desc(a, s);
  const int H = S.h, W = S.w;
  const int HW = H * W;
  const int lb = blockIdx.x - S.block0;
  const int per = S.tiles_x * S.tiles_y;
  const int n = lb / per, t = lb - n * per;
  const int ty0 = (t / S.tiles_x) * FTY, tx0 = (t % S.tiles_x) * FTX;
  const float* pp = S.pred + (long)n * HW * 4;
  const float* img = S.img + (long)n * 6 * HW;
  const int gh = H - 2, gw = W - 2;
  const float Wh = (float)W * 0.5f;
  float* const recp = pick(a.rec, s);
  constexpr int KP = FTY * FTX / FNT;  // pixels per thread and view
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  stage_pred<FTY, FTX, FNT>(pp, H, W, ty0, tx0, sP);
  init_tabs<FTY, FTX>(tb, H, W, ty0, tx0);
  __syncthreads();
  for (int v = 0; v < 2; ++v) {
    const float sign = v == 0 ? -1.f : 1.f;
    stage_view<FTY, FTX, false, FNT>(img + v * 3 * HW, img + (1 - v) * 3 * HW, H, W, HW, ty0, tx0,
                                v, tb, sP, sI, sR, nullptr);
    __syncthreads();
    // DSSIM on the valid grid: mean_c clamp((1 - SSIM_c)/2, 0, 1)
    for (int i = tid; i < FT::GY * FT::GX; i += FNT) {
      const int r = i / FT::GX, q = i - (i / FT::GX) * FT::GX;
      const int gy = ty0 - 2 + r, gx = tx0 - 2 + q;
      float dv = 0.f;
      if (gy >= 0 && gy < gh && gx >= 0 && gx < gw) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const Stats st = win_stats<FT::RX>(sI[c], sR[c], r, q);
          const float ss = fdiv((2 * st.mx * st.my + C1) * (2 * st.vxy + C2),
                                (st.mx * st.mx + st.my * st.my + C1) * (st.vx + st.vy + C2));
          dv += fminf(fmaxf((1.f - ss) * 0.5f, 0.f), 1.f);
        }
        dv *= (1.f / 3.f);
      }
      sD[r][q] = dv;
    }
    __syncthreads();
    int ly[KP], lx[KP];
    Samp td[KP], ts[KP];
    float dvv[KP], sgv[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int i = tid + k * FNT;
      ly[k] = i / FTX;
      lx[k] = i - (i / FTX) * FTX;
      const float4 p = sP[ly[k] + 2][lx[k] + 2];
      dvv[k] = comp(p, v);
      sgv[k] = comp(p, 2 + v);
      td[k] = warp_tab(tb.lin[lx[k] + 2], tb.row[ly[k] + 2], sign * dvv[k], Wh);
      ts[k] = warp_tab(tb.lin[lx[k] + 2], tb.row[ly[k] + 2], sign * sgv[k], Wh);
    }
    float wd[KP], ws_[KP];
    cons_samples<KP>(pp + (1 - v), H, W, td, wd, nullptr);
    if (a.ecw != 0.f) cons_samples<KP>(pp + (1 - v), H, W, ts, ws_, nullptr);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int y = ty0 + ly[k], x = tx0 + lx[k];
      if (y >= H || x >= W) continue;
      const int rr = ly[k] + 2, qq = lx[k] + 2;
      const float up = dssim_up<FT::GX>(sD, tb.uy[ly[k]], tb.ux[lx[k]]);
      float l1 = 0.f, gxi = 0.f, gyi = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float iv = sI[c][rr][qq];
        l1 += fabsf(iv - sR[c][rr][qq]);
        gxi += fabsf(iv - sI[c][rr][qq + 1]);
        gyi += fabsf(iv - sI[c][rr + 1][qq]);
      }
      if (x == W - 1) gxi = 0.f;  // replicate-padded gradient (loss.py:208-218)
      if (y == H - 1) gyi = 0.f;
      const float ev = a.alpha * up + (1.f - a.alpha) * (l1 * (1.f / 3.f));
      if (a.emap != nullptr && s == a.nscales - 1)
        a.emap[(n * 2 + v) * HW + y * W + x] = ev;
      if (recp != nullptr)
#pragma unroll
        for (int c = 0; c < 3; ++c) recp[(n * 6 + v * 3 + c) * HW + y * W + x] = sR[c][rr][qq];
      acc[0] += ev;
      const float wxs = __expf(-gxi * (1.f / 3.f)), wys = __expf(-gyi * (1.f / 3.f));
      const float4 p0 = sP[rr][qq], px1 = sP[rr][qq + 1], py1 = sP[rr + 1][qq];
      // edge-aware smoothness of disparity v (and of uncertainty v if weighted)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = v + 2 * kk;
        if (kk == 1 && a.esw == 0.f) continue;
        const float dv = comp(p0, ch);
        const float dgx = x < W - 1 ? dv - comp(px1, ch) : 0.f;
        const float dgy = y < H - 1 ? dv - comp(py1, ch) : 0.f;
        acc[kk == 0 ? 2 : 5] += fabsf(dgx * wxs) + fabsf(dgy * wys);
      }
      // consistency: d_v / sigma_v vs the opposite disparity warped by it (F5)
      acc[1] += fabsf(dvv[k] - wd[k]);
      const float sg = sgv[k];
      if (a.ecw != 0.f) acc[4] += fabsf(sg - ws_[k]);
      if (a.loss_type == 1) acc[3] += fdiv(ev, sg) + __logf(sg);
      else if (a.loss_type == 2) acc[3] += fdiv(ev, __expf(-sg)) + sg;
      else acc[3] += fabsf(sg - ev);
    }
    __syncthreads();
  }
  loss_partials<FNT>(a, acc, red);
}

// ------------------------------------------------------------ backward -----
// (1) the consistency terms' gradient w.r.t. the WARPED operand (the
// opposite disparity): a scatter along the row.  One workgroup per strip of
// STR rows (full width) accumulates, in LDS, the contributions of every
// source pixel whose bilinear taps land in its rows -- sources in rows
// [y0-1, y0+STR] -- and stores them once, into channels 0/1 of each target
// pixel's own gradient slot (loss_grad_kernel's thread for that pixel reads
// them and then stores the final float4).
constexpr int STR = 8;
constexpr int SCT = 1024;  // threads per scatter workgroup

// COMBINE: the forward was loss_grad_kernel<true>; complete its per-unit-gout
// partials: dpred = (gout_d * gpart.xy + scatter, gout_e * gpart.zw).
template <bool COMBINE>
__global__ void __launch_bounds__(SCT) loss_scatter_kernel(LArgs a) {
  // The warp's row taps do not depend on the shift (row_w), so the scatter
  // is separable: each source row r first scatters along x into its own
  // accumulator X_r[ch][x] (2 LDS adds per term instead of 4), then target
  // row T sums (1-n_r) X_r over the rows with y0(r) = T and n_r X_r over
  // those with y0(r) + 1 = T.
  // The row accumulators are fixed point (int32 LDS atomics, which run at
  // the LDS's integer rate; f32 LDS atomics measured 2x slower for the whole
  // kernel): a source pixel adds gg_d * e (|gg_d| <= |kcd|) and, with an
  // error-consistency weight, gg_s * e (|gg_s| <= |kce|) into the SAME target
  // channel, e + w = 1 per source, so a row sums at most W * kmax into one
  // target with kmax = |kcd| + |kce|.  Units of kmax * 2^-sh with
  // sh = 30 - ceil(log2 W) keep that at most 2^30 (int32 headroom 2x);
  // the quantum is kmax * 2^-sh (5e-7 kmax at W = 512) and the integer sums
  // are exact, i.e. independent of the atomics' order.
  extern __shared__ int acc[];  // [STR + 2 source rows][2 target ch][W]
  const int tid = threadIdx.x;
  const int s = scale_of(a, blockIdx.x);
  const LScale S = scale_desc(a, s);
  const int H = S.h, W = S.w;
  const int HW = H * W;
  const int lb = blockIdx.x - S.block0;
  const int n = lb / S.tiles_y, y0 = (lb - n * S.tiles_y) * STR;
  const float* pp = S.pred + (long)n * HW * 4;
  const double np = (double)a.N * HW;
  const float kcd = (float)(gval(a.gout_d) * a.w_cons / np);
  const float kce = (float)(gval(a.gout_e) * a.w_err * a.ecw / np);
  const float Wh = (float)W * 0.5f;
  const float stepx = W > 1 ? 1.f / (float)(W - 1) : 0.f;
  const int halfw = W / 2;
  const int r0 = max(0, y0 - 1), r1 = min(H, y0 + STR + 1);
  const int nr = r1 - r0;
  // the d term (kcd) and the sigma term (kce) of one source land in the same
  // target channel: their magnitudes add in the bound
  const float kmax = fabsf(kcd) + (a.ecw != 0.f ? fabsf(kce) : 0.f);
  const int sh = 30 - (W > 1 ? 32 - __clz(W - 1) : 0);
  const float toq = kmax > 0.f ? ldexpf(1.f, sh) / kmax : 0.f;
  const float fromq = ldexpf(kmax, -sh);
  for (int i = tid; i < nr * 2 * W; i += SCT) acc[i] = 0;
  __syncthreads();
  for (int i = tid; i < nr * W; i += SCT) {
    const int ri = i / W, x = i - ri * W;
    const int y = r0 + ri;
    const RowW rw = row_w(y, H);
    const float4 p = *reinterpret_cast<const float4*>(pp + (y * W + x) * 4);
    const float linx = lin01s(x, W, halfw, stepx);
    Samp t[4];
    float val[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // (view, term): (0,d) (1,d) (0,sigma) (1,sigma)
      const int v = j & 1;
      val[j] = comp(p, j < 2 ? v : 2 + v);
      t[j] = warp_tab(linx, rw, (v == 0 ? -1.f : 1.f) * val[j], Wh);
    }
    float wv[4];
    cons_samples<1>(pp + 1, H, W, t, wv, nullptr);          // view 0 samples d_R
    cons_samples<1>(pp + 0, H, W, t + 1, wv + 1, nullptr);  // view 1 samples d_L
    if (a.ecw != 0.f) {
      cons_samples<1>(pp + 1, H, W, t + 2, wv + 2, nullptr);
      cons_samples<1>(pp + 0, H, W, t + 3, wv + 3, nullptr);
    }
    int* X = acc + ri * 2 * W;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= 2 && a.ecw == 0.f) break;
      const int v = j & 1;
      const float gg = -sgnf(val[j] - wv[j]) * (j < 2 ? kcd : kce) * toq;
      if (gg == 0.f) continue;
      int* Xc = X + (1 - v) * W;  // target channel = the warped (opposite) disparity
      const int xa = t[j].x0;
      if (xa >= 0 && xa < W) atomicAdd(&Xc[xa], __float2int_rn(gg * t[j].e));
      if (xa + 1 >= 0 && xa + 1 < W) atomicAdd(&Xc[xa + 1], __float2int_rn(gg * t[j].w));
    }
  }
  __syncthreads();
  float* sa = S.dpred + ((long)n * HW + (long)y0 * W) * 4;
  const float* gp = COMBINE ? S.gpart + ((long)n * HW + (long)y0 * W) * 4 : nullptr;
  const float gd = COMBINE ? gval(a.gout_d) : 0.f, ge = COMBINE ? gval(a.gout_e) : 0.f;
  const int rows = min(STR, H - y0);
  for (int i = tid; i < rows * W; i += SCT) {
    const int T = y0 + i / W, x = i % W;
    float g0 = 0.f, g1 = 0.f;
    for (int r = max(r0, T - 2); r <= min(r1 - 1, T + 2); ++r) {
      const RowW rw = row_w(r, H);
      const float wgt = rw.y0 == T ? 1.f - rw.n : (rw.y0 + 1 == T ? rw.n : 0.f);
      if (wgt == 0.f) continue;
      const int* X = acc + (r - r0) * 2 * W;
      g0 += wgt * (float)X[x];
      g1 += wgt * (float)X[W + x];
    }
    g0 *= fromq;
    g1 *= fromq;
    if (COMBINE) {
      const float4 p = *reinterpret_cast<const float4*>(gp + i * 4);
      *reinterpret_cast<float4*>(sa + i * 4) =
          make_float4(gd * p.x + g0, gd * p.y + g1, ge * p.z, ge * p.w);
    } else {
      *reinterpret_cast<float2*>(sa + i * 4) = make_float2(g0, g1);
    }
  }
}

// (2) every other gradient, per TY x TX tile (both views), plus the scatter sums.
// FUSED: the forward pass of a step that will differentiate the loss.  The
// same tile work also yields the six loss terms (loss_fwd_kernel's sums), and
// the gradient is stored per unit gout -- channels 0/1 the d(disp_loss)/d(d_v)
// part without the scatter, channels 2/3 d(error_loss)/d(sigma_v) -- into
// gpart; the backward's scatter launch scales and completes it
// (loss_scatter_kernel<true>).  Every gradient term is linear in exactly one
// of gout_d / gout_e, so this is the backward at any gout.
constexpr int BTY = 16, BTX = 32, BNT = 512;
using BT = Tile<BTY, BTX>;

template <bool FUSED>
__global__ void __launch_bounds__(BNT, 2) loss_grad_kernel(LArgs a) {
  __shared__ float4 sP[BT::RY][BT::RX];
  __shared__ float sI[3][BT::RY][BT::RX], sR[3][BT::RY][BT::RX];
  __shared__ float sX[3][BTY][BTX];           // d recon_c / d ix at the pixels
  __shared__ float sA[3][3][BT::GY][BT::GX];  // per channel: a1, a2 (x y_q), a3 (x x_q)
  __shared__ float sD[BT::GY][BT::GX];
  __shared__ float sUy[BT::GY], sUx[BT::GX];
  __shared__ Tabs<BTY, BTX> tb;
  __shared__ double red[FUSED ? 6 : 1][BNT / 64];
  const int tid = threadIdx.x;
  const int s = scale_of(a, blockIdx.x);
  const LScale S = scale_desc(a, s);
  const int H = S.h, W = S.w;
  const int HW = H * W;
  const int lb = blockIdx.x - S.block0;
  const int per = S.tiles_x * S.tiles_y;
  const int n = lb / per, t = lb - n * per;
  const int ty0 = (t / S.tiles_x) * BTY, tx0 = (t % S.tiles_x) * BTX;
  const float* pp = S.pred + (long)n * HW * 4;
  const float* img = S.img + (long)n * 6 * HW;
  const int gh = H - 2, gw = W - 2;
  const float Wh = (float)W * 0.5f;
  const double np = (double)a.N * HW;
  const float gd = FUSED ? 1.f : gval(a.gout_d), ge = FUSED ? 1.f : gval(a.gout_e);
  const float kW = (float)(gd * a.w_wssim / np);  // d total / d sum_p (e_L + e_R)
  const float kcd = (float)(gd * a.w_cons / np);
  const float kce = (float)(ge * a.w_err * a.ecw / np);
  const float ksd = (float)(gd * a.w_smooth / np / (double)(1 << s));
  const float kse = (float)(ge * a.w_err * a.esw / np);
  const float kn = (float)(ge * a.w_err / (2.0 * np));
  // one pixel per thread and view
  const int ly = tid / BTX, lx = tid - (tid / BTX) * BTX;
  const int y = ty0 + ly, x = tx0 + lx;
  const bool ok = y < H && x < W;
  const int rr = ly + 2, qq = lx + 2;
  float* dslot = (FUSED ? S.gpart : S.dpred) + ((long)n * HW + (long)min(y, H - 1) * W + min(x, W - 1)) * 4;
  const float2 sav = FUSED ? make_float2(0.f, 0.f) : *reinterpret_cast<const float2*>(dslot);
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // FUSED: the forward's loss terms
  float* const recp = FUSED ? pick(a.rec, s) : nullptr;

  stage_pred<BTY, BTX, BNT>(pp, H, W, ty0, tx0, sP);
  init_tabs<BTY, BTX>(tb, H, W, ty0, tx0);
  if (tid < BT::GY) {
    const int gy = ty0 - 2 + tid;
    sUy[tid] = (gy >= 0 && gy < gh) ? up_adj_sum(gy, gh, H) : 0.f;
  } else if (tid >= 64 && tid < 64 + BT::GX) {
    const int gx = tx0 - 2 + (tid - 64);
    sUx[tid - 64] = (gx >= 0 && gx < gw) ? up_adj_sum(gx, gw, W) : 0.f;
  }
  __syncthreads();
  float4 outv = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int v = 0; v < 2; ++v) {
    const float sign = v == 0 ? -1.f : 1.f;
    stage_view<BTY, BTX, true, BNT>(img + v * 3 * HW, img + (1 - v) * 3 * HW, H, W, HW, ty0, tx0, v,
                               tb, sP, sI, sR, sX);
    __syncthreads();
    // per grid point: DSSIM (for the NLL's error map) and the SSIM
    // gradient coefficients
    for (int i = tid; i < BT::GY * BT::GX; i += BNT) {
      const int r = i / BT::GX, q = i - (i / BT::GX) * BT::GX;
      const int gy = ty0 - 2 + r, gx = tx0 - 2 + q;
      float dsum = 0.f;
      const bool valid = gy >= 0 && gy < gh && gx >= 0 && gx < gw;
      const float kk = kW * a.alpha * sUy[r] * sUx[q] * (-0.5f / 27.f);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float a1 = 0.f, a2 = 0.f, a3 = 0.f;
        if (valid) {
          const Stats st = win_stats<BT::RX>(sI[c], sR[c], r, q);
          const float A1 = 2 * st.mx * st.my + C1, A2 = 2 * st.vxy + C2;
          const float B1 = st.mx * st.mx + st.my * st.my + C1, B2 = st.vx + st.vy + C2;
          const float inv = fdiv(1.f, B1 * B2);
          const float Sv = (A1 * A2) * inv;
          const float dss = (1.f - Sv) * 0.5f;
          dsum += fminf(fmaxf(dss, 0.f), 1.f);
          if (dss >= 0.f && dss <= 1.f) {
            const float dA1 = A2 * inv, dA2 = A1 * inv;
            const float dB1 = -Sv * fdiv(1.f, B1), dB2 = -Sv * fdiv(1.f, B2);
            const float dP1 = 2 * st.mx * dA1 - 2 * st.mx * dA2 + 2 * st.my * dB1 - 2 * st.my * dB2;
            // k = d total / d SSIM_c(g) = kW * alpha * U(g) / 3 * (-1/2), per 1/9 of the window
            a1 = kk * dP1;
            a2 = kk * 2.f * dB2;
            a3 = kk * 2.f * dA2;
          }
        }
        sA[c][0][r][q] = a1;
        sA[c][1][r][q] = a2;
        sA[c][2][r][q] = a3;
      }
      sD[r][q] = dsum * (1.f / 3.f);
    }
    __syncthreads();
    const float4 p0 = sP[rr][qq];
    const float dv = comp(p0, v), sg = comp(p0, 2 + v);
    Samp tt[2];
    tt[0] = warp_tab(tb.lin[qq], tb.row[rr], sign * dv, Wh);
    tt[1] = warp_tab(tb.lin[qq], tb.row[rr], sign * sg, Wh);
    float wv[2], dx[2];
    cons_samples<2>(pp + (1 - v), H, W, tt, wv, dx);
    float gdv = v == 0 ? sav.x : sav.y, gsv = 0.f;
    if (ok) {
      // ---- WSSIM through the recon: dL/dR_c, then the warp derivative
      float l1 = 0.f;
      {
        const float kL1 = kW * (1.f - a.alpha) * (1.f / 3.f);
#pragma unroll 1
        for (int c = 0; c < 3; ++c) {
          const float iv = sI[c][rr][qq], rv = sR[c][rr][qq];
          l1 += fabsf(iv - rv);
          float g = kL1 * sgnf(rv - iv);
#pragma unroll
          for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int w = 0; w < 3; ++w) {
              const int r = ly + u, q = lx + w;  // grid point (y-2+u, x-2+w)
              g += sA[c][0][r][q] + sA[c][1][r][q] * rv + sA[c][2][r][q] * iv;
            }
          gdv += g * sX[c][ly][lx] * sign * (float)W;
        }
      }
      // ---- disparity consistency, own operand (the warped one came from the scatter)
      gdv += sgnf(dv - wv[0]) * kcd * (1.f - dx[0] * sign * (float)W);
      if (FUSED) acc[1] += fabsf(dv - wv[0]);
      // ---- error consistency: sigma_v vs warp(d_opp, sign*sigma_v) (F5)
      if (a.ecw != 0.f) {
        gsv += sgnf(sg - wv[1]) * kce * (1.f - dx[1] * sign * (float)W);
        if (FUSED) acc[4] += fabsf(sg - wv[1]);
      }
      // ---- smoothness (loss.py:191-264) of d_v (and sigma_v if weighted)
      {
        auto wgt = [&](int ry, int rx, int dy, int dxx) {
          float g = 0.f;
#pragma unroll
          for (int c = 0; c < 3; ++c) g += fabsf(sI[c][ry][rx] - sI[c][ry + dy][rx + dxx]);
          return __expf(-g * (1.f / 3.f));
        };
        float wx0 = 0.f, wx1 = 0.f, wy0 = 0.f, wy1 = 0.f;  // at q and q-1 (x), q and q-w (y)
        if (x < W - 1) wx0 = wgt(rr, qq, 0, 1);
        if (x > 0) wx1 = wgt(rr, qq - 1, 0, 1);
        if (y < H - 1) wy0 = wgt(rr, qq, 1, 0);
        if (y > 0) wy1 = wgt(rr - 1, qq, 1, 0);
        const float4 pxp = sP[rr][qq + 1], pxm = sP[rr][qq - 1];
        const float4 pyp = sP[rr + 1][qq], pym = sP[rr - 1][qq];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int ch = v + 2 * k;
          if (k == 1 && a.esw == 0.f) continue;
          const float d0 = comp(p0, ch);
          float g = 0.f;
          if (x < W - 1) g += sgnf((d0 - comp(pxp, ch)) * wx0) * wx0;
          if (x > 0) g -= sgnf((comp(pxm, ch) - d0) * wx1) * wx1;
          if (y < H - 1) g += sgnf((d0 - comp(pyp, ch)) * wy0) * wy0;
          if (y > 0) g -= sgnf((comp(pym, ch) - d0) * wy1) * wy1;
          if (k == 0) gdv += ksd * g;
          else gsv += kse * g;
          if (FUSED) {  // forward smoothness (wx0 / wy0 are 0 at the far edges, as dgx / dgy are)
            const float dgx = x < W - 1 ? d0 - comp(pxp, ch) : 0.f;
            const float dgy = y < H - 1 ? d0 - comp(pyp, ch) : 0.f;
            acc[k == 0 ? 2 : 5] += fabsf(dgx * wx0) + fabsf(dgy * wy0);
          }
        }
      }
      // ---- NLL on sigma_v with the detached error map (loss.py:389-403)
      {
        const float up = dssim_up<BT::GX>(sD, tb.uy[ly], tb.ux[lx]);
        const float ev = a.alpha * up + (1.f - a.alpha) * (l1 * (1.f / 3.f));
        if (FUSED) {
          acc[0] += ev;
          if (a.loss_type == 1) acc[3] += fdiv(ev, sg) + __logf(sg);
          else if (a.loss_type == 2) acc[3] += fdiv(ev, __expf(-sg)) + sg;
          else acc[3] += fabsf(sg - ev);
          if (a.emap != nullptr && s == a.nscales - 1) a.emap[(n * 2 + v) * HW + y * W + x] = ev;
          if (recp != nullptr)
#pragma unroll
            for (int c = 0; c < 3; ++c) recp[(n * 6 + v * 3 + c) * HW + y * W + x] = sR[c][rr][qq];
        }
        float g;
        if (a.loss_type == 1) g = fdiv(1.f, sg) - fdiv(ev, sg * sg);
        else if (a.loss_type == 2) g = 0.5f * (ev * __expf(sg) + 1.f);
        else g = sgnf(sg - ev);
        gsv += kn * g;
      }
    }
    if (v == 0) { outv.x = gdv; outv.z = gsv; }
    else { outv.y = gdv; outv.w = gsv; }
    __syncthreads();
  }
  if (ok) *reinterpret_cast<float4*>(dslot) = outv;
  if constexpr (FUSED) loss_partials<BNT>(a, acc, red);
}

constexpr int ETY = 16, ETX = 64;
using ET = Tile<ETY, ETX>;

// WeightedSSIMLoss.image_error with an explicit recon (evaluation,
// reference train/evaluate.py:151 -> train/loss.py:96-131): out [N][2][H][W]
__global__ void __launch_bounds__(256) image_error_kernel(const float* __restrict__ img,
                                                          const float* __restrict__ rec, int N,
                                                          int H, int W, float alpha,
                                                          float* __restrict__ out, int tiles_x,
                                                          int tiles_y) {
  __shared__ float sI[3][ET::RY][ET::RX], sR[3][ET::RY][ET::RX];
  __shared__ float sD[ET::GY][ET::GX];
  const int tid = threadIdx.x;
  const long HW = (long)H * W;
  const int per = tiles_x * tiles_y;
  const int n = blockIdx.x / per, t = blockIdx.x - n * per;
  const int ty0 = (t / tiles_x) * ETY, tx0 = (t % tiles_x) * ETX;
  const int gh = H - 2, gw = W - 2;
  for (int v = 0; v < 2; ++v) {
    const float* Iv = img + ((long)n * 6 + v * 3) * HW;
    const float* Rv = rec + ((long)n * 6 + v * 3) * HW;
    for (int i = tid; i < ET::RY * ET::RX; i += 256) {
      const int r = i / ET::RX, q = i - (i / ET::RX) * ET::RX;
      const int y = ty0 - 2 + r, x = tx0 - 2 + q;
      const bool in = y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        sI[c][r][q] = in ? Iv[c * HW + (long)y * W + x] : 0.f;
        sR[c][r][q] = in ? Rv[c * HW + (long)y * W + x] : 0.f;
      }
    }
    __syncthreads();
    for (int i = tid; i < ET::GY * ET::GX; i += 256) {
      const int r = i / ET::GX, q = i - (i / ET::GX) * ET::GX;
      const int gy = ty0 - 2 + r, gx = tx0 - 2 + q;
      float dv = 0.f;
      if (gy >= 0 && gy < gh && gx >= 0 && gx < gw) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float ss = ssim_of(win_stats<ET::RX>(sI[c], sR[c], r, q));
          dv += fminf(fmaxf((1.f - ss) * 0.5f, 0.f), 1.f);
        }
        dv /= 3.f;
      }
      sD[r][q] = dv;
    }
    __syncthreads();
    for (int i = tid; i < ETY * ETX; i += 256) {
      const int ly = i / ETX, lx = i - (i / ETX) * ETX;
      const int y = ty0 + ly, x = tx0 + lx;
      if (y >= H || x >= W) continue;
      int y0, y1, x0, x1;
      float wy, wx_;
      up_index(y, gh, H, y0, y1, wy);
      up_index(x, gw, W, x0, x1, wx_);
      const int r0 = y0 - (ty0 - 2), r1 = y1 - (ty0 - 2);
      const int q0 = x0 - (tx0 - 2), q1 = x1 - (tx0 - 2);
      const float up = (1.f - wy) * ((1.f - wx_) * sD[r0][q0] + wx_ * sD[r0][q1]) +
                       wy * ((1.f - wx_) * sD[r1][q0] + wx_ * sD[r1][q1]);
      float l1 = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c) l1 += fabsf(sI[c][ly + 2][lx + 2] - sR[c][ly + 2][lx + 2]);
      out[((long)n * 2 + v) * HW + (long)y * W + x] = alpha * up + (1.f - alpha) * (l1 / 3.f);
    }
    __syncthreads();
  }
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// fill the per-scale geometry of a loss launch; returns the block count
int loss_setup(LArgs& a, int nscales, int N, int H0, int W0, const float* const* img,
               const float* const* pred, float* const* dpred, int tile_y, int tile_x) {
  a.nscales = nscales;
  a.N = N;
  int blocks = 0;
  for (int s = 0; s < nscales; ++s) {
    a.img[s] = img[s];
    a.pred[s] = pred[s];
    a.dpred[s] = dpred ? dpred[s] : nullptr;
    a.h[s] = H0 >> s;
    a.w[s] = W0 >> s;
    a.tiles_x[s] = tile_x > 0 ? ceil_div(a.w[s], tile_x) : 1;  // tile_x 0: full rows
    a.tiles_y[s] = ceil_div(a.h[s], tile_y);
    a.block0[s] = blocks;
    blocks += N * a.tiles_x[s] * a.tiles_y[s];
  }
  a.nblocks = blocks;
  return blocks;
}

}  // namespace

extern "C" {

int um_pyramid(const float* x, int NC, int H, int W, int nlevels, float* const* out,
               hipStream_t st) {
  UM_CHECK_ARG(nlevels >= 1 && nlevels <= MAXS, "um_pyramid: %d levels (1..%d)", nlevels, MAXS);
  UM_CHECK_ARG(((long)H * W) % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out[0]) & 15) == 0,
               "um_pyramid: level 0 needs 16-byte aligned planes of a multiple of 4 pixels");
  PyrArgs a{};
  a.x = x;
  a.NC = NC;
  a.H = H;
  a.W = W;
  a.nlev = nlevels;
  a.off[0] = 0;
  a.off[1] = (long)NC * H * W / 4;
  for (int l = 0; l < nlevels; ++l) {
    a.out[l] = out[l];
    if (l >= 1) a.off[l + 1] = a.off[l] + (long)NC * (H >> l) * (W >> l);
  }
  hipLaunchKernelGGL(pyramid_kernel, dim3(grid_for(a.off[nlevels])), dim3(256), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_warp(const float* img, int N, int C, int H, int W, const float* disp, long disp_sn,
            long disp_sp, float sign, float* out, hipStream_t st) {
  hipLaunchKernelGGL(warp_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, st, img, N, C, H,
                     W, disp, disp_sn, disp_sp, sign, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_warp_bwd(const float* img, int N, int C, int H, int W, const float* disp, long disp_sn,
                long disp_sp, float sign, const float* gout, float* gdisp, long g_sn, long g_sp,
                hipStream_t st) {
  hipLaunchKernelGGL(warp_bwd_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, st, img, N,
                     C, H, W, disp, disp_sn, disp_sp, sign, gout, gdisp, g_sn, g_sp);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_recon_pyramid(int nlevels, int N, int H, int W, const float* const* img,
                     const float* const* pred, const long* pred_strides, float* const* out,
                     hipStream_t st) {
  UM_CHECK_ARG(nlevels >= 1 && nlevels <= MAXS, "um_recon_pyramid: %d levels", nlevels);
  ReconArgs a{};
  a.N = N;
  a.H = H;
  a.W = W;
  a.nlev = nlevels;
  a.off[0] = 0;
  for (int l = 0; l < nlevels; ++l) {
    a.img[l] = img[l];
    a.pred[l] = pred[l];
    a.out[l] = out[l];
    a.psn[l] = pred_strides[3 * l];
    a.psc[l] = pred_strides[3 * l + 1];
    a.psp[l] = pred_strides[3 * l + 2];
    a.off[l + 1] = a.off[l] + (long)N * (H >> l) * (W >> l);
  }
  hipLaunchKernelGGL(recon_kernel, dim3(grid_for(a.off[nlevels])), dim3(256), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

long um_loss_ws(int nscales, int N, int H, int W) {
  LArgs a{};
  const float* dummy[MAXS] = {};
  if (nscales < 1 || nscales > MAXS) return 0;
  // partials for the smaller tiles of the fused forward (>= the plain forward's)
  return (long)loss_setup(a, nscales, N, H, W, dummy, dummy, nullptr, BTY, BTX) * 8 *
         sizeof(double);
}

int um_loss_fwd(int nscales, int N, int H, int W, const float* const* img,
                const float* const* pred, float alpha, int loss_type, float esw, float ecw,
                float w_wssim, float w_cons, float w_smooth, float w_err, double* ws,
                float* emap_last, float* const* recon_out, float* out, float* disp_loss,
                float* error_loss, float* const* gpart, hipStream_t st) {
  UM_CHECK_ARG(nscales >= 1 && nscales <= MAXS, "um_loss_fwd: %d scales (1..%d)", nscales, MAXS);
  UM_CHECK_ARG((H >> (nscales - 1)) >= 3 && (W >> (nscales - 1)) >= 3,
               "um_loss_fwd: image %dx%d too small for %d scales", H, W, nscales);
  LArgs a{};
  const int blocks = gpart ? loss_setup(a, nscales, N, H, W, img, pred, nullptr, BTY, BTX)
                           : loss_setup(a, nscales, N, H, W, img, pred, nullptr, FTY, FTX);
  a.alpha = alpha; a.loss_type = loss_type; a.esw = esw; a.ecw = ecw;
  a.w_wssim = w_wssim; a.w_cons = w_cons; a.w_smooth = w_smooth; a.w_err = w_err;
  a.parts = ws;
  a.emap = emap_last;
  for (int l = 0; l < nscales; ++l) a.rec[l] = recon_out ? recon_out[l] : nullptr;
  a.out = out;
  a.disp_loss = disp_loss;
  a.error_loss = error_loss;
  if (gpart) {
    for (int l = 0; l < nscales; ++l) a.gpart[l] = gpart[l];
    hipLaunchKernelGGL(loss_grad_kernel<true>, dim3(blocks), dim3(BNT), 0, st, a);
  } else {
    hipLaunchKernelGGL(loss_fwd_kernel, dim3(blocks), dim3(FNT), 0, st, a);
  }
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(RNT), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_loss_bwd(int nscales, int N, int H, int W, const float* const* img,
                const float* const* pred, float alpha, int loss_type, float esw, float ecw,
                float w_wssim, float w_cons, float w_smooth, float w_err,
                const float* gout_disp, const float* gout_err, const float* const* gpart,
                float* const* dpred, hipStream_t st) {
  UM_CHECK_ARG(nscales >= 1 && nscales <= MAXS, "um_loss_bwd: %d scales (1..%d)", nscales, MAXS);
  UM_CHECK_ARG((H >> (nscales - 1)) >= 3 && (W >> (nscales - 1)) >= 3,
               "um_loss_bwd: image %dx%d too small for %d scales", H, W, nscales);
  const size_t lds = (size_t)(STR + 2) * W * 2 * sizeof(int);
  UM_CHECK_ARG(lds <= 128 * 1024, "um_loss_bwd: width %d too large", W);
  LArgs a{};
  a.alpha = alpha; a.loss_type = loss_type; a.esw = esw; a.ecw = ecw;
  a.w_wssim = w_wssim; a.w_cons = w_cons; a.w_smooth = w_smooth; a.w_err = w_err;
  a.gout_d = gout_disp;
  a.gout_e = gout_err;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&loss_scatter_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&loss_scatter_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    attr = true;
  }
  int blocks = loss_setup(a, nscales, N, H, W, img, pred, dpred, STR, 0);
  if (gpart) {
    // the fused forward computed every other term: the scatter completes them
    for (int l = 0; l < nscales; ++l) a.gpart[l] = const_cast<float*>(gpart[l]);
    hipLaunchKernelGGL(loss_scatter_kernel<true>, dim3(blocks), dim3(SCT), lds, st, a);
  } else {
    // (1) consistency scatter sums into channels 0/1 of dpred, (2) the rest
    hipLaunchKernelGGL(loss_scatter_kernel<false>, dim3(blocks), dim3(SCT), lds, st, a);
    blocks = loss_setup(a, nscales, N, H, W, img, pred, dpred, BTY, BTX);
    hipLaunchKernelGGL(loss_grad_kernel<false>, dim3(blocks), dim3(BNT), 0, st, a);
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_image_error(const float* img, const float* rec, int N, int H, int W, float alpha,
                   float* out, hipStream_t st) {
  UM_CHECK_ARG(H >= 3 && W >= 3, "um_image_error: image %dx%d too small", H, W);
  const int tx = ceil_div(W, FTX), ty = ceil_div(H, FTY);
  hipLaunchKernelGGL(image_error_kernel, dim3(N * tx * ty), dim3(256), 0, st, img, rec, N, H, W,
                     alpha, out, tx, ty);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
