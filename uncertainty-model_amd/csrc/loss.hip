// Monodepth-style loss stack with uncertainty, forward + analytic backward.
// Reference: train/utils.py:27-135 (pyramid, bilinear warp) and
// train/loss.py:15-264,340-434,512-568 (WSSIM, L-R consistency, edge-aware
// smoothness, reprojection-error NLL, Tukra total).
//
// Images are NCHW f32 [N][6][h][w] (left = channels 0-2, right = 3-5).
// Predictions are the disp head's NHWC f32 [N][h][w][4] (pixel stride pld):
// channel 0/1 = left/right disparity, 2/3 = left/right uncertainty.
//
// Warp (F6): sample x = ((2*(lin(j)+shift) - 1) + 1) * W/2 - 0.5 with
// lin = torch.linspace(0,1,W) in f32, y likewise with shift 0; bilinear,
// zero padding (grid_sample align_corners=False).
#include "common.h"

namespace {

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

constexpr float C1 = 0.01f * 0.01f;
constexpr float C2 = 0.03f * 0.03f;

// ---------------------------------------------------------------- pyramid --
__global__ void pyramid_kernel(const float* __restrict__ x, int NC, int H, int W,
                               float* __restrict__ out, int h, int w) {
  const long total = (long)NC * h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int xo = i % w;
    const int yo = (i / w) % h;
    const long pl = i / ((long)w * h);
    const float* p = x + pl * H * W;
    int y0, y1, x0, x1;
    float ly, lx;
    up_index(yo, H, h, y0, y1, ly);
    up_index(xo, W, w, x0, x1, lx);
    const float v = (1.f - ly) * ((1.f - lx) * p[(long)y0 * W + x0] + lx * p[(long)y0 * W + x1]) +
                    ly * ((1.f - lx) * p[(long)y1 * W + x0] + lx * p[(long)y1 * W + x1]);
    out[i] = v;
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

// ------------------------------------------------------------------ DSSIM --
// D[n][v][gy][gx] = mean_c clamp((1 - SSIM_c)/2, 0, 1) over the 3x3 valid window
__global__ void dssim_kernel(const float* __restrict__ img, const float* __restrict__ rec, int N,
                             int H, int W, float* __restrict__ D) {
  const int gh = H - 2, gw = W - 2;
  const long total = (long)N * 2 * gh * gw;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int gx = i % gw;
    const int gy = (i / gw) % gh;
    const int v = (i / ((long)gw * gh)) % 2;
    const int n = i / ((long)gw * gh * 2);
    float acc = 0.f;
    for (int c = 0; c < 3; ++c) {
      const long pl = ((long)n * 6 + v * 3 + c) * H * W;
      float sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          const long o = pl + (long)(gy + a) * W + gx + b;
          const float xv = img[o], yv = rec[o];
          sx += xv; sy += yv; sxx += xv * xv; syy += yv * yv; sxy += xv * yv;
        }
      const float mx = sx / 9.f, my = sy / 9.f;
      const float vx = sxx / 9.f - mx * mx, vy = syy / 9.f - my * my, vxy = sxy / 9.f - mx * my;
      const float ss = ((2 * mx * my + C1) * (2 * vxy + C2)) / ((mx * mx + my * my + C1) * (vx + vy + C2));
      acc += fminf(fmaxf((1.f - ss) * 0.5f, 0.f), 1.f);
    }
    D[i] = acc / 3.f;
  }
}

struct LossP {
  const float* img;
  const float* rec;
  const float* pred;
  int pld;
  const float* D;
  float* e;
  int N, H, W;
  float alpha;
  int loss_type;  // 0 l1, 1 bayesian, 2 log_bayesian
  float esw, ecw;  // error-loss smoothness / consistency weights
};

// per-pixel forward terms; partials[block][8]:
// 0 wssim, 1 consistency, 2 smoothness, 3 nll, 4 err-consistency, 5 err-smoothness
__global__ void terms_kernel(LossP a, float* __restrict__ parts) {
  const int H = a.H, W = a.W;
  const long total = (long)a.N * H * W;
  float acc[6] = {0, 0, 0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = i % W;
    const int y = (i / W) % H;
    const int n = i / ((long)W * H);
    const float* pp = a.pred + (long)n * H * W * a.pld;
    const float* p = pp + ((long)y * W + x) * a.pld;
    int y0, y1, x0, x1;
    float ly, lx;
    up_index(y, H - 2, H, y0, y1, ly);
    up_index(x, W - 2, W, x0, x1, lx);
    for (int v = 0; v < 2; ++v) {
      const float* Dv = a.D + ((long)n * 2 + v) * (H - 2) * (W - 2);
      const int gw = W - 2;
      const float up = (1.f - ly) * ((1.f - lx) * Dv[y0 * gw + x0] + lx * Dv[y0 * gw + x1]) +
                       ly * ((1.f - lx) * Dv[y1 * gw + x0] + lx * Dv[y1 * gw + x1]);
      float l1 = 0.f;
      float gxi = 0.f, gyi = 0.f;
      for (int c = 0; c < 3; ++c) {
        const long pl = ((long)n * 6 + v * 3 + c) * H * W;
        const float iv = a.img[pl + (long)y * W + x];
        l1 += fabsf(iv - a.rec[pl + (long)y * W + x]);
        if (x < W - 1) gxi += fabsf(iv - a.img[pl + (long)y * W + x + 1]);
        if (y < H - 1) gyi += fabsf(iv - a.img[pl + (long)(y + 1) * W + x]);
      }
      const float ev = a.alpha * up + (1.f - a.alpha) * (l1 / 3.f);
      a.e[(((long)n * 2 + v) * H + y) * W + x] = ev;
      acc[0] += ev;
      const float wx = __expf(-gxi / 3.f), wy = __expf(-gyi / 3.f);
      // smoothness of disparity v and of uncertainty v
      for (int k = 0; k < 2; ++k) {
        const int ch = v + 2 * k;
        if (k == 1 && a.esw == 0.f) continue;
        const float dv = p[ch];
        const float dgx = x < W - 1 ? dv - p[a.pld + ch] : 0.f;
        const float dgy = y < H - 1 ? dv - p[(long)W * a.pld + ch] : 0.f;
        acc[k == 0 ? 2 : 5] += fabsf(dgx * wx) + fabsf(dgy * wy);
      }
      // consistency: disparity v vs opposite disparity warped by (+-) d_v / sigma_v
      const float sign = v == 0 ? -1.f : 1.f;
      const float* opp = pp + (1 - v);  // opposite disparity plane, stride pld
      {
        const float dv = p[v];
        const Samp t = warp_at(x, y, sign * dv, W, H);
        acc[1] += fabsf(dv - sample(opp, t, H, W, a.pld, nullptr));
      }
      if (a.ecw != 0.f) {
        const float sv = p[2 + v];
        const Samp t = warp_at(x, y, sign * sv, W, H);
        acc[4] += fabsf(sv - sample(opp, t, H, W, a.pld, nullptr));
      }
      const float sg = p[2 + v];
      if (a.loss_type == 1) acc[3] += ev / sg + __logf(sg);
      else if (a.loss_type == 2) acc[3] += ev / __expf(-sg) + sg;
      else acc[3] += fabsf(sg - ev);
    }
  }
  __shared__ float red[6][4];
  for (int k = 0; k < 6; ++k) {
    const float t = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = t;
  }
  __syncthreads();
  if (threadIdx.x < 6)
    parts[(long)blockIdx.x * 8 + threadIdx.x] =
        red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
}

struct FinalP {
  const float* parts[4];
  int nparts[4];
  double npix[4];  // N*h*w per scale
  int nscales;
  float w_wssim, w_cons, w_smooth, w_err, esw, ecw;
  int loss_type;
};

// out: [0] disp_loss [1] error_loss [2] wssim [3] consistency [4] smoothness [5] error
__global__ void __launch_bounds__(1024) finalize_kernel(FinalP f, float* __restrict__ out) {
  // 16 waves; wave w sums (scale, term) pairs w and w + 16 over the partial rows
  __shared__ double tot[4][6];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int pr = wave; pr < 4 * 6; pr += 16) {
    const int sc = pr / 6, k = pr % 6;
    if (sc >= f.nscales) continue;
    const float* q = f.parts[sc] + k;
    const int np = f.nparts[sc];
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
    int p = lane;
    for (; p + 192 < np; p += 256) {
      t0 += q[(long)p * 8];
      t1 += q[(long)(p + 64) * 8];
      t2 += q[(long)(p + 128) * 8];
      t3 += q[(long)(p + 192) * 8];
    }
    for (; p < np; p += 64) t0 += q[(long)p * 8];
    double t = (t0 + t1) + (t2 + t3);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) tot[sc][k] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ws = 0, cs = 0, sm = 0, er = 0;
    for (int i = 0; i < f.nscales; ++i) {
      const double np = f.npix[i];
      ws += tot[i][0] / np;
      cs += tot[i][1] / np;
      sm += tot[i][2] / np / (double)(1 << i);
      double e = tot[i][3] / (2.0 * np);
      if (f.loss_type == 2) e *= 0.5;
      e += f.esw * tot[i][5] / np + f.ecw * tot[i][4] / np;
      er += e;
    }
    out[0] = (float)(ws * f.w_wssim + cs * f.w_cons + sm * f.w_smooth);
    out[1] = (float)(er * f.w_err);
    out[2] = (float)ws;
    out[3] = (float)cs;
    out[4] = (float)sm;
    out[5] = (float)er;
  }
}

// ---------------------------------------------------------------- backward --
struct BwdP {
  LossP l;
  float* dpred;  // [N][H][W][pld] f32: own terms stored, then the scatter pass adds
  const float* gout;  // [2]: d total / d disp_loss, d / d error_loss (device scalars)
  float w_wssim, w_cons, w_smooth, w_err;
  float smooth_div;  // 2^scale
};

constexpr int TB = 16;           // output tile
constexpr int TI = TB + 4;       // image tile (halo 2)
constexpr int TG = TB + 2;       // grid-point tile

__global__ void __launch_bounds__(256) loss_bwd_kernel(BwdP b) {
  const LossP& a = b.l;
  const int H = a.H, W = a.W, pld = a.pld;
  const int nv = blockIdx.z;
  const int n = nv >> 1, v = nv & 1;
  const int ty0 = blockIdx.y * TB, tx0 = blockIdx.x * TB;
  const int tid = threadIdx.x;
  __shared__ float sI[3][TI][TI], sR[3][TI][TI];
  __shared__ float sA[3][3][TG][TG];  // per channel: a1, a2 (x y_q), a3 (x x_q)
  __shared__ float sUy[TG], sUx[TG];

  const float gd = b.gout[0], ge = b.gout[1];
  const double npix = (double)a.N * H * W;
  const float kW = (float)(gd * b.w_wssim / npix);  // d total / d sum_p (e_L + e_R)

  // stage image + recon tile (rows ty0-2 .. ty0+TB+1)
  for (int i = tid; i < 3 * TI * TI; i += 256) {
    const int c = i / (TI * TI), r = (i / TI) % TI, q = i % TI;
    const int y = ty0 - 2 + r, x = tx0 - 2 + q;
    float iv = 0.f, rv = 0.f;
    if (y >= 0 && y < H && x >= 0 && x < W) {
      const long o = (((long)n * 6 + v * 3 + c) * H + y) * W + x;
      iv = a.img[o];
      rv = a.rec[o];
    }
    sI[c][r][q] = iv;
    sR[c][r][q] = rv;
  }
  const int gh = H - 2, gw = W - 2;
  if (tid < TG) {
    const int gy = ty0 - 2 + tid;
    sUy[tid] = (gy >= 0 && gy < gh) ? up_adj_sum(gy, gh, H) : 0.f;
  } else if (tid >= 64 && tid < 64 + TG) {
    const int gx = tx0 - 2 + (tid - 64);
    sUx[tid - 64] = (gx >= 0 && gx < gw) ? up_adj_sum(gx, gw, W) : 0.f;
  }
  __syncthreads();
  // SSIM coefficients per grid point (gy, gx) = (ty0-2+r, tx0-2+q)
  for (int i = tid; i < 3 * TG * TG; i += 256) {
    const int c = i / (TG * TG), r = (i / TG) % TG, q = i % TG;
    const int gy = ty0 - 2 + r, gx = tx0 - 2 + q;
    float a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (gy >= 0 && gy < gh && gx >= 0 && gx < gw) {
      float sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
      for (int u = 0; u < 3; ++u)
        for (int w = 0; w < 3; ++w) {
          const float xv = sI[c][r + u][q + w], yv = sR[c][r + u][q + w];
          sx += xv; sy += yv; sxx += xv * xv; syy += yv * yv; sxy += xv * yv;
        }
      const float mx = sx / 9.f, my = sy / 9.f;
      const float vx = sxx / 9.f - mx * mx, vy = syy / 9.f - my * my, vxy = sxy / 9.f - mx * my;
      const float A1 = 2 * mx * my + C1, A2 = 2 * vxy + C2;
      const float B1 = mx * mx + my * my + C1, B2 = vx + vy + C2;
      const float S = (A1 * A2) / (B1 * B2);
      const float dss = (1.f - S) * 0.5f;
      if (dss >= 0.f && dss <= 1.f) {
        const float inv = 1.f / (B1 * B2);
        const float dA1 = A2 * inv, dA2 = A1 * inv, dB1 = -S / B1, dB2 = -S / B2;
        const float dP1 = 2 * mx * dA1 - 2 * mx * dA2 + 2 * my * dB1 - 2 * my * dB2;
        const float dP2 = dB2;
        const float dP3 = 2 * dA2;
        // k = d total / d SSIM_c(g) = kW * alpha * U(g) / 3 * (-1/2)
        const float k = kW * a.alpha * sUy[r] * sUx[q] / 3.f * -0.5f / 9.f;
        a1 = k * dP1;
        a2 = k * 2.f * dP2;
        a3 = k * dP3;
      }
    }
    sA[c][0][r][q] = a1;
    sA[c][1][r][q] = a2;
    sA[c][2][r][q] = a3;
  }
  __syncthreads();

  const int ly = tid / TB, lx = tid % TB;
  const int y = ty0 + ly, x = tx0 + lx;
  if (y >= H || x >= W) return;
  const float* pp = a.pred + (long)n * H * W * pld;
  const float* p = pp + ((long)y * W + x) * pld;
  float* dp = b.dpred + (long)n * H * W * pld;
  const float sign = v == 0 ? -1.f : 1.f;
  float gdv = 0.f, gsv = 0.f;

  // ---- WSSIM through the recon: dR_c then the warp derivative
  {
    const float dv = p[v];
    const Samp t = warp_at(x, y, sign * dv, W, H);
    const float kL1 = kW * (1.f - a.alpha) / 3.f;
    for (int c = 0; c < 3; ++c) {
      const float iv = sI[c][ly + 2][lx + 2], rv = sR[c][ly + 2][lx + 2];
      float g = kL1 * sgnf(rv - iv);
      for (int u = 0; u < 3; ++u)
        for (int w = 0; w < 3; ++w) {
          const int r = ly + u, q = lx + w;  // grid point (y-2+u, x-2+w) -> tile index
          g += sA[c][0][r][q] + sA[c][1][r][q] * rv + sA[c][2][r][q] * iv;
        }
      // recon_v,c = warp(opposite image channel c, shift = sign * d_v)
      const float* op = a.img + ((long)n * 6 + (1 - v) * 3 + c) * H * W;
      float dix;
      sample(op, t, H, W, 1, &dix);
      gdv += g * dix * sign * (float)W;
    }
  }
  // ---- disparity consistency (loss.py:154-188), d_v vs warp(d_opp, sign*d_v)
  {
    const float kc = (float)(gd * b.w_cons / npix);
    const float dv = p[v];
    const Samp t = warp_at(x, y, sign * dv, W, H);
    float dix;
    const float wv = sample(pp + (1 - v), t, H, W, pld, &dix);
    const float s = sgnf(dv - wv) * kc;
    gdv += s * (1.f - dix * sign * (float)W);  // the d_opp part: loss_scatter_kernel
  }
  // ---- error consistency: sigma_v vs warp(d_opp, sign*sigma_v) (F5)
  if (a.ecw != 0.f) {
    const float kc = (float)(ge * b.w_err * a.ecw / npix);
    const float sv = p[2 + v];
    const Samp t = warp_at(x, y, sign * sv, W, H);
    float dix;
    const float wv = sample(pp + (1 - v), t, H, W, pld, &dix);
    const float s = sgnf(sv - wv) * kc;
    gsv += s * (1.f - dix * sign * (float)W);
  }
  // ---- smoothness (loss.py:191-264) of d_v (and sigma_v if weighted)
  {
    // edge weights from the staged image tile (tile index = pixel + 2)
    auto wgt = [&](int ry, int rx, int dy, int dx) {
      float g = 0.f;
      for (int c = 0; c < 3; ++c) g += fabsf(sI[c][ry][rx] - sI[c][ry + dy][rx + dx]);
      return __expf(-g / 3.f);
    };
    float wxs[2] = {0.f, 0.f}, wys[2] = {0.f, 0.f};  // at q and q-1 (x), q and q-w (y)
    if (x < W - 1) wxs[0] = wgt(ly + 2, lx + 2, 0, 1);
    if (x > 0) wxs[1] = wgt(ly + 2, lx + 1, 0, 1);
    if (y < H - 1) wys[0] = wgt(ly + 2, lx + 2, 1, 0);
    if (y > 0) wys[1] = wgt(ly + 1, lx + 2, 1, 0);
    for (int k = 0; k < 2; ++k) {
      const int ch = v + 2 * k;
      float kc;
      if (k == 0) kc = (float)(gd * b.w_smooth / npix / b.smooth_div);
      else {
        if (a.esw == 0.f) continue;
        kc = (float)(ge * b.w_err * a.esw / npix);
      }
      const float d0 = p[ch];
      float g = 0.f;
      if (x < W - 1) { const float t = (d0 - p[pld + ch]) * wxs[0]; g += sgnf(t) * wxs[0]; }
      if (x > 0) { const float t = (p[-pld + ch] - d0) * wxs[1]; g -= sgnf(t) * wxs[1]; }
      if (y < H - 1) { const float t = (d0 - p[(long)W * pld + ch]) * wys[0]; g += sgnf(t) * wys[0]; }
      if (y > 0) { const float t = (p[-(long)W * pld + ch] - d0) * wys[1]; g -= sgnf(t) * wys[1]; }
      if (k == 0) gdv += kc * g; else gsv += kc * g;
    }
  }
  // ---- NLL on sigma_v with the detached error map (loss.py:389-403)
  {
    const float kn = (float)(ge * b.w_err / (2.0 * npix));
    const float sg = p[2 + v];
    const float ev = a.e[(((long)n * 2 + v) * H + y) * W + x];
    float g;
    if (a.loss_type == 1) g = -ev / (sg * sg) + 1.f / sg;
    else if (a.loss_type == 2) g = 0.5f * (ev * __expf(sg) + 1.f);
    else g = sgnf(sg - ev);
    gsv += kn * g;
  }
  dp[((long)y * W + x) * pld + v] = gdv;
  dp[((long)y * W + x) * pld + 2 + v] = gsv;
}

// Consistency terms' gradient w.r.t. the OPPOSITE disparity (the warped
// operand): a data-dependent scatter.  The warp moves rows by < 1 (sample
// y = y*H/(H-1) - 0.5), so a strip of RS rows scatters into rows y0-1 ..
// y0+RS only: accumulate them in LDS (ds_add_f32), then add rows no other
// strip reaches with plain read-modify-writes and the 4 shared border rows
// with global atomics.  Runs after loss_bwd_kernel (which stored the own terms).
constexpr int RS = 8;
__global__ void __launch_bounds__(256) loss_scatter_kernel(BwdP b) {
  extern __shared__ float acc[];  // [2 channels][RS + 2][W]
  const LossP& a = b.l;
  const int H = a.H, W = a.W, pld = a.pld;
  const int n = blockIdx.y;
  const int y0 = blockIdx.x * RS;
  const int nrow = RS + 2;
  for (int i = threadIdx.x; i < 2 * nrow * W; i += 256) acc[i] = 0.f;
  __syncthreads();
  const float gd = b.gout[0], ge = b.gout[1];
  const double npix = (double)a.N * H * W;
  const float kcd = (float)(gd * b.w_cons / npix);
  const float kce = (float)(ge * b.w_err * a.ecw / npix);
  const float* pp = a.pred + (long)n * H * W * pld;
  const int rows = min(RS, H - y0);
  for (int i = threadIdx.x; i < 2 * rows * W; i += 256) {
    const int v = i / (rows * W);
    const int r = i - v * rows * W;
    const int y = y0 + r / W, x = r % W;
    const float sign = v == 0 ? -1.f : 1.f;
    const float* p = pp + ((long)y * W + x) * pld;
    float* buf = acc + (1 - v) * nrow * W;
    for (int k = 0; k < 2; ++k) {
      float kc, val;
      if (k == 0) { kc = kcd; val = p[v]; }
      else { if (a.ecw == 0.f) break; kc = kce; val = p[2 + v]; }
      const Samp t = warp_at(x, y, sign * val, W, H);
      const float wv = sample(pp + (1 - v), t, H, W, pld, nullptr);
      const float g = -sgnf(val - wv) * kc;
      if (g == 0.f) continue;
      const int xs[2] = {t.x0, t.x0 + 1}, ys[2] = {t.y0, t.y0 + 1};
      const float wx[2] = {t.e, t.w}, wy[2] = {t.s, t.n};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int yy = ys[u], xx = xs[q];
          if (xx >= 0 && xx < W && yy >= 0 && yy < H)
            atomicAdd(&buf[(yy - (y0 - 1)) * W + xx], g * wy[u] * wx[q]);
        }
    }
  }
  __syncthreads();
  float* dp = b.dpred + (long)n * H * W * pld;
  for (int i = threadIdx.x; i < 2 * nrow * W; i += 256) {
    const int ch = i / (nrow * W);
    const int r = (i / W) % nrow;
    const int x = i % W;
    const int yy = y0 - 1 + r;
    if (yy < 0 || yy >= H) continue;
    const float v = acc[i];
    if (v == 0.f) continue;
    float* o = dp + ((long)yy * W + x) * pld + ch;
    if (r >= 2 && r <= RS - 1) *o += v;  // rows y0+1 .. y0+RS-2: this strip only
    else atomicAdd(o, v);
  }
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

int um_pyramid_level(const float* x, int NC, int H, int W, float* out, int h, int w,
                     hipStream_t st) {
  hipLaunchKernelGGL(pyramid_kernel, dim3(grid_for((long)NC * h * w)), dim3(256), 0, st, x, NC, H,
                     W, out, h, w);
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

int um_loss_parts(int N, int H, int W) { return grid_for((long)N * H * W); }

int um_loss_fwd_scale(const float* img, const float* rec, const float* pred, int pld, int N,
                      int H, int W, float alpha, int loss_type, float esw, float ecw, float* D,
                      float* e, float* parts, hipStream_t st) {
  UM_CHECK_ARG(H >= 3 && W >= 3, "um_loss_fwd_scale: image %dx%d too small", H, W);
  hipLaunchKernelGGL(dssim_kernel, dim3(grid_for((long)N * 2 * (H - 2) * (W - 2))), dim3(256), 0,
                     st, img, rec, N, H, W, D);
  LossP a{img, rec, pred, pld, D, e, N, H, W, alpha, loss_type, esw, ecw};
  hipLaunchKernelGGL(terms_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, st, a, parts);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_loss_finalize(int nscales, const float* const* parts, const int* nparts,
                     const double* npix, float w_wssim, float w_cons, float w_smooth, float w_err,
                     float esw, float ecw, int loss_type, float* out, hipStream_t st) {
  UM_CHECK_ARG(nscales >= 1 && nscales <= 4, "um_loss_finalize: nscales %d", nscales);
  FinalP f{};
  for (int i = 0; i < nscales; ++i) {
    f.parts[i] = parts[i];
    f.nparts[i] = nparts[i];
    f.npix[i] = npix[i];
  }
  f.nscales = nscales;
  f.w_wssim = w_wssim; f.w_cons = w_cons; f.w_smooth = w_smooth; f.w_err = w_err;
  f.esw = esw; f.ecw = ecw; f.loss_type = loss_type;
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1024), 0, st, f, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_loss_bwd_scale(const float* img, const float* rec, const float* pred, int pld, int N,
                      int H, int W, float alpha, int loss_type, float esw, float ecw,
                      const float* e, const float* gout, float w_wssim, float w_cons,
                      float w_smooth, float w_err, float smooth_div, float* dpred,
                      hipStream_t st) {
  BwdP b{};
  b.l = LossP{img, rec, pred, pld, nullptr, const_cast<float*>(e), N, H, W, alpha, loss_type,
              esw, ecw};
  b.dpred = dpred;
  b.gout = gout;
  b.w_wssim = w_wssim; b.w_cons = w_cons; b.w_smooth = w_smooth; b.w_err = w_err;
  b.smooth_div = smooth_div;
  dim3 grid(ceil_div(W, TB), ceil_div(H, TB), N * 2);
  hipLaunchKernelGGL(loss_bwd_kernel, grid, dim3(256), 0, st, b);
  const size_t lds = (size_t)2 * (RS + 2) * W * sizeof(float);
  UM_CHECK_ARG(lds <= 150 * 1024, "um_loss_bwd_scale: width %d too large", W);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&loss_scatter_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(loss_scatter_kernel, dim3(ceil_div(H, RS), N), dim3(256), lds, st, b);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
