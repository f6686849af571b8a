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

#include <cstdlib>

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

// value of source s, channel cc, at destination pixel (n, y, x)
__device__ __forceinline__ float cat_value(const CatSrc& s, int n, int y, int x, int H, int W,
                                           int cc) {
  float v;
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
                          (y & 1) * 2 + (x & 1), s.dtype);
  }
  if (s.scale) v *= s.scale[n * s.C + cc];
  return v;
}

__device__ __forceinline__ void ld8_any(const void* p, long off, int dt, float* v) {
  if (dt == UM_BF16) load8(reinterpret_cast<const bf16_t*>(p) + off, v);
  else load8(reinterpret_cast<const float*>(p) + off, v);
}

// 8 channels [cc, cc+8) of source pixel `off` as f32, lanes >= C zeroed.
// ld % 8 == 0: one 16/32-byte load (channels past C up to ceil8(C) <= ld
// exist in the row); C <= 4 with an f32 row of 4 (the disparity): one float4.
struct F8 {
  float v[8];
};
__device__ __forceinline__ F8 src8(const CatSrc& s, long off, int cc) {
  F8 r;
  if ((s.ld & 7) == 0) {
    if (s.dtype == UM_BF16) load8(reinterpret_cast<const bf16_t*>(s.ptr) + off + cc, r.v);
    else load8(reinterpret_cast<const float*>(s.ptr) + off + cc, r.v);
  } else {
    const float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(s.ptr) + off);
    r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
    r.v[4] = r.v[5] = r.v[6] = r.v[7] = 0.f;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) r.v[e] = (cc + e < s.C) ? r.v[e] : 0.f;
  return r;
}

// One launch per concat source: thread per (pixel, 8 destination channels)
// of the source's span [coff, coff + ceil8(C)) (sources start at 8-aligned
// offsets, so the spans tile the concat; lanes >= C are written as 0).
// Vector loads for COPY/UP2 rows with ld % 8 == 0 or the 4-channel f32
// disparity, and for PSHUF (the 32 source channels 4cc .. 4cc+31 holding
// the group's sub-pixel values); per-element fallback otherwise.
// the 8 channels [cc, cc+8) of source s at destination pixel (n, y, x)
template <int OP>
__device__ __forceinline__ void cat_vals(const CatSrc& s, int n, int y, int x, int H, int W,
                                         int cc, float* v) {
  const bool vec_ok = (OP == UM_CAT_PSHUF)
                          ? ((s.ld & 7) == 0 && (s.C & 7) == 0)
                          : ((s.ld & 7) == 0 || (s.C <= 4 && (s.ld & 3) == 0 && s.dtype == UM_F32));
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  if (!vec_ok) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (cc + e < s.C) v[e] = cat_value(s, n, y, x, H, W, cc + e);  // gate inside
    return;
  }
  if (OP == UM_CAT_COPY) {
    const F8 t = src8(s, ((long)(n * H + y) * W + x) * s.ld, cc);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t.v[e];
  } else if (OP == UM_CAT_UP2) {
    int y0, y1, x0, x1;
    float ly, lx;
    up_index(y, s.h, H, y0, y1, ly);
    up_index(x, s.w, W, x0, x1, lx);
    const long b = (long)n * s.h;
    const F8 v00 = src8(s, ((b + y0) * s.w + x0) * s.ld, cc);
    const F8 v01 = src8(s, ((b + y0) * s.w + x1) * s.ld, cc);
    const F8 v10 = src8(s, ((b + y1) * s.w + x0) * s.ld, cc);
    const F8 v11 = src8(s, ((b + y1) * s.w + x1) * s.ld, cc);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = (1.f - ly) * ((1.f - lx) * v00.v[e] + lx * v01.v[e]) +
             ly * ((1.f - lx) * v10.v[e] + lx * v11.v[e]);
  } else {  // PSHUF: src [N][H/2][W/2][4C], channel 4c + (y&1)*2 + (x&1)
    const long off = ((long)(n * s.h + (y >> 1)) * s.w + (x >> 1)) * s.ld + 4 * cc;
    const int sub = (y & 1) * 2 + (x & 1);
    float q[32];
#pragma unroll
    for (int j = 0; j < 4; ++j) ld8_any(s.ptr, off + 8 * j, s.dtype, q + 8 * j);
#pragma unroll
    for (int e = 0; e < 8; ++e)  // selects, not a dynamically indexed register array
      v[e] = sub == 0 ? q[4 * e] : sub == 1 ? q[4 * e + 1] : sub == 2 ? q[4 * e + 2] : q[4 * e + 3];
  }
  if (s.scale) {
    const float* g = s.scale + n * s.C + cc;
    if ((s.C & 3) == 0 && cc + 8 <= s.C && (reinterpret_cast<uintptr_t>(s.scale) & 15) == 0) {
      // the gate row's 8 values as two 16-byte loads
      const float4 g0 = *reinterpret_cast<const float4*>(g);
      const float4 g1 = *reinterpret_cast<const float4*>(g + 4);
      v[0] *= g0.x; v[1] *= g0.y; v[2] *= g0.z; v[3] *= g0.w;
      v[4] *= g1.x; v[5] *= g1.y; v[6] *= g1.z; v[7] *= g1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (cc + e < s.C) v[e] *= g[e];
    }
  }
}

// One launch per concat source: thread per (pixel, 8 destination channels)
// of the source's span [coff, coff + ceil8(C)) (sources start at 8-aligned
// offsets, so the spans tile the concat; lanes >= C are written as 0).
// Grid (row items / 256, H, N).
template <typename T, int OP>
__global__ void __launch_bounds__(256) cat_src_kernel(CatSrc s, int N, int H, int W,
                                                       T* __restrict__ dst, int ld) {
  const int cg = (s.C + 7) / 8;
  const int y = blockIdx.y, n = blockIdx.z;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * cg) return;
  const int x = i / cg;
  const int cc = (i - x * cg) * 8;
  float v[8];
  cat_vals<OP>(s, n, y, x, H, W, cc, v);
  store8(dst + (((long)n * H + y) * W + x) * ld + s.coff + cc, v);
}

// ALL sources of a concat in one launch: thread per (pixel, 8-channel group
// of the whole concat), so a pixel's Ctot channels leave as one contiguous
// row from adjacent lanes (full cache lines, each written once) instead of
// one partial-line pass per source.  Grid (W * Ctot/8 / 256, H, N).
template <typename T>
__global__ void __launch_bounds__(256) cat_all_kernel(CatArgs a, int N, int H, int W,
                                                       T* __restrict__ dst, int ld, int ng) {
  const int y = blockIdx.y, n = blockIdx.z;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * ng) return;
  const int x = i / ng;
  const int gi = i - x * ng;
  int k = 0;
#pragma unroll
  for (int j = 1; j < MAX_SRC; ++j)
    if (j < a.nsrc && a.s[j].coff <= gi * 8) k = j;
  // constant-offset selects into the kernel arguments (no dynamic indexing)
  const CatSrc* sp = &a.s[0];
#pragma unroll
  for (int j = 1; j < MAX_SRC; ++j) sp = k == j ? &a.s[j] : sp;
  const CatSrc& s = *sp;
  const int cc = gi * 8 - s.coff;
  float v[8];
  if (s.op == UM_CAT_COPY) cat_vals<UM_CAT_COPY>(s, n, y, x, H, W, cc, v);
  else if (s.op == UM_CAT_UP2) cat_vals<UM_CAT_UP2>(s, n, y, x, H, W, cc, v);
  else cat_vals<UM_CAT_PSHUF>(s, n, y, x, H, W, cc, v);
  store8(dst + (((long)n * H + y) * W + x) * ld + gi * 8, v);
}

// ---- backward: RowMap blocks (channel groups x pixel lanes) over a chunk of
// `chunk` source pixels of one image n (bwd_chunk); grid (chunks, 1, N)
// source pixels per block: ~2048 blocks overall, 16..256 pixels each
inline int bwd_chunk(long P, int N) {
  const long want = ((long)P * N + 2047) / 2048;
  int c = 16;
  while (c < want && c < 256) c <<= 1;
  return c;
}

__device__ __forceinline__ void st8_any(void* p, long off, int dt, const float* v, int acc) {
  float o[8];
  if (dt == UM_BF16) {
    bf16_t* q = reinterpret_cast<bf16_t*>(p) + off;
    if (acc) {
      load8(q, o);
      for (int e = 0; e < 8; ++e) o[e] += v[e];
      store8(q, o);
    } else {
      store8(q, v);
    }
  } else {
    float* q = reinterpret_cast<float*>(p) + off;
    if (acc) {
      load8(q, o);
      for (int e = 0; e < 8; ++e) o[e] += v[e];
      store8(q, o);
    } else {
      store8(q, v);
    }
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

// weight with which high-res index i samples low-res index j under the x2
// align_corners=True upsample (in -> out); 0 outside [0, out)
__device__ __forceinline__ float up_w(int i, int j, int in, int out) {
  if (i < 0 || i >= out) return 0.f;
  int i0, i1;
  float l1;
  up_index(i, in, out, i0, i1, l1);
  float w = 0.f;
  if (i0 == j) w += 1.f - l1;
  if (i1 == j) w += l1;
  return w;
}

// COPY (op 0) / UP2 (op 1) source gradient, vectorised over 8 channels:
//   gv = (op==COPY) g[pix, coff+c] : sum_taps w * g[hi-res tap, coff+c]
//   dsrc (+)= gv * gate ;  dgate[n][c] += sum_pix gv * src
template <typename T, int OP>
__global__ void __launch_bounds__(256) cat_bwd_kernel(const T* __restrict__ g, int ldg, int coff,
                                                      int H, int W, CatSrc s, void* dsrc, int ldd,
                                                      int dsd, int acc,
                                                      float* __restrict__ dscale, int chunk) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.z;
  const int cg = s.C / 8;
  const RowMap rm(cg);
  const long P = (long)s.h * s.w;
  const long p0 = (long)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int gi = g0 + rm.g;
    const int c = gi * 8;
    float ds[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && gi < cg) {
      float sc[8] = {1, 1, 1, 1, 1, 1, 1, 1};
      if (s.scale) load8(s.scale + n * s.C + c, sc);
      for (long p = p0 + rm.lane; p < p1; p += rm.lanes) {
        float gv[8];
        if (OP == UM_CAT_COPY) {
          load8(g + ((long)n * P + p) * ldg + coff + c, gv);
        } else if (s.h >= 4 && s.w >= 4) {
          // branch-free 6x6 window: high-res rows/cols i with floor(sc*i) in
          // {j-1, j} start at floor((j-1)/sc) and span < 6 when the low-res
          // side is >= 4 (sc = (in-1)/(out-1) > 0.4); weights 0 outside, so
          // all 36 loads are independent (no branch around a load)
          const int py = p / s.w, px = p % s.w;
          const float scy = (float)(s.h - 1) / (float)(H - 1), scx = (float)(s.w - 1) / (float)(W - 1);
          const int iy0 = max(0, (int)floorf((py - 1) / scy));
          const int ix0 = max(0, (int)floorf((px - 1) / scx));
          float wy[6], wx[6];
          int ry[6], rx[6];
#pragma unroll
          for (int u = 0; u < 6; ++u) {
            wy[u] = up_w(iy0 + u, py, s.h, H);
            ry[u] = min(iy0 + u, H - 1);
            wx[u] = up_w(ix0 + u, px, s.w, W);
            rx[u] = min(ix0 + u, W - 1);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = 0.f;
#pragma unroll
          for (int u = 0; u < 6; ++u) {
            const T* row = g + ((long)(n * H + ry[u]) * W) * ldg + coff + c;
#pragma unroll
            for (int v = 0; v < 6; ++v) {
              float t[8];
              load8(row + (long)rx[v] * ldg, t);
              const float w = wy[u] * wx[v];
#pragma unroll
              for (int e = 0; e < 8; ++e) gv[e] += w * t[e];
            }
          }
        } else {
          const int py = p / s.w, px = p % s.w;
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = 0.f;
          // high-res rows/cols that sample low-res (py, px) lie in [2j-2, 2j+4]
          float wx[7];
#pragma unroll
          for (int v = 0; v < 7; ++v) wx[v] = up_w(2 * px - 2 + v, px, s.w, W);
#pragma unroll
          for (int u = 0; u < 7; ++u) {
            const float wy = up_w(2 * py - 2 + u, py, s.h, H);
            if (wy == 0.f) continue;
            const T* row = g + ((long)(n * H + 2 * py - 2 + u) * W + 2 * px - 2) * ldg + coff + c;
#pragma unroll
            for (int v = 0; v < 7; ++v) {
              if (wx[v] == 0.f) continue;
              float t[8];
              load8(row + (long)v * ldg, t);
              const float w = wy * wx[v];
#pragma unroll
              for (int e = 0; e < 8; ++e) gv[e] += w * t[e];
            }
          }
        }
        const long sp = (long)n * P + p;
        if (dsrc) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = gv[e] * sc[e];
          st8_any(dsrc, sp * ldd + c, dsd, o, acc);
        }
        if (dscale) {
          float sv[8];
          ld8_any(s.ptr, sp * s.ld + c, s.dtype, sv);
#pragma unroll
          for (int e = 0; e < 8; ++e) ds[e] += gv[e] * sv[e];
        }
      }
    }
    if (dscale) {
      lane_reduce<8>(red, rm, ds);
      if (rm.lane == 0 && gi < cg)
#pragma unroll
        for (int e = 0; e < 8; ++e)  // per-block partial (no same-address atomics)
          dscale[((long)n * gridDim.x + blockIdx.x) * s.C + c + e] = ds[e];
    }
  }
}

// scalar path for sources whose channels are not 8-aligned in the concat
// (the 4-channel disparity; the skip placed after the 3-channel image):
// thread = (channel c = t % Cl, pixel lane t / Cl), per-block gate sums.
template <typename T, int OP>
__global__ void __launch_bounds__(256) cat_bwd_scalar_kernel(const T* __restrict__ g, int ldg,
                                                             int coff, int H, int W, CatSrc s,
                                                             void* dsrc, int ldd, int dsd,
                                                             int acc, float* __restrict__ dscale,
                                                             int chunk) {
  __shared__ float red[256];
  const int n = blockIdx.z;
  const int Cl = s.C < 256 ? s.C : 256;
  const int lanes = 256 / Cl;
  const int cl = threadIdx.x % Cl, lane = threadIdx.x / Cl;
  const long P = (long)s.h * s.w;
  const long p0 = (long)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  for (int c0 = 0; c0 < s.C; c0 += Cl) {
    const int c = c0 + cl;
    float ds = 0.f;
    if (lane < lanes && c < s.C) {
      const float sc = s.scale ? s.scale[n * s.C + c] : 1.f;
      for (long p = p0 + lane; p < p1; p += lanes) {
        float gv;
        if (OP == UM_CAT_COPY) {
          gv = to_f32(g[((long)n * P + p) * ldg + coff + c]);
        } else {
          const int py = p / s.w, px = p % s.w;
          gv = 0.f;
#pragma unroll
          for (int u = 0; u < 7; ++u) {
            const float wy = up_w(2 * py - 2 + u, py, s.h, H);
            if (wy == 0.f) continue;
#pragma unroll
            for (int v = 0; v < 7; ++v) {
              const float wx = up_w(2 * px - 2 + v, px, s.w, W);
              if (wx == 0.f) continue;
              gv += wy * wx * to_f32(g[((long)(n * H + 2 * py - 2 + u) * W + 2 * px - 2 + v) * ldg +
                                       coff + c]);
            }
          }
        }
        const long sp = (long)n * P + p;
        if (dsrc) st_any(dsrc, sp * ldd + c, dsd, gv * sc, acc);
        if (dscale) ds += gv * ld_any(s.ptr, sp * s.ld + c, s.dtype);
      }
    }
    if (dscale) {
      red[threadIdx.x] = ds;
      __syncthreads();
      if (lane == 0 && c < s.C) {
        for (int r = 1; r < lanes; ++r) ds += red[r * Cl + cl];
        dscale[((long)n * gridDim.x + blockIdx.x) * s.C + c] = ds;
      }
      __syncthreads();
    }
  }
}

// UP2 adjoint of a 4-channel source (the disparity maps) at 4-aligned channel
// offsets: thread = one source pixel, all 4 channels per tap as one 8-byte
// (bf16) / 16-byte (f32) load.  Only high-res taps X in [2x-1, 2x+2] (and Y
// likewise) carry nonzero weight under the x2 align_corners upsample (the
// scalar path scans 2x-2 .. 2x+4), so the 16 loads are issued together with
// clamped addresses and zero weights, then summed in the scalar path's order
// (u, then v; adding exact zeros leaves the sums bit-identical).
template <typename T>
__global__ void __launch_bounds__(256) cat_bwd_up2c4_kernel(const T* __restrict__ g, int ldg,
                                                            int coff, int H, int W, CatSrc s,
                                                            void* dsrc, int ldd, int dsd, int acc,
                                                            float* __restrict__ dscale, int chunk) {
  __shared__ float red[4][256];
  const int n = blockIdx.z;
  const long P = (long)s.h * s.w;
  const long p0 = (long)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  float sc[4] = {1.f, 1.f, 1.f, 1.f};
  if (s.scale)
#pragma unroll
    for (int c = 0; c < 4; ++c) sc[c] = s.scale[n * 4 + c];
  float ds[4] = {0.f, 0.f, 0.f, 0.f};
  for (long p = p0 + threadIdx.x; p < p1; p += 256) {
    const int py = p / s.w, px = p % s.w;
    float wy[4], wx[4];
    int yy[4], xx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      wy[u] = up_w(2 * py - 1 + u, py, s.h, H);
      yy[u] = min(max(2 * py - 1 + u, 0), H - 1);
      wx[u] = up_w(2 * px - 1 + u, px, s.w, W);
      xx[u] = min(max(2 * px - 1 + u, 0), W - 1);
    }
    float t[4][4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const long off = ((long)(n * H + yy[u]) * W + xx[v]) * ldg + coff;
        if constexpr (sizeof(T) == 2) {
          const uint2 q = *reinterpret_cast<const uint2*>(g + off);
          t[u][v][0] = __uint_as_float(q.x << 16);
          t[u][v][1] = __uint_as_float(q.x & 0xffff0000u);
          t[u][v][2] = __uint_as_float(q.y << 16);
          t[u][v][3] = __uint_as_float(q.y & 0xffff0000u);
        } else {
          const float4 f = *reinterpret_cast<const float4*>(g + off);
          t[u][v][0] = f.x; t[u][v][1] = f.y; t[u][v][2] = f.z; t[u][v][3] = f.w;
        }
      }
    float gv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int c = 0; c < 4; ++c) gv[c] += wy[u] * wx[v] * t[u][v][c];
    const long sp = (long)n * P + p;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (dsrc) st_any(dsrc, sp * ldd + c, dsd, gv[c] * sc[c], acc);
      if (dscale) ds[c] += gv[c] * ld_any(s.ptr, sp * s.ld + c, s.dtype);
    }
  }
  if (dscale) {
#pragma unroll
    for (int c = 0; c < 4; ++c) red[c][threadIdx.x] = ds[c];
    __syncthreads();
    if (threadIdx.x < 4) {
      float t = 0.f;
      for (int i = 0; i < 256; ++i) t += red[threadIdx.x][i];
      dscale[((long)n * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = t;
    }
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

// the same with 8 concat channels per thread (C, coff, ldd multiples of 8):
// four 16-byte loads (the 2x2 sub-pixels), the 32 source values of channels
// [4*c0, 4*c0 + 32) as four 8-element stores
template <typename T>
__global__ void cat_bwd_pshuf8_kernel(const T* __restrict__ g, int ldg, int coff, int H, int W,
                                      CatSrc s, void* dsrc, int ldd, int dsd, int acc) {
  const int n = blockIdx.z;
  const int C8 = s.C / 8;
  const long P = (long)s.h * s.w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P * C8;
       i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long p = i / C8;
    const int py = p / s.w, px = p % s.w;
    float v[4][8];
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      const int yy = 2 * py + (sub >> 1), xx = 2 * px + (sub & 1);
      load8(g + ((long)(n * H + yy) * W + xx) * ldg + coff + c8 * 8, v[sub]);
    }
    const long base = ((long)n * P + p) * ldd + c8 * 32;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const float w[8] = {v[0][2 * o], v[1][2 * o], v[2][2 * o], v[3][2 * o],
                          v[0][2 * o + 1], v[1][2 * o + 1], v[2][2 * o + 1], v[3][2 * o + 1]};
      st8_any(dsrc, base + o * 8, dsd, w, acc);
    }
  }
}

// ---- SE
constexpr int MEAN_PIX = 2048;  // pixels per block
// out[n][c] += mean over a pixel chunk (out zeroed by the caller): thread =
// (8-channel group, pixel lane), 16-byte loads, 2 pixels in flight
template <typename T>
__global__ void __launch_bounds__(256) channel_mean_kernel(const T* __restrict__ x, int ld, long S,
                                                            int C, float* __restrict__ out) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.y;
  const int cg = C / 8;
  const RowMap rm(cg);
  const long p0 = (long)blockIdx.x * MEAN_PIX, p1 = min(S, p0 + MEAN_PIX);
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && g < cg) {
      const T* base = x + (long)n * S * ld + g * 8;
      long p = p0 + rm.lane;
      for (; p + rm.lanes < p1; p += 2 * rm.lanes) {
        float u[8], v[8];
        load8(base + p * ld, u);
        load8(base + (p + rm.lanes) * ld, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += u[e] + v[e];
      }
      if (p < p1) {
        float u[8];
        load8(base + p * ld, u);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += u[e];
      }
    }
    lane_reduce<8>(red, rm, acc);
    if (rm.lane == 0 && g < cg)
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&out[n * C + g * 8 + e], acc[e] / (float)S);
  }
}

// one block per image: pooled = (sum of the image's pool partial rows) / HW
// (written out for the backward), then the excite MLP.  The partial rows are
// summed by column lanes x row lanes (256 threads) and combined in LDS.
__global__ void __launch_bounds__(256) se_mlp_fwd_kernel(
    const float* __restrict__ parts, int nparts, float inv_hw, float* __restrict__ pooled,
    const float* __restrict__ w1, const float* __restrict__ w2, int C, int R,
    float* __restrict__ z1, float* __restrict__ s) {
  extern __shared__ float sh[];
  const int n = blockIdx.x;
  float* p = sh;            // [C]
  float* z = sh + C;        // [R]
  float* red = z + R;       // [256]
  const int CU = C < 256 ? C : 256;
  const int L = 256 / CU;
  const int u = threadIdx.x % CU, l = threadIdx.x / CU;
  for (int c0 = 0; c0 < C; c0 += CU) {
    const int c = c0 + u;
    float t = 0.f;
    if (l < L && c < C) {
      // 8 independent partial sums: 8 loads in flight per thread (the
      // grid is one block per image, so this loop is latency-bound)
      const float* q = parts + (long)n * nparts * C + c;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int b = l;
      for (; b + 7 * L < nparts; b += 8 * L) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += q[(long)(b + k * L) * C];
      }
      for (; b < nparts; b += L) acc[0] += q[(long)b * C];
      t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    red[threadIdx.x] = t;
    __syncthreads();
    if (l == 0 && c < C) {
      for (int k = 1; k < L; ++k) t += red[k * CU + u];
      t *= inv_hw;
      p[c] = t;
      pooled[n * C + c] = t;
    }
    __syncthreads();
  }
  // z = relu(W1 p): LP lanes per output row (all R rows in one pass for R <=
  // 256 / LP), each lane 4 inputs per 16-byte load with every load of its
  // slice issued before the sums -- one round of load latency instead of
  // R / 4 dependent wave rounds
  int LP = 64;
  while (LP > 1 && LP * R > 256) LP >>= 1;
  const int vec = (C % 4 == 0) ? 4 : 1;
  for (int r0 = 0; r0 < R; r0 += 256 / LP) {
    const int r = r0 + (int)threadIdx.x / LP, j = threadIdx.x % LP;
    float t = 0.f;
    if (r < R) {
      const float* wr = w1 + (long)r * C;
      if (vec == 4) {
#pragma unroll 4
        for (int c = j * 4; c < C; c += LP * 4) {
          const float4 a = *reinterpret_cast<const float4*>(wr + c);
          t += a.x * p[c] + a.y * p[c + 1] + a.z * p[c + 2] + a.w * p[c + 3];
        }
      } else {
        for (int c = j; c < C; c += LP) t += wr[c] * p[c];
      }
    }
    for (int o = LP >> 1; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (r < R && j == 0) {
      t = fmaxf(t, 0.f);
      z[r] = t;
      z1[n * R + r] = t;
    }
  }
  __syncthreads();
  // s = sigmoid(W2 z): thread per output channel, its W2 row (R contiguous
  // floats) in 16-byte loads
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* wc = w2 + (long)c * R;
    float t = 0.f;
    if (R % 4 == 0) {
      for (int r = 0; r < R; r += 4) {
        const float4 a = *reinterpret_cast<const float4*>(wc + r);
        t += a.x * z[r] + a.y * z[r + 1] + a.z * z[r + 2] + a.w * z[r + 3];
      }
    } else {
      for (int r = 0; r < R; ++r) t += wc[r] * z[r];
    }
    s[n * C + c] = sigmoidf_(t);
  }
}

// dw1 [R][C], dw2 [C][R] written (not accumulated); dpool_scaled[n][c] = dpool / S
// SE excite backward, two launches:
//  (1) dz[n][r] = relu'(z1) * sum_c w2[c][r] * ds[n][c] s(1-s): one wave per
//      (n, r), lanes over c;
//  (2) one thread per output of dw2[c][r] += sum_n dl2[n][c] z1[n][r],
//      dw1[r][c] += sum_n dz[n][r] pooled[n][c] and
//      dpool[n][c] = inv_S * sum_r w1[r][c] dz[n][r]
__global__ void __launch_bounds__(256) se_dz_kernel(int N, int C, int R, const float* __restrict__ ds,
                                                     const float* __restrict__ s,
                                                     const float* __restrict__ z1,
                                                     const float* __restrict__ w2,
                                                     float* __restrict__ dz) {
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (pair >= N * R) return;
  const int n = pair / R, r = pair % R;
  float t = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float sv = s[n * C + c];
    t += w2[c * R + r] * ds[n * C + c] * sv * (1.f - sv);
  }
  t = wave_sum(t);
  if (lane == 0) dz[pair] = z1[pair] > 0.f ? t : 0.f;
}

__global__ void __launch_bounds__(256) se_wgrad_kernel(int N, int C, int R, const float* __restrict__ ds,
                                                        const float* __restrict__ s,
                                                        const float* __restrict__ z1,
                                                        const float* __restrict__ pooled,
                                                        const float* __restrict__ w1,
                                                        const float* __restrict__ dz,
                                                        float* __restrict__ dw1,
                                                        float* __restrict__ dw2,
                                                        float* __restrict__ dpool, float inv_S) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long CR = (long)C * R;
  if (i < CR) {  // dw2[c][r]
    const int c = i / R, r = i % R;
    float t = 0.f;
    for (int n = 0; n < N; ++n) {
      const float sv = s[n * C + c];
      t += ds[n * C + c] * sv * (1.f - sv) * z1[n * R + r];
    }
    dw2[i] = t;
  } else if (i < 2 * CR) {  // dw1[r][c]
    const long j = i - CR;
    const int r = j / C, c = j % C;
    float t = 0.f;
    for (int n = 0; n < N; ++n) t += dz[n * R + r] * pooled[n * C + c];
    dw1[j] = t;
  } else if (i < 2 * CR + (long)N * C) {  // dpool[n][c]
    const long j = i - 2 * CR;
    const int n = j / C, c = j % C;
    float t = 0.f;
    for (int r = 0; r < R; ++r) t += w1[r * C + c] * dz[n * R + r];
    dpool[j] = t * inv_S;
  }
}

// dscale[n][c] (+)= sum_b parts[n][b][c]: block = (cl channels) x (256/cl
// b-lanes), grid (ceil(C/cl), N)
__global__ void __launch_bounds__(256) parts_accum_kernel(const float* __restrict__ parts, int B,
                                                          int C, float* __restrict__ out, int cl,
                                                          int store) {
  __shared__ float red[256];
  const int lanes = 256 / cl;
  const int n = blockIdx.y;
  const int c = blockIdx.x * cl + (threadIdx.x % cl);
  const int lane = threadIdx.x / cl;
  float t0 = 0.f, t1 = 0.f;
  if (c < C) {
    const float* p = parts + (long)n * B * C + c;
    int b = lane;
    for (; b + lanes < B; b += 2 * lanes) {
      t0 += p[(long)b * C];
      t1 += p[(long)(b + lanes) * C];
    }
    if (b < B) t0 += p[(long)b * C];
  }
  float t = t0 + t1;
  red[threadIdx.x] = t;
  __syncthreads();
  if (lane == 0 && c < C) {
    for (int q = 1; q < lanes; ++q) t += red[q * cl + (threadIdx.x % cl)];
    out[n * C + c] = store ? t : out[n * C + c] + t;
  }
}


// tuning key cat_fused (default 0): all sources of a concat in one launch.
// Measured slower (decoder concats 514 -> 693 us per step, 716 -> 705
// pairs/s): waves spanning several sources run every source's path, and the
// per-source launches already write whole 16-byte lanes
bool cat_fused() {
  static const int v = (int)umamd::tuning_env("cat_fused", 0);
  return v != 0;
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
  UM_CHECK_ARG(Ctot % 8 == 0 && ld % 8 == 0, "um_concat_build: Ctot/ld %% 8");
  int covered = 0;
  if (cat_fused()) {
    for (int i = 0; i < nsrc; ++i) {
      UM_CHECK_ARG(a.s[i].coff == covered && a.s[i].coff % 8 == 0,
                   "um_concat_build: source %d must start at the 8-aligned end of the previous", i);
      covered = a.s[i].coff + (a.s[i].C + 7) / 8 * 8;
    }
    UM_CHECK_ARG(covered == Ctot, "um_concat_build: sources cover %d of %d channels", covered, Ctot);
    const int ng = Ctot / 8;
    const dim3 g(ceil_div((long)W * ng, 256), H, N);
    if (dtype == UM_BF16)
      hipLaunchKernelGGL(cat_all_kernel<bf16_t>, g, dim3(256), 0, st, a, N, H, W, (bf16_t*)dst, ld, ng);
    else
      hipLaunchKernelGGL(cat_all_kernel<float>, g, dim3(256), 0, st, a, N, H, W, (float*)dst, ld, ng);
    UM_LAUNCH_CHECK();
    return UM_OK;
  }
  for (int i = 0; i < nsrc; ++i) {
    const CatSrc& s = a.s[i];
    UM_CHECK_ARG(s.coff == covered && s.coff % 8 == 0,
                 "um_concat_build: source %d must start at the 8-aligned end of the previous", i);
    covered = s.coff + (s.C + 7) / 8 * 8;
    const dim3 g(ceil_div((long)W * ((s.C + 7) / 8), 256), H, N);
#define CAT_LAUNCH(T, OP) \
  hipLaunchKernelGGL((cat_src_kernel<T, OP>), g, dim3(256), 0, st, s, N, H, W, (T*)dst, ld)
    if (dtype == UM_BF16) {
      if (s.op == UM_CAT_COPY) CAT_LAUNCH(bf16_t, UM_CAT_COPY);
      else if (s.op == UM_CAT_UP2) CAT_LAUNCH(bf16_t, UM_CAT_UP2);
      else CAT_LAUNCH(bf16_t, UM_CAT_PSHUF);
    } else {
      if (s.op == UM_CAT_COPY) CAT_LAUNCH(float, UM_CAT_COPY);
      else if (s.op == UM_CAT_UP2) CAT_LAUNCH(float, UM_CAT_UP2);
      else CAT_LAUNCH(float, UM_CAT_PSHUF);
    }
#undef CAT_LAUNCH
  }
  UM_CHECK_ARG(covered == Ctot, "um_concat_build: sources cover %d of %d channels", covered, Ctot);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

long um_concat_bwd_ws(int N, int h, int w, int C) {
  const long P = (long)h * w;
  return (long)N * ceil_div(P, bwd_chunk(P, N)) * C;
}

int um_concat_bwd_src(int dtype, int N, int H, int W, const void* g, int ldg,
                      const um_cat_src* src, void* dsrc, int ldd, int dsrc_dtype, int accumulate,
                      float* dscale, float* ws, hipStream_t st) {
  // accumulate bit 0: dsrc (+=); bit 1: dscale is WRITTEN (=) instead of added
  // to (no zero fill of the gate gradient beforehand)
  const int store_scale = (accumulate >> 1) & 1;
  accumulate &= 1;
  const um_cat_src& s0 = *src;
  CatSrc s{s0.ptr, s0.scale, s0.C, s0.ld, s0.op, s0.coff, s0.dtype, s0.h, s0.w};
  UM_CHECK_ARG(ldg % 8 == 0, "um_concat_bwd_src: ldg %% 8");
  if (s.op == UM_CAT_PSHUF) {
    UM_CHECK_ARG(dsrc != nullptr && dscale == nullptr, "um_concat_bwd_src: pshuf args");
    if (s.C % 8 == 0 && s.coff % 8 == 0 && ldd % 8 == 0) {
      const long per_n8 = (long)s.h * s.w * s.C / 8;
      dim3 grid8((unsigned)std::min<long>((per_n8 + 255) / 256, 2048), 1, N);
      if (dtype == UM_BF16)
        hipLaunchKernelGGL(cat_bwd_pshuf8_kernel<bf16_t>, grid8, dim3(256), 0, st,
                           (const bf16_t*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate);
      else
        hipLaunchKernelGGL(cat_bwd_pshuf8_kernel<float>, grid8, dim3(256), 0, st,
                           (const float*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate);
      UM_LAUNCH_CHECK();
      return UM_OK;
    }
    const long per_n = (long)s.h * s.w * 4 * s.C;
    dim3 grid((unsigned)std::min<long>((per_n + 255) / 256, 2048), 1, N);
    if (dtype == UM_BF16)
      hipLaunchKernelGGL(cat_bwd_pshuf_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)g,
                         ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate);
    else
      hipLaunchKernelGGL(cat_bwd_pshuf_kernel<float>, grid, dim3(256), 0, st, (const float*)g, ldg,
                         s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate);
    UM_LAUNCH_CHECK();
    return UM_OK;
  }
  const long P = (long)s.h * s.w;
  const bool vec = (s.C % 8 == 0) && (s.coff % 8 == 0) && (ldd % 8 == 0 || !dsrc) &&
                   (s.ld % 8 == 0 || !dscale);
  const int chunk = bwd_chunk(P, N);
  const int nblk = ceil_div(P, chunk);
  UM_CHECK_ARG(!dscale || ws, "um_concat_bwd_src: gate gradient needs the workspace");
  float* parts = dscale ? ws : nullptr;
  if (!vec && s.op == UM_CAT_UP2 && s.C == 4 && s.coff % 4 == 0 && H == 2 * s.h &&
      W == 2 * s.w) {
    dim3 grid(nblk, 1, N);
    if (dtype == UM_BF16)
      hipLaunchKernelGGL(cat_bwd_up2c4_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)g,
                         ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, parts, chunk);
    else
      hipLaunchKernelGGL(cat_bwd_up2c4_kernel<float>, grid, dim3(256), 0, st, (const float*)g, ldg,
                         s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, parts, chunk);
  } else if (!vec) {
    dim3 grid(nblk, 1, N);
#define UM_CAT_SCALAR(T_, OP_)                                                               \
    hipLaunchKernelGGL((cat_bwd_scalar_kernel<T_, OP_>), grid, dim3(256), 0, st, (const T_*)g, \
                       ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype, accumulate, parts, chunk)
    if (dtype == UM_BF16) {
      if (s.op == UM_CAT_COPY) UM_CAT_SCALAR(bf16_t, UM_CAT_COPY); else UM_CAT_SCALAR(bf16_t, UM_CAT_UP2);
    } else {
      if (s.op == UM_CAT_COPY) UM_CAT_SCALAR(float, UM_CAT_COPY); else UM_CAT_SCALAR(float, UM_CAT_UP2);
    }
#undef UM_CAT_SCALAR
  } else {
    dim3 grid(nblk, 1, N);
    if (s.op == UM_CAT_COPY) {
      if (dtype == UM_BF16)
        hipLaunchKernelGGL((cat_bwd_kernel<bf16_t, UM_CAT_COPY>), grid, dim3(256), 0, st,
                           (const bf16_t*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate, parts, chunk);
      else
        hipLaunchKernelGGL((cat_bwd_kernel<float, UM_CAT_COPY>), grid, dim3(256), 0, st,
                           (const float*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate, parts, chunk);
    } else {
      if (dtype == UM_BF16)
        hipLaunchKernelGGL((cat_bwd_kernel<bf16_t, UM_CAT_UP2>), grid, dim3(256), 0, st,
                           (const bf16_t*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate, parts, chunk);
      else
        hipLaunchKernelGGL((cat_bwd_kernel<float, UM_CAT_UP2>), grid, dim3(256), 0, st,
                           (const float*)g, ldg, s.coff, H, W, s, dsrc, ldd, dsrc_dtype,
                           accumulate, parts, chunk);
    }
  }
  if (dscale) {  // per-block partials -> dscale (+=)
    int cl = 1;
    while (cl < s.C && cl < 64) cl <<= 1;
    hipLaunchKernelGGL(parts_accum_kernel, dim3(ceil_div(s.C, cl), N), dim3(256), 0, st, parts,
                       nblk, s.C, dscale, cl, store_scale);
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_channel_mean(int dtype, int N, long S, int C, const void* x, int ld, float* out,
                    hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0 && ld % 8 == 0, "um_channel_mean: C/ld %% 8");
  dim3 grid(ceil_div(S, MEAN_PIX), N);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(channel_mean_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, ld,
                       S, C, out);
  else
    hipLaunchKernelGGL(channel_mean_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ld, S,
                       C, out);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_se_mlp_fwd(int N, int C, int R, const float* pool_parts, int parts_per_image,
                  float inv_hw, float* pooled, const float* w1, const float* w2, float* z1,
                  float* s, hipStream_t st) {
  hipLaunchKernelGGL(se_mlp_fwd_kernel, dim3(N), dim3(256), (C + R + 256) * sizeof(float), st,
                     pool_parts, parts_per_image, inv_hw, pooled, w1, w2, C, R, z1, s);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_se_mlp_bwd(int N, int C, int R, const float* ds, const float* s, const float* z1,
                  const float* pooled, const float* w1, const float* w2, float* dw1, float* dw2,
                  float* dpool_scaled, float* dz, float inv_S, hipStream_t st) {
  hipLaunchKernelGGL(se_dz_kernel, dim3(ceil_div((long)N * R, 4)), dim3(256), 0, st, N, C, R, ds, s,
                     z1, w2, dz);
  const long outs = 2l * C * R + (long)N * C;
  hipLaunchKernelGGL(se_wgrad_kernel, dim3(ceil_div(outs, 256)), dim3(256), 0, st, N, C, R, ds, s,
                     z1, pooled, w1, dz, dw1, dw2, dpool_scaled, inv_S);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
