// Disparity/uncertainty heads, bf16 (gfx950): the 4-output 3x3 reflect-pad
// conv + scale*sigmoid of reference model/layers/decoder.py:244-247, forward
// and input gradient, with the split-bf16 weights of um_pack_weight_split
// (rows 0-3 = bf16(w), rows 4-7 = bf16(w - bf16(w))).
//
// A 4-output conv is a GEMM with 8 (split) columns: on the 256-row implicit
// GEMM tiles it needed split-K plus a partial-sum epilogue (the 32x64 head:
// 15.9 us GEMM + 21.7 us epilogue + 4.9 us finish) and the data gradient
// padded the 8 dlogit channels of each tap to a 32-deep MFMA step (55-86 us
// + a border pass of 11-15 us).  Here both directions are one pass:
//   - 16-pixel strips (W % 16 == 0), MFMA operands loaded straight from
//     global into registers (lane = pixel, 16 contiguous bytes of channels),
//     the weights staged once per persistent workgroup in LDS (stream1x1's
//     conflict-free 64-byte rows) or held in registers;
//   - forward: D = W . X^T (v_mfma_f32_16x16x32_bf16, weights as the A
//     operand, 8 of 16 rows live): a lane ends with 4 hi rows (kq = 0) or 4
//     lo rows (kq = 1) of one pixel; one shuffle adds the halves, the
//     epilogue adds the bias and applies scale*sigmoid, and the 4 disparity
//     channels leave as one 16-byte store -- no f32 z round trip, no finish
//     launch.  C <= 64: a wave walks a column of U output rows x 16 pixels,
//     loading each of its U + 2 input rows ONCE per channel chunk; the
//     column taps are that row moved one lane by DPP row shifts (the strip's
//     outer neighbours loaded by lanes 0 / 15 only).  C = 128 / 256 (64k /
//     16k pixels): the 9 C/32 k-steps of a strip are split over the 4 waves
//     of a workgroup and meet in LDS, so the small grids reach every SIMD;
//   - data gradient: D = W^T . dL^T with one tap ROW per 32-deep k-step (kq =
//     tap column x 8 dlogit channels), so a column of U output rows needs U + 2
//     input-row loads; the reflect adjoint is folded into the operand load
//     (interior pixels: one 16-byte load; rows/cols 1 and n-2 add their
//     mirror sources, f32 sum rounded once to bf16) -- no zero-pad pass +
//     border pass.  Output rows go through LDS and leave as 16-byte rows
//     (1 KB per instruction at C = 32), optional accumulate.
#include <algorithm>

#include "common.h"

namespace {

constexpr int DH_NTAP = 9;

// 64-byte row `row` of plane `ks` (nr rows per plane), 16-byte chunk c8,
// swizzled as stream1x1 / igemm's Img<bf16, 32>
__device__ __forceinline__ int dh_img(int ks, int nr, int row, int c8) {
  return (ks * nr + row) * 32 + ((c8 ^ ((4 - ((row >> 2) & 3)) & 3)) << 3);
}

struct DHFwd {
  const bf16_t* x;
  const bf16_t* wf;  // [8][3][3][C]
  const float* bias;
  float* d;
  int N, H, W, C, ldx, ldd;
  float scale;
};

// KS = C / 32 channel chunks; KW = waves sharing one strip's k-steps (1 or
// 4); U = strips per wave per iteration
template <int KS, int KW, int U>
__global__ void __launch_bounds__(256) dhead_fwd_kernel(DHFwd a, int nstrips) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sW[];  // [9*KS][8][32]
  __shared__ float red[KW > 1 ? 4 : 1][KW > 1 ? U * 32 * 4 : 1];
  constexpr int NKS = DH_NTAP * KS;               // k-steps of a strip
  constexpr int NK = (NKS + KW - 1) / KW;         // k-steps per wave
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < NKS * 8 * 4; i += 256) {
    const int kstep = i >> 5, r = (i >> 2) & 7, c8 = i & 3;
    const int tap = kstep / KS, ks = kstep - tap * KS;
    const uint4 v =
        *reinterpret_cast<const uint4*>(a.wf + ((long)r * DH_NTAP + tap) * a.C + ks * 32 + c8 * 8);
    *reinterpret_cast<uint4*>(&sW[dh_img(kstep, 8, r, c8)]) = v;
  }
  __syncthreads();
  const int px = lane & 15, kq = lane >> 4;
  const int kw = KW > 1 ? w : 0;
  const long HW = (long)a.H * a.W;
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) bv = *reinterpret_cast<const float4*>(a.bias);
  const long per_iter = KW > 1 ? (long)gridDim.x * U : (long)gridDim.x * 4 * U;
  for (long s0 = KW > 1 ? (long)blockIdx.x * U : ((long)blockIdx.x * 4 + w) * U; s0 < nstrips;
       s0 += per_iter) {
    bf16x8_t b[U][NK];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = (s0 + u) * 16 + px;
      const bool in = s0 + u < nstrips;
      const int n = (int)(m / HW);
      const int rem = (int)(m - n * HW);
      const int h = rem / a.W, wc = rem - h * a.W;
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        const int kstep = kw + j * KW;
        const int tap = kstep / KS, ks = kstep - tap * KS;
        if (in && kstep < NKS) {
          const int tr = tap / 3, tc = tap - tr * 3;
          const int hh = reflect_idx(h + tr - 1, a.H), ww = reflect_idx(wc + tc - 1, a.W);
          b[u][j] = *reinterpret_cast<const bf16x8_t*>(
              a.x + ((long)n * HW + (long)hh * a.W + ww) * a.ldx + ks * 32 + kq * 8);
        } else {
          b[u][j] = bf16x8_t{};
        }
      }
    }
    f32x4_t acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int kstep = kw + j * KW;
      if (kstep >= NKS) break;
      bf16x8_t af = bf16x8_t{};
      if (px < 8) af = *reinterpret_cast<const bf16x8_t*>(&sW[dh_img(kstep, 8, px, kq)]);
#pragma unroll
      for (int u = 0; u < U; ++u)
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[u][j], acc[u], 0, 0, 0);
    }
    if constexpr (KW > 1) {  // the 4 waves' partial sums of rows 0-7 meet in LDS
      if (kq < 2)
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[w][(u * 32 + lane) * 4 + e] = acc[u][e];
      __syncthreads();
      if (w == 0 && kq < 2)
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[u][e] = red[0][(u * 32 + lane) * 4 + e] + red[1][(u * 32 + lane) * 4 + e] +
                        red[2][(u * 32 + lane) * 4 + e] + red[3][(u * 32 + lane) * 4 + e];
      __syncthreads();
      if (w != 0) continue;
    }
    // lane (px, kq=0): hi rows 0-3 of pixel px; lane + 16: the lo rows
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[u][e] + __shfl(acc[u][e], lane + 16, 64);
      const long m = (s0 + u) * 16 + px;
      if (kq == 0 && s0 + u < nstrips)
        *reinterpret_cast<float4*>(a.d + m * a.ldd) =
            make_float4(a.scale * sigmoidf_(v[0] + bv.x), a.scale * sigmoidf_(v[1] + bv.y),
                        a.scale * sigmoidf_(v[2] + bv.z), a.scale * sigmoidf_(v[3] + bv.w));
    }
  }
}

// Narrow inputs (C <= 64): a wave owns a column of U output rows x 16
// pixels.  The rows overlap in their taps, so the wave loads the U + 2 input
// rows it needs once per column shift (3 (U + 2) KS fragments instead of
// 9 U KS): the 9-fold tap re-reads had made the cache hierarchy, not HBM, the
// limit (256x512 C32: 41.8 us for 80 MB).
template <int KS, int U>
__global__ void __launch_bounds__(256) dhead_fwd_col_kernel(DHFwd a, int units) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sW[];  // [9*KS][8][32]
  constexpr int NKS = DH_NTAP * KS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < NKS * 8 * 4; i += 256) {
    const int kstep = i >> 5, r = (i >> 2) & 7, c8 = i & 3;
    const int tap = kstep / KS, ks = kstep - tap * KS;
    const uint4 v =
        *reinterpret_cast<const uint4*>(a.wf + ((long)r * DH_NTAP + tap) * a.C + ks * 32 + c8 * 8);
    *reinterpret_cast<uint4*>(&sW[dh_img(kstep, 8, r, c8)]) = v;
  }
  __syncthreads();
  const int px = lane & 15, kq = lane >> 4;
  const int hb = (a.H + U - 1) / U, wb = a.W / 16;
  const long HW = (long)a.H * a.W;
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) bv = *reinterpret_cast<const float4*>(a.bias);
  for (int t = blockIdx.x * 4 + w; t < units; t += gridDim.x * 4) {
    const int n = t / (hb * wb), rem = t - n * hb * wb;
    const int h0 = (rem / wb) * U, w0 = (rem % wb) * 16;
    const bf16_t* xn = a.x + (long)n * HW * a.ldx;
    bf16x8_t b[U + 2][3][KS];
#pragma unroll
    for (int j = 0; j < U + 2; ++j) {
      const int hh = reflect_idx(min(h0 - 1 + j, a.H), a.H);
#pragma unroll
      for (int tc = 0; tc < 3; ++tc) {
        const int ww = reflect_idx(w0 + px + tc - 1, a.W);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          b[j][tc][ks] = *reinterpret_cast<const bf16x8_t*>(
              xn + ((long)hh * a.W + ww) * a.ldx + ks * 32 + kq * 8);
      }
    }
    f32x4_t acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < DH_NTAP; ++tap)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8_t af = bf16x8_t{};
        if (px < 8) af = *reinterpret_cast<const bf16x8_t*>(&sW[dh_img(tap * KS + ks, 8, px, kq)]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[u + tap / 3][tap % 3][ks], acc[u],
                                                           0, 0, 0);
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[u][e] + __shfl(acc[u][e], lane + 16, 64);
      if (kq == 0 && h0 + u < a.H)
        *reinterpret_cast<float4*>(a.d + ((long)n * HW + (long)(h0 + u) * a.W + w0 + px) * a.ldd) =
            make_float4(a.scale * sigmoidf_(v[0] + bv.x), a.scale * sigmoidf_(v[1] + bv.y),
                        a.scale * sigmoidf_(v[2] + bv.z), a.scale * sigmoidf_(v[3] + bv.w));
    }
  }
}

typedef __attribute__((ext_vector_type(4))) int i32x4_t;

// row_shr:1 (SHL = false: lane px <- px - 1) or row_shl:1 (lane px <- px + 1)
// within each 16-lane row; the row's first (last) lane takes `edge`
template <bool SHL>
__device__ __forceinline__ bf16x8_t dh_shift(bf16x8_t v, bf16x8_t edge) {
  const i32x4_t s = __builtin_bit_cast(i32x4_t, v), e = __builtin_bit_cast(i32x4_t, edge);
  i32x4_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r[i] = __builtin_amdgcn_update_dpp(e[i], s[i], SHL ? 0x101 : 0x111, 0xf, 0xf, false);
  return __builtin_bit_cast(bf16x8_t, r);
}

// The column kernel with ONE load per input row and channel chunk: the
// column taps tc = 0 / 2 are the row's fragments moved one lane right / left
// by DPP row shifts, the strip's outer neighbours (w0 - 1, w0 + 16) loaded by
// lanes 0 and 15 of each row only.  Loads issue before the weight staging.
template <int KS, int U>
__global__ void __launch_bounds__(256) dhead_fwd_dpp_kernel(DHFwd a, int units) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sW[];  // [9*KS][8][32]
  constexpr int NKS = DH_NTAP * KS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int px = lane & 15, kq = lane >> 4;
  const int hb = (a.H + U - 1) / U, wb = a.W / 16;
  const long HW = (long)a.H * a.W;
  bf16x8_t b[U + 2][KS], e[U + 2][KS];
  auto load = [&](int t, int& n, int& h0, int& w0) {
    n = t / (hb * wb);
    const int rem = t - n * hb * wb;
    h0 = (rem / wb) * U;
    w0 = (rem % wb) * 16;
    const bf16_t* xn = a.x + (long)n * HW * a.ldx;
    const bool edge = px == 0 || px == 15;
    const int we = reflect_idx(px == 0 ? w0 - 1 : w0 + 16, a.W);
#pragma unroll
    for (int j = 0; j < U + 2; ++j) {
      const int hh = reflect_idx(min(h0 - 1 + j, a.H), a.H);
      const bf16_t* row = xn + (long)hh * a.W * a.ldx + kq * 8;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        b[j][ks] = *reinterpret_cast<const bf16x8_t*>(row + (long)(w0 + px) * a.ldx + ks * 32);
        e[j][ks] = edge ? *reinterpret_cast<const bf16x8_t*>(row + (long)we * a.ldx + ks * 32)
                        : bf16x8_t{};
      }
    }
  };
  int t = blockIdx.x * 4 + w, n = 0, h0 = 0, w0 = 0;
  if (t < units) load(t, n, h0, w0);
  for (int i = tid; i < NKS * 8 * 4; i += 256) {
    const int kstep = i >> 5, r = (i >> 2) & 7, c8 = i & 3;
    const int tap = kstep / KS, ks = kstep - tap * KS;
    const uint4 v =
        *reinterpret_cast<const uint4*>(a.wf + ((long)r * DH_NTAP + tap) * a.C + ks * 32 + c8 * 8);
    *reinterpret_cast<uint4*>(&sW[dh_img(kstep, 8, r, c8)]) = v;
  }
  __syncthreads();
  // one channel chunk: the 9 tap fragments of this lane's weight row stay in
  // registers for the whole persistent loop (no LDS read per MFMA)
  constexpr bool AREG = KS == 1;
  bf16x8_t wa[AREG ? DH_NTAP : 1];
  if constexpr (AREG) {
#pragma unroll
    for (int k = 0; k < DH_NTAP; ++k)
      wa[k] = px < 8 ? *reinterpret_cast<const bf16x8_t*>(&sW[dh_img(k, 8, px, kq)]) : bf16x8_t{};
  }
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) bv = *reinterpret_cast<const float4*>(a.bias);
  for (; t < units; t += gridDim.x * 4) {
    f32x4_t acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < U + 2; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8_t f1 = b[j][ks];
        const bf16x8_t f0 = dh_shift<false>(f1, e[j][ks]);
        const bf16x8_t f2 = dh_shift<true>(f1, e[j][ks]);
        // input row j feeds output rows u = j - tr for tap rows tr = 0..2
#pragma unroll
        for (int tr = 0; tr < 3; ++tr) {
          const int u = j - tr;
          if (u < 0 || u >= U) continue;
#pragma unroll
          for (int tc = 0; tc < 3; ++tc) {
            bf16x8_t af = bf16x8_t{};
            if constexpr (AREG)
              af = wa[tr * 3 + tc];
            else if (px < 8)
              af = *reinterpret_cast<const bf16x8_t*>(
                  &sW[dh_img((tr * 3 + tc) * KS + ks, 8, px, kq)]);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, tc == 0 ? f0 : (tc == 1 ? f1 : f2),
                                                             acc[u], 0, 0, 0);
          }
        }
      }
    const int n_ = n, h0_ = h0, w0_ = w0;
    if (t + (int)gridDim.x * 4 < units) load(t + gridDim.x * 4, n, h0, w0);  // next unit in flight
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc[u][q] + __shfl(acc[u][q], lane + 16, 64);
      if (kq == 0 && h0_ + u < a.H)
        *reinterpret_cast<float4*>(a.d + ((long)n_ * HW + (long)(h0_ + u) * a.W + w0_ + px) * a.ldd) =
            make_float4(a.scale * sigmoidf_(v[0] + bv.x), a.scale * sigmoidf_(v[1] + bv.y),
                        a.scale * sigmoidf_(v[2] + bv.z), a.scale * sigmoidf_(v[3] + bv.w));
    }
  }
}

struct DHDgrad {
  const bf16_t* dl;  // [M][8] dlogit (channels 4-7 = 0-3: the split rows)
  const bf16_t* wT;  // [C][3][3][8]
  bf16_t* dx;
  int N, H, W, C, ldl, ldx, accumulate;
};

// the 8 dlogit channels of reflect-pad tap (tr, tc) summed over every output
// pixel whose (padded) tap reads input pixel (h, wc): the regular source
// (h - tr + 1, wc - tc + 1) and, next to the border, the mirror sources
// (pad row -1 = row 1, pad row H = row H-2; likewise columns)
__device__ __forceinline__ bf16x8_t dh_dl_frag(const DHDgrad& a, long nbase, int h, int wc, int tr,
                                              int tc) {
  const int r1 = h - tr + 1, c1 = wc - tc + 1;
  const bool v1 = r1 >= 0 && r1 < a.H, u1 = c1 >= 0 && c1 < a.W;
  const int r2 = (h == 1 && tr == 0) ? 0 : ((h == a.H - 2 && tr == 2) ? a.H - 1 : -1);
  const int c2 = (wc == 1 && tc == 0) ? 0 : ((wc == a.W - 2 && tc == 2) ? a.W - 1 : -1);
  auto at = [&](int r, int c) { return a.dl + (nbase + (long)r * a.W + c) * a.ldl; };
  if (r2 < 0 && c2 < 0) {
    if (v1 && u1) return *reinterpret_cast<const bf16x8_t*>(at(r1, c1));
    return bf16x8_t{};
  }
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add = [&](int r, int c) {
    float v[8];
    load8(at(r, c), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += v[e];
  };
  if (v1 && u1) add(r1, c1);
  if (v1 && c2 >= 0) add(r1, c2);
  if (r2 >= 0 && u1) add(r2, c1);
  if (r2 >= 0 && c2 >= 0) add(r2, c2);
  bf16x8_t f;
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (__bf16)s[e];
  return f;
}

// NB = C / 16 output-channel blocks; U strips per wave per iteration
template <int NB, int U>
__global__ void __launch_bounds__(256) dhead_dgrad_kernel(DHDgrad a, int nstrips) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sA[];  // [3][C][32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NR = NB * 16;
  for (int i = tid; i < 3 * NR * 4; i += 256) {
    const int ks = i / (NR * 4), r = (i >> 2) % NR, c8 = i & 3;
    const int tap = ks * 4 + c8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (tap < DH_NTAP) v = *reinterpret_cast<const uint4*>(a.wT + ((long)r * DH_NTAP + tap) * 8);
    *reinterpret_cast<uint4*>(&sA[dh_img(ks, NR, r, c8)]) = v;
  }
  __syncthreads();
  const int px = lane & 15, kq = lane >> 4;
  const long HW = (long)a.H * a.W;
  const long per_iter = (long)gridDim.x * 4 * U;
  for (long s0 = ((long)blockIdx.x * 4 + w) * U; s0 < nstrips; s0 += per_iter) {
    bf16x8_t b[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = (s0 + u) * 16 + px;
      const bool in = s0 + u < nstrips;
      const int n = (int)(m / HW);
      const int rem = (int)(m - n * HW);
      const int h = rem / a.W, wc = rem - h * a.W;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int tap = ks * 4 + kq;
        b[u][ks] = (in && tap < DH_NTAP) ? dh_dl_frag(a, (long)n * HW, h, wc, tap / 3, tap % 3)
                                         : bf16x8_t{};
      }
    }
#pragma unroll 2
    for (int nb = 0; nb < NB; ++nb) {
      f32x4_t acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(&sA[dh_img(ks, NR, nb * 16 + px, kq)]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[u][ks], acc[u], 0, 0, 0);
      }
      // lane: pixel (s0 + u) * 16 + px, channels nb*16 + 4kq .. + 3
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s0 + u >= nstrips) continue;
        const long m = (s0 + u) * 16 + px;
        bf16_t* o = a.dx + m * a.ldx + nb * 16 + kq * 4;
        float v[4] = {acc[u][0], acc[u][1], acc[u][2], acc[u][3]};
        if (a.accumulate) {
          const uint2 p = *reinterpret_cast<const uint2*>(o);
          v[0] += __uint_as_float(p.x << 16);
          v[1] += __uint_as_float(p.x & 0xffff0000u);
          v[2] += __uint_as_float(p.y << 16);
          v[3] += __uint_as_float(p.y & 0xffff0000u);
        }
        store4(o, v);
      }
    }
  }
}

// Narrow outputs (C <= 64): a wave owns a column of U rows x 16 pixels and
// the k-step is one tap ROW (kq = tap column, 8 dlogit channels; kq = 3 is
// zero), so the U x 3 row-tap fragments come from U + 2 input-row loads:
// L[j] = dL row h0 + j - 1 at column w - kq + 1 (+ its column mirror next to
// the border), B(u, tr) = L[u - tr + 2] (+ the row mirror at rows 1, H-2).
// STG: the output tile of one row (16 pixels x C) goes through this wave's
// LDS slice and leaves as 16-byte rows (1 KB contiguous per instruction at
// C = 32) instead of 8-byte stores of 4 channels per lane.
template <int NB, int U, bool STG>
__global__ void __launch_bounds__(256) dhead_dgrad_col_kernel(DHDgrad a, int units) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sA[];  // [3 (tr)][C][32 (tc x 8)]
  constexpr int SROW = NB * 16 + 8;  // staged row (elements): 16 bytes of padding
  __shared__ __attribute__((aligned(16))) bf16_t sO[STG ? 4 : 1][STG ? 16 * SROW : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NR = NB * 16;
  for (int i = tid; i < 3 * NR * 4; i += 256) {
    const int tr = i / (NR * 4), r = (i >> 2) % NR, c8 = i & 3;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (c8 < 3) v = *reinterpret_cast<const uint4*>(a.wT + ((long)r * DH_NTAP + tr * 3 + c8) * 8);
    *reinterpret_cast<uint4*>(&sA[dh_img(tr, NR, r, c8)]) = v;
  }
  __syncthreads();
  const int px = lane & 15, kq = lane >> 4;
  const int hb = (a.H + U - 1) / U, wb = a.W / 16;
  const long HW = (long)a.H * a.W;
  for (int t = blockIdx.x * 4 + w; t < units; t += gridDim.x * 4) {
    const int n = t / (hb * wb), rem = t - n * hb * wb;
    const int h0 = (rem / wb) * U, w0 = (rem % wb) * 16;
    const bf16_t* dln = a.dl + (long)n * HW * a.ldl;
    // this lane's source columns: regular wc - kq + 1 and the mirror
    const int wc = w0 + px;
    const int c1 = wc - kq + 1;
    const bool u1 = kq < 3 && c1 >= 0 && c1 < a.W;
    const int c2 = (kq == 0 && wc == 1) ? 0 : ((kq == 2 && wc == a.W - 2) ? a.W - 1 : -1);
    bf16x8_t L[U + 2];
#pragma unroll
    for (int j = 0; j < U + 2; ++j) {
      const int r = h0 + j - 1;
      const bool rv = r >= 0 && r < a.H;
      if (c2 < 0) {
        L[j] = (rv && u1) ? *reinterpret_cast<const bf16x8_t*>(dln + ((long)r * a.W + c1) * a.ldl)
                          : bf16x8_t{};
      } else {
        float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, v[8];
        if (rv && u1) {
          load8(dln + ((long)r * a.W + c1) * a.ldl, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) s8[e] += v[e];
        }
        if (rv) {
          load8(dln + ((long)r * a.W + c2) * a.ldl, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) s8[e] += v[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) L[j][e] = (__bf16)s8[e];
      }
    }
    // row mirrors (uniform per wave): output row 1 also reads dL row 0
    // through tap row 0, row H-2 reads row H-1 through tap row 2
    const int um1 = h0 == 0 ? 1 : -1;              // u with h0 + u == 1, tr == 0: + L[1]
    const int um2 = (a.H - 2 >= h0 && a.H - 2 < h0 + U) ? a.H - 2 - h0 : -1;  // tr == 2: + L[u + 2]
    auto bfrag = [&](int u, int tr) -> bf16x8_t {
      const bf16x8_t base = L[u - tr + 2];
      int extra = -1;
      if (tr == 0 && u == um1) extra = 1;
      if (tr == 2 && u == um2) extra = u + 2;
      if (extra < 0) return base;
      bf16x8_t f;
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = (__bf16)((float)base[e] + (float)L[extra][e]);
      return f;
    };
    if constexpr (STG) {
      // the 3 x NB weight fragments of this lane, in registers (NB <= 4)
      bf16x8_t wa[3][NB];
#pragma unroll
      for (int tr = 0; tr < 3; ++tr)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          wa[tr][nb] = *reinterpret_cast<const bf16x8_t*>(&sA[dh_img(tr, NR, nb * 16 + px, kq)]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int tr = 0; tr < 3; ++tr) {
            const bf16x8_t af = wa[tr][nb];
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfrag(u, tr), acc, 0, 0, 0);
          }
          const float v[4] = {acc[0], acc[1], acc[2], acc[3]};
          store4(&sO[w][px * SROW + nb * 16 + kq * 4], v);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (h0 + u < a.H) {
          constexpr int CH = NB * 2;  // 16-byte chunks per pixel
#pragma unroll
          for (int i = lane; i < 16 * CH; i += 64) {
            const int p = i / CH, q = i - p * CH;
            bf16_t* o = a.dx + ((long)n * HW + (long)(h0 + u) * a.W + w0 + p) * a.ldx + q * 8;
            uint4 v = *reinterpret_cast<const uint4*>(&sO[w][p * SROW + q * 8]);
            if (a.accumulate) {
              float f[8], g[8];
              load8(reinterpret_cast<const bf16_t*>(&v), f);
              load8(o, g);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] += g[e];
              store8(o, f);
            } else {
              *reinterpret_cast<uint4*>(o) = v;
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      continue;
    }
#pragma unroll 2
    for (int nb = 0; nb < NB; ++nb) {
      f32x4_t acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tr = 0; tr < 3; ++tr) {
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(&sA[dh_img(tr, NR, nb * 16 + px, kq)]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfrag(u, tr), acc[u], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (h0 + u >= a.H) continue;
        bf16_t* o = a.dx + ((long)n * HW + (long)(h0 + u) * a.W + wc) * a.ldx + nb * 16 + kq * 4;
        float v[4] = {acc[u][0], acc[u][1], acc[u][2], acc[u][3]};
        if (a.accumulate) {
          const uint2 p = *reinterpret_cast<const uint2*>(o);
          v[0] += __uint_as_float(p.x << 16);
          v[1] += __uint_as_float(p.x & 0xffff0000u);
          v[2] += __uint_as_float(p.y << 16);
          v[3] += __uint_as_float(p.y & 0xffff0000u);
        }
        store4(o, v);
      }
    }
  }
}

inline bool dh_al(const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; }

int dh_grid(long work_items) { return (int)std::max<long>(1, std::min<long>(work_items, 2048)); }

}  // namespace

extern "C" {

int um_disp_head_ok(int N, int H, int W, int C, int ldx) {
  return N > 0 && H >= 4 && W >= 4 && W % 16 == 0 && (C == 32 || C == 64 || C == 128 || C == 256) &&
         ldx % 8 == 0 && ldx >= C;
}

int um_disp_head_fwd(int N, int H, int W, int C, const void* x, int ldx, const void* wf,
                     const float* bias, float scale, float* d, int ldd, hipStream_t st) {
  UM_CHECK_ARG(um_disp_head_ok(N, H, W, C, ldx), "um_disp_head_fwd: shape N=%d H=%d W=%d C=%d ldx=%d",
               N, H, W, C, ldx);
  UM_CHECK_ARG(x && wf && d && ldd % 4 == 0 && dh_al(x, 16) && dh_al(wf, 16) && dh_al(d, 16) &&
                   (bias == nullptr || dh_al(bias, 16)),
               "um_disp_head_fwd: pointers / ldd");
  DHFwd a{(const bf16_t*)x, (const bf16_t*)wf, bias, d, N, H, W, C, ldx, ldd, scale};
  const long nstrips = (long)N * H * W / 16;
  const size_t lds = (size_t)DH_NTAP * (C / 32) * 8 * 32 * sizeof(bf16_t);
  // measured (tools/head_micro.py, B=8 C2 heads): the DPP column kernel for
  // C = 32 / 64 / 128 (28.5 -> 25.4 / 27.6 -> 19.7 us over the tap-shift
  // loads; 21.3 -> 12.1 us over the k-split strips at C = 128), the k-split
  // strip kernel for C = 256 (16k pixels).  dh_fwd = 1: the shift-load column
  // kernel; dh_fwd128 = 0: the k-split strips at C = 128
  static const int var = (int)umamd::tuning_env("dh_fwd", 0);
  static const int var128 = (int)umamd::tuning_env("dh_fwd128", 1);
  auto col_units = [&](int U) { return N * ((H + U - 1) / U) * (W / 16); };
  switch (C) {
    case 32:
      if (var == 1)
        hipLaunchKernelGGL((dhead_fwd_col_kernel<1, 4>), dim3(dh_grid((col_units(4) + 3) / 4)),
                           dim3(256), lds, st, a, col_units(4));
      else
        hipLaunchKernelGGL((dhead_fwd_dpp_kernel<1, 4>), dim3(dh_grid((col_units(4) + 3) / 4)),
                           dim3(256), lds, st, a, col_units(4));
      break;
    case 64:
      if (var == 1)
        hipLaunchKernelGGL((dhead_fwd_col_kernel<2, 2>), dim3(dh_grid((col_units(2) + 3) / 4)),
                           dim3(256), lds, st, a, col_units(2));
      else
        hipLaunchKernelGGL((dhead_fwd_dpp_kernel<2, 4>), dim3(dh_grid((col_units(4) + 3) / 4)),
                           dim3(256), lds, st, a, col_units(4));
      break;
    case 128:
      if (var128 == 1)
        hipLaunchKernelGGL((dhead_fwd_dpp_kernel<4, 2>), dim3(dh_grid((col_units(2) + 3) / 4)),
                           dim3(256), lds, st, a, col_units(2));
      else
        hipLaunchKernelGGL((dhead_fwd_kernel<4, 4, 1>), dim3(dh_grid(nstrips)), dim3(256), lds, st,
                           a, (int)nstrips);
      break;
    default:
      hipLaunchKernelGGL((dhead_fwd_kernel<8, 4, 1>), dim3(dh_grid(nstrips)), dim3(256), lds, st, a,
                         (int)nstrips);
      break;
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_disp_head_dgrad(int N, int H, int W, int C, const void* dl, int ldl, const void* wT,
                       void* dx, int ldx, int accumulate, hipStream_t st) {
  UM_CHECK_ARG(um_disp_head_ok(N, H, W, C, ldx), "um_disp_head_dgrad: shape N=%d H=%d W=%d C=%d ldx=%d",
               N, H, W, C, ldx);
  UM_CHECK_ARG(dl && wT && dx && ldl % 8 == 0 && dh_al(dl, 16) && dh_al(wT, 16) && dh_al(dx, 8),
               "um_disp_head_dgrad: pointers / ldl");
  DHDgrad a{(const bf16_t*)dl, (const bf16_t*)wT, (bf16_t*)dx, N, H, W, C, ldl, ldx, accumulate};
  const long nstrips = (long)N * H * W / 16;
  const size_t lds = (size_t)3 * C * 32 * sizeof(bf16_t);
#define UM_DHD(NB_, U_)                                                                        \
  hipLaunchKernelGGL((dhead_dgrad_kernel<NB_, U_>), dim3(dh_grid((nstrips + 4 * U_ - 1) / (4 * U_))), \
                     dim3(256), lds, st, a, (int)nstrips)
#define UM_DHC(NB_, U_, S_)                                                                     \
  {                                                                                             \
    const int units = N * ((H + U_ - 1) / U_) * (W / 16);                                       \
    hipLaunchKernelGGL((dhead_dgrad_col_kernel<NB_, U_, S_>), dim3(dh_grid((units + 3) / 4)),    \
                       dim3(256), lds, st, a, units);                                           \
  }
  // measured: LDS-staged 16-byte rows (STG) 36.8 -> 23.6 us (C = 32, U = 8) and
  // 21.2 -> 12.1 us (C = 64, U = 4) over 8-byte stores; dh_dgrad = 0: unstaged
  static const int var = (int)umamd::tuning_env("dh_dgrad", 1);
  switch (C) {
    case 32:
      if (var == 0) UM_DHC(2, 8, false) else UM_DHC(2, 8, true)
      break;
    case 64:
      if (var == 0) UM_DHC(4, 8, false) else UM_DHC(4, 4, true)
      break;
    case 128: UM_DHD(8, 1); break;
    default: UM_DHD(16, 1); break;
  }
#undef UM_DHD
#undef UM_DHC
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
