// Tap-major implicit-GEMM convolution on MFMA (gfx950), forward and
// stride-1 data gradient.
//
//   forward : Y[m=(n,p,q)][k] = sum_{r,s,c} X[n, p*st-pad+r, q*st-pad+s, c] * Wf[k][r][s][c]
//   dgrad   : DX[m=(n,i,j)][c] = sum_{r',s',k} DY[n, i-p'+r', j-p'+s', k] * WT[c][R-1-r'][R-1-s'][k]
//             (p' = R-1-pad: the transposed conv is a forward conv over DY
//             with flipped taps; reflect padding adds the fold sources of
//             the border pixels, see gather())
//
// Reduction order: taps (r, s) outer, channels inner in BK-wide chunks, so a
// k-step is one tap and one channel chunk and the gather needs no division:
// the source pixel of a GEMM row moves by (r, s) and the channel by c0.
// Reference ops: every nn.Conv2d of model/layers/{encoder,decoder,attention}.py
// and its input gradient.
//
// Block: 256 threads = 4 waves, BM x BN output tile, each wave a
// (BM/WM) x (BN/WN) grid of 16x16 MFMA tiles.  A (pixels x BK) and B
// (channels x BK) are register-staged into a double-buffered LDS image (one
// barrier per k-step, next step's global loads in flight during the MFMAs).
// bf16 images use 16-byte-chunk XOR swizzles that make every 16x16x32
// fragment read (ds_read_b128) bank-conflict free (checked exhaustively
// against the gfx950 lane groups).  Blocks are remapped so each XCD walks a
// contiguous run of tiles (neighbouring pixel tiles share halo rows in L2).
//
// Split-K (small-M layers: deep encoder stages have 128-4096 pixels): the
// k-steps are split over blockIdx.z, partial tiles go to an f32 workspace
// [split][M][NC] and splitk_epilogue_kernel sums them and applies the
// epilogue (bias, BN partial statistics, residual, sigmoid-scale).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "igemm.h"
#include "halo_conv.h"
#include "stream1x1.h"

namespace {

using umamd::IgArgs;

// BN partial-statistics row block (um_conv_stats_parts): a.stats_rows, 128 or
// 64 (the 64x64-tile plans); BM is a multiple of it.

// ------------------------------------------------------------ LDS images --
template <typename T, int BK> struct Img;
template <> struct Img<bf16_t, 32> {  // 64-B rows; chunk ^ {0,3,2,1}[(row>>2)&3]
  static constexpr int ROW = 32;
  __device__ static int off(int row, int c8) {
    return row * 32 + ((c8 ^ ((4 - ((row >> 2) & 3)) & 3)) << 3);
  }
};
template <> struct Img<bf16_t, 64> {  // 128-B rows; chunk ^ (row & 7)
  static constexpr int ROW = 64;
  __device__ static int off(int row, int c8) { return row * 64 + ((c8 ^ (row & 7)) << 3); }
};
template <> struct Img<float, 32> {  // 144-B rows (padded)
  static constexpr int ROW = 36;
  __device__ static int off(int row, int c8) { return row * 36 + c8 * 8; }
};

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { bf16x8_t v; };
template <> struct Frag<float> { float v[8]; };

__device__ __forceinline__ void lds_frag(const bf16_t* p, Frag<bf16_t>& f) {
  f.v = *reinterpret_cast<const bf16x8_t*>(p);
}
__device__ __forceinline__ void lds_frag(const float* p, Frag<float>& f) {
  const float4 x = *reinterpret_cast<const float4*>(p);
  const float4 y = *reinterpret_cast<const float4*>(p + 4);
  f.v[0] = x.x; f.v[1] = x.y; f.v[2] = x.z; f.v[3] = x.w;
  f.v[4] = y.x; f.v[5] = y.y; f.v[6] = y.z; f.v[7] = y.w;
}
__device__ __forceinline__ void mfma(f32x4_t& acc, const Frag<bf16_t>& x, const Frag<bf16_t>& y) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.v, y.v, acc, 0, 0, 0);
}
// f32: 8 x 16x16x4 with lane group g, element e -> k = 8g + e on both operands
__device__ __forceinline__ void mfma(f32x4_t& acc, const Frag<float>& x, const Frag<float>& y) {
#pragma unroll
  for (int e = 0; e < 8; ++e)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.v[e], y.v[e], acc, 0, 0, 0);
}

__device__ __forceinline__ void add8(const bf16_t* p, float* v) {
  float t[8];
  load8(p, t);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] += t[i];
}
__device__ __forceinline__ void add8(const float* p, float* v) {
  float t[8];
  load8(p, t);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] += t[i];
}
__device__ __forceinline__ void to_raw(const float* v, Raw8<bf16_t>& r) {
  r.v.x = pack_bf16x2(v[0], v[1]);
  r.v.y = pack_bf16x2(v[2], v[3]);
  r.v.z = pack_bf16x2(v[4], v[5]);
  r.v.w = pack_bf16x2(v[6], v[7]);
}
__device__ __forceinline__ void to_raw(const float* v, Raw8<float>& r) {
  r.a = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                   __float_as_uint(v[3]));
  r.b = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                   __float_as_uint(v[7]));
}

// one A row (GEMM row = output pixel) as seen by the gather
struct ARow {
  long base;   // element offset of the image (n) in the source
  int y0, x0;  // source coords of tap (0,0)
  bool ok;
};

// MODE: 0 plain rows, 1 parity class rows (stride-2 data gradient), 2 the
// border list of the reflect fold (IgArgs::border)
template <int MODE>
__device__ __forceinline__ ARow decode_row(const IgArgs& a, int m) {
  constexpr bool CLS = MODE == 1;
  ARow w;
  w.ok = m < a.M;
  const int mm = w.ok ? m : 0;
  if constexpr (MODE == 2) {
    int n, y, x;
    border_pixel(a, mm, n, y, x);
    w.base = (long)n * a.ah * a.aw * a.lda;
    w.y0 = y - a.pad;
    w.x0 = x - a.pad;
    return w;
  }
  const int hw = a.oh * a.ow;
  const int n = mm / hw;
  const int rem = mm - n * hw;
  const int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
  w.base = (long)n * a.ah * a.aw * a.lda;
  w.y0 = oy * a.stride - a.pad;
  w.x0 = ox * a.stride - (CLS ? a.padx : a.pad);
  return w;
}

// element offset of output row m (class mode: the row (n, i', j') of parity
// class (ay, ax) is output pixel (n, 2i'+ay, 2j'+ax) of the full image)
template <int MODE>
__device__ __forceinline__ long out_row(const IgArgs& a, int m) {
  constexpr bool CLS = MODE == 1;
  if constexpr (MODE == 2) {
    int n, y, x;
    border_pixel(a, m, n, y, x);
    return (((long)n * a.oh + y) * a.ow + x) * a.ld_out;
  }
  if (!CLS) return (long)m * a.ld_out;
  const int hw = a.oh * a.ow;
  const int n = m / hw, rem = m - n * hw;
  const int i = rem / a.ow, j = rem - (rem / a.ow) * a.ow;
  return (((long)n * a.outH + 2 * i + a.ay) * a.outW + 2 * j + a.ax) * a.ld_out;
}

template <int MODE, typename T>
__device__ __forceinline__ void gather(const IgArgs& a, const T* __restrict__ src, const ARow& w,
                                       int r, int s, int c, Raw8<T>& out) {
  constexpr bool CLS = MODE == 1, BRD = MODE == 2;
  raw_zero(out);
  if (!w.ok || c >= a.ach) return;
  int yy = CLS ? w.y0 - r : w.y0 + r, xx = CLS ? w.x0 - s : w.x0 + s;
  if (a.pmode == umamd::IG_PAD_REFLECT) {
    yy = reflect_idx(yy, a.ah);
    xx = reflect_idx(xx, a.aw);
    raw_load8(src + w.base + ((long)yy * a.aw + xx) * a.lda + c, out);
    return;
  }
  const bool iny = yy >= 0 && yy < a.ah, inx = xx >= 0 && xx < a.aw;
  if (a.pmode == umamd::IG_PAD_ZERO) {
    if (iny && inx) raw_load8(src + w.base + ((long)yy * a.aw + xx) * a.lda + c, out);
    return;
  }
  // IG_FOLD (reflect-padded transpose).  The forward read X[refl(o + r - pad)],
  // so output pixel i also receives from o = -i - p' + r' (1 <= i <= pad) and
  // o = 2(H-1) - i - p' + r' (H-1-pad <= i <= H-2); here a.pad = p'.
  const int oy = w.y0 + a.pad, ox = w.x0 + a.pad;
  const int H = a.oh, W = a.ow, fp = a.fold_pad;
  const bool lo_y = oy >= 1 && oy <= fp, hi_y = oy >= H - 1 - fp && oy <= H - 2;
  const bool lo_x = ox >= 1 && ox <= fp, hi_x = ox >= W - 1 - fp && ox <= W - 2;
  if (!(lo_y || hi_y || lo_x || hi_x)) {
    if (iny && inx && !BRD) raw_load8(src + w.base + ((long)yy * a.aw + xx) * a.lda + c, out);
    return;
  }
  int ys[3], xs[3], ny = 0, nx = 0;
  if (iny) ys[ny++] = yy;
  if (lo_y) { const int t = -oy - a.pad + r; if (t >= 0 && t < a.ah) ys[ny++] = t; }
  if (hi_y) { const int t = 2 * (H - 1) - oy - a.pad + r; if (t >= 0 && t < a.ah) ys[ny++] = t; }
  if (inx) xs[nx++] = xx;
  if (lo_x) { const int t = -ox - a.pad + s; if (t >= 0 && t < a.aw) xs[nx++] = t; }
  if (hi_x) { const int t = 2 * (W - 1) - ox - a.pad + s; if (t >= 0 && t < a.aw) xs[nx++] = t; }
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // border-list mode: the plain (zero-pad) source was summed by the same-size
  // data gradient already
  const bool skip0 = BRD && iny && inx;
  for (int u = 0; u < ny; ++u)
    for (int q = 0; q < nx; ++q)
      if (!(skip0 && u == 0 && q == 0))
        add8(src + w.base + ((long)ys[u] * a.aw + xs[q]) * a.lda + c, v);
  to_raw(v, out);
}

// Epilogue shared by the register-staged and the LDS-DMA main loops: split-K
// partial tile, or bias / residual / sigmoid-scale / stores and the BN
// partial statistics (sStat: WM x BN x 2 floats of LDS).
// sOut (optional, BM x BN elements of T in LDS): outputs of type T are
// staged there and leave as 16-byte rows (8 channels per lane) instead of
// the MFMA layout's 2-byte column scatter -- the 1x1 convs and data
// gradients are store-bound (dx at full resolution is 2/3 of their bytes).
template <typename T, int BM, int BN, int WM, int WN, bool SPLIT, int MODE>
__device__ __forceinline__ void igemm_epilogue(const IgArgs& a, float* __restrict__ ws,
                                               f32x4_t (&acc)[BM / WM / 16][BN / WN / 16],
                                               int bm, int bn, float* sStatp, T* sOut) {
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  auto sStat = reinterpret_cast<float(*)[BN][2]>(sStatp);
  const int col_l = lane & 15;
  const int row_g = (lane >> 4) * 4;
  if (SPLIT) {
    float* o = ws + (long)blockIdx.z * a.M * a.NC;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = bn + wn * (BN / WN) + j * 16 + col_l;
      if (n >= a.NC) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = bm + wm * (BM / WM) + i * 16 + row_g + q;
          if (m < a.M) o[(long)m * a.NC + n] = acc[i][j][q];
        }
    }
    return;
  }
  const bool stageable = sOut != nullptr && !a.out_f32 && a.NC % 8 == 0 &&
                         a.ld_out % 8 == 0;
  // accumulate + statistics slots (the decoder skip conv's feature-map half
  // onto up2(z)): the statistics of the SUM are taken in the 16-byte row
  // store (WN == 1: one wave per row of sStat) instead of a 2-byte
  // read-modify-write per element in the MFMA layout
  constexpr bool kRows = WN == 1 && 256 % (BN / 8) == 0;  // a thread keeps one column group
  const bool stat_rows = kRows && stageable && a.accumulate && a.epilogue == UM_EPI_STATS &&
                         a.stat_slots;
  const bool staged = stageable && (!(a.accumulate && a.epilogue == UM_EPI_STATS) || stat_rows);
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = bn + wn * (BN / WN) + j * 16 + col_l;
    const bool nok = n < a.NC;
    const float bv = (a.bias != nullptr && nok) ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = bm + wm * (BM / WM) + i * 16 + row_g + q;
        if (!nok || m >= a.M) continue;
        float v = acc[i][j][q] + bv;
        const long off = out_row<MODE>(a, m) + n;
        if (a.epilogue == UM_EPI_RESIDUAL)
          v += to_f32(reinterpret_cast<const T*>(a.residual)[(long)m * a.ldr + n]);
        if (a.epilogue == UM_EPI_SIGMOID_SCALE) v = a.epi_scale * sigmoidf_(v);
        if (a.out_f32) {
          float* o = reinterpret_cast<float*>(a.out) + off;
          if (a.accumulate) v += *o;
          *o = v;
        } else if (staged) {  // accumulate (if any) happens at the row store
          sOut[(m - bm) * BN + (n - bn)] = from_f32<T>(v);
        } else {
          T* o = reinterpret_cast<T*>(a.out) + off;
          if (a.accumulate) v += to_f32(*o);
          *o = from_f32<T>(v);
        }
        csum[j] += v;
        csq[j] += v * v;
      }
  }
  if (a.epilogue == UM_EPI_STATS && !stat_rows) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float sm = csum[j], sq = csq[j];
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      sq += __shfl_xor(sq, 16, 64);
      sq += __shfl_xor(sq, 32, 64);
      if (lane < 16) {
        sStat[wm][wn * (BN / WN) + j * 16 + lane][0] = sm;
        sStat[wm][wn * (BN / WN) + j * 16 + lane][1] = sq;
      }
    }
    __syncthreads();
    // stats row blocks of SR rows (BM % SR == 0): waves of rows [w*BM/WM, (w+1)*BM/WM)
    constexpr int WROWS = BM / WM;
    if (a.stat_slots) {  // the whole tile's sums: one f64 atomic per (column, value)
      stat_slots_count(reinterpret_cast<double*>(a.stats), a.NC, a.M);
      stat_slots_add_row(reinterpret_cast<double*>(a.stats), bm / BM, a.NC, bn,
                         min(BN, a.NC - bn), [&](int i) {
                           float v = 0.f;
#pragma unroll
                           for (int w = 0; w < WM; ++w) v += sStat[w][i >> 1][i & 1];
                           return v;
                         });
    } else {
      const int SR = a.stats_rows;
      const int NSB = BM / SR;
      for (int c = tid; c < BN * NSB; c += (int)blockDim.x) {
        const int col = c % BN, sb = c / BN;
        const int n = bn + col;
        if (n >= a.NC || bm + sb * SR >= a.M) continue;
        float sm = 0.f, sq = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w)
          if ((w * WROWS) / SR == sb) { sm += sStat[w][col][0]; sq += sStat[w][col][1]; }
        float* o = a.stats + ((long)(bm / SR + sb) * a.NC + n) * 2;
        o[0] = sm;
        o[1] = sq;
      }
    }
  }
  if (staged) {
    __syncthreads();
    constexpr int CPR = BN / 8;
    float ps[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = tid; c < BM * CPR; c += (int)blockDim.x) {
      const int r = c / CPR, c8 = (c - r * CPR) * 8;
      const int m = bm + r, n = bn + c8;
      if (m >= a.M || n >= a.NC) continue;
      T* o = reinterpret_cast<T*>(a.out) + out_row<MODE>(a, m) + n;
      if (a.accumulate) {
        float x[8], y[8];
        load8(&sOut[r * BN + c8], x);
        load8(o, y);
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] += y[e];
        store8(o, x);
        if (stat_rows)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            ps[e] += x[e];
            pq[e] += x[e] * x[e];
          }
      } else {
        Raw8<T> v;
        raw_load8(&sOut[r * BN + c8], v);
        raw_store8(o, v);
      }
    }
    if constexpr (kRows) if (stat_rows) {
      // lanes of one wave with the same column group: lane % CPR
#pragma unroll
      for (int sh = CPR; sh < 64; sh <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ps[e] += __shfl_xor(ps[e], sh, 64);
          pq[e] += __shfl_xor(pq[e], sh, 64);
        }
      if (lane < CPR)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sStat[wave][lane * 8 + e][0] = ps[e];
          sStat[wave][lane * 8 + e][1] = pq[e];
        }
      __syncthreads();
      stat_slots_count(reinterpret_cast<double*>(a.stats), a.NC, a.M);
      stat_slots_add_row(reinterpret_cast<double*>(a.stats), bm / BM, a.NC, bn,
                         min(BN, a.NC - bn), [&](int i) {
                           float v = 0.f;
#pragma unroll
                           for (int w = 0; w < WM; ++w) v += sStat[w][i >> 1][i & 1];
                           return v;
                         });
    }
  }
}

// the XCD-aware tile order: blocks b, b+8, b+16... (one XCD) take
// consecutive tiles
__device__ __forceinline__ int xcd_tile(int t, int nb) {
  if (nb >= 16) {
    const int xcd = t & 7, q = nb >> 3, rr = nb & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  return t;
}

template <typename T, int BK, int BM, int BN, int WM, int WN, bool SPLIT, int MODE>
__device__ __forceinline__ void igemm_tile(const IgArgs& a, float* __restrict__ ws, int steps,
                                           int steps_per_split, int ntn, int t, int ntiles);

template <typename T, int BK, int BM, int BN, int WM, int WN, bool SPLIT, int MODE>
__global__ void __launch_bounds__(256) igemm_kernel(IgArgs a, float* __restrict__ ws,
                                                     int steps, int steps_per_split, int ntn) {
  igemm_tile<T, BK, BM, BN, WM, WN, SPLIT, MODE>(a, ws, steps, steps_per_split, ntn,
                                                 xcd_tile(blockIdx.x, gridDim.x), gridDim.x);
}

// The four parity classes of a stride-2 data gradient in ONE launch: class c
// owns tiles [start[c], start[c+1]) of the grid (same column tiling, its own
// rows, taps and output parity), so the four short-K GEMMs fill the chip
// together instead of four launches of one tile per CU each (+ their split-K
// epilogues).
template <typename T, int BK, int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256) igemm_cls4_kernel(IgArgs a0, IgArgs a1, IgArgs a2, IgArgs a3,
                                                          int4 start, int4 steps, int ntn) {
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  const int c = t < start.y ? 0 : (t < start.z ? 1 : (t < start.w ? 2 : 3));
  const IgArgs* ap = c == 0 ? &a0 : (c == 1 ? &a1 : (c == 2 ? &a2 : &a3));
  const int s0 = c == 0 ? start.x : (c == 1 ? start.y : (c == 2 ? start.z : start.w));
  const int s1 = c == 0 ? start.y : (c == 1 ? start.z : (c == 2 ? start.w : (int)gridDim.x));
  const int st = c == 0 ? steps.x : (c == 1 ? steps.y : (c == 2 ? steps.z : steps.w));
  igemm_tile<T, BK, BM, BN, WM, WN, false, 1>(*ap, nullptr, st, st, ntn, t - s0, s1 - s0);
}

template <typename T, int BK, int BM, int BN, int WM, int WN, bool SPLIT, int MODE>
__device__ __forceinline__ void igemm_tile(const IgArgs& a, float* __restrict__ ws, int steps,
                                           int steps_per_split, int ntn, int t, int ntiles) {
  constexpr bool CLS = MODE == 1;
  using I = Img<T, BK>;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int CPR = BK / 8;  // 8-element chunks per LDS row
  constexpr int A_CH = BM * CPR, B_CH = BN * CPR;
  static_assert(A_CH % 256 == 0, "A chunks per thread");
  constexpr int A_PER = A_CH / 256;
  constexpr int B_PER = (B_CH + 255) / 256;
  static_assert(WM * WN == 4, "4 waves");

  // one LDS array: the two A and B stages, reused by the staged epilogue
  constexpr int SMEM = 2 * (BM + BN) * I::ROW;
  __shared__ __attribute__((aligned(16))) T smem[SMEM];
  T(*sA)[BM * I::ROW] = reinterpret_cast<T(*)[BM * I::ROW]>(smem);
  T(*sB)[BN * I::ROW] = reinterpret_cast<T(*)[BN * I::ROW]>(smem + 2 * BM * I::ROW);
  __shared__ float sStat[WM][BN][2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // row-major tile order (an XCD's contiguous t range shares row tiles, so
  // reads a slice of A and all of B) unless the weights outweigh the
  // gathered image (deep layers): then column-major, each XCD's L2 holds a
  // slice of B and the whole (small) A
  int bm, bn;
  if (a.colmajor) {
    const int ntm = ntiles / ntn;
    bn = (t / ntm) * BN;
    bm = (t - (t / ntm) * ntm) * BM;
  } else {
    bm = (t / ntn) * BM;
    bn = (t - (t / ntn) * ntn) * BN;
  }

  const T* __restrict__ asrc = reinterpret_cast<const T*>(a.a);
  const T* __restrict__ bsrc = reinterpret_cast<const T*>(a.b);

  ARow arow[A_PER];
  int akc[A_PER], arow_i[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int c = tid + i * 256;
    arow_i[i] = c / CPR;
    akc[i] = c % CPR;
    arow[i] = decode_row<MODE>(a, bm + arow_i[i]);
  }
  int brow_i[B_PER], bkc[B_PER];
  bool bok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int c = tid + i * 256;
    brow_i[i] = c / CPR;
    bkc[i] = c % CPR;
    bok[i] = c < B_CH && bn + brow_i[i] < a.NC;
  }

  const int s_begin = SPLIT ? blockIdx.z * steps_per_split : 0;
  const int s_end = SPLIT ? min(steps, s_begin + steps_per_split) : steps;
  const int nchunk = (a.ach + BK - 1) / BK;
  int tap = s_begin / nchunk;
  int c0 = (s_begin - tap * nchunk) * BK;
  const int RX = CLS ? a.Rx : a.R;
  int r = tap / RX, s = tap - (tap / RX) * RX;

  // tap packing (a.tappack: 8-channel operands, BK = 32): a k-step holds 4
  // taps x 8 channels instead of one tap's 8 channels + 24 zero columns, so
  // the 7x7 first conv and the 8-channel heads' data gradients take 1/4 of
  // the k-steps.  Chunk q of step st is tap 4*st + q, channels 0..7.
  const int taps = a.R * RX;
  int tb = s_begin * CPR;
  auto tap_b = [&](int r_, int s_) {
    return CLS ? (a.r0y + 2 * r_) * a.wR + (a.r0x + 2 * s_)
               : (a.flip ? (a.R - 1 - r_) * a.R + (a.R - 1 - s_) : r_ * a.R + s_);
  };

  Raw8<T> ra[A_PER], rb[B_PER];
  auto load = [&]() {
    if (a.tappack) {
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const int tp = tb + akc[i];
        const int r_ = tp / RX, s_ = tp - (tp / RX) * RX;
        if (tp < taps) gather<MODE>(a, asrc, arow[i], r_, s_, 0, ra[i]);
        else raw_zero(ra[i]);
      }
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        raw_zero(rb[i]);
        const int tp = tb + bkc[i];
        const int r_ = tp / RX, s_ = tp - (tp / RX) * RX;
        if (bok[i] && tp < taps)
          raw_load8(bsrc + (long)(bn + brow_i[i]) * a.ldb + (long)tap_b(r_, s_) * 8, rb[i]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) gather<MODE>(a, asrc, arow[i], r, s, c0 + akc[i] * 8, ra[i]);
    const int btap = CLS ? (a.r0y + 2 * r) * a.wR + (a.r0x + 2 * s)
                         : (a.flip ? (a.R - 1 - r) * a.R + (a.R - 1 - s) : r * a.R + s);
    const long boff = (long)btap * a.ach;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      raw_zero(rb[i]);
      const int c = c0 + bkc[i] * 8;
      if (bok[i] && c < a.ach) raw_load8(bsrc + (long)(bn + brow_i[i]) * a.ldb + boff + c, rb[i]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) raw_store8(&sA[buf][I::off(arow_i[i], akc[i])], ra[i]);
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      if (tid + i * 256 < B_CH) raw_store8(&sB[buf][I::off(brow_i[i], bkc[i])], rb[i]);
  };
  auto advance = [&]() {
    tb += CPR;
    c0 += BK;
    if (c0 >= a.ach) {
      c0 = 0;
      if (++s == RX) { s = 0; ++r; }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fg = lane >> 4;
  if (s_begin < s_end) {
    load();
    store(0);
    advance();
  }
  __syncthreads();
  for (int st = s_begin; st < s_end; ++st) {
    const int cur = (st - s_begin) & 1;
    const bool more = st + 1 < s_end;
    if (more) load();
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      Frag<T> fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        lds_frag(&sA[cur][I::off(wm * (BM / WM) + i * 16 + frow, kk * 4 + fg)], fa[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        lds_frag(&sB[cur][I::off(wn * (BN / WN) + j * 16 + frow, kk * 4 + fg)], fb[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma(acc[i][j], fa[i], fb[j]);
    }
    if (more) {
      store(cur ^ 1);
      advance();
    }
    __syncthreads();
  }

  igemm_epilogue<T, BM, BN, WM, WN, SPLIT, MODE>(a, ws, acc, bm, bn, &sStat[0][0][0],
                                               BM * BN <= SMEM ? smem : nullptr);
}

// ---------------------------------------------------------------------------
// LDS-DMA main loop (bf16, BK = 64, no reflect fold): A and B tiles go
// global -> LDS with global_load_lds_dwordx4, NST stages deep, so a block
// keeps NST-1 k-steps of loads in flight instead of one register set.
// The LDS image is the register path's Img<bf16, 64> (chunk ^ (row & 7)): one
// wave instruction fills 8 rows x 128 B lane-linearly, so lane L loads the
// global chunk (L & 7) ^ (row & 7) of row L >> 3.  Out-of-range rows, padding
// taps and channel chunks past ach read a zero page.  All LDS is one
// __shared__ array, waits are counted (vmcnt never 0 inside the loop) and the
// barriers are raw s_barrier, so the DMA stays in flight across them.
__device__ __attribute__((aligned(16))) unsigned int g_zero_page[4];

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(later, N) k-steps of PER loads each are outstanding
template <int PER, int N>
__device__ __forceinline__ void wait_later(int later) {
  if constexpr (N == 0) {
    wait_vm<0>();
  } else {
    if (later >= N) wait_vm<N * PER>();
    else wait_later<PER, N - 1>(later);
  }
}

template <int MODE>
__device__ __forceinline__ const bf16_t* gather_ptr(const IgArgs& a, const bf16_t* src,
                                                     const ARow& w, int r, int s, int c) {
  constexpr bool CLS = MODE == 1;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_page);
  if (!w.ok || c >= a.ach) return zero;
  int yy = CLS ? w.y0 - r : w.y0 + r, xx = CLS ? w.x0 - s : w.x0 + s;
  if (a.pmode == umamd::IG_PAD_REFLECT) {
    yy = reflect_idx(yy, a.ah);
    xx = reflect_idx(xx, a.aw);
  } else if (yy < 0 || yy >= a.ah || xx < 0 || xx >= a.aw) {
    return zero;
  }
  return src + w.base + ((long)yy * a.aw + xx) * a.lda + c;
}

// NW = 4 or 8 waves; with 8, a 64x64 tile gives each wave a 16x32 sub-tile
// and every SIMD two waves of the block to overlap the per-step latencies.
// NST stages: 3 (48 KB for 64x64, several blocks per CU) or deeper for grids
// of at most ~1-2 blocks per CU, whose k-loop is pure load latency (knob
// glds_deep: 6 stages = 5 k-steps in flight, 96 KB).
// XCD-aware tile order: the dispatcher deals workgroups round-robin over the
// 8 XCDs, so give each XCD a contiguous range of tiles (shared rows in its L2)
__device__ __forceinline__ int glds_xcd_tile(int t, int nb) {
  if (nb < 16) return t;
  const int xcd = t & 7, q = nb >> 3, rr = nb & 7;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
}

// one 64-deep-k tile t of ntiles (the launch's own grid, or one parity class's
// share of a 4-class launch); split index blockIdx.z
template <int BM, int BN, int NW, bool SPLIT, int MODE, int NST>
__device__ __forceinline__ void glds_tile(const IgArgs& a, float* __restrict__ ws, int steps,
                                          int steps_per_split, int ntn, int t, int ntiles) {
  constexpr bool CLS = MODE == 1;
  static_assert(MODE != 2, "the reflect fold gathers through registers");
  constexpr int BK = 64, WM = NW == 8 ? 4 : 2, WN = 2;
  using I = Img<bf16_t, BK>;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int STAGE = (BM + BN) * BK;  // elements
  constexpr int A_INS = BM / 8 / NW, B_INS = BN / 8 / NW;  // 8-row glds per wave per k-step
  static_assert(A_INS >= 1 && B_INS >= 1, "rows per wave");
  constexpr int PER = A_INS + B_INS;
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile");
  static_assert(NST * STAGE * 2 >= WM * BN * 2 * 4, "stats scratch fits the staging LDS");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // row-major tile order (an XCD's contiguous t range shares row tiles, so
  // reads a slice of A and all of B) unless the weights outweigh the
  // gathered image (deep layers): then column-major, each XCD's L2 holds a
  // slice of B and the whole (small) A
  int bm, bn;
  if (a.colmajor) {
    const int ntm = ntiles / ntn;
    bn = (t / ntm) * BN;
    bm = (t - (t / ntm) * ntm) * BM;
  } else {
    bm = (t / ntn) * BM;
    bn = (t - (t / ntn) * ntn) * BN;
  }
  const bf16_t* __restrict__ asrc = reinterpret_cast<const bf16_t*>(a.a);
  const bf16_t* __restrict__ bsrc = reinterpret_cast<const bf16_t*>(a.b);
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_page);

  // this lane's rows: A rows wave*(BM/4) + 8i + (lane >> 3), B likewise
  const int lr = lane >> 3, lp = lane & 7;
  ARow arow[A_INS];
  int ac8[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int row = wave * (BM / NW) + i * 8 + lr;
    ac8[i] = lp ^ (row & 7);
    arow[i] = decode_row<MODE>(a, bm + row);
  }
  int bc8[B_INS];
  long boff_row[B_INS];
  bool bok[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int row = wave * (BN / NW) + i * 8 + lr;
    bc8[i] = lp ^ (row & 7);
    bok[i] = bn + row < a.NC;
    boff_row[i] = (long)(bn + row) * a.ldb;
  }

  const int s_begin = SPLIT ? blockIdx.z * steps_per_split : 0;
  const int s_end = SPLIT ? min(steps, s_begin + steps_per_split) : steps;
  const int nsteps = s_end - s_begin;
  const int nchunk = (a.ach + BK - 1) / BK;
  int tap = s_begin / nchunk;
  int c0 = (s_begin - tap * nchunk) * BK;
  const int RX = CLS ? a.Rx : a.R;
  int r = tap / RX, s = tap - (tap / RX) * RX;

  // issue the k-step at the cursor (r, s, c0) into stage `st`, then advance
  auto issue = [&](int st) {
    bf16_t* base = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const bf16_t* g = gather_ptr<MODE>(a, asrc, arow[i], r, s, c0 + ac8[i] * 8);
      __builtin_amdgcn_global_load_lds(
          g, (__attribute__((address_space(3))) void*)(base + (wave * (BM / NW) + i * 8) * BK), 16,
          0, 0);
    }
    const int btap = CLS ? (a.r0y + 2 * r) * a.wR + (a.r0x + 2 * s)
                         : (a.flip ? (a.R - 1 - r) * a.R + (a.R - 1 - s) : r * a.R + s);
    const long boff = (long)btap * a.ach;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int c = c0 + bc8[i] * 8;
      const bf16_t* g = (bok[i] && c < a.ach) ? bsrc + boff_row[i] + boff + c : zero;
      __builtin_amdgcn_global_load_lds(
          g,
          (__attribute__((address_space(3))) void*)(base + BM * BK +
                                                    (wave * (BN / NW) + i * 8) * BK),
          16, 0, 0);
    }
    c0 += BK;
    if (c0 >= a.ach) {
      c0 = 0;
      if (++s == RX) { s = 0; ++r; }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fg = lane >> 4;
  const int npro = nsteps < NST ? nsteps : NST;
  for (int p = 0; p < npro; ++p) issue(p);
  for (int k = 0; k < nsteps; ++k) {
    // this wave's loads of step k have landed when at most the later issued
    // steps' loads are outstanding
    wait_later<PER, NST - 1>(nsteps - 1 - k);
    __builtin_amdgcn_s_barrier();  // every wave's DMA for step k is in LDS
    const int cur = k % NST;
    const bf16_t* sA = smem + cur * STAGE;
    const bf16_t* sB = sA + BM * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      Frag<bf16_t> fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        lds_frag(&sA[I::off(wm * (BM / WM) + i * 16 + frow, kk * 4 + fg)], fa[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        lds_frag(&sB[I::off(wn * (BN / WN) + j * 16 + frow, kk * 4 + fg)], fb[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma(acc[i][j], fa[i], fb[j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage `cur` is free again
    if (k + NST < nsteps) issue(cur);
  }
  // all DMA retired (the last iteration waited vmcnt(0)); reuse LDS for stats
  __syncthreads();
  constexpr int STAT_ELEMS = (WM * BN * 2 * 4 + 15) / 16 * 8;  // bf16 elements, 16-B aligned
  static_assert(STAT_ELEMS + BM * BN <= NST * STAGE, "staged epilogue fits the staging LDS");
  igemm_epilogue<bf16_t, BM, BN, WM, WN, SPLIT, MODE>(a, ws, acc, bm, bn,
                                                     reinterpret_cast<float*>(smem),
                                                     smem + STAT_ELEMS);
  static_assert(WM * WN == NW, "waves");
}

template <int BM, int BN, int NW, bool SPLIT, int MODE, int NST>
__global__ void __launch_bounds__(NW * 64) igemm_glds_kernel(IgArgs a, float* __restrict__ ws,
                                                              int steps, int steps_per_split,
                                                              int ntn) {
  glds_tile<BM, BN, NW, SPLIT, MODE, NST>(a, ws, steps, steps_per_split, ntn,
                                          glds_xcd_tile(blockIdx.x, gridDim.x), gridDim.x);
}

// The four parity classes of a stride-2 data gradient as ONE launch of 64x64
// LDS-DMA tiles: class c owns tiles [start[c], start[c+1]) and splits
// [0, splits[c]) of the z range, with its own workspace slice.  The class is
// chosen by uniform branches on kernel arguments (indexing the four by-value
// IgArgs through a pointer spilled ~200 SGPRs in the register-path variant).
template <int BN, int NW, bool SPLIT, int NST>
__global__ void __launch_bounds__(NW * 64) igemm_glds_cls4_kernel(IgArgs a0, IgArgs a1, IgArgs a2,
                                                               IgArgs a3, int4 start, int4 steps,
                                                               int4 per, int4 splits, int4 ntiles,
                                                               int ntn, float* __restrict__ ws,
                                                               long4 wsoff) {
  const int t = glds_xcd_tile(blockIdx.x, gridDim.x);
  const int z = blockIdx.z;
  if (t < start.y) {
    if (z < splits.x)
      glds_tile<64, BN, NW, SPLIT, 1, NST>(a0, ws + wsoff.x, steps.x, per.x, ntn, t - start.x,
                                          ntiles.x);
  } else if (t < start.z) {
    if (z < splits.y)
      glds_tile<64, BN, NW, SPLIT, 1, NST>(a1, ws + wsoff.y, steps.y, per.y, ntn, t - start.y,
                                          ntiles.y);
  } else if (t < start.w) {
    if (z < splits.z)
      glds_tile<64, BN, NW, SPLIT, 1, NST>(a2, ws + wsoff.z, steps.z, per.z, ntn, t - start.z,
                                          ntiles.z);
  } else {
    if (z < splits.w)
      glds_tile<64, BN, NW, SPLIT, 1, NST>(a3, ws + wsoff.w, steps.w, per.w, ntn, t - start.w,
                                          ntiles.w);
  }
}

// sum the split-K partials and apply the epilogue.  Block = a.stats_rows rows x
// 64 columns: thread (g, lane) owns columns 4g..4g+3 and rows lane, lane+16, ...
constexpr int EPI_COLS = 64;
// rows: the block's row count -- a.stats_rows when the epilogue takes BN
// statistics (one partial row per statistics row block), else EPI_ROWS (more,
// smaller blocks: one row per thread, the partial loads of all rows in flight)
constexpr int EPI_ROWS = 16;
template <typename T, int MODE>
__device__ __forceinline__ void splitk_epi_rows(const IgArgs& a, const float* __restrict__ ws,
                                                int splits, int bx, int rows) {
  __shared__ float red[16][16][8];
  const int g = threadIdx.x & 15, lane = threadIdx.x >> 4;
  const int n = blockIdx.y * EPI_COLS + g * 4;  // NC % 4 == 0 (host-checked)
  const long m0 = (long)bx * rows;
  const long m1 = min((long)a.M, m0 + rows);
  const long zs = (long)a.M * a.NC;
  const bool act = n < a.NC;
  // 4 consecutive outputs as one 16-byte (f32) / 8-byte (bf16) access
  const bool vec4 = (a.ld_out & 3) == 0 &&
                    (reinterpret_cast<uintptr_t>(a.out) & (a.out_f32 || sizeof(T) == 4 ? 15 : 7)) == 0;
  float sm[4] = {0, 0, 0, 0}, sq[4] = {0, 0, 0, 0};
  if (act) {
    float bv[4] = {0, 0, 0, 0};
    if (a.bias)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = a.bias[n + e];
    for (long m = m0 + lane; m < m1; m += 16) {
      const float* p = ws + m * a.NC + n;
      float4 x = *reinterpret_cast<const float4*>(p);
      int z = 1;
      for (; z + 1 < splits; z += 2) {  // two partials in flight
        const float4 y0 = *reinterpret_cast<const float4*>(p + z * zs);
        const float4 y1 = *reinterpret_cast<const float4*>(p + (z + 1) * zs);
        x.x += y0.x + y1.x; x.y += y0.y + y1.y; x.z += y0.z + y1.z; x.w += y0.w + y1.w;
      }
      if (z < splits) {
        const float4 y0 = *reinterpret_cast<const float4*>(p + z * zs);
        x.x += y0.x; x.y += y0.y; x.z += y0.z; x.w += y0.w;
      }
      float v[4] = {x.x + bv[0], x.y + bv[1], x.z + bv[2], x.w + bv[3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.epilogue == UM_EPI_RESIDUAL)
          v[e] += to_f32(reinterpret_cast<const T*>(a.residual)[m * a.ldr + n + e]);
        if (a.epilogue == UM_EPI_SIGMOID_SCALE) v[e] = a.epi_scale * sigmoidf_(v[e]);
      }
      // the row's output offset once (the border mode maps it through the
      // reflect list), then the 4 columns as one vector access when aligned
      const long off = out_row<MODE>(a, (int)m) + n;
      if (vec4) {
        if (a.out_f32) {
          float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + off);
          if (a.accumulate) {
            const float4 p = *o;
            v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
          }
          *o = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (sizeof(T) == 2) {
          uint2* o = reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.out) + off);
          if (a.accumulate) {
            const uint2 p = *o;
            v[0] += __uint_as_float(p.x << 16);
            v[1] += __uint_as_float(p.x & 0xffff0000u);
            v[2] += __uint_as_float(p.y << 16);
            v[3] += __uint_as_float(p.y & 0xffff0000u);
          }
          *o = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        } else {
          float4* o = reinterpret_cast<float4*>(reinterpret_cast<T*>(a.out) + off);
          if (a.accumulate) {
            const float4 p = *o;
            v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
          }
          *o = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (a.out_f32) {
            float* o = reinterpret_cast<float*>(a.out) + off + e;
            if (a.accumulate) v[e] += *o;
            *o = v[e];
          } else {
            T* o = reinterpret_cast<T*>(a.out) + off + e;
            if (a.accumulate) v[e] += to_f32(*o);
            *o = from_f32<T>(v[e]);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sm[e] += v[e];
        sq[e] += v[e] * v[e];
      }
    }
  }
  if (a.epilogue != UM_EPI_STATS) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) { red[lane][g][e] = sm[e]; red[lane][g][4 + e] = sq[e]; }
  __syncthreads();
  if (lane == 0 && act) {
    for (int l = 1; l < 16; ++l)
#pragma unroll
      for (int e = 0; e < 4; ++e) { sm[e] += red[l][g][e]; sq[e] += red[l][g][4 + e]; }
    if (!a.stat_slots) {
      float* o = a.stats + ((long)bx * a.NC + n) * 2;
#pragma unroll
      for (int e = 0; e < 4; ++e) { o[2 * e] = sm[e]; o[2 * e + 1] = sq[e]; }
    }
  }
  if (a.stat_slots) {  // stage the 64 column pairs, then contiguous f64 atomics
    __shared__ float tot[EPI_COLS * 2];
    if (lane == 0)
#pragma unroll
      for (int e = 0; e < 4; ++e) { tot[(g * 4 + e) * 2] = sm[e]; tot[(g * 4 + e) * 2 + 1] = sq[e]; }
    __syncthreads();
    const int c0 = blockIdx.y * EPI_COLS;
    stat_slots_count(reinterpret_cast<double*>(a.stats), a.NC, a.M);
    stat_slots_add_row(reinterpret_cast<double*>(a.stats), bx, a.NC, c0,
                       min(EPI_COLS, a.NC - c0), [&](int i) { return tot[i]; });
  }
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(IgArgs a, const float* __restrict__ ws,
                                                               int splits, int rows) {
  splitk_epi_rows<T, MODE>(a, ws, splits, blockIdx.x, rows);
}

// the split-K sums of igemm_glds_cls4_kernel: class c owns row blocks
// [rstart[c], rstart[c+1])
template <typename T>
__global__ void __launch_bounds__(256) splitk_epilogue_cls4_kernel(IgArgs a0, IgArgs a1, IgArgs a2,
                                                                    IgArgs a3, int4 rstart,
                                                                    int4 splits,
                                                                    const float* __restrict__ ws,
                                                                    long4 wsoff) {
  const int b = blockIdx.x;
  if (b < rstart.y) splitk_epi_rows<T, 1>(a0, ws + wsoff.x, splits.x, b - rstart.x, a0.stats_rows);
  else if (b < rstart.z) splitk_epi_rows<T, 1>(a1, ws + wsoff.y, splits.y, b - rstart.y, a1.stats_rows);
  else if (b < rstart.w) splitk_epi_rows<T, 1>(a2, ws + wsoff.z, splits.z, b - rstart.z, a2.stats_rows);
  else splitk_epi_rows<T, 1>(a3, ws + wsoff.w, splits.w, b - rstart.w, a3.stats_rows);
}

struct Plan {
  int bk, bm, bn, wm, wn, splits, steps, per;
};

// tuning knobs (read once; defaults below, UMAMD_TUNING="key=value,..." for
// sweeps, um_set_tuning at run time for tests)
struct Knobs {
  int small, small_tiles, split_below, split_target, split_minsteps, halo, halo_min_tiles, odd_bn, bk64;
  int glds_split_below, glds_split_target;
  int glds;
  int glds_deep, glds_deep_blocks;
  int xcd_col;
  int tappack;
  int cls4;
  int cls_glds;
  int pad_dgrad;
  int fold_split_nc;
  int halo_max_nc;
  int halo_pf2;
  int halo_persist, halo_grid, halo_res_kb;
  int halo_staged;
  int border_valu;
  int s1x1, s1x1_small;
  Knobs() {
    auto env = [](const char* n, int d) { return (int)umamd::tuning_env(n, d); };
    small = env("small", 1);
    // measured on MI355X (bench step, tools/sweep.sh): the deep layers' main
    // loops are load-latency bound (one double-buffered stage in flight per
    // block, ~1 us per k-step at 1 block per CU), so more, smaller and split
    // tiles help: 160/320/8/256 -> 600/1024/4/1024 took 578 -> 599 pairs/s
    small_tiles = env("small_tiles", 1024);
    split_below = env("split_below", 600);
    split_target = env("split_target", 1024);
    // the 8-wave LDS-DMA loop (glds bit 2) hides more of a 64x64-tile
    // block's own latency: measured per conv (tools/ig_micro.sh), split only
    // below 256 tiles and to ~512 blocks -- 16x32x256->256 27 -> 24 us,
    // 32x64x128->128 27 -> 19 us, 8x16x512->512 28 -> 25 us.  The register
    // path (reflect-fold data gradients, f32) keeps the thresholds above.
    glds_split_below = env("glds_split_below", 256);
    glds_split_target = env("glds_split_target", 512);
    split_minsteps = env("split_minsteps", 4);
    halo = env("halo", 1);
    halo_min_tiles = env("halo_min_tiles", 256);
    // widest output (columns) the halo kernel takes: 64 = one column block
    // (round 2); up to 192 adds 96/128-wide 3x3 blocks and column grids
    halo_max_nc = env("halo_max_nc", 192);
    odd_bn = env("odd_bn", 1);
    // bit 0: 64-deep k-steps for the 64x64 tiles, bit 1: for the 128-row tiles
    bk64 = env("bk64", 3);
    // bit 0: LDS-DMA main loop for the 64x64 tiles, bit 1: for the 128-row
    // tiles, bit 2: 8 waves per 64x64 tile.  Step sweep (tools/sweep.sh):
    // 0 -> 653.6, 7 -> 654.8, 5 -> 661.3 pairs/s (the 128-row tiles keep the
    // register path: 3 LDS stages of 128-row tiles leave 1 block per CU)
    glds = env("glds", 5);
    // 6-stage LDS-DMA loop for 8-wave 64x64 grids of at most this many
    // blocks (one 96 KB block per CU); 3 = off.  Step sweep: 3 -> 721,
    // 6 -> 715 pairs/s (unsplit deep grids 713-717): five k-steps in flight
    // do not shorten the deep layers' k-loop, so latency is not its limit
    glds_deep = env("glds_deep", 3);
    glds_deep_blocks = env("glds_deep_blocks", 256);
    // column-major tile order for weight-heavy GEMMs (0 off, 1 auto, 2 on):
    // per conv and per step within noise (714 vs 713 pairs/s), off
    xcd_col = env("xcd_col", 0);
    // 8-channel operands: bit 0 packs 4 taps per 32-deep k-step, bit 1 also
    // routes them past the halo kernel.  First conv (7x7 s2, C8) 93 -> 51 us;
    // step 711 -> 715-716 pairs/s with 1 or 3 (the heads' halo path is as fast)
    tappack = env("tappack", 1);
    // the four parity classes of a stride-2 data gradient as one launch
    cls4 = env("cls4", 1);
    // the four parity classes of a stride-2 data gradient as one launch of
    // LDS-DMA tiles instead of 256-row register tiles (bit 0: NC a multiple
    // of 64 on 64x64 tiles: 64x128 C64 K128 59 -> 28 us, 32x64 C128 K256
    // 50 -> 24, 16x32 C256 K512 57 -> 28; bit 1: NC = 32 on 64x32 tiles with
    // 4 waves: 128x256 C32 K64 5x5 79 -> 63 us; MI355X, tools/gpu_s2_micro.sh)
    cls_glds = env("cls_glds", 3);
    // reflect data gradient as a zero-pad transposed conv onto the padded
    // input + a fold pass (0 off, 1 the wide layers, 2 all)
    pad_dgrad = env("pad_dgrad", 1);
    // per conv (tools/conv_table.py): split form 256x512 C48 171 -> 117 us,
    // C32 K8 125 -> 85; one pass stays ahead from C = 128 up (16x32 C640:
    // 106 vs 140, 8x16 C512: 53 vs 79)
    fold_split_nc = env("fold_split_nc", 64);
    // halo conv: weight tap rows loaded two rows ahead (halo_conv.hip PF2)
    halo_pf2 = env("halo_pf2", 0);
    // halo conv as persistent workgroups (resident count x this; 0 = one
    // tile per workgroup) that prefetch the next tile's halo; halo_grid > 0
    // caps the grid (tests: several tiles per workgroup on small images)
    halo_persist = env("halo_persist", 1);
    halo_grid = env("halo_grid", 0);
    // 3x3 halo convs keep all their tap weights in LDS (per workgroup, for
    // all its tiles) when they need at most this many KB; 0 = stream rows
    halo_res_kb = env("halo_res_kb", 48);
    // halo conv bf16 outputs through LDS as 16-byte rows (halo_conv.hip)
    halo_staged = env("halo_staged", 1);
    // reflect fold of the split-form data gradient: a VALU pass over the
    // border list (conv.hip reflect_border_kernel) instead of the GEMM
    border_valu = env("border_valu", 1);
    // high-resolution 1x1 convs (M >= 16k, C <= 256, N <= 192) on the
    // streaming kernel (stream1x1.hip) instead of 256-row GEMM tiles
    s1x1 = env("s1x1", 1);
    // small-M 1x1 convs (stream1x1.hip s1x1_small_kernel, M < 16k pixels)
    s1x1_small = env("s1x1_small", 1);
  }
};
Knobs& knobs() {
  static Knobs k;
  return k;
}

// Deep layers (few 128x128 tiles) use 64x64 tiles: 4x the workgroups, more of
// them per CU (32 KB of LDS each), so more loads in flight per CU instead of
// a split-K round trip through an f32 workspace.  Depends on (M, NC) only so
// um_conv_stats_parts can follow it.
bool small_tiles(int M, int NC) {
  const Knobs& k = knobs();
  return k.small && NC > 64 && (long)ceil_div(M, 128) * ceil_div(NC, 128) < k.small_tiles;
}

void split_plan(Plan& p, int M, int NC, int taps, int ach, long ws_bytes, bool glds);

// glds: the launch will take the LDS-DMA loop (its split thresholds); the
// workspace query passes false, whose split counts bound the LDS-DMA ones
Plan make_plan(int dtype, int M, int NC, int taps, int ach, long ws_bytes, bool glds) {
  const Knobs& kn = knobs();
  Plan p{};
  p.bk = 32;
  if (NC <= 16) { p.bm = 256; p.bn = 16; p.wm = 4; p.wn = 1; }
  else if (NC <= 32) { p.bm = 256; p.bn = 32; p.wm = 4; p.wn = 1; }
  else if (NC <= 48 && kn.odd_bn) { p.bm = 256; p.bn = 48; p.wm = 4; p.wn = 1; }
  else if (NC <= 64) { p.bm = 256; p.bn = 64; p.wm = 4; p.wn = 1; }
  else if (small_tiles(M, NC)) {
    p.bm = 64; p.bn = 64; p.wm = 2; p.wn = 2;
    if (dtype == UM_BF16 && ach % 64 == 0 && (kn.bk64 & 1)) p.bk = 64;
  } else {
    // 128-row tiles; the column width that pads the fewest columns.  The
    // data gradient's NC is the conv's INPUT channel count, which after the
    // decoder concats is 72/88/160/168/320: 96- and 160-wide tiles cut the
    // padded MFMA work from up to 44 % to at most 12.5 % there.
    p.bm = 128; p.bn = 128; p.wm = 2; p.wn = 2;
    if (kn.odd_bn) {
      auto padded = [&](int bn) { return (long)ceil_div(NC, bn) * bn; };
      if (padded(96) < padded(p.bn)) p.bn = 96;
      if (padded(160) < padded(p.bn)) p.bn = 160;
    }
    if (dtype == UM_BF16 && ach % 64 == 0 && (kn.bk64 & 2)) p.bk = 64;  // 64-83 KB of LDS: 1-2 blocks/CU
  }
  split_plan(p, M, NC, taps, ach, ws_bytes, glds);
  return p;
}

// tap packing applies to 8-channel operands on the 32-deep register path
bool tappack_ok(int ach, int bk) { return (knobs().tappack & 1) && ach == 8 && bk == 32; }

void split_plan(Plan& p, int M, int NC, int taps, int ach, long ws_bytes, bool glds) {
  const Knobs& kn = knobs();
  p.steps = tappack_ok(ach, p.bk) ? ceil_div(taps, p.bk / 8) : taps * ((ach + p.bk - 1) / p.bk);
  // Split grids that leave CUs with too few blocks to hide load latency: the
  // partials cost an f32 write + read of splits*M*NC (about 1 us per 8 MB
  // each way), so aim at ~1024 blocks, >= 4 k-steps per split and <= 32 MB
  // of partials.
  const long tiles = (long)ceil_div(M, p.bm) * ceil_div(NC, p.bn);
  p.splits = 1;
  const int below = glds ? kn.glds_split_below : kn.split_below;
  const int target = glds ? kn.glds_split_target : kn.split_target;
  if (tiles < below && NC % 4 == 0) {
    long sp = (target + tiles - 1) / tiles;
    sp = std::min<long>(sp, p.steps / kn.split_minsteps);
    sp = std::min<long>(sp, (32l << 20) / ((long)M * NC * 4));
    if (ws_bytes >= 0) sp = std::min<long>(sp, ws_bytes / ((long)M * NC * 4));
    if (sp >= 2) p.splits = (int)sp;
  }
  p.per = ceil_div(p.steps, p.splits);
  p.splits = ceil_div(p.steps, p.per);  // no empty splits
}

template <typename T, int BK, int BM, int BN, int WM, int WN, int MODE>
int launch_cls(const IgArgs& a, const Plan& p, float* ws, hipStream_t st) {
  const int ntm = ceil_div(a.M, BM), ntn = ceil_div(a.NC, BN);
  if constexpr (sizeof(T) == 2 && BK == 64 && WM == 2 && WN == 2 && MODE != 2) {
    if (a.pmode != umamd::IG_FOLD && (knobs().glds & (BM == 64 ? 1 : 2))) {
      const bool w8 = BM == 64 && (knobs().glds & 4);
      const long blocks = (long)ntm * ntn * p.splits;
      const bool deep = BM == 64 && w8 && knobs().glds_deep > 3 && blocks <= knobs().glds_deep_blocks;
      constexpr int DEEP = BM == 64 ? 6 : 3;  // 96 KB of stages: 64x64 tiles only
      const IgArgs& g = a;
      const dim3 grid(ntm * ntn, 1, p.splits);
      if (deep && p.splits > 1)
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 8, true, MODE, DEEP>), grid, dim3(512), 0, st, g,
                           ws, p.steps, p.per, ntn);
      else if (deep)
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 8, false, MODE, DEEP>), grid, dim3(512), 0, st, g,
                           ws, p.steps, p.per, ntn);
      else if (w8 && p.splits > 1)
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 8, true, MODE, 3>), grid, dim3(512), 0, st, g, ws,
                           p.steps, p.per, ntn);
      else if (w8)
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 8, false, MODE, 3>), grid, dim3(512), 0, st, g, ws,
                           p.steps, p.per, ntn);
      else if (p.splits > 1)
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 4, true, MODE, 3>), grid, dim3(256), 0, st, g, ws,
                           p.steps, p.per, ntn);
      else
        hipLaunchKernelGGL((igemm_glds_kernel<BM, BN, 4, false, MODE, 3>), grid, dim3(256), 0, st, g, ws,
                           p.steps, p.per, ntn);
      if (p.splits > 1) {
        const int er = a.epilogue == UM_EPI_STATS ? a.stats_rows : EPI_ROWS;
        hipLaunchKernelGGL((splitk_epilogue_kernel<T, MODE>),
                           dim3(ceil_div(a.M, er), ceil_div(a.NC, EPI_COLS)), dim3(256), 0, st, a,
                           (const float*)ws, p.splits, er);
      }
      UM_LAUNCH_CHECK();
      return UM_OK;
    }
  }
  if (p.splits > 1) {
    hipLaunchKernelGGL((igemm_kernel<T, BK, BM, BN, WM, WN, true, MODE>),
                       dim3(ntm * ntn, 1, p.splits), dim3(256), 0, st, a, ws, p.steps, p.per, ntn);
    const int er = a.epilogue == UM_EPI_STATS ? a.stats_rows : EPI_ROWS;
    hipLaunchKernelGGL((splitk_epilogue_kernel<T, MODE>),
                       dim3(ceil_div(a.M, er), ceil_div(a.NC, EPI_COLS)), dim3(256), 0, st, a,
                       (const float*)ws, p.splits, er);
  } else {
    hipLaunchKernelGGL((igemm_kernel<T, BK, BM, BN, WM, WN, false, MODE>), dim3(ntm * ntn, 1, 1),
                       dim3(256), 0, st, a, ws, p.steps, p.per, ntn);
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

template <typename T, int BK, int BM, int BN, int WM, int WN>
int launch(const IgArgs& a, const Plan& p, float* ws, hipStream_t st) {
  return a.cls ? launch_cls<T, BK, BM, BN, WM, WN, 1>(a, p, ws, st)
               : launch_cls<T, BK, BM, BN, WM, WN, 0>(a, p, ws, st);
}

template <typename T>
int dispatch_tiles(const IgArgs& a, const Plan& p, float* ws, hipStream_t st) {
  if (p.bn == 16) return launch<T, 32, 256, 16, 4, 1>(a, p, ws, st);
  if (p.bn == 32) return launch<T, 32, 256, 32, 4, 1>(a, p, ws, st);
  if (p.bn == 48) return launch<T, 32, 256, 48, 4, 1>(a, p, ws, st);
  if (p.bn == 96) {
    if constexpr (sizeof(T) == 2)
      if (p.bk == 64) return launch<T, 64, 128, 96, 2, 2>(a, p, ws, st);
    return launch<T, 32, 128, 96, 2, 2>(a, p, ws, st);
  }
  if (p.bn == 160) {
    if constexpr (sizeof(T) == 2)
      if (p.bk == 64) return launch<T, 64, 128, 160, 2, 2>(a, p, ws, st);
    return launch<T, 32, 128, 160, 2, 2>(a, p, ws, st);
  }
  if (p.bn == 64 && p.bm == 256) return launch<T, 32, 256, 64, 4, 1>(a, p, ws, st);
  if (p.bm == 64) {
    if constexpr (sizeof(T) == 2)
      if (p.bk == 64) return launch<T, 64, 64, 64, 2, 2>(a, p, ws, st);
    return launch<T, 32, 64, 64, 2, 2>(a, p, ws, st);
  }
  if constexpr (sizeof(T) == 2)
    if (p.bk == 64) return launch<T, 64, 128, 128, 2, 2>(a, p, ws, st);
  return launch<T, 32, 128, 128, 2, 2>(a, p, ws, st);
}

}  // namespace

namespace umamd {

int igemm_fold_split_nc() { return knobs().fold_split_nc; }

// the zero-pad pass of a reflect data gradient in split form would run on
// the halo kernel ("same" 3x3/5x5/7x7, 8x32 tiles, enough of them)
bool igemm_halo_dgrad(int dtype, int N, int H, int W, int C, int R) {
  const Knobs& k = knobs();
  if (!k.halo || dtype != UM_BF16 || (R != 3 && R != 5 && R != 7)) return false;
  if (H % 8 || W % 32 || C > k.halo_max_nc || C % 8) return false;
  return (long)N * (H / 8) * (W / 32) >= k.halo_min_tiles;
}
int igemm_pad_dgrad() { return knobs().pad_dgrad; }
int igemm_halo_pf2() { return knobs().halo_pf2; }
int igemm_halo_persist() { return knobs().halo_persist; }
int igemm_halo_grid() { return knobs().halo_grid; }
int igemm_halo_res_kb() { return knobs().halo_res_kb; }
int igemm_halo_staged() { return knobs().halo_staged; }
int igemm_border_valu() { return knobs().border_valu; }

int igemm_border_list(IgArgs& a) {
  const int H = a.oh, W = a.ow, p = a.fold_pad;
  auto receives = [p](int i, int n) { return (i >= 1 && i <= p) || (i >= n - 1 - p && i <= n - 2); };
  a.border = 1;
  a.nrr = a.nrc = 0;
  for (int i = 0; i < H && a.nrr < 4; ++i)
    if (receives(i, H)) a.rr[a.nrr++] = i;
  for (int j = 0; j < W && a.nrc < 4; ++j)
    if (receives(j, W)) a.rc[a.nrc++] = j;
  return a.nrr * W + (H - a.nrr) * a.nrc;
}

long igemm_ws_bytes(int dtype, int M, int NC, int taps, int ach) {
  const Plan p = make_plan(dtype, M, NC, taps, ach, -1, false);
  return p.splits > 1 ? (long)p.splits * M * NC * 4 : 0;
}

// split-K workspace of the reflect fold's border-list GEMM (igemm_run's
// a.border plan: 64x64 register tiles, 32-deep k-steps)
long igemm_border_ws_bytes(int dtype, int M, int NC, int taps, int ach) {
  (void)dtype;
  Plan p{};
  p.bk = 32; p.bm = 64; p.bn = 64; p.wm = 2; p.wn = 2;
  split_plan(p, M, NC, taps, ach, -1, false);
  return p.splits > 1 ? (long)p.splits * M * NC * 4 : 0;
}

int igemm_stats_rows(int M, int NC) { return small_tiles(M, NC) ? 64 : 128; }

int igemm_run(int dtype, const IgArgs& a_in, float* ws, long ws_bytes, hipStream_t st) {
  if (a_in.M == 0) return UM_OK;
  IgArgs a = a_in;
  a.stats_rows = igemm_stats_rows(a.M, a.NC);
  {
    // column-major tile order when B (NC x taps x ach) is larger than the
    // gathered image A (M x ach): knob xcd_col 0 = never, 1 = auto, 2 = always
    const int xc = knobs().xcd_col;
    const long abytes = (long)a.M * a.ach, bbytes = (long)a.NC * a.R * a.Rx * a.ach;
    a.colmajor = xc == 2 || (xc == 1 && bbytes > abytes);
  }
  if (a.border) {
    // the reflect fold's border list: a few thousand rows, one small plan
    Plan p{};
    p.bk = 32; p.bm = 64; p.bn = 64; p.wm = 2; p.wn = 2;
    split_plan(p, a.M, a.NC, a.R * a.Rx, a.ach, ws ? ws_bytes : 0, false);
    a.tappack = tappack_ok(a.ach, p.bk);
    if (dtype == UM_BF16) return launch_cls<bf16_t, 32, 64, 64, 2, 2, 2>(a, p, ws, st);
    return launch_cls<float, 32, 64, 64, 2, 2, 2>(a, p, ws, st);
  }
  if (knobs().s1x1 && stream1x1_applicable(dtype, a)) return stream1x1_run(a, st);
  if (knobs().s1x1_small && s1x1_small_applicable(dtype, a)) return s1x1_small_run(a, st);
  // 8-channel operands take the tap-packed GEMM instead of the halo kernel
  // (which stages 32-channel chunks) unless tappack bit 1 is clear
  const bool pack_first = (knobs().tappack & 3) == 3 && a.ach == 8;
  if (knobs().halo && !pack_first &&
      halo_applicable(dtype, a, knobs().halo_min_tiles, knobs().halo_max_nc))
    return halo_run(a, st);
  // the LDS-DMA loop serves the bf16 64x64 tiles without the reflect fold
  Plan p = make_plan(dtype, a.M, a.NC, a.R * a.Rx, a.ach, ws ? ws_bytes : 0, false);
  if (dtype == UM_BF16 && p.bm == 64 && p.bk == 64 && a.pmode != IG_FOLD && (knobs().glds & 1))
    p = make_plan(dtype, a.M, a.NC, a.R * a.Rx, a.ach, ws ? ws_bytes : 0, true);
  a.tappack = tappack_ok(a.ach, p.bk);
  if (dtype == UM_BF16) return dispatch_tiles<bf16_t>(a, p, ws, st);
  return dispatch_tiles<float>(a, p, ws, st);
}

// the four parity classes of a stride-2 data gradient on 64x64 LDS-DMA tiles
// in one launch (+ one split-K epilogue launch): per-class tile ranges,
// per-class split counts (the split target over the classes' tiles together,
// each class capped by its own k-steps) and workspace slices
struct Cls4Plan {
  int ntn;
  int start[5], ntiles[4], steps[4], per[4], splits[4];
  long wsoff[4];  // f32 elements
  long ws;        // bytes (0: no split)
};

// column tile of the 4-class launch: 64 (8 waves), or 32 (4 waves) when NC is 32
static int cls4_bn(int NC) { return NC % 64 == 0 ? 64 : 32; }

static Cls4Plan cls4_glds_plan(const int (&M)[4], const int (&taps)[4], int NC, int ach,
                               long ws_bytes) {
  const Knobs& kn = knobs();
  Cls4Plan p{};
  p.ntn = ceil_div(NC, cls4_bn(NC));
  long tiles = 0, rows = 0;
  for (int c = 0; c < 4; ++c) {
    p.ntiles[c] = ceil_div(M[c], 64) * p.ntn;
    p.start[c + 1] = p.start[c] + p.ntiles[c];
    p.steps[c] = taps[c] * ceil_div(ach, 64);
    tiles += p.ntiles[c];
    rows += M[c];
  }
  long sp = 1;
  if (tiles < kn.glds_split_below && NC % 4 == 0 && rows > 0) {
    sp = (kn.glds_split_target + tiles - 1) / tiles;
    sp = std::min<long>(sp, (32l << 20) / (rows * NC * 4));
    if (ws_bytes >= 0) sp = std::min<long>(sp, ws_bytes / (rows * NC * 4));
  }
  long off = 0;
  bool split = false;
  for (int c = 0; c < 4; ++c) {
    long sc = sp >= 2 ? std::min<long>(sp, p.steps[c] / kn.split_minsteps) : 1;
    if (sc < 1) sc = 1;
    p.per[c] = std::max(1, ceil_div(p.steps[c], sc));
    p.splits[c] = std::max(1, ceil_div(p.steps[c], p.per[c]));
    split |= p.splits[c] > 1;
    p.wsoff[c] = off;
    off += (long)p.splits[c] * M[c] * NC;
  }
  p.ws = split ? off * 4 : 0;
  return p;
}

static bool cls4_glds_ok(int dtype, const IgArgs (&as)[4]) {
  if (!knobs().cls4 || !knobs().cls_glds || !(knobs().glds & 1) || dtype != UM_BF16) return false;
  for (const auto& a : as)
    if (a.M <= 0 || (a.NC % 64 && !(a.NC == 32 && (knobs().cls_glds & 2))) || a.ach % 64 ||
        a.pmode != IG_PAD_ZERO)
      return false;
  return true;
}

long igemm_cls4_ws_bytes(int dtype, const int (&M)[4], const int (&taps)[4], int NC, int ach) {
  if (!knobs().cls4 || !knobs().cls_glds || dtype != UM_BF16 || ach % 64 ||
      (NC % 64 && !(NC == 32 && (knobs().cls_glds & 2))))
    return 0;
  return cls4_glds_plan(M, taps, NC, ach, -1).ws;
}

static int run_cls4_glds(IgArgs (&as)[4], float* ws, long ws_bytes, hipStream_t st) {
  int M[4], taps[4];
  for (int c = 0; c < 4; ++c) {
    M[c] = as[c].M;
    taps[c] = as[c].R * as[c].Rx;
  }
  const int NC = as[0].NC, ach = as[0].ach;
  const Cls4Plan p = cls4_glds_plan(M, taps, NC, ach, ws ? ws_bytes : 0);
  const bool split = p.ws > 0;
  int zmax = 1;
  int rstart[5] = {0, 0, 0, 0, 0};
  for (int c = 0; c < 4; ++c) {
    IgArgs& a = as[c];
    a.stats_rows = igemm_stats_rows(a.M, a.NC);
    const int xc = knobs().xcd_col;
    const long abytes = (long)a.M * a.ach, bbytes = (long)a.NC * a.R * a.Rx * a.ach;
    a.colmajor = xc == 2 || (xc == 1 && bbytes > abytes);
    a.tappack = 0;
    zmax = std::max(zmax, p.splits[c]);
    rstart[c + 1] = rstart[c] + ceil_div(a.M, a.stats_rows);
  }
  const dim3 grid(p.start[4], 1, split ? zmax : 1);
  const int4 s4 = make_int4(p.start[0], p.start[1], p.start[2], p.start[3]);
  const int4 k4 = make_int4(p.steps[0], p.steps[1], p.steps[2], p.steps[3]);
  const int4 per4 = make_int4(p.per[0], p.per[1], p.per[2], p.per[3]);
  const int4 sp4 = split ? make_int4(p.splits[0], p.splits[1], p.splits[2], p.splits[3])
                         : make_int4(1, 1, 1, 1);
  const int4 nt4 = make_int4(p.ntiles[0], p.ntiles[1], p.ntiles[2], p.ntiles[3]);
  const long4 off4 = make_long4(p.wsoff[0], p.wsoff[1], p.wsoff[2], p.wsoff[3]);
  const long blocks = (long)p.start[4] * (split ? zmax : 1);
  const bool deep = knobs().glds_deep > 3 && blocks <= knobs().glds_deep_blocks;
#define UM_GC4(SP_, NST_)                                                                         \
  do {                                                                                            \
    if (cls4_bn(NC) == 32)                                                                        \
      hipLaunchKernelGGL((igemm_glds_cls4_kernel<32, 4, SP_, NST_>), grid, dim3(256), 0, st,      \
                         as[0], as[1], as[2], as[3], s4, k4, per4, sp4, nt4, p.ntn, ws, off4);    \
    else                                                                                          \
      hipLaunchKernelGGL((igemm_glds_cls4_kernel<64, 8, SP_, NST_>), grid, dim3(512), 0, st,      \
                         as[0], as[1], as[2], as[3], s4, k4, per4, sp4, nt4, p.ntn, ws, off4);    \
  } while (0)
  if (split && deep) UM_GC4(true, 6);
  else if (split) UM_GC4(true, 3);
  else if (deep) UM_GC4(false, 6);
  else UM_GC4(false, 3);
#undef UM_GC4
  if (split) {
    const int4 r4 = make_int4(rstart[0], rstart[1], rstart[2], rstart[3]);
    hipLaunchKernelGGL(splitk_epilogue_cls4_kernel<bf16_t>, dim3(rstart[4], ceil_div(NC, EPI_COLS)),
                       dim3(256), 0, st, as[0], as[1], as[2], as[3], r4, sp4, (const float*)ws,
                       off4);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("igemm_run_cls4: %s", hipGetErrorString(e));
    return -UM_ERR_HIP;
  }
  return 1;
}

// the four parity classes of a stride-2 data gradient in one launch (bf16,
// 256-row register tiles when the LDS-DMA form does not apply); returns 1
// when launched, 0 when the caller should launch the classes one by one, or
// an error code < 0
int igemm_run_cls4(int dtype, IgArgs (&as)[4], float* ws, long ws_bytes, hipStream_t st) {
  if (cls4_glds_ok(dtype, as)) return run_cls4_glds(as, ws, ws_bytes, st);
  if (!knobs().cls4 || dtype != UM_BF16) return 0;
  for (auto& a : as)
    if (a.M <= 0) return 0;
  const Plan p0 = make_plan(dtype, as[0].M, as[0].NC, as[0].R * as[0].Rx, as[0].ach, 0, false);
  if (p0.bm != 256 || p0.bk != 32) return 0;
  int start[5] = {0, 0, 0, 0, 0}, steps[4];
  const int ntn = ceil_div(as[0].NC, p0.bn);
  for (int c = 0; c < 4; ++c) {
    IgArgs& a = as[c];
    a.stats_rows = igemm_stats_rows(a.M, a.NC);
    a.colmajor = 0;
    Plan p = p0;
    split_plan(p, a.M, a.NC, a.R * a.Rx, a.ach, 0, false);  // no workspace: no split
    a.tappack = tappack_ok(a.ach, p.bk);
    steps[c] = p.steps;
    start[c + 1] = start[c] + ceil_div(a.M, 256) * ntn;
  }
  const dim3 grid(start[4]);
  const int4 s4 = make_int4(start[0], start[1], start[2], start[3]);
  const int4 k4 = make_int4(steps[0], steps[1], steps[2], steps[3]);
#define UM_CLS4(BN_)                                                                       \
  hipLaunchKernelGGL((igemm_cls4_kernel<bf16_t, 32, 256, BN_, 4, 1>), grid, dim3(256), 0, st, \
                     as[0], as[1], as[2], as[3], s4, k4, ntn)
  if (p0.bn == 16) UM_CLS4(16);
  else if (p0.bn == 32) UM_CLS4(32);
  else if (p0.bn == 48) UM_CLS4(48);
  else UM_CLS4(64);
#undef UM_CLS4
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("igemm_run_cls4: %s", hipGetErrorString(e));
    return -UM_ERR_HIP;
  }
  return 1;
}

}  // namespace umamd

// tuning knobs at run time (tests force code paths; sweeps): returns the old
// value, or -1 for an unknown key
extern "C" int um_set_tuning(const char* key, int value) {
  Knobs& k = knobs();
  int* f = nullptr;
  if (!strcmp(key, "halo")) f = &k.halo;
  else if (!strcmp(key, "halo_min_tiles")) f = &k.halo_min_tiles;
  else if (!strcmp(key, "small")) f = &k.small;
  else if (!strcmp(key, "small_tiles")) f = &k.small_tiles;
  else if (!strcmp(key, "split_below")) f = &k.split_below;
  else if (!strcmp(key, "split_target")) f = &k.split_target;
  else if (!strcmp(key, "glds_split_below")) f = &k.glds_split_below;
  else if (!strcmp(key, "glds_split_target")) f = &k.glds_split_target;
  else if (!strcmp(key, "split_minsteps")) f = &k.split_minsteps;
  else if (!strcmp(key, "odd_bn")) f = &k.odd_bn;
  else if (!strcmp(key, "bk64")) f = &k.bk64;
  else if (!strcmp(key, "glds")) f = &k.glds;
  else if (!strcmp(key, "glds_deep")) f = &k.glds_deep;
  else if (!strcmp(key, "xcd_col")) f = &k.xcd_col;
  else if (!strcmp(key, "tappack")) f = &k.tappack;
  else if (!strcmp(key, "cls4")) f = &k.cls4;
  else if (!strcmp(key, "cls_glds")) f = &k.cls_glds;
  else if (!strcmp(key, "pad_dgrad")) f = &k.pad_dgrad;
  else if (!strcmp(key, "glds_deep_blocks")) f = &k.glds_deep_blocks;
  else if (!strcmp(key, "fold_split_nc")) f = &k.fold_split_nc;
  else if (!strcmp(key, "halo_max_nc")) f = &k.halo_max_nc;
  else if (!strcmp(key, "halo_pf2")) f = &k.halo_pf2;
  else if (!strcmp(key, "halo_persist")) f = &k.halo_persist;
  else if (!strcmp(key, "halo_grid")) f = &k.halo_grid;
  else if (!strcmp(key, "halo_res_kb")) f = &k.halo_res_kb;
  else if (!strcmp(key, "halo_staged")) f = &k.halo_staged;
  else if (!strcmp(key, "border_valu")) f = &k.border_valu;
  else if (!strcmp(key, "s1x1")) f = &k.s1x1;
  else if (!strcmp(key, "s1x1_small")) f = &k.s1x1_small;
  if (!f) return -1;
  const int old = *f;
  *f = value;
  return old;
}
