// Implicit-GEMM convolutions on MFMA for gfx950 (CDNA4): C-ABI entries, the
// weight gradient, weight packing and column reductions.  Forward convs and
// stride-1 data gradients run on the tap-major kernel of igemm.hip; the
// general gather kernel below serves the stride-2 data gradient.
//
// General kernel (forward form kept for reference, dgrad form in use):
//   forward  : Y[m=(n,p,q)][k]  = sum_{(r,s,c)} X[n, p*st-pad+r, q*st-pad+s, c] * Wf[k][r][s][c]
//   dgrad    : DX[m=(n,h,w)][c] = sum_{(r,s,k)} DY[src(n,h,w,r,s)][k] * WT[c][r][s][k]
// where src() inverts the forward gather: the stride-2 parity filter and the
// reflect-pad fold (a border pixel of X feeds two padded taps).
// The weight gradient is a separate template whose operands are both
// pixel-major, transposed into LDS.
//
// Tiles: BM x BN output, BK = 32 reduction step, 256 threads = 4 waves, each
// wave a (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA fragments.  LDS rows are
// padded by 8 elements.  One LDS buffer + register prefetch of the next tile.
//
// bf16: v_mfma_f32_16x16x32_bf16 (lane l: A[l&15][8(l>>4)+j], j<8).
// f32 : 8 x v_mfma_f32_16x16x4_f32 per BK step with the k-permutation
//       "lane group g, element e -> k = 8g+e" on both operands (exact f32).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "igemm.h"
#include "wgrad_halo.h"
#include "wgrad_tr.h"

namespace {

constexpr int BK = 32;

// input-channel segments of a packed weight: reference channels
// [src0, src0+len) live at packed channels [dst0, dst0+len); other packed
// channels are zero (used to keep concat segments 8-channel aligned)
constexpr int MAX_SEG = 4;
struct Segs {
  int n;
  int src0[MAX_SEG], dst0[MAX_SEG], len[MAX_SEG];
};
__device__ __forceinline__ int seg_src(const Segs& g, int c) {  // packed -> reference, or -1
  // unrolled over static indices (segments do not overlap): a runtime index
  // would put a by-value Segs in scratch
  int r = -1;
#pragma unroll
  for (int i = 0; i < MAX_SEG; ++i)
    if (i < g.n && c >= g.dst0[i] && c < g.dst0[i] + g.len[i]) r = g.src0[i] + c - g.dst0[i];
  return r;
}
constexpr int LDK = BK + 8;  // padded LDS row (elements)

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { bf16x8_t v; };
template <> struct Frag<float> { float v[8]; };

__device__ __forceinline__ void lds_frag(const bf16_t* p, Frag<bf16_t>& f) {
  f.v = *reinterpret_cast<const bf16x8_t*>(p);
}
__device__ __forceinline__ void lds_frag(const float* p, Frag<float>& f) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
  f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
}
__device__ __forceinline__ void mfma(f32x4_t& acc, const Frag<bf16_t>& a, const Frag<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mfma(f32x4_t& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int e = 0; e < 8; ++e)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[e], b.v[e], acc, 0, 0, 0);
}

// add 8 raw elements into an f32 accumulator (used by the reflect fold)
__device__ __forceinline__ void accum8(const bf16_t* p, float* v) {
  float t[8];
  load8(p, t);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] += t[i];
}
__device__ __forceinline__ void accum8(const float* p, float* v) {
  float t[8];
  load8(p, t);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] += t[i];
}
__device__ __forceinline__ void f32_to_raw(const float* v, Raw8<bf16_t>& r) {
  r.v.x = pack_bf16x2(v[0], v[1]);
  r.v.y = pack_bf16x2(v[2], v[3]);
  r.v.z = pack_bf16x2(v[4], v[5]);
  r.v.w = pack_bf16x2(v[6], v[7]);
}
__device__ __forceinline__ void f32_to_raw(const float* v, Raw8<float>& r) {
  r.a = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                   __float_as_uint(v[3]));
  r.b = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                   __float_as_uint(v[7]));
}

// sources in [0, n) of a dgrad tap: forward used index r(o*st + tap - pad) = i
__device__ __forceinline__ int dgrad_sources(int i, int tap, int n_in, int n_out, int st,
                                             int pad, int reflect, int* srcs) {
  int cnt = 0;
  int cand[3];
  int nc = 1;
  cand[0] = i;
  if (reflect) {
    if (i >= 1 && i <= pad) cand[nc++] = -i;
    if (i >= n_in - 1 - pad && i <= n_in - 2) cand[nc++] = 2 * (n_in - 1) - i;
  }
  for (int c = 0; c < nc; ++c) {
    const int t = cand[c] + pad - tap;  // = o * st
    if (t < 0) continue;
    if (st == 2) {
      if (t & 1) continue;
      const int o = t >> 1;
      if (o < n_out) srcs[cnt++] = o;
    } else {
      if (t < n_out) srcs[cnt++] = t;
    }
  }
  return cnt;
}

struct WgradArgs {
  int N, H, W, C, ldx, K, R, stride, pad, pad_mode, P, Q, ldy;
  const void* x;
  const void* dy;
  float* slabs;
  int M, RRC, m_per_split;
};

template <typename T, int BM, int BN>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs a) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_CH = BK * BM / 8;  // dy chunks: 32 m x BM/8 k-chunks
  constexpr int B_CH = BK * BN / 8;
  constexpr int A_PER = (A_CH + 255) / 256, B_PER = (B_CH + 255) / 256;
  __shared__ __attribute__((aligned(16))) T sA[BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[BN * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bk = blockIdx.x * BM;  // output-channel tile
  const int bj = blockIdx.y * BN;  // (r,s,c) tile
  const int m_begin = blockIdx.z * a.m_per_split;
  const int m_end = min(a.M, m_begin + a.m_per_split);
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ DY = reinterpret_cast<const T*>(a.dy);

  // fixed column chunks per thread
  int a_m[A_PER], a_c[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int c = tid + i * 256;
    a_m[i] = c / (BM / 8);
    a_c[i] = (c % (BM / 8)) * 8;
  }
  int b_m[B_PER], b_j[B_PER], b_r[B_PER], b_s[B_PER], b_ch[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int c = tid + i * 256;
    b_m[i] = c / (BN / 8);
    b_j[i] = (c % (BN / 8)) * 8;
    const int j = bj + b_j[i];
    b_ok[i] = (c < B_CH) && (j < a.RRC);
    const int jj = b_ok[i] ? j : 0;
    const int tap = jj / a.C;
    b_ch[i] = jj - tap * a.C;
    b_r[i] = tap / a.R;
    b_s[i] = tap - b_r[i] * a.R;
  }

  float va[A_PER][8], vb[B_PER][8];
  const int pq = a.P * a.Q;
  auto load_tiles = [&](int m0) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int m = m0 + a_m[i];
      const int k = bk + a_c[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) va[i][e] = 0.f;
      if (tid + i * 256 < A_CH && m < m_end && k < a.K) load8(DY + (long)m * a.ldy + k, va[i]);
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int m = m0 + b_m[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) vb[i][e] = 0.f;
      if (!b_ok[i] || m >= m_end) continue;
      const int n = m / pq;
      const int rr = m - n * pq;
      const int p = rr / a.Q, q = rr - (rr / a.Q) * a.Q;
      int yy = p * a.stride - a.pad + b_r[i], xx = q * a.stride - a.pad + b_s[i];
      if (a.pad_mode == UM_PAD_REFLECT) {
        yy = reflect_idx(yy, a.H);
        xx = reflect_idx(xx, a.W);
      } else if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W) {
        continue;
      }
      load8(X + ((long)(n * a.H + yy) * a.W + xx) * a.ldx + b_ch[i], vb[i]);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fk = (lane >> 4) * 8;
  if (m_begin < m_end) load_tiles(m_begin);
  for (int m0 = m_begin; m0 < m_end; m0 += BK) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
      if (tid + i * 256 < A_CH)
#pragma unroll
        for (int e = 0; e < 8; ++e) sA[(a_c[i] + e) * LDK + a_m[i]] = from_f32<T>(va[i][e]);
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      if (tid + i * 256 < B_CH)
#pragma unroll
        for (int e = 0; e < 8; ++e) sB[(b_j[i] + e) * LDK + b_m[i]] = from_f32<T>(vb[i][e]);
    __syncthreads();
    if (m0 + BK < m_end) load_tiles(m0 + BK);
    Frag<T> fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) lds_frag(&sA[(wm * (BM / WM) + i * 16 + frow) * LDK + fk], fa[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) lds_frag(&sB[(wn * (BN / WN) + j * 16 + frow) * LDK + fk], fb[j]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(acc[i][j], fa[i], fb[j]);
  }

  float* out = a.slabs + (long)blockIdx.z * a.K * a.RRC;
  const int col_l = lane & 15, row_g = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = bk + wm * (BM / WM) + i * 16 + row_g + r;
        const int jj = bj + wn * (BN / WN) + j * 16 + col_l;
        if (k < a.K && jj < a.RRC) out[(long)k * a.RRC + jj] = acc[i][j][r];
      }
}

template <typename T, int BM, int BN>
int launch_wgrad(const WgradArgs& a, int splits, hipStream_t st) {
  dim3 grid(ceil_div(a.K, BM), ceil_div(a.RRC, BN), splits);
  hipLaunchKernelGGL((wgrad_kernel<T, BM, BN>), grid, dim3(256), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// ---- bf16 weight gradient: both operands pixel-major in memory.  Each thread
// loads an 8(m) x 8(col) bf16 block (8 x 16 B), transposes it in registers
// (v_perm) and writes 8 x ds_write_b128 rows of 8 consecutive m, so the MFMA
// fragments (8 consecutive reduction elements per lane) read with
// ds_read_b128.  Tile BM (out channels) x 128 (r,s,c) x 64 pixels, 4 waves.
constexpr int WBK = 64;
constexpr int WLDK = WBK + 8;

__device__ __forceinline__ void transpose8x8_bf16(const uint4* in, uint4* out) {
  // in[r] = row r (8 bf16 of consecutive cols); out[e] = col e (8 bf16 of consecutive rows)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in);  // w[r*4 + d]
  uint32_t* o = reinterpret_cast<uint32_t*>(out);              // o[e*4 + q]
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t x = w[(2 * q) * 4 + (e >> 1)], y = w[(2 * q + 1) * 4 + (e >> 1)];
      o[e * 4 + q] = (e & 1) ? __builtin_amdgcn_perm(y, x, 0x07060302u)
                             : __builtin_amdgcn_perm(y, x, 0x05040100u);
    }
}

template <int BM>
__global__ void __launch_bounds__(256) wgrad_bf16_kernel(WgradArgs a) {
  constexpr int BN = 128;
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_BLK = BM;       // (BM/8) x (WBK/8)
  constexpr int B_BLK = BN;       // (BN/8) x (WBK/8)
  static_assert(A_BLK + B_BLK <= 256, "one 8x8 block per thread");
  __shared__ __attribute__((aligned(16))) bf16_t sA[BM * WLDK];
  __shared__ __attribute__((aligned(16))) bf16_t sB[BN * WLDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bk = blockIdx.x * BM;
  const int bj = blockIdx.y * BN;
  const int m_begin = blockIdx.z * a.m_per_split;
  const int m_end = min(a.M, m_begin + a.m_per_split);
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ DY = reinterpret_cast<const bf16_t*>(a.dy);

  // block role
  const bool isA = tid < A_BLK;
  const bool isB = !isA && tid < A_BLK + B_BLK;
  int cb = 0, mb = 0;  // column block, m block
  if (isA) { cb = tid % (BM / 8); mb = tid / (BM / 8); }
  if (isB) { const int t = tid - A_BLK; cb = t % (BN / 8); mb = t / (BN / 8); }
  // B column decode (one tap, 8 channels)
  int br = 0, bs = 0, bch = 0;
  bool bok = false;
  if (isB) {
    const int j = bj + cb * 8;
    bok = j < a.RRC;
    const int jj = bok ? j : 0;
    const int tap = jj / a.C;
    bch = jj - tap * a.C;
    br = tap / a.R;
    bs = tap - br * a.R;
  }
  const bool aok = isA && (bk + cb * 8 < a.K);
  const int pq = a.P * a.Q;

  uint4 blk[8];
  auto load = [&](int m0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      blk[r] = make_uint4(0, 0, 0, 0);
      const int m = m0 + mb * 8 + r;
      if (m >= m_end) continue;
      if (isA) {
        if (aok) blk[r] = *reinterpret_cast<const uint4*>(DY + (long)m * a.ldy + bk + cb * 8);
      } else if (isB && bok) {
        const int n = m / pq;
        const int rr = m - n * pq;
        const int p = rr / a.Q, q = rr - (rr / a.Q) * a.Q;
        int yy = p * a.stride - a.pad + br, xx = q * a.stride - a.pad + bs;
        if (a.pad_mode == UM_PAD_REFLECT) {
          yy = reflect_idx(yy, a.H);
          xx = reflect_idx(xx, a.W);
        } else if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W) {
          continue;
        }
        blk[r] = *reinterpret_cast<const uint4*>(X + ((long)(n * a.H + yy) * a.W + xx) * a.ldx + bch);
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fk = (lane >> 4) * 8;
  if (m_begin < m_end) load(m_begin);
  for (int m0 = m_begin; m0 < m_end; m0 += WBK) {
    uint4 tr[8];
    transpose8x8_bf16(blk, tr);
    __syncthreads();
    if (isA || isB) {
      bf16_t* dst = isA ? sA : sB;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<uint4*>(dst + (cb * 8 + e) * WLDK + mb * 8) = tr[e];
    }
    __syncthreads();
    if (m0 + WBK < m_end) load(m0 + WBK);
#pragma unroll
    for (int kk = 0; kk < WBK; kk += 32) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8_t*>(
            &sA[(wm * (BM / WM) + i * 16 + frow) * WLDK + kk + fk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8_t*>(
            &sB[(wn * (BN / WN) + j * 16 + frow) * WLDK + kk + fk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  float* out = a.slabs + (long)blockIdx.z * a.K * a.RRC;
  const int col_l = lane & 15, row_g = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = bk + wm * (BM / WM) + i * 16 + row_g + r;
        const int jj = bj + wn * (BN / WN) + j * 16 + col_l;
        if (k < a.K && jj < a.RRC) out[(long)k * a.RRC + jj] = acc[i][j][r];
      }
}

// ---- 1x1 weight gradient of narrow layers (K, C in {8, 16, 32, 64}, K*C <=
// W1_MAX), a VALU streaming pass: lane (kb, cb) of the L = K/8 * C/8 lanes
// that share a pixel owns the 8x8 block dW[kb*8 .. +7][cb*8 .. +7]; a wave
// covers 64/L pixels per step and reads each pixel's dy and x rows once, as
// 16-byte loads (HBM-bound; the MFMA tiles above are 128 columns wide, 1/16
// full at C = 8).  One f32 partial [K][C] per workgroup into the slabs.
// MI355X (tools/conv_micro.py, wgrad + slab reduce): 256x512 C8 K32 120 ->
// 27 us; past K*C = 512 the FMAs per pixel make it VALU/latency-bound
// (128x256 C32 K32 41 -> 37, C64 K32 41 -> 63 us), so those keep the MFMA tiles.
constexpr int W1_NT = 256, W1_MAX = 512;

__device__ __forceinline__ void bf16x8_to_f32(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

template <int L>
__global__ void __launch_bounds__(W1_NT) wgrad_1x1_kernel(WgradArgs a) {
  constexpr int PW = 64 / L, U = 4;
  __shared__ float red[W1_MAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane / L, sub = lane - (lane / L) * L;
  const int ncb = a.C / 8;
  const int kb = sub / ncb, cb = sub - (sub / ncb) * ncb;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(a.x) + cb * 8;
  const bf16_t* __restrict__ DY = reinterpret_cast<const bf16_t*>(a.dy) + kb * 8;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const long step = (long)gridDim.x * (W1_NT / 64) * PW;
  long p = ((long)blockIdx.x * (W1_NT / 64) + wave) * PW + slot;
  for (; p < a.M; p += U * step) {
    uint4 dv[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long q = p + u * step;
      const bool ok = q < a.M;
      dv[u] = ok ? *reinterpret_cast<const uint4*>(DY + q * a.ldy) : make_uint4(0, 0, 0, 0);
      xv[u] = ok ? *reinterpret_cast<const uint4*>(X + q * a.ldx) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d[8], x[8];
      bf16x8_to_f32(dv[u], d);
      bf16x8_to_f32(xv[u], x);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(d[i], x[j], acc[i][j]);
    }
  }
  // sum the wave's pixel slots (lanes sub, sub + L, ...), then the 4 waves in turn
#pragma unroll
  for (int o = L; o < 64; o <<= 1)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] += __shfl_xor(acc[i][j], o, 64);
  const int KC = a.K * a.C;
  for (int w = 0; w < W1_NT / 64; ++w) {
    if (wave == w && slot == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float* r = &red[(kb * 8 + i) * a.C + cb * 8 + j];
          *r = (w == 0 ? 0.f : *r) + acc[i][j];
        }
    }
    __syncthreads();
  }
  float* out = a.slabs + (long)blockIdx.x * KC;
  for (int i = threadIdx.x; i < KC; i += W1_NT) out[i] = red[i];
}

static bool wgrad_1x1_ok(int dtype, int C, int K, int R, int stride, int pad, int ldx, int ldy) {
  auto p2 = [](int v) { return v == 8 || v == 16 || v == 32 || v == 64; };
  static const bool on = umamd::tuning_env("w1x1", 1) != 0;  // read once (common.h)
  return dtype == UM_BF16 && on && R == 1 && stride == 1 && pad == 0 &&
         p2(C) && p2(K) && K * C <= W1_MAX && ldx % 8 == 0 && ldy % 8 == 0;
}

// workgroups (= slabs) of the 1x1 pass: ~4 pixel steps per wave at least
static int wgrad_1x1_blocks(long M) {
  return (int)std::max<long>(1, std::min<long>(512, (M + 2047) / 2048));
}

template <int BM>
int launch_wgrad_bf16(const WgradArgs& a, int splits, hipStream_t st) {
  dim3 grid(ceil_div(a.K, BM), ceil_div(a.RRC, 128), splits);
  hipLaunchKernelGGL(wgrad_bf16_kernel<BM>, grid, dim3(256), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// slab index i = (k, r, s, c) [K][R][R][C] -> dw[k][c][r][s].  Block = EB
// elements x L split lanes (L * EB = 256); a thread sums splits lane,
// lane + L, ... (4 accumulators), the L partial sums meet in LDS.  Reads are
// coalesced along the elements.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slabs,
                                                           int splits, int K, int Kreal, int R,
                                                           int C, int Creal, float* __restrict__ dw,
                                                           int accumulate, Segs sg, int L) {
  __shared__ float red[256];
  const int EB = 256 / L;
  const int le = threadIdx.x % EB, lane = threadIdx.x / EB;
  const long RRC = (long)R * R * C;
  const long total = (long)Kreal * RRC;
  const long zs = (long)K * RRC;
  for (long i0 = (long)blockIdx.x * EB; i0 < total; i0 += (long)gridDim.x * EB) {
    const long i = i0 + le;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (i < total) {
      int z = lane;
      for (; z + 3 * L < splits; z += 4 * L) {
        v0 += slabs[z * zs + i];
        v1 += slabs[(z + L) * zs + i];
        v2 += slabs[(z + 2 * L) * zs + i];
        v3 += slabs[(z + 3 * L) * zs + i];
      }
      for (; z < splits; z += L) v0 += slabs[z * zs + i];
    }
    float v = (v0 + v1) + (v2 + v3);
    if (L > 1) {
      red[threadIdx.x] = v;
      __syncthreads();
      if (lane == 0)
        for (int q = 1; q < L; ++q) v += red[q * EB + le];
      __syncthreads();
    }
    if (lane == 0 && i < total) {
      const int c = seg_src(sg, (int)(i % C));
      if (c >= 0) {
        const int rs = (i / C) % (R * R);
        const int k = i / RRC;
        const long o = ((long)k * Creal + c) * R * R + rs;
        dw[o] = accumulate ? dw[o] + v : v;
      }
    }
  }
}

// The same reduction when R*R*C % 4 == 0 (every slab row starts 16-byte
// aligned): a thread owns 4 consecutive elements, reads float4 and keeps
// four of them in flight per round, so a wave moves 1 KB per load instead of
// 256 B and the reduction runs at streaming rate instead of load latency.
// All offsets fit 32 bits (checked by the caller).
__device__ __forceinline__ void wgrad_reduce4_body(const float* __restrict__ slabs, int splits,
                                                   int K, int Kreal, int R, int C, int Creal,
                                                   float* __restrict__ dw, int accumulate,
                                                   const Segs& sg, int L, int blk, int nblk,
                                                   float4* red) {
  const int EB = 256 / L;
  const int le = threadIdx.x % EB, lane = threadIdx.x / EB;
  const int RR = R * R, RRC = RR * C;
  const int total4 = Kreal * RRC / 4;
  const int zs4 = K * RRC / 4;
  const int step = L * zs4;
  const float4* __restrict__ s4 = reinterpret_cast<const float4*>(slabs);
  for (int i0 = blk * EB; i0 < total4; i0 += nblk * EB) {
    const int i = i0 + le;
    float4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0, v2 = v0, v3 = v0;
    if (i < total4) {
      const float4* p = s4 + lane * zs4 + i;
      int z = lane;
      for (; z + 3 * L < splits; z += 4 * L, p += 4l * step) {
        const float4 a0 = p[0], a1 = p[step], a2 = p[2 * step], a3 = p[3 * step];
        v0 += a0;
        v1 += a1;
        v2 += a2;
        v3 += a3;
      }
      for (; z < splits; z += L, p += step) v0 += p[0];
    }
    float4 v = (v0 + v1) + (v2 + v3);
    if (L > 1) {
      red[threadIdx.x] = v;
      __syncthreads();
      if (lane == 0)
        for (int q = 1; q < L; ++q) v += red[q * EB + le];
      __syncthreads();
    }
    if (lane == 0 && i < total4) {
      const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * i + e;
        const int k = j / RRC, rem = j - k * RRC;
        const int rs = rem / C, cp = rem - rs * C;
        const int c = seg_src(sg, cp);
        if (c >= 0) {
          const int o = (k * Creal + c) * RR + rs;
          dw[o] = accumulate ? dw[o] + vs[e] : vs[e];
        }
      }
    }
  }
}

// Slab reduce of the large 3x3..7x7 weights (>= 256K elements): block (64-
// channel chunk, output row k) sums the splits of slab rows [k][rs][c0, c0+64)
// for every tap into an LDS tile, then writes dW[k][c][rs] of its chunk as
// one contiguous run.  The float4 reduce's 4-byte stores at stride R*R leave
// partially written lines all over the 2-13 MB weight in every XCD's L2
// (15-19 us per 3x3/512 layer for ~37 MB of slab traffic).
constexpr int WRT_CW = 64;
__global__ void __launch_bounds__(256) wgrad_reduce_t_kernel(const float* __restrict__ slabs,
                                                             int splits, int K, int R, int C,
                                                             int Creal, float* __restrict__ dw,
                                                             int accumulate, Segs sg) {
  extern __shared__ float tile[];  // [R*R][WRT_CW + 1]
  const int k = blockIdx.y, c0 = blockIdx.x * WRT_CW;
  const int RR = R * R, RRC = RR * C;
  const int cw = min(WRT_CW, C - c0);
  const long zs = (long)K * RRC;
  const float* __restrict__ base = slabs + (long)k * RRC + c0;
  const int n = RR * WRT_CW;
  for (int e = threadIdx.x; e < n; e += 256) {
    const int rs = e / WRT_CW, cl = e - rs * WRT_CW;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (cl < cw) {
      const float* p = base + rs * C + cl;
      int z = 0;
      for (; z + 3 < splits; z += 4, p += 4 * zs) {
        v0 += p[0];
        v1 += p[zs];
        v2 += p[2 * zs];
        v3 += p[3 * zs];
      }
      for (; z < splits; ++z, p += zs) v0 += p[0];
    }
    tile[rs * (WRT_CW + 1) + cl] = (v0 + v1) + (v2 + v3);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < n; q += 256) {
    const int cl = q / RR, rs = q - cl * RR;
    if (cl >= cw) continue;
    const int c = seg_src(sg, c0 + cl);
    if (c < 0) continue;
    const long o = ((long)k * Creal + c) * RR + rs;
    const float v = tile[rs * (WRT_CW + 1) + cl];
    dw[o] = accumulate ? dw[o] + v : v;
  }
}

__global__ void __launch_bounds__(256) wgrad_reduce4_kernel(const float* __restrict__ slabs,
                                                            int splits, int K, int Kreal, int R,
                                                            int C, int Creal,
                                                            float* __restrict__ dw,
                                                            int accumulate, Segs sg, int L) {
  __shared__ float4 red[256];
  wgrad_reduce4_body(slabs, splits, K, Kreal, R, C, Creal, dw, accumulate, sg, L, blockIdx.x,
                     gridDim.x, red);
}

// split-bf16 value of a packed row: rows [0, K) the weight rounded to the
// activation type, rows [K, 2K) (split packs only) its rounding residual, so
// that a GEMM over both row sets summed in f32 sees the f32 weight to ~2^-17
template <typename T>
__device__ __forceinline__ float split_part(float v, bool lo) {
  return lo ? v - to_f32(from_f32<T>(v)) : v;
}

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int K, int Creal, int R, int C,
                                   T* __restrict__ wf, T* __restrict__ wT, int ldT, Segs sg,
                                   int split) {
  const int K2 = split ? 2 * K : K;
  const long total = (long)K2 * R * R * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    // i indexes wf [K2][R][R][C]
    const int c = i % C;
    const int s = (i / C) % R;
    const int r = (i / ((long)C * R)) % R;
    const int k2 = i / ((long)C * R * R);
    const int k = k2 < K ? k2 : k2 - K;
    const int cs = seg_src(sg, c);
    const float v = split_part<T>(cs >= 0 ? w[(((long)k * Creal + cs) * R + r) * R + s] : 0.f,
                                  k2 >= K);
    if (wf) wf[i] = from_f32<T>(v);
    if (wT) wT[((long)c * R * R + r * R + s) * ldT + k2] = from_f32<T>(v);
  }
}

// per-block column sums of y[M][C] (C % 8 == 0) -> parts[blk][C]
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ y, int M, int C,
                                                     int ld, float* __restrict__ parts,
                                                     int rows_per_block) {
  __shared__ float red[256 * 8];
  const int cg = C / 8;
  const RowMap rm(cg);
  const long m0 = (long)blockIdx.x * rows_per_block;
  const long m1 = min((long)M, m0 + rows_per_block);
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && g < cg)
#pragma unroll 4
      for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
        float v[8];
        load8(y + m * ld + g * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    lane_reduce<8>(red, rm, acc);
    if (rm.lane == 0 && g < cg) store8(parts + (long)blockIdx.x * C + g * 8, acc);
  }
}

// Several bias gradients (column sums) in two launches: the weight-gradient
// side stream's flush batches them (umamd.functional._colsum_grad).  Phase 1:
// descriptor d owns workgroups [first[d], first[d+1]), each one row chunk of
// y -> its partial row parts[blk][C] (as colsum_kernel); phase 2: one
// workgroup per (descriptor, 64 columns) sums the partial rows in f64.
struct CsDesc {
  const void* y;
  float* parts;
  float* out;
  int M, C, ld, nparts, rows, creal;
};
struct CsBatch {
  int n, dtype;
  int first[UM_CSUM_MAX + 1];
  CsDesc d[UM_CSUM_MAX];
};

#define CSEL(expr)                                          \
  ({                                                        \
    auto v_ = b.d[0].expr;                                  \
    _Pragma("unroll") for (int j = 1; j < UM_CSUM_MAX; ++j) \
      if (j == i) v_ = b.d[j].expr;                         \
    v_;                                                     \
  })

template <typename T>
__global__ void __launch_bounds__(256) colsum_batch_kernel(CsBatch b) {
  __shared__ float red[256 * 8];
  int i = 0;
#pragma unroll
  for (int j = 1; j < UM_CSUM_MAX; ++j)
    if (j < b.n && (int)blockIdx.x >= b.first[j]) i = j;
  int f0 = 0;
#pragma unroll
  for (int j = 0; j < UM_CSUM_MAX; ++j)
    if (j == i) f0 = b.first[j];
  const T* __restrict__ y = reinterpret_cast<const T*>(CSEL(y));
  float* __restrict__ parts = CSEL(parts);
  const int M = CSEL(M), C = CSEL(C), ld = CSEL(ld), rows = CSEL(rows);
  const int blk = blockIdx.x - f0;
  const int cg = C / 8;
  const RowMap rm(cg);
  const long m0 = (long)blk * rows;
  const long m1 = min((long)M, m0 + rows);
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && g < cg)
#pragma unroll 4
      for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
        float v[8];
        load8(y + m * ld + g * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    lane_reduce<8>(red, rm, acc);
    if (rm.lane == 0 && g < cg) store8(parts + (long)blk * C + g * 8, acc);
  }
}

// grid (descriptors, column chunks of 32): 32 columns x 8 row lanes, each
// lane with 4 independent f64 accumulators (the partial rows are up to ~2k
// deep: one dependent load chain per lane was 42 us per launch)
__global__ void __launch_bounds__(256) colsum_fin_batch_kernel(CsBatch b) {
  const int i = blockIdx.x;
  if (i >= b.n) return;
  const float* __restrict__ parts = CSEL(parts);
  float* __restrict__ out = CSEL(out);
  const int C = CSEL(C), np = CSEL(nparts), creal = CSEL(creal);
  __shared__ double red[8][32];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.y * 32 + cl;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < C) {
    int r = rl;
    for (; r + 24 < np; r += 32) {
      s0 += parts[(long)r * C + c];
      s1 += parts[(long)(r + 8) * C + c];
      s2 += parts[(long)(r + 16) * C + c];
      s3 += parts[(long)(r + 24) * C + c];
    }
    for (; r < np; r += 8) s0 += parts[(long)r * C + c];
  }
  red[rl][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rl == 0 && c < creal) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    out[c] = (float)t;
  }
}
#undef CSEL

// out[c] (+)= sum_r p[r*stride + c]: block = cl channel lanes (cl = C up to
// 64, power of two) x 256/cl row lanes, 8 independent accumulators per
// thread, f64 lane combine
// Reflect-pad data gradient, padded form: dxp[n][Y][X] (the gradient of the
// reflect-padded input, (H+2p) x (W+2p), from a zero-pad transposed conv
// on the fast GEMM paths) folded onto dx: x_pad[Y] = x[refl(Y - p)], so
// The reflect fold of a split-form data gradient as a VALU pass over the
// border list (umamd::border_pixel): border pixel (n, i, j) of dx adds, for
// every tap (r, s), the dy sources that reach it only through the reflect
// pad -- rows -i - p' + r (1 <= i <= pad) and 2(H-1) - i - p' + r
// (H-1-pad <= i <= H-2), columns likewise, p' = a.pad = R-1-pad, every
// (row, column) pair but the plain one -- times the flipped tap's weights.
// The same sums as the register GEMM's border mode (igemm.hip gather, IG_FOLD
// + border), without its per-k-step gather chain: thread per (border pixel,
// 8 dx channels), all of a pair's dy chunks and weight rows loaded before
// they are summed.
template <typename T>
__global__ void __launch_bounds__(256) reflect_border_kernel(umamd::IgArgs a) {
  const int cg = a.NC / 8;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)a.M * cg) return;
  const int m = (int)(gid / cg), c0 = (int)(gid - (long)m * cg) * 8;
  int n, oy, ox;
  umamd::border_pixel(a, m, n, oy, ox);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.a) + (long)n * a.ah * a.aw * a.lda;
  const T* __restrict__ wT = reinterpret_cast<const T*>(a.b);
  const int H = a.oh, W = a.ow, fp = a.fold_pad, R = a.R, K = a.ach;
  const bool lo_y = oy >= 1 && oy <= fp, hi_y = oy >= H - 1 - fp && oy <= H - 2;
  const bool lo_x = ox >= 1 && ox <= fp, hi_x = ox >= W - 1 - fp && ox <= W - 2;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < R; ++r) {
    const int yy = oy - a.pad + r;
    int ys[3], ny = 0;
    const bool iny = yy >= 0 && yy < a.ah;
    if (iny) ys[ny++] = yy;
    if (lo_y) { const int t = -oy - a.pad + r; if (t >= 0 && t < a.ah) ys[ny++] = t; }
    if (hi_y) { const int t = 2 * (H - 1) - oy - a.pad + r; if (t >= 0 && t < a.ah) ys[ny++] = t; }
    for (int s = 0; s < R; ++s) {
      const int xx = ox - a.pad + s;
      int xs[3], nx = 0;
      const bool inx = xx >= 0 && xx < a.aw;
      if (inx) xs[nx++] = xx;
      if (lo_x) { const int t = -ox - a.pad + s; if (t >= 0 && t < a.aw) xs[nx++] = t; }
      if (hi_x) { const int t = 2 * (W - 1) - ox - a.pad + s; if (t >= 0 && t < a.aw) xs[nx++] = t; }
      const int btap = (R - 1 - r) * R + (R - 1 - s);
      for (int u = 0; u < ny; ++u)
        for (int q = 0; q < nx; ++q) {
          if (u == 0 && q == 0 && iny && inx) continue;  // the zero-pad pass summed it
          const T* src = dy + ((long)ys[u] * a.aw + xs[q]) * a.lda;
          for (int k0 = 0; k0 < K; k0 += 8) {
            float dv[8], wv[8][8];
            load8(src + k0, dv);
#pragma unroll
            for (int e = 0; e < 8; ++e) load8(wT + (long)(c0 + e) * a.ldb + (long)btap * K + k0, wv[e]);
#pragma unroll
            for (int e = 0; e < 8; ++e)
#pragma unroll
              for (int kk = 0; kk < 8; ++kk) acc[e] += dv[kk] * wv[e][kk];
          }
        }
    }
  }
  T* o = reinterpret_cast<T*>(a.out) + (((long)n * H + oy) * W + ox) * a.ld_out + c0;
  float t[8];
  load8(o, t);  // the zero-pad pass wrote these pixels: always accumulate
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] += acc[e];
  store8(o, t);
}

// dx[i] sums dxp[i + p], dxp[p - i] (1 <= i <= p) and dxp[2(H-1) + p - i]
// (H-1-p <= i <= H-2), separably in y and x.  Thread per (pixel, 8 channels).
template <typename T>
__global__ void __launch_bounds__(256) reflect_fold_kernel(const T* __restrict__ dxp, int N, int H,
                                                           int W, int C, int p, T* __restrict__ dx,
                                                           int ldx, int accumulate) {
  const int cg = C / 8;
  const int y = blockIdx.y, n = blockIdx.z;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * cg) return;
  const int x = i / cg, c = (i - x * cg) * 8;
  const int Hp = H + 2 * p, Wp = W + 2 * p;
  int ys[3], xs[3], ny = 0, nx = 0;
  ys[ny++] = y + p;
  if (y >= 1 && y <= p) ys[ny++] = p - y;
  if (y >= H - 1 - p && y <= H - 2) ys[ny++] = 2 * (H - 1) + p - y;
  xs[nx++] = x + p;
  if (x >= 1 && x <= p) xs[nx++] = p - x;
  if (x >= W - 1 - p && x <= W - 2) xs[nx++] = 2 * (W - 1) + p - x;
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const T* base = dxp + (long)n * Hp * Wp * C + c;
  for (int u = 0; u < ny; ++u)
    for (int q = 0; q < nx; ++q) {
      float t[8];
      load8(base + ((long)ys[u] * Wp + xs[q]) * C, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
  T* o = dx + (((long)n * H + y) * W + x) * ldx + c;
  if (accumulate) {
    float t[8];
    load8(o, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  store8(o, v);
}

// the padded form applies (knob pad_dgrad: 0 off, 1 for dx wider than
// fold_split_nc -- the layers the one-pass fold gather served --, 2 all)
// -- except where the split form's zero-pad pass runs on the halo kernel (its
// 64..192-wide column blocks: 128x256 C88 and 64x128 C168 decoder layers)
bool split_form(int dtype, int N, int H, int W, int C, int R) {
  return C <= umamd::igemm_fold_split_nc() || umamd::igemm_halo_dgrad(dtype, N, H, W, C, R);
}

bool pad_dgrad_applies(int dtype, int N, int C, int R, int pad, int pad_mode, int stride, int P,
                       int Q, int H, int W) {
  const int kn = umamd::igemm_pad_dgrad();
  if (kn == 0 || pad_mode != UM_PAD_REFLECT || stride != 1 || pad <= 0 || pad >= H || pad >= W) return false;
  if (P != H || Q != W || C % 8) return false;
  return kn == 2 || !split_form(dtype, N, H, W, C, R);
}

long pad_dgrad_bytes(int dtype, int N, int H, int W, int C, int R, int K, int pad, long* gemm_off) {
  const long Hp = H + 2 * pad, Wp = W + 2 * pad;
  const long esz = dtype == UM_BF16 ? 2 : 4;
  const long buf = (N * Hp * Wp * C * esz + 255) / 256 * 256;
  if (gemm_off) *gemm_off = buf;
  return buf + umamd::igemm_ws_bytes(dtype, (int)(N * Hp * Wp), C, R * R, K);
}

}  // namespace

extern "C" {

long um_conv_dgrad_ws_pad(int dtype, int N, int H, int W, int C, int R, int K, int stride, int pad,
                          int pad_mode) {
  const long base = um_conv_dgrad_ws(dtype, N, H, W, C, R, K, stride);
  if (pad_dgrad_applies(dtype, N, C, R, pad, pad_mode, stride, H, W, H, W))
    return std::max(base, pad_dgrad_bytes(dtype, N, H, W, C, R, K, pad, nullptr));
  // split form of a reflect data gradient: the border-list GEMM of the fold
  // splits its k-loop too (a few thousand rows x 9 taps: unsplit, 96-256
  // workgroups ran 24-53 us behind a 30-87 us main pass), unless the fold is
  // the VALU pass (um_conv2d_dgrad)
  static const int border_split = (int)umamd::tuning_env("border_split", 1);
  if (border_split && pad_mode == UM_PAD_REFLECT && pad > 0 && stride == 1 &&
      split_form(dtype, N, H, W, C, R)) {
    const int bv = umamd::igemm_border_valu();
    if (!((bv == 2 || (bv == 1 && K <= 8)) && C % 8 == 0 && K % 8 == 0)) {
      umamd::IgArgs a{};
      a.oh = H; a.ow = W; a.fold_pad = pad;
      const long mb = (long)N * umamd::igemm_border_list(a);
      // after the main pass's own workspace (its plan stays as sized by base)
      return base + umamd::igemm_border_ws_bytes(dtype, (int)mb, C, R * R, K);
    }
  }
  return base;
}

int um_conv_stats_parts(int M, int K) {
  return ceil_div(M, umamd::igemm_stats_rows(M, K));
}

long um_conv_fwd_ws(int dtype, int N, int P, int Q, int K, int R, int C) {
  return umamd::igemm_ws_bytes(dtype, N * P * Q, K, R * R, C);
}

long um_conv_dgrad_ws(int dtype, int N, int H, int W, int C, int R, int K, int stride) {
  if (stride == 1) return umamd::igemm_ws_bytes(dtype, N * H * W, C, R * R, K);
  long b = 0;  // the largest parity class (the launches reuse one workspace)
  const int taps = ((R + 1) / 2) * ((R + 1) / 2);
  b = std::max(b, umamd::igemm_ws_bytes(dtype, N * ((H + 1) / 2) * ((W + 1) / 2), C, taps, K));
  // ... or the four classes in one launch, each with its own slice (both pad
  // parities: the tap counts per class swap with it)
  for (int pad = 0; pad < 2; ++pad) {
    int M[4], tp[4];
    for (int ay = 0; ay < 2; ++ay)
      for (int ax = 0; ax < 2; ++ax) {
        const int r0y = (ay + pad) & 1, r0x = (ax + pad) & 1;
        M[2 * ay + ax] = N * ((H - ay + 1) / 2) * ((W - ax + 1) / 2);
        tp[2 * ay + ax] = ((R - r0y + 1) / 2) * ((R - r0x + 1) / 2);
      }
    b = std::max(b, umamd::igemm_cls4_ws_bytes(dtype, M, tp, C, K));
  }
  return b;
}

static int conv2d_fwd(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                      const void* wf, const float* bias, int K, int R, int stride, int pad,
                      int pad_mode, int P, int Q, int ydtype, void* y, int ldy, int epilogue,
                      float epi_scale, const void* residual, int ldr, float* stats, void* ws,
                      long ws_bytes, int accumulate, hipStream_t st);

int um_conv2d_fwd(int dtype, int N, int H, int W, int C, int ldx, const void* x, const void* wf,
                  const float* bias, int K, int R, int stride, int pad, int pad_mode, int P,
                  int Q, int ydtype, void* y, int ldy, int epilogue, float epi_scale,
                  const void* residual, int ldr, float* stats, void* ws, long ws_bytes,
                  hipStream_t st) {
  return conv2d_fwd(dtype, N, H, W, C, ldx, x, wf, bias, K, R, stride, pad, pad_mode, P, Q, ydtype,
                    y, ldy, epilogue, epi_scale, residual, ldr, stats, ws, ws_bytes, 0, st);
}

}  // extern "C"

namespace {
// The decoder skip conv's feature-map half when the feature map is narrow
// (C <= 16: the image at 256x512): y = W x + bias + up2(z)
// and the BN statistics slots of y in ONE VALU pass.  The GEMM route (an
// upsample pass into y, then an accumulating 1x1 GEMM with 256-row tiles on
// an 8..32-deep reduction) moves y three times and runs the MFMA tiles on a
// reduction they cannot fill; here x and z are read once and y written once.
// Thread = (pixel, 8 output channels): the K/8 groups of a pixel are
// consecutive lanes (one contiguous run per pixel); W in LDS as f32 (the
// lanes of a wave read G distinct rows: broadcast reads).
template <typename T, typename TY, int C>
__global__ void __launch_bounds__(256) conv1x1_up2_kernel(
    const T* __restrict__ x, int ldx, const T* __restrict__ wf, const float* __restrict__ bias,
    int K, int H, int W, long M, TY* __restrict__ y, int ldy, const TY* __restrict__ z, int h,
    int w, int ldz, double* __restrict__ slots) {
  extern __shared__ float sm[];  // W [K][C] f32, the statistics [4 waves][K][2], zr [w][K]
  float* sW = sm;
  float* sS = sm + K * C;
  float* zr = sS + 8 * K;  // this row's vertical interpolation of z (f32)
  for (int i = threadIdx.x; i < K * C; i += 256) sW[i] = to_f32(wf[i]);
  __syncthreads();
  const int G = K / 8;  // 256 % G == 0 (host): a thread keeps its group
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = threadIdx.x % G, k0 = g * 8;
  float b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = bias ? bias[k0 + e] : 0.f;
  const float scy = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  const float scx = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  float ps[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // one output row (n, oy) per block iteration: 32-bit index math only, the
  // vertical taps and weights once per row
  const int rows = (int)(M / W), items = W * G, gs = __ffs(G) - 1;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int n = row / H, oy = row - n * H;
    const float fy = scy * (float)oy;
    const int y0 = min((int)fy, h - 1);
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0);
    const float ly = fy - (float)y0;
    // the two z rows of this output row, interpolated vertically ONCE into
    // LDS (each z value was re-read by ~4 output pixels through the L1)
    {
      const TY* __restrict__ z0 = z + ((long)n * h + y0) * w * ldz;
      const TY* __restrict__ z1 = z + ((long)n * h + y1) * w * ldz;
      __syncthreads();  // the previous row's readers are done
      for (int i = threadIdx.x; i < w * G; i += 256) {
        const int x = i >> gs, kk = (i & (G - 1)) * 8;
        float a[8], c[8];
        load8(z0 + (long)x * ldz + kk, a);
        load8(z1 + (long)x * ldz + kk, c);
        float4* d = reinterpret_cast<float4*>(zr + x * K + kk);
        d[0] = make_float4((1.f - ly) * a[0] + ly * c[0], (1.f - ly) * a[1] + ly * c[1],
                           (1.f - ly) * a[2] + ly * c[2], (1.f - ly) * a[3] + ly * c[3]);
        d[1] = make_float4((1.f - ly) * a[4] + ly * c[4], (1.f - ly) * a[5] + ly * c[5],
                           (1.f - ly) * a[6] + ly * c[6], (1.f - ly) * a[7] + ly * c[7]);
      }
      __syncthreads();
    }
    const long mrow = (long)row * W;
    for (int i = threadIdx.x; i < items; i += 256) {
      const int ox = i >> gs;  // G is a power of two
      // re-read W from LDS per pixel (broadcast reads) instead of keeping 8*C
      // weights live in VGPRs (170-250 VGPRs, 2 waves per SIMD)
      asm volatile("" ::: "memory");
      const long m = mrow + ox;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = b[e];
#pragma unroll
      for (int c = 0; c < C; c += 8) {
        float xv[8];
        load8(x + m * ldx + c, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float4 w0 = *reinterpret_cast<const float4*>(&sW[(k0 + e) * C + c]);
          const float4 w1 = *reinterpret_cast<const float4*>(&sW[(k0 + e) * C + c + 4]);
          v[e] += w0.x * xv[0] + w0.y * xv[1] + w0.z * xv[2] + w0.w * xv[3] + w1.x * xv[4] +
                  w1.y * xv[5] + w1.z * xv[6] + w1.w * xv[7];
        }
      }
      // torch upsample_bilinear2d(align_corners=True), as the concat kernel
      const float fx = scx * (float)ox;
      const int x0 = min((int)fx, w - 1);
      const int x1 = x0 + (x0 < w - 1 ? 1 : 0);
      const float lx = fx - (float)x0;
      const float4* r0 = reinterpret_cast<const float4*>(zr + x0 * K + k0);
      const float4* r1 = reinterpret_cast<const float4*>(zr + x1 * K + k0);
      const float4 p0 = r0[0], p1 = r0[1], q0 = r1[0], q1 = r1[1];
      const float a0[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
      const float a1[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += (1.f - lx) * a0[e] + lx * a1[e];
      store8(y + m * ldy + k0, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ps[e] += v[e];
        pq[e] += v[e] * v[e];
      }
    }
  }
  if (slots == nullptr) return;
  // lanes of a wave with the same group: lane % G
  for (int sh = G; sh < 64; sh <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ps[e] += __shfl_xor(ps[e], sh, 64);
      pq[e] += __shfl_xor(pq[e], sh, 64);
    }
  if (lane < G)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sS[(wave * K + k0 + e) * 2] = ps[e];
      sS[(wave * K + k0 + e) * 2 + 1] = pq[e];
    }
  __syncthreads();
  stat_slots_count(slots, K, M);
  stat_slots_add_row(slots, blockIdx.x, K, 0, K, [&](int i) {
    return sS[i] + sS[2 * K + i] + sS[4 * K + i] + sS[6 * K + i];
  });
}

template <typename T, typename TY>
int launch_conv1x1_up2(int C, const void* x, int ldx, const void* wf, const float* bias, int K,
                       int N, int H, int W, void* y, int ldy, const void* z, int h, int w, int ldz,
                       double* slots, hipStream_t st) {
  const long M = (long)N * H * W;
  const int grid = std::min(N * H, 4096);
  const size_t shm = ((size_t)K * C + 8 * (size_t)K + (size_t)w * K) * sizeof(float);
  UM_CHECK_ARG(shm <= 160 * 1024, "um_conv2d_fwd_up2: low-resolution row too wide (%d x %d)", w, K);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_up2_kernel<T, TY, 8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_up2_kernel<T, TY, 16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
#define UM_C1UP(CC)                                                                            \
  hipLaunchKernelGGL((conv1x1_up2_kernel<T, TY, CC>), dim3(grid), dim3(256), shm, st,           \
                     (const T*)x, ldx, (const T*)wf, bias, K, H, W, M, (TY*)y, ldy, (const TY*)z, \
                     h, w, ldz, slots)
  if (C == 8) UM_C1UP(8); else UM_C1UP(16);
#undef UM_C1UP
  UM_LAUNCH_CHECK();
  return UM_OK;
}
}  // namespace

extern "C" {

int um_conv2d_fwd_up2(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                      const void* wf, const float* bias, int K, int P, int Q, void* y, int ldy,
                      int epilogue, float* stats, const void* up2, int up2_h, int up2_w,
                      int up2_ld, hipStream_t st) {
  // UM_Y_ACT: y and up2 in the activation dtype, else f32
  const int ydt = (dtype & UM_Y_ACT) ? (dtype & ~UM_Y_ACT) : UM_F32;
  dtype &= ~UM_Y_ACT;
  UM_CHECK_ARG(up2 != nullptr && up2_h >= 1 && up2_w >= 1 && up2_ld >= K,
               "um_conv2d_fwd_up2: low-resolution map");
  UM_CHECK_ARG(epilogue == UM_EPI_NONE || epilogue == UM_EPI_STATS ||
                   epilogue == UM_EPI_STAT_SLOTS,
               "um_conv2d_fwd_up2: epilogue");
  UM_CHECK_ARG(K % 8 == 0 && ldy % 8 == 0 && up2_ld % 8 == 0 && P == H && Q == W,
               "um_conv2d_fwd_up2: K / strides must be multiples of 8, 1x1 same-size conv");
  static const int valu = (int)umamd::tuning_env("up2_valu", 1);
  const int G = K / 8;
  if (valu && C % 8 == 0 && C <= 16 && K <= 128 && 256 % G == 0 && ldx % 8 == 0 &&
      (epilogue == UM_EPI_NONE || epilogue == UM_EPI_STAT_SLOTS)) {
    double* sl = epilogue == UM_EPI_STAT_SLOTS ? reinterpret_cast<double*>(stats) : nullptr;
    if (dtype == UM_BF16 && ydt == UM_BF16)
      return launch_conv1x1_up2<bf16_t, bf16_t>(C, x, ldx, wf, bias, K, N, H, W, y, ldy, up2,
                                                up2_h, up2_w, up2_ld, sl, st);
    if (dtype == UM_BF16)
      return launch_conv1x1_up2<bf16_t, float>(C, x, ldx, wf, bias, K, N, H, W, y, ldy, up2,
                                               up2_h, up2_w, up2_ld, sl, st);
    return launch_conv1x1_up2<float, float>(C, x, ldx, wf, bias, K, N, H, W, y, ldy, up2, up2_h,
                                            up2_w, up2_ld, sl, st);
  }
  // y = up2(z) by one vectorised upsample pass (the concat kernel with one
  // UP2 source), then the GEMM ADDS W x + bias into y, with the BN
  // statistics taken on the sum in its epilogue (an in-epilogue gather of the
  // 4 taps per element measured 142 us for the 256x512 stage vs ~60 here)
  um_cat_src src{};
  src.ptr = up2; src.scale = nullptr; src.C = K; src.ld = up2_ld; src.op = UM_CAT_UP2;
  src.coff = 0; src.dtype = ydt; src.h = up2_h; src.w = up2_w;
  const int rc = um_concat_build(ydt, N, H, W, y, ldy, K, 1, &src, st);
  if (rc != UM_OK) return rc;
  return conv2d_fwd(dtype, N, H, W, C, ldx, x, wf, bias, K, 1, 1, 0, UM_PAD_ZERO, P, Q, ydt, y,
                    ldy, epilogue, 1.f, nullptr, 0, stats, nullptr, 0, 1, st);
}

static int conv2d_fwd(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                      const void* wf, const float* bias, int K, int R, int stride, int pad,
                      int pad_mode, int P, int Q, int ydtype, void* y, int ldy, int epilogue,
                      float epi_scale, const void* residual, int ldr, float* stats, void* ws,
                      long ws_bytes, int accumulate, hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0 && ldx % 8 == 0, "um_conv2d_fwd: C (%d) and ldx (%d) must be multiples of 8", C, ldx);
  UM_CHECK_ARG(stride == 1 || stride == 2, "um_conv2d_fwd: stride %d", stride);
  UM_CHECK_ARG(P == (H + 2 * pad - R) / stride + 1 && Q == (W + 2 * pad - R) / stride + 1,
               "um_conv2d_fwd: output size mismatch");
  UM_CHECK_ARG(pad_mode == UM_PAD_ZERO || pad < H, "um_conv2d_fwd: reflect pad too large");
  UM_CHECK_ARG((epilogue != UM_EPI_STATS && epilogue != UM_EPI_STAT_SLOTS) || stats != nullptr,
               "um_conv2d_fwd: stats buffer missing");
  UM_CHECK_ARG(epilogue != UM_EPI_RESIDUAL || residual != nullptr, "um_conv2d_fwd: residual missing");
  UM_CHECK_ARG(ydtype == dtype || ydtype == UM_F32, "um_conv2d_fwd: ydtype must be dtype or f32");
  umamd::IgArgs a{};
  a.a = x; a.ah = H; a.aw = W; a.ach = C; a.lda = ldx;
  a.on = N; a.oh = P; a.ow = Q;
  a.R = R; a.stride = stride; a.pad = pad;
  a.Rx = R; a.padx = pad; a.tsign = 1; a.wR = R;
  a.pmode = pad_mode == UM_PAD_REFLECT ? umamd::IG_PAD_REFLECT : umamd::IG_PAD_ZERO;
  a.fold_pad = 0; a.flip = 0;
  a.b = wf; a.ldb = (long)R * R * C;
  a.NC = K; a.M = N * P * Q;
  a.bias = bias; a.out = y; a.ld_out = ldy; a.out_f32 = (ydtype == UM_F32);
  a.epilogue = epilogue == UM_EPI_STAT_SLOTS ? UM_EPI_STATS : epilogue;
  a.stat_slots = epilogue == UM_EPI_STAT_SLOTS;
  a.accumulate = accumulate; a.epi_scale = epi_scale;
  a.residual = residual; a.ldr = ldr; a.stats = stats;
  return umamd::igemm_run(dtype, a, (float*)ws, ws_bytes, st);
}

int um_conv2d_dgrad(int dtype, int N, int H, int W, int C, int ldx, void* dx, int accumulate,
                    const void* wT, int K, int R, int stride, int pad, int pad_mode, int P,
                    int Q, const void* dy, int ldy, void* ws, long ws_bytes, hipStream_t st) {
  UM_CHECK_ARG(K % 8 == 0 && ldy % 8 == 0, "um_conv2d_dgrad: K (%d) and ldy (%d) must be multiples of 8", K, ldy);
  UM_CHECK_ARG(stride == 1 || stride == 2, "um_conv2d_dgrad: stride %d", stride);
  UM_CHECK_ARG(pad_mode == UM_PAD_ZERO || stride == 1, "um_conv2d_dgrad: reflect needs stride 1");
  if (stride == 1) {
    UM_CHECK_ARG(P == H + 2 * pad - R + 1 && Q == W + 2 * pad - R + 1, "um_conv2d_dgrad: size");
    UM_CHECK_ARG(pad_mode == UM_PAD_ZERO || (P == H && Q == W && pad <= 1),
                 "um_conv2d_dgrad: reflect transpose needs a same-size conv with pad <= 1");
    long goff = 0;
    if (pad_dgrad_applies(dtype, N, C, R, pad, pad_mode, stride, P, Q, H, W) && ws != nullptr &&
        ws_bytes >= pad_dgrad_bytes(dtype, N, H, W, C, R, K, pad, &goff)) {
      // padded form: zero-pad transposed conv onto the (H+2p) x (W+2p) padded
      // input (halo / LDS-DMA / register GEMM paths), then the reflect fold
      const int Hp = H + 2 * pad, Wp = W + 2 * pad;
      umamd::IgArgs a{};
      a.a = dy; a.ah = P; a.aw = Q; a.ach = K; a.lda = ldy;
      a.on = N; a.oh = Hp; a.ow = Wp;
      a.R = R; a.stride = 1; a.pad = R - 1;
      a.Rx = R; a.padx = R - 1; a.tsign = 1; a.wR = R;
      a.pmode = umamd::IG_PAD_ZERO; a.fold_pad = 0; a.flip = 1;
      a.b = wT; a.ldb = (long)R * R * K;
      a.NC = C; a.M = N * Hp * Wp;
      a.bias = nullptr; a.out = ws; a.ld_out = C; a.out_f32 = (dtype == UM_F32);
      a.epilogue = UM_EPI_NONE; a.accumulate = 0; a.epi_scale = 1.f;
      a.residual = nullptr; a.ldr = 0; a.stats = nullptr;
      int rc = umamd::igemm_run(dtype, a, reinterpret_cast<float*>((char*)ws + goff), ws_bytes - goff, st);
      if (rc != UM_OK) return rc;
      const dim3 g(ceil_div((long)W * (C / 8), 256), H, N);
      if (dtype == UM_BF16)
        hipLaunchKernelGGL(reflect_fold_kernel<bf16_t>, g, dim3(256), 0, st, (const bf16_t*)ws, N, H, W,
                           C, pad, (bf16_t*)dx, ldx, accumulate);
      else
        hipLaunchKernelGGL(reflect_fold_kernel<float>, g, dim3(256), 0, st, (const float*)ws, N, H, W,
                           C, pad, (float*)dx, ldx, accumulate);
      UM_LAUNCH_CHECK();
      return UM_OK;
    }
    umamd::IgArgs a{};
    a.a = dy; a.ah = P; a.aw = Q; a.ach = K; a.lda = ldy;
    a.on = N; a.oh = H; a.ow = W;
    a.R = R; a.stride = 1; a.pad = R - 1 - pad;
    a.Rx = R; a.padx = R - 1 - pad; a.tsign = 1; a.wR = R;
    // reflect pad, split form (narrow dx: the zero-pad pass takes the halo /
    // 256-row tiles, 117 vs 171 us at 256x512 C48) or one fold pass (wide dx:
    // the deep layers' border list is 18-34 % of their pixels)
    const bool fold1 = pad_mode == UM_PAD_REFLECT && pad > 0 && !split_form(dtype, N, H, W, C, R);
    a.pmode = fold1 ? umamd::IG_FOLD : umamd::IG_PAD_ZERO;
    a.fold_pad = fold1 ? pad : 0; a.flip = 1;
    a.b = wT; a.ldb = (long)R * R * K;
    a.NC = C; a.M = N * H * W;
    a.bias = nullptr; a.out = dx; a.ld_out = ldx; a.out_f32 = (dtype == UM_F32);
    a.epilogue = UM_EPI_NONE; a.accumulate = accumulate; a.epi_scale = 1.f;
    a.residual = nullptr; a.ldr = 0; a.stats = nullptr;
    // the (zero-pad) transposed conv over every pixel (all fast paths apply) ...
    // (its workspace: the first `base` bytes; the border GEMM's split
    // partials follow them, um_conv_dgrad_ws_pad)
    const long base = um_conv_dgrad_ws(dtype, N, H, W, C, R, K, stride);
    int rc = umamd::igemm_run(dtype, a, (float*)ws, ws ? std::min(ws_bytes, base) : 0, st);
    if (rc != UM_OK || fold1 || pad_mode != UM_PAD_REFLECT || pad == 0) return rc;
    // ... then the reflect fold: the pixels rows/columns 1..pad and H-1-pad..H-2
    // also receive the gradient of the padded taps that mirrored them.  A
    // small GEMM over that border list sums only those sources into dx.
    a.pmode = umamd::IG_FOLD;
    a.fold_pad = pad;
    a.accumulate = 1;
    a.M = N * umamd::igemm_border_list(a);
    // 8-channel dy (the disparity heads): the border list as a VALU pass,
    // else as a register-path GEMM (igemm.hip).  Micro-benchmark on MI355X
    // (tools/border_micro.sh r04aa): 256x512 C32 K8 80.9 -> 77.2 us, 128x256
    // C64 K8 59.5 -> 55.5; at K = 32 / 64 the GEMM stays ahead (144 vs 163,
    // 59 vs 83 us).  Knob border_valu: 0 never, 1 K <= 8, 2 always
    const int bv = umamd::igemm_border_valu();
    if ((bv == 2 || (bv == 1 && K <= 8)) && C % 8 == 0 && K % 8 == 0 && ldx % 8 == 0 && a.M > 0) {
      const long threads = (long)a.M * (C / 8);
      if (dtype == UM_BF16)
        hipLaunchKernelGGL(reflect_border_kernel<bf16_t>, dim3(ceil_div(threads, 256)), dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL(reflect_border_kernel<float>, dim3(ceil_div(threads, 256)), dim3(256), 0, st, a);
      UM_LAUNCH_CHECK();
      return UM_OK;
    }
    const long rest = ws != nullptr ? ws_bytes - base : 0;
    return umamd::igemm_run(dtype, a, rest > 0 ? (float*)((char*)ws + base) : nullptr,
                            rest > 0 ? rest : 0, st);
  }
  // stride 2 (zero padding): four parity classes (ay, ax) of dx pixels, each
  // a stride-1 gather over dy with the weight taps of matching parity:
  // dx[2i'+ay] = sum_t dy[i' + offy - t] * w[r0y + 2t], r0y = (ay+pad) % 2,
  // offy = (ay + pad - r0y) / 2 (and likewise in x)
  UM_CHECK_ARG(P == (H + 2 * pad - R) / 2 + 1 && Q == (W + 2 * pad - R) / 2 + 1,
               "um_conv2d_dgrad: size");
  umamd::IgArgs cls[4];
  for (int ay = 0; ay < 2; ++ay)
    for (int ax = 0; ax < 2; ++ax) {
      umamd::IgArgs& a = cls[2 * ay + ax];
      a = umamd::IgArgs{};
      const int r0y = (ay + pad) & 1, r0x = (ax + pad) & 1;
      const int nty = (R - r0y + 1) / 2, ntx = (R - r0x + 1) / 2;
      const int Hc = (H - ay + 1) / 2, Wc = (W - ax + 1) / 2;
      if (Hc <= 0 || Wc <= 0) continue;  // M stays 0: nothing to launch
      a.a = dy; a.ah = P; a.aw = Q; a.ach = K; a.lda = ldy;
      a.on = N; a.oh = Hc; a.ow = Wc;
      a.R = nty; a.Rx = ntx; a.stride = 1; a.tsign = -1;
      a.pad = -((ay + pad - r0y) / 2); a.padx = -((ax + pad - r0x) / 2);
      a.pmode = umamd::IG_PAD_ZERO; a.fold_pad = 0; a.flip = 0;
      a.cls = 1; a.wR = R; a.r0y = r0y; a.r0x = r0x; a.ay = ay; a.ax = ax; a.outH = H; a.outW = W;
      a.b = wT; a.ldb = (long)R * R * K;
      a.NC = C; a.M = N * Hc * Wc;
      a.bias = nullptr; a.out = dx; a.ld_out = ldx; a.out_f32 = (dtype == UM_F32);
      a.epilogue = UM_EPI_NONE; a.accumulate = accumulate; a.epi_scale = 1.f;
      a.residual = nullptr; a.ldr = 0; a.stats = nullptr;
    }
  const int one = umamd::igemm_run_cls4(dtype, cls, (float*)ws, ws_bytes, st);
  if (one < 0) return -one;
  if (one == 1) return UM_OK;
  for (auto& a : cls) {
    const int rc = umamd::igemm_run(dtype, a, (float*)ws, ws_bytes, st);  // M == 0: no-op
    if (rc != UM_OK) return rc;
  }
  return UM_OK;
}

static int wgrad_bm(int K) { return K <= 32 ? 32 : (K <= 64 ? 64 : 128); }

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    n = (hipGetDevice(&dev) == hipSuccess &&
         hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            ? v
            : 256;
    (void)hipGetLastError();
  }
  return n;
}

static int generic_wgrad_splits(int M, int K, int RRC, bool tr) {
  // tiles of the bf16 kernels (the f32 kernel uses 64x64 tiles; same split count)
  const int bm = tr ? umamd::wgrad_tr_bm(K) : wgrad_bm(K);
  const long tiles = (long)ceil_div(K, bm) * ceil_div(RRC, 128);
  // target workgroups over the chip: for the transposed-read kernel ONE round
  // of resident workgroups (occupancy x CUs; 768 was 1.5 rounds of the
  // 2-per-CU instance), else 768 (UMAMD_TUNING wsplit_blocks for sweeps)
  static const long fixed = umamd::tuning_env("wsplit_blocks", 0);
  const long target = fixed > 0 ? fixed
                      : tr      ? (long)umamd::wgrad_tr_blocks_per_cu(K) * cu_count()
                                : 768;
  long splits = tr && fixed <= 0 ? std::max<long>(1, target / tiles) : (target + tiles - 1) / tiles;
  const long max_by_m = (M + 255) / 256;  // >= 256 pixels per split
  if (splits > max_by_m) splits = max_by_m;
  const long max_by_bytes = (32l << 20) / ((long)K * RRC * 4);  // <= 32 MB of slabs
  if (splits > max_by_bytes) splits = max_by_bytes;
  if (splits < 1) splits = 1;
  return (int)splits;
}

int um_conv_wgrad_splits(int dtype, int N, int H, int W, int C, int ldx, int K, int R,
                         int stride, int pad, int pad_mode, int P, int Q, int ldy) {
  if (wgrad_1x1_ok(dtype, C, K, R, stride, pad, ldx, ldy)) return wgrad_1x1_blocks((long)N * P * Q);
  if (dtype == UM_BF16 && ldx % 8 == 0 && ldy % 8 == 0) {
    const int h = umamd::hwgrad_splits(N, H, W, C, ldx, K, R, stride, pad,
                                       pad_mode == UM_PAD_REFLECT, P, Q, ldy);
    if (h > 0) return h;
  }
  return generic_wgrad_splits(N * P * Q, K, R * R * C, dtype == UM_BF16 && K > 32);
}

int um_conv2d_wgrad(int dtype, int N, int H, int W, int C, int ldx, const void* x, int K, int R,
                    int stride, int pad, int pad_mode, int P, int Q, const void* dy, int ldy,
                    float* slabs, int splits, hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0 && K % 8 == 0, "um_conv2d_wgrad: C (%d), K (%d) must be multiples of 8", C, K);
  UM_CHECK_ARG(splits >= 1, "um_conv2d_wgrad: splits");
  UM_CHECK_ARG(splits == um_conv_wgrad_splits(dtype, N, H, W, C, ldx, K, R, stride, pad, pad_mode,
                                              P, Q, ldy),
               "um_conv2d_wgrad: splits must come from um_conv_wgrad_splits");
  if (dtype == UM_BF16 && ldx % 8 == 0 && ldy % 8 == 0 &&
      umamd::hwgrad_splits(N, H, W, C, ldx, K, R, stride, pad, pad_mode == UM_PAD_REFLECT, P, Q,
                           ldy) == splits) {
    if (umamd::hwgrad_run(x, N, H, W, C, ldx, K, R, stride, pad, pad_mode == UM_PAD_REFLECT, P,
                          Q, dy, ldy, slabs, splits, st) == UM_OK)
      return UM_OK;
    umamd::set_error("um_conv2d_wgrad: halo kernel launch failed");
    return UM_ERR_HIP;
  }
  if (dtype == UM_BF16 && K > 32 && !wgrad_1x1_ok(dtype, C, K, R, stride, pad, ldx, ldy)) {
    UM_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0, "um_conv2d_wgrad: ld %% 8");
    return umamd::wgrad_tr_run(x, N, H, W, C, ldx, K, R, stride, pad, pad_mode == UM_PAD_REFLECT,
                               P, Q, dy, ldy, slabs, splits, st);
  }
  WgradArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.K = K; a.R = R; a.stride = stride;
  a.pad = pad; a.pad_mode = pad_mode; a.P = P; a.Q = Q; a.ldy = ldy;
  a.x = x; a.dy = dy; a.slabs = slabs;
  a.M = N * P * Q; a.RRC = R * R * C;
  a.m_per_split = ceil_div(ceil_div(a.M, splits), WBK) * WBK;
  if (wgrad_1x1_ok(dtype, C, K, R, stride, pad, ldx, ldy)) {
    const int L = (K / 8) * (C / 8);
    const dim3 grid(splits);
    switch (L) {
      case 1: hipLaunchKernelGGL(wgrad_1x1_kernel<1>, grid, dim3(W1_NT), 0, st, a); break;
      case 2: hipLaunchKernelGGL(wgrad_1x1_kernel<2>, grid, dim3(W1_NT), 0, st, a); break;
      case 4: hipLaunchKernelGGL(wgrad_1x1_kernel<4>, grid, dim3(W1_NT), 0, st, a); break;
      case 8: hipLaunchKernelGGL(wgrad_1x1_kernel<8>, grid, dim3(W1_NT), 0, st, a); break;
      case 16: hipLaunchKernelGGL(wgrad_1x1_kernel<16>, grid, dim3(W1_NT), 0, st, a); break;
      default: hipLaunchKernelGGL(wgrad_1x1_kernel<32>, grid, dim3(W1_NT), 0, st, a); break;
    }
    UM_LAUNCH_CHECK();
    return UM_OK;
  }
  if (dtype == UM_BF16) {
    UM_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0, "um_conv2d_wgrad: ld %% 8");
    const int bm = wgrad_bm(K);
    if (bm == 32) return launch_wgrad_bf16<32>(a, splits, st);
    if (bm == 64) return launch_wgrad_bf16<64>(a, splits, st);
    return launch_wgrad_bf16<128>(a, splits, st);
  }
  return launch_wgrad<float, 64, 64>(a, splits, st);
}

static int make_segs(Segs& g, int nseg, const int* src0, const int* dst0, const int* len,
                     int Creal, int C) {
  if (nseg <= 0) {
    g.n = 1;
    g.src0[0] = 0; g.dst0[0] = 0; g.len[0] = Creal;
    return 1;
  }
  if (nseg > MAX_SEG) return 0;
  g.n = nseg;
  for (int i = 0; i < nseg; ++i) {
    g.src0[i] = src0[i]; g.dst0[i] = dst0[i]; g.len[i] = len[i];
    if (src0[i] + len[i] > Creal || dst0[i] + len[i] > C) return 0;
  }
  return 1;
}

int um_conv_wgrad_reduce_seg(const float* slabs, int splits, int K, int Kreal, int R, int C,
                             int Creal, float* dw, int accumulate, int nseg, const int* src0,
                             const int* dst0, const int* len, hipStream_t st) {
  UM_CHECK_ARG(Kreal <= K && (nseg > 0 || Creal <= C), "um_conv_wgrad_reduce: sizes");
  Segs g{};
  UM_CHECK_ARG(make_segs(g, nseg, src0, dst0, len, Creal, C), "um_conv_wgrad_reduce: segments");
  const long total = (long)Kreal * R * R * C;
  const long RRC = (long)R * R * C;
  static const int wred_t = (int)umamd::tuning_env("wred_t", 1);
  if (wred_t && R > 1 && total >= (1l << 18)) {
    const size_t shm = (size_t)R * R * (WRT_CW + 1) * sizeof(float);
    hipLaunchKernelGGL(wgrad_reduce_t_kernel, dim3(ceil_div(C, WRT_CW), Kreal), dim3(256), shm, st,
                       slabs, splits, K, R, C, Creal, dw, accumulate, g);
    UM_LAUNCH_CHECK();
    return UM_OK;
  }
  if (RRC % 4 == 0 && (long)splits * K * RRC < (1l << 33)) {
    const long total4 = total / 4;
    int L = 1;
    while (L < 32 && L * 4 <= splits && (total4 * L) / 256 < 2048) L <<= 1;
    const int EB = 256 / L;
    const int blocks = (int)std::min<long>((total4 + EB - 1) / EB, 8192);
    hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3(blocks), dim3(256), 0, st, slabs, splits, K,
                       Kreal, R, C, Creal, dw, accumulate, g, L);
    UM_LAUNCH_CHECK();
    return UM_OK;
  }
  // split lanes: enough that ~2048 blocks x EB elements cover the slab, and
  // <= splits / 4 so each lane still sums >= 4 partials
  int L = 1;
  while (L < 32 && L * 4 <= splits && (total * L) / 256 < 2048) L <<= 1;
  const int EB = 256 / L;
  const int blocks = (int)std::min<long>((total + EB - 1) / EB, 8192);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, slabs, splits, K, Kreal,
                     R, C, Creal, dw, accumulate, g, L);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_conv_wgrad_reduce(const float* slabs, int splits, int K, int Kreal, int R, int C,
                         int Creal, float* dw, int accumulate, hipStream_t st) {
  return um_conv_wgrad_reduce_seg(slabs, splits, K, Kreal, R, C, Creal, dw, accumulate, 0,
                                  nullptr, nullptr, nullptr, st);
}

int um_pack_weight_seg(int dtype, const float* w, int K, int Creal, int R, int C, void* wf,
                       void* wT, int ldT, int nseg, const int* src0, const int* dst0,
                       const int* len, hipStream_t st) {
  // segments may place a part of the reference channels only (the decoder's
  // skip / feature-map halves of one 1x1 weight); without them all Creal
  UM_CHECK_ARG(nseg > 0 || C >= Creal, "um_pack_weight: C < Creal");
  Segs g{};
  UM_CHECK_ARG(make_segs(g, nseg, src0, dst0, len, Creal, C), "um_pack_weight: segments");
  const long total = (long)K * R * R * C;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, w, K, Creal,
                       R, C, (bf16_t*)wf, (bf16_t*)wT, ldT, g, 0);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(blocks), dim3(256), 0, st, w, K, Creal, R,
                       C, (float*)wf, (float*)wT, ldT, g, 0);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_pack_weight(int dtype, const float* w, int K, int Creal, int R, int C, void* wf, void* wT,
                   int ldT, hipStream_t st) {
  return um_pack_weight_seg(dtype, w, K, Creal, R, C, wf, wT, ldT, 0, nullptr, nullptr, nullptr,
                            st);
}

int um_pack_weight_split(const float* w, int K, int Creal, int R, int C, void* wf, void* wT,
                         int ldT, hipStream_t st) {
  UM_CHECK_ARG(C >= Creal && (wT == nullptr || ldT >= 2 * K), "um_pack_weight_split: C / ldT");
  Segs g{};
  UM_CHECK_ARG(make_segs(g, 0, nullptr, nullptr, nullptr, Creal, C), "um_pack_weight_split");
  const long total = 2L * K * R * R * C;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, w, K, Creal, R,
                     C, (bf16_t*)wf, (bf16_t*)wT, ldT, g, 1);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_colsum_batch(int dtype, const um_csum_desc* descs, int n, hipStream_t st) {
  UM_CHECK_ARG(descs != nullptr && n >= 0 && n <= UM_CSUM_MAX, "um_colsum_batch: n");
  if (n == 0) return UM_OK;
  CsBatch b{};
  b.n = n;
  b.dtype = dtype;
  int blocks = 0, maxc = 0;
  for (int i = 0; i < n; ++i) {
    const um_csum_desc& e = descs[i];
    UM_CHECK_ARG(e.y && e.parts && e.out && e.M > 0 && e.C % 8 == 0 && e.ld % 8 == 0 &&
                     e.creal <= e.C && e.nparts == parts_for(e.M),
                 "um_colsum_batch: descriptor %d", i);
    CsDesc& d = b.d[i];
    d.y = e.y; d.parts = e.parts; d.out = e.out;
    d.M = e.M; d.C = e.C; d.ld = e.ld; d.nparts = e.nparts; d.rows = rows_per_part(e.M);
    d.creal = e.creal;
    b.first[i] = blocks;
    blocks += e.nparts;
    maxc = std::max(maxc, e.C);
  }
  b.first[n] = blocks;
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(colsum_batch_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, b);
  else
    hipLaunchKernelGGL(colsum_batch_kernel<float>, dim3(blocks), dim3(256), 0, st, b);
  hipLaunchKernelGGL(colsum_fin_batch_kernel, dim3(n, ceil_div(maxc, 32)), dim3(256), 0, st, b);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_colsum_parts(int M) { return parts_for(M); }

int um_colsum(int dtype, int M, int C, int ld, const void* y, float* parts, hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0 && ld % 8 == 0, "um_colsum: C/ld %% 8");
  const int blocks = parts_for(M);
  const int rows = rows_per_part(M);
  if (M == 0) return UM_OK;
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)y, M,
                       C, ld, parts, rows);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)y, M,
                       C, ld, parts, rows);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"

// ------------------------------------------------------- batched repack --
// One launch refreshes the packed copies of every conv weight (see
// um_pack_batch in umamd.h).  Workgroup = 32 output channels (k) x ct(R)
// input channels (c) x all R*R taps: the source block w[k][c0..c0+ct)[taps]
// is one contiguous run per k (coalesced f32 reads), staged in LDS, then
// written as wf rows (c contiguous) and, transposed, as wT rows (k
// contiguous, 64-byte segments).
namespace {

constexpr int PK = 32;  // k per workgroup
__host__ __device__ constexpr int pack_ct(int R) {  // c per workgroup: 32*ct*R*R <= 8192
  return R <= 1 ? 64 : (R <= 3 ? 16 : (R <= 5 ? 8 : 4));
}

// One (32 k x CT c) tile of one weight per workgroup.  The filter size is a
// compile-time constant (R in {1, 3, 5, 7}: every conv of the model) so the
// (k, c, tap) index splits are multiplies and shifts, not integer divisions.
template <typename T, int R>
__device__ __forceinline__ void pack_tile(const um_pack_desc& d, int t, float* tile) {
  constexpr int RR = R * R, CT = pack_ct(R);
  constexpr int per_k = CT * RR;  // staged values per k row
  constexpr int ldt = per_k + 1;  // odd LDS row stride
  constexpr int n = PK * per_k;
  const int nct = (d.C + CT - 1) / CT;
  const int k0 = (t / nct) * PK, c0 = (t % nct) * CT;
  const int K2 = d.split ? 2 * d.K : d.K;  // packed rows (split: [hi | lo])
  // whole channel block present and no segment map: each k row of the tile is
  // one contiguous, 16-byte aligned run of CT*RR floats -> float4 loads, four
  // independent ones in flight per thread (the scalar gather below ran the
  // 180 MB repack at 1.8 TB/s)
  const bool vec = d.nseg <= 0 && c0 + CT <= d.Creal && (d.Creal * RR) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(d.w) & 15) == 0;
  if (vec) {
    constexpr int Q4 = per_k / 4;  // float4 per k row
    static_assert(per_k % 4 == 0, "k row of float4");
    constexpr int N4 = PK * Q4, U = 4;
    for (int i0 = threadIdx.x; i0 < N4; i0 += U * 256) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 256;
        const int kk = i / Q4, q = i - kk * Q4;
        const int k2 = k0 + kk;
        const int k = k2 < d.K ? k2 : k2 - d.K;
        v[u] = (i < N4 && k2 < K2)
                   ? *reinterpret_cast<const float4*>(d.w + ((long)k * d.Creal + c0) * RR + 4 * q)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 256;
        if (i >= N4) break;
        const int kk = i / Q4, q = i - kk * Q4;
        const bool lo = k0 + kk >= d.K;
        float* t = tile + kk * ldt + 4 * q;
        t[0] = split_part<T>(v[u].x, lo);
        t[1] = split_part<T>(v[u].y, lo);
        t[2] = split_part<T>(v[u].z, lo);
        t[3] = split_part<T>(v[u].w, lo);
      }
    }
  }
  for (int i = vec ? n : threadIdx.x; i < n; i += 256) {
    const int kk = i / per_k, rem = i - kk * per_k;
    const int cc = rem / RR, tap = rem - cc * RR;
    const int k2 = k0 + kk, c = c0 + cc;
    const int k = k2 < d.K ? k2 : k2 - d.K;
    float v = 0.f;
    if (k2 < K2 && c < d.C) {
      int cs = -1;
      if (d.nseg <= 0) cs = c < d.Creal ? c : -1;
      else
#pragma unroll
        for (int g = 0; g < UM_PACK_MAXSEG; ++g)  // static indices: no scratch copy of d
          if (g < d.nseg && c >= d.dst0[g] && c < d.dst0[g] + d.len[g])
            cs = d.src0[g] + c - d.dst0[g];
      if (cs >= 0) v = split_part<T>(d.w[((long)k * d.Creal + cs) * RR + tap], k2 >= d.K);
    }
    tile[kk * ldt + cc * RR + tap] = v;
  }
  __syncthreads();
  T* wf = reinterpret_cast<T*>(d.wf);
  T* wT = reinterpret_cast<T*>(d.wT);
  // vector stores: wf in runs of 4 channels (C is a multiple of 8, CT of 4),
  // wT in runs of 8 output channels (scalar where a run leaves [0, K) or ldT
  // is not a multiple of 8).  LDS reads: consecutive lanes step by RR (wf) or
  // ldt (wT), both odd, so they spread over the banks.
  if (wf)
    for (int i = threadIdx.x; i < n / 4; i += 256) {  // (kk, tap, c4): c fastest
      const int kk = i / (per_k / 4), rem = i - kk * (per_k / 4);
      const int tap = rem / (CT / 4), c4 = (rem - tap * (CT / 4)) * 4;
      const int k = k0 + kk, c = c0 + c4;
      if (k >= K2 || c >= d.C) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tile[kk * ldt + (c4 + e) * RR + tap];
      store4(wf + ((long)k * RR + tap) * d.C + c, v);
    }
  if (wT) {
    const bool vec = (d.ldT & 7) == 0;
    for (int i = threadIdx.x; i < n / 8; i += 256) {  // (cc, tap, k8): k fastest
      const int cc = i / (RR * PK / 8), rem = i - cc * (RR * PK / 8);
      const int tap = rem / (PK / 8), k8 = (rem - tap * (PK / 8)) * 8;
      const int k = k0 + k8, c = c0 + cc;
      if (c >= d.C || k >= K2) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[(k8 + e) * ldt + cc * RR + tap];
      T* o = wT + ((long)c * RR + tap) * d.ldT + k;
      if (vec && k + 8 <= K2) {
        store8(o, v);
      } else {
        for (int e = 0; e < 8 && k + e < K2; ++e) o[e] = from_f32<T>(v[e]);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) pack_batch_kernel(const um_pack_desc* __restrict__ table,
                                                         const int* __restrict__ blk2desc) {
  __shared__ float tile[8192 + 64];
  const um_pack_desc d = table[blk2desc[blockIdx.x]];
  const int t = blockIdx.x - d.block0;
  switch (d.R) {
    case 1: pack_tile<T, 1>(d, t, tile); break;
    case 3: pack_tile<T, 3>(d, t, tile); break;
    case 5: pack_tile<T, 5>(d, t, tile); break;
    case 7: pack_tile<T, 7>(d, t, tile); break;
    default: break;  // rejected on the host (um_pack_batch)
  }
}

}  // namespace

extern "C" int um_pack_tiles(int K, int C, int R) {
  return ceil_div(K, PK) * ceil_div(C, pack_ct(R));
}

extern "C" int um_pack_batch(int dtype, const um_pack_desc* table, int ndesc,
                             const int* blk2desc, int nblocks, hipStream_t st) {
  UM_CHECK_ARG(table != nullptr && blk2desc != nullptr && ndesc > 0, "um_pack_batch: table");
  // (split descriptors are bf16-only; the table is device memory, so the
  // binding checks that: umamd/packer.py)
  if (nblocks <= 0) return UM_OK;
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(pack_batch_kernel<bf16_t>, dim3(nblocks), dim3(256), 0, st, table,
                       blk2desc);
  else
    hipLaunchKernelGGL(pack_batch_kernel<float>, dim3(nblocks), dim3(256), 0, st, table,
                       blk2desc);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

extern "C" int um_pack_desc_size(void) { return (int)sizeof(um_pack_desc); }
