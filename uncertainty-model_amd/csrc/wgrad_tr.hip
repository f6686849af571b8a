// Implicit-GEMM weight gradient with transposed LDS reads (bf16, gfx950).
//
//   dW[k][j] = sum_m DY[m][k] * X(m, j),  j = (r, s, c),  m = output pixel
//
// The reduction runs over pixels, while both operands are stored
// pixel-major (NHWC), so each k-step (32 pixels) stages plain 16-byte rows:
//   sA[px][BM output channels]  (DY)
//   sB[px][128 columns (r,s,c)]  (X gathered at the column's tap)
// and the MFMA fragments (8 consecutive pixels of one channel / column per
// lane) come out of ds_read_b64_tr_b16 pairs.  The images swizzle 32-byte
// channel chunks by pixel-row bits (the parity masks found conflict-free for
// 8- and 4-chunk rows), double-buffered, one barrier per k-step, the next
// step's global loads in flight during the MFMAs.  Pixel coordinates advance
// incrementally (no division in the loop).  Split over pixels into f32 slabs
// [split][K][R*R*C] as the other weight-gradient kernels; wgrad_reduce_kernel
// sums them.  Used for the bf16 convs the halo kernel does not cover (deep
// layers with many channels or small maps).
#include <algorithm>
#include <cstdlib>

#include <atomic>

#include "common.h"
#include "wgrad_tr.h"

namespace {

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

constexpr int TBN = 128;  // (r,s,c) columns per block

struct TrArgs {
  const bf16_t* x;
  const bf16_t* dy;
  float* slabs;
  int N, H, W, C, ldx, K, R, stride, pad, reflect, P, Q, ldy;
  int M, RRC, m_per_split;
};

__device__ __forceinline__ int bit(int v, int b) { return (v >> b) & 1; }
// chunk swizzle for an image of `nch` 16-channel chunks per pixel row
template <int NCH>
__device__ __forceinline__ int swz(int row) {
  if (NCH == 8) return bit(row, 0) | (bit(row, 1) << 1) | (bit(row, 3) << 2);
  if (NCH == 4) return bit(row, 1) | (bit(row, 3) << 1);
  return 0;
}
template <int NCH>
__device__ __forceinline__ int img_off(int row, int c8) {  // element offset of 8-ch chunk c8
  return row * NCH * 16 + (((c8 >> 1) ^ swz<NCH>(row)) << 4) + ((c8 & 1) << 3);
}

__device__ __forceinline__ bf16x4_t tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (__attribute__((address_space(3))) bf16x4_t*)(p));
}

// pixel coordinates advanced by a fixed step without division
struct Pix {
  int n, p, q;
  bool ok;
};
__device__ __forceinline__ Pix pix_at(long m, int P, int Q, long mend) {
  Pix x;
  x.ok = m < mend;
  const long mm = x.ok ? m : 0;
  const long pq = (long)P * Q;
  x.n = (int)(mm / pq);
  const int r = (int)(mm - x.n * pq);
  x.p = r / Q;
  x.q = r - x.p * Q;
  return x;
}
__device__ __forceinline__ void pix_adv(Pix& x, int step, int P, int Q, long m, long mend) {
  x.q += step;
  while (x.q >= Q) {
    x.q -= Q;
    if (++x.p == P) { x.p = 0; ++x.n; }
  }
  x.ok = m < mend;
}

// TBK pixels per k-step (a multiple of the MFMA's 32): the loads of step
// s+1 are in flight during the MFMAs of step s, so a larger step hides more
// of the global-load latency per barrier (these GEMMs are latency-bound at
// one or two blocks per CU).
template <int BM, int TBK>
__global__ void __launch_bounds__(256) wgrad_tr_kernel(TrArgs a) {
  constexpr int NCA = BM / 16, NCB = TBN / 16;  // 16-channel chunks per image row
  constexpr int TM = BM / 32, TN = 4;           // 2x2 waves, 16x16 tiles
  constexpr int A_PER = TBK * BM / 8 / 256;     // 8-channel chunks per thread per step
  constexpr int B_PER = TBK * TBN / 8 / 256;
  constexpr int KS = TBK / 32;                  // MFMA k-substeps per step
  static_assert(A_PER >= 1 && B_PER >= 2 && TBK % 32 == 0, "tiles");
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][TBK * BM];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][TBK * TBN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int bk = blockIdx.x * BM;   // output-channel tile
  const int bj = blockIdx.y * TBN;  // (r,s,c) tile
  const long m_begin = (long)blockIdx.z * a.m_per_split;
  const long m_end = min((long)a.M, m_begin + a.m_per_split);

  // staging assignments: A chunk u -> (row, c8), B likewise
  int arow[A_PER], ac8[A_PER];
  bool aok[A_PER];
  Pix apx[A_PER];
#pragma unroll
  for (int u = 0; u < A_PER; ++u) {
    const int id = tid + u * 256;
    arow[u] = id / (BM / 8);
    ac8[u] = id % (BM / 8);
    aok[u] = bk + ac8[u] * 8 < a.K;
    apx[u] = pix_at(m_begin + arow[u], a.P, a.Q, m_end);
  }
  int brow[B_PER], bc8[B_PER], bry[B_PER], brx[B_PER], bch[B_PER];
  bool bok[B_PER];
  Pix bpx[B_PER];
#pragma unroll
  for (int u = 0; u < B_PER; ++u) {
    const int id = tid + u * 256;
    brow[u] = id / (TBN / 8);
    bc8[u] = id % (TBN / 8);
    const int j = bj + bc8[u] * 8;
    bok[u] = j < a.RRC;
    const int jj = bok[u] ? j : 0;
    const int tap = jj / a.C;
    bch[u] = jj - tap * a.C;
    bry[u] = tap / a.R;
    brx[u] = tap - bry[u] * a.R;
    bpx[u] = pix_at(m_begin + brow[u], a.P, a.Q, m_end);
  }

  uint4 ra[A_PER], rb[B_PER];
  auto load = [&]() {
#pragma unroll
    for (int u = 0; u < A_PER; ++u) {
      ra[u] = make_uint4(0, 0, 0, 0);
      if (apx[u].ok && aok[u])
        ra[u] = *reinterpret_cast<const uint4*>(
            a.dy + ((long)(apx[u].n * a.P + apx[u].p) * a.Q + apx[u].q) * a.ldy + bk + ac8[u] * 8);
    }
#pragma unroll
    for (int u = 0; u < B_PER; ++u) {
      rb[u] = make_uint4(0, 0, 0, 0);
      if (!bpx[u].ok || !bok[u]) continue;
      int yy = bpx[u].p * a.stride - a.pad + bry[u], xx = bpx[u].q * a.stride - a.pad + brx[u];
      if (a.reflect) {
        yy = reflect_idx(yy, a.H);
        xx = reflect_idx(xx, a.W);
      } else if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W) {
        continue;
      }
      rb[u] = *reinterpret_cast<const uint4*>(
          a.x + ((long)(bpx[u].n * a.H + yy) * a.W + xx) * a.ldx + bch[u]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < A_PER; ++u)
      *reinterpret_cast<uint4*>(&sA[buf][img_off<NCA>(arow[u], ac8[u])]) = ra[u];
#pragma unroll
    for (int u = 0; u < B_PER; ++u)
      *reinterpret_cast<uint4*>(&sB[buf][img_off<NCB>(brow[u], bc8[u])]) = rb[u];
  };
  auto advance = [&](long m0) {
#pragma unroll
    for (int u = 0; u < A_PER; ++u) pix_adv(apx[u], TBK, a.P, a.Q, m0 + arow[u], m_end);
#pragma unroll
    for (int u = 0; u < B_PER; ++u) pix_adv(bpx[u], TBK, a.P, a.Q, m0 + brow[u], m_end);
  };

  // transposed-read offsets (elements, relative to a buffer): rows 8g+q and +4
  int oa[TM][2], ob[TN][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + q4 + 4 * h;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ct = (wm * (BM / 2) + i * 16) / 16;
      oa[i][h] = row * NCA * 16 + ((ct ^ swz<NCA>(row)) << 4) + 4 * p4;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int ct = (wn * 64 + j * 16) / 16;
      ob[j][h] = row * NCB * 16 + ((ct ^ swz<NCB>(row)) << 4) + 4 * p4;
    }
  }

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (m_begin < m_end) {
    load();
    store(0);
    advance(m_begin + TBK);
  }
  __syncthreads();
  int cur = 0;
  for (long m0 = m_begin; m0 < m_end; m0 += TBK) {
    const bool more = m0 + TBK < m_end;
    if (more) load();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // 32 more pixel rows: row bits 0..3 (the swizzle's) are unchanged
      const int da = ks * 32 * NCA * 16, db = ks * 32 * NCB * 16;
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x4_t lo = tr_read(&sA[cur][oa[i][0] + da]);
        const bf16x4_t hi = tr_read(&sA[cur][oa[i][1] + da]);
        fa[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bf16x4_t lo = tr_read(&sB[cur][ob[j][0] + db]);
        const bf16x4_t hi = tr_read(&sB[cur][ob[j][1] + db]);
        fb[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store(cur ^ 1);
      advance(m0 + 2 * TBK);
    }
    __syncthreads();
    cur ^= 1;
  }

  float* out = a.slabs + (long)blockIdx.z * a.K * a.RRC;
  const int col = lane & 15, row4 = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = bk + wm * (BM / 2) + i * 16 + row4 + e;
        const int jj = bj + wn * 64 + j * 16 + col;
        if (k < a.K && jj < a.RRC) out[(long)k * a.RRC + jj] = acc[i][j][e];
      }
}

}  // namespace

namespace umamd {

int wgrad_tr_bm(int K) { return K <= 64 ? 64 : 128; }

// pixels per k-step (tuning key wtr_tbk: 32, 64 or 128)
int wgrad_tr_tbk() {
  static const int v = [] {
    const int t = (int)umamd::tuning_env("wtr_tbk", 32);
    return (t == 64 || t == 128) ? t : 32;
  }();
  return v;
}

// resident 256-thread workgroups per CU of the instance wgrad_tr_run picks for K
int wgrad_tr_blocks_per_cu(int K) {
  const int bm = wgrad_tr_bm(K), tbk = wgrad_tr_tbk();
  // cached per instance (bm, tbk): queried on every weight-gradient plan
  static std::atomic<int> cache[2][3] = {{{0}, {0}, {0}}, {{0}, {0}, {0}}};
  std::atomic<int>& slot = cache[bm == 128][tbk == 32 ? 0 : (tbk == 64 ? 1 : 2)];
  if (const int c = slot.load(std::memory_order_relaxed)) return c;
  const void* f = nullptr;
#define UM_WTRF(BM_, TBK_) \
  if (bm == BM_ && tbk == TBK_) f = reinterpret_cast<const void*>(&wgrad_tr_kernel<BM_, TBK_>);
  UM_WTRF(64, 32) UM_WTRF(64, 64) UM_WTRF(64, 128)
  UM_WTRF(128, 32) UM_WTRF(128, 64) UM_WTRF(128, 128)
#undef UM_WTRF
  int n = 0;
  if (f == nullptr || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) {
    (void)hipGetLastError();
    n = 1;
  }
  n = std::max(1, n);
  slot.store(n, std::memory_order_relaxed);
  return n;
}

int wgrad_tr_run(const void* x, int N, int H, int W, int C, int ldx, int K, int R, int stride,
                 int pad, int reflect, int P, int Q, const void* dy, int ldy, float* slabs,
                 int splits, hipStream_t st) {
  TrArgs a{};
  a.x = reinterpret_cast<const bf16_t*>(x);
  a.dy = reinterpret_cast<const bf16_t*>(dy);
  a.slabs = slabs;
  a.N = N; a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.K = K; a.R = R; a.stride = stride;
  a.pad = pad; a.reflect = reflect; a.P = P; a.Q = Q; a.ldy = ldy;
  a.M = N * P * Q;
  a.RRC = R * R * C;
  const int tbk = wgrad_tr_tbk();
  a.m_per_split = ceil_div(ceil_div(a.M, splits), tbk) * tbk;
  const int bm = wgrad_tr_bm(K);
  dim3 grid(ceil_div(K, bm), ceil_div(a.RRC, TBN), splits);
#define UM_WTR(BM_, TBK_)                                                                 \
  if (bm == BM_ && tbk == TBK_) {                                                         \
    hipLaunchKernelGGL((wgrad_tr_kernel<BM_, TBK_>), grid, dim3(256), 0, st, a);          \
    UM_LAUNCH_CHECK();                                                                    \
    return UM_OK;                                                                         \
  }
  UM_WTR(64, 32) UM_WTR(64, 64) UM_WTR(64, 128)
  UM_WTR(128, 32) UM_WTR(128, 64) UM_WTR(128, 128)
#undef UM_WTR
  umamd::set_error("wgrad_tr: no kernel for bm %d tbk %d", bm, tbk);
  return UM_ERR_ARG;
}

}  // namespace umamd
