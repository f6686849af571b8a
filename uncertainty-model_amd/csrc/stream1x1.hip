// Streaming 1x1 convolution for the HBM-bound high-resolution layers (bf16,
// gfx950): out[m][n] = sum_c A[m][c] W[n][c] (+ bias, + residual, + out)
// over M >= 16k pixels with few channels (C <= 256, N <= 192).
//
// At these shapes a 1x1 conv is one pass over its activations and outputs
// (AI 16-48 FLOP/B): the tiled implicit GEMM (igemm.hip, 256-row
// tiles) spends its time in per-tile prologue/epilogue latency (30-35 us for
// 50-70 MB).  Here:
//   - the whole weight (N x C bf16, <= 32 KB) is staged once per workgroup in
//     LDS (igemm's conflict-free 64-byte-row swizzle) and the workgroups are
//     persistent: wave w of block b takes the 16-pixel strips b*8+2w, ...;
//   - the MFMA runs transposed, D = W . A^T (v_mfma_f32_16x16x32_bf16 with
//     the weights as the A operand): the activation fragments are the NHWC
//     rows themselves (lane = pixel, 16 contiguous bytes of channels, loaded
//     straight from global into registers: no LDS for the streamed operand),
//     and each lane ends up holding 4 CONSECUTIVE output channels of one
//     pixel, stored as one 8-byte (bf16) or 16-byte (f32) vector;
//   - two strips per wave in flight (32 pixels x C channels of loads), the
//     next n-chunk of 4 blocks reuses the loaded fragments;
//   - BN statistics (the decoder skip conv's f32 pre-BN output, accumulated
//     onto up2(z): statistics of the SUM) stay in registers for all strips
//     of the workgroup and leave as one f64 slot atomic per channel.
// Reference ops: the 1x1 nn.Conv2d of model/layers/attention.py:37-40 (keys,
// queries, values, reprojection) and of the DecoderStage squeeze-excite
// ConvELUBlock (model/layers/decoder.py:228-238), forward and input gradient.
#include <algorithm>

#include "common.h"
#include "igemm.h"
#include "stream1x1.h"

namespace {

using umamd::IgArgs;

constexpr int S1U = 2;      // 16-pixel strips per wave per iteration
constexpr int S1MAXNB = 12; // output channels <= 192
constexpr int S1STATNB = 8; // statistics: output channels <= 128

// plane ks (32 reduction channels) of nr weight rows, 64-byte rows whose
// 16-byte chunks are swizzled as igemm's Img<bf16, 32>
__device__ __forceinline__ int wimg(int ks, int nr, int row, int c8) {
  return (ks * nr + row) * 32 + ((c8 ^ ((4 - ((row >> 2) & 3)) & 3)) << 3);
}

__device__ __forceinline__ void add4(const bf16_t* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] += __uint_as_float(u.x << 16);
  v[1] += __uint_as_float(u.x & 0xffff0000u);
  v[2] += __uint_as_float(u.y << 16);
  v[3] += __uint_as_float(u.y & 0xffff0000u);
}

template <int KS, bool F32, bool STATS>
__global__ void __launch_bounds__(256) stream1x1_kernel(IgArgs a, int nb, long nstrips) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sW[];  // KS x nr x 32
  __shared__ float sStat[STATS ? 4 : 1][STATS ? S1STATNB * 16 : 1][2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nr = nb * 16;
  const bf16_t* __restrict__ wsrc = reinterpret_cast<const bf16_t*>(a.b);
  for (int i = tid; i < nr * KS * 4; i += 256) {
    const int n = i / (KS * 4), c8 = i - n * (KS * 4), c = c8 * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < a.NC && c < a.ach) v = *reinterpret_cast<const uint4*>(wsrc + (long)n * a.ldb + c);
    *reinterpret_cast<uint4*>(&sW[wimg(c8 >> 2, nr, n, c8 & 3)]) = v;
  }
  __syncthreads();
  const bf16_t* __restrict__ act = reinterpret_cast<const bf16_t*>(a.a);
  const int px = lane & 15, kq = lane >> 4;
  float st1[STATS ? S1STATNB : 1][4], st2[STATS ? S1STATNB : 1][4];
  if constexpr (STATS) {
#pragma unroll
    for (int b = 0; b < S1STATNB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st1[b][j] = st2[b][j] = 0.f;
  }
  const long stride = (long)gridDim.x * 4 * S1U;
  for (long t0 = ((long)blockIdx.x * 4 + w) * S1U; t0 < nstrips; t0 += stride) {
    bf16x8_t af[S1U][KS];
#pragma unroll
    for (int u = 0; u < S1U; ++u) {
      const long m = (t0 + u) * 16 + px;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c = ks * 32 + kq * 8;
        if (m < a.M && c < a.ach)
          af[u][ks] = *reinterpret_cast<const bf16x8_t*>(act + m * a.lda + c);
        else
          af[u][ks] = bf16x8_t{};
      }
    }
#pragma unroll
    for (int nc = 0; nc < S1MAXNB; nc += 4) {
      if (nc >= nb) break;
      f32x4_t acc[S1U][4];
#pragma unroll
      for (int u = 0; u < S1U; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[u][q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (nc + q >= nb) break;
          const bf16x8_t wf =
              *reinterpret_cast<const bf16x8_t*>(&sW[wimg(ks, nr, (nc + q) * 16 + px, kq)]);
#pragma unroll
          for (int u = 0; u < S1U; ++u)
            acc[u][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af[u][ks], acc[u][q], 0, 0, 0);
        }
      // lane: pixel (t0 + u) * 16 + px, channels n .. n + 3 of block nc + q
#pragma unroll
      for (int u = 0; u < S1U; ++u) {
        const long m = (t0 + u) * 16 + px;
        if (m >= a.M) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (nc + q >= nb) break;
          const int n = (nc + q) * 16 + kq * 4;
          float v[4] = {acc[u][q][0], acc[u][q][1], acc[u][q][2], acc[u][q][3]};
          if (a.bias != nullptr) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] += a.bias[n + j];
          }
          if (a.epilogue == UM_EPI_RESIDUAL)
            add4(reinterpret_cast<const bf16_t*>(a.residual) + m * a.ldr + n, v);
          if constexpr (F32) {
            float* o = reinterpret_cast<float*>(a.out) + m * a.ld_out + n;
            if (a.accumulate) {
              const float4 p = *reinterpret_cast<const float4*>(o);
              v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
            }
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + m * a.ld_out + n;
            if (a.accumulate) add4(o, v);
            uint2 r;
            r.x = pack_bf16x2(v[0], v[1]);
            r.y = pack_bf16x2(v[2], v[3]);
            *reinterpret_cast<uint2*>(o) = r;
          }
          if constexpr (STATS) {
            if (nc + q < S1STATNB) {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                st1[nc + q][j] += v[j];
                st2[nc + q][j] += v[j] * v[j];
              }
            }
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    // the 16 lanes of a channel group (same kq) hold 16 pixels' sums
#pragma unroll
    for (int b = 0; b < S1STATNB; ++b) {
      if (b >= nb) break;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = st1[b][j], y = st2[b][j];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          x += __shfl_xor(x, o, 64);
          y += __shfl_xor(y, o, 64);
        }
        if (px == 0) {
          sStat[w][b * 16 + kq * 4 + j][0] = x;
          sStat[w][b * 16 + kq * 4 + j][1] = y;
        }
      }
    }
    __syncthreads();
    double* slots = reinterpret_cast<double*>(a.stats);
    stat_slots_count(slots, a.NC, a.M);
    stat_slots_add_row(slots, blockIdx.x, a.NC, 0, a.NC, [&](int i) {
      return sStat[0][i >> 1][i & 1] + sStat[1][i >> 1][i & 1] + sStat[2][i >> 1][i & 1] +
             sStat[3][i >> 1][i & 1];
    });
  }
}

// Small-M 1x1 convolutions (round 6): the deep 8x16 .. 32x64 layers (M = 1k
// .. 16k pixels, C <= 512 reduction channels, N up to 1536: the attention's
// fused K/Q/V and reprojection, the decoder's first squeeze-excite 1x1, and
// their data gradients).  On 64x64 GEMM tiles these were 16-32 sequential
// k-steps per block with split-K epilogues (9-22 us for 0.5-1.6 GFLOP).  Here
// a workgroup owns NG 16-channel output blocks (grid.y) and stages only their
// weights (NG*16 rows x C, <= 64 KB) in LDS; each wave takes 16-pixel strips
// whose KS activation fragments (the whole reduction) it loads into registers
// at once -- one round of load latency per strip, no k-loop barrier -- then
// runs the KS x NG MFMAs (D = W . A^T as stream1x1_kernel: each lane ends with
// 4 consecutive output channels of one pixel) and the same epilogues (bias,
// residual, f32 output, accumulate, BN statistics into f64 slots).
template <int KS, int NG, bool F32, bool STATS>
__global__ void __launch_bounds__(256) s1x1_small_kernel(IgArgs a, long nstrips) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sW[];  // KS x (NG*16) x 32
  __shared__ float sStat[STATS ? 4 : 1][STATS ? NG * 16 : 1][2];
  constexpr int NR = NG * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.y * NR;  // this workgroup's first output channel
  const bf16_t* __restrict__ wsrc = reinterpret_cast<const bf16_t*>(a.b);
  for (int i = tid; i < NR * KS * 4; i += 256) {
    const int n = i / (KS * 4), c8 = i - n * (KS * 4), c = c8 * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n0 + n < a.NC && c < a.ach) v = *reinterpret_cast<const uint4*>(wsrc + (long)(n0 + n) * a.ldb + c);
    *reinterpret_cast<uint4*>(&sW[wimg(c8 >> 2, NR, n, c8 & 3)]) = v;
  }
  __syncthreads();
  const bf16_t* __restrict__ act = reinterpret_cast<const bf16_t*>(a.a);
  const int px = lane & 15, kq = lane >> 4;
  float st1[STATS ? NG : 1][4], st2[STATS ? NG : 1][4];
  if constexpr (STATS) {
#pragma unroll
    for (int b = 0; b < NG; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st1[b][j] = st2[b][j] = 0.f;
  }
  for (long t = (long)blockIdx.x * 4 + w; t < nstrips; t += (long)gridDim.x * 4) {
    const long m = t * 16 + px;
    bf16x8_t af[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c = ks * 32 + kq * 8;
      af[ks] = (m < a.M && c < a.ach) ? *reinterpret_cast<const bf16x8_t*>(act + m * a.lda + c)
                                      : bf16x8_t{};
    }
    f32x4_t acc[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) acc[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(&sW[wimg(ks, NR, q * 16 + px, kq)]);
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af[ks], acc[q], 0, 0, 0);
      }
    if (m >= a.M) continue;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const int n = n0 + q * 16 + kq * 4;
      if (n >= a.NC) break;
      float v[4] = {acc[q][0], acc[q][1], acc[q][2], acc[q][3]};
      if (a.bias != nullptr) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += a.bias[n + j];
      }
      if (a.epilogue == UM_EPI_RESIDUAL)
        add4(reinterpret_cast<const bf16_t*>(a.residual) + m * a.ldr + n, v);
      if constexpr (F32) {
        float* o = reinterpret_cast<float*>(a.out) + m * a.ld_out + n;
        if (a.accumulate) {
          const float4 p = *reinterpret_cast<const float4*>(o);
          v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
        }
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + m * a.ld_out + n;
        if (a.accumulate) add4(o, v);
        uint2 r;
        r.x = pack_bf16x2(v[0], v[1]);
        r.y = pack_bf16x2(v[2], v[3]);
        *reinterpret_cast<uint2*>(o) = r;
      }
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st1[q][j] += v[j];
          st2[q][j] += v[j] * v[j];
        }
      }
    }
  }
  if constexpr (STATS) {
#pragma unroll
    for (int b = 0; b < NG; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = st1[b][j], y = st2[b][j];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          x += __shfl_xor(x, o, 64);
          y += __shfl_xor(y, o, 64);
        }
        if (px == 0) {
          sStat[w][b * 16 + kq * 4 + j][0] = x;
          sStat[w][b * 16 + kq * 4 + j][1] = y;
        }
      }
    __syncthreads();
    double* slots = reinterpret_cast<double*>(a.stats);
    stat_slots_count(slots, a.NC, a.M);
    stat_slots_add_row(slots, blockIdx.x, a.NC, n0, min(NR, a.NC - n0), [&](int i) {
      return sStat[0][i >> 1][i & 1] + sStat[1][i >> 1][i & 1] + sStat[2][i >> 1][i & 1] +
             sStat[3][i >> 1][i & 1];
    });
  }
}

}  // namespace

namespace umamd {

static int s1x1_ks(int ach) {
  const int k = (ach + 31) / 32;
  return k <= 1 ? 1 : (k <= 2 ? 2 : (k <= 4 ? 4 : (k <= 8 ? 8 : 0)));
}

bool stream1x1_applicable(int dtype, const IgArgs& a) {
  if (dtype != UM_BF16 || a.R != 1 || a.Rx != 1 || a.stride != 1 || a.pad != 0 || a.padx != 0 ||
      a.cls || a.border || a.pmode != IG_PAD_ZERO || a.oh != a.ah || a.ow != a.aw)
    return false;
  if (a.M < 16384 || a.ach % 8 || a.lda % 8 || a.ld_out % 8 || a.NC % 16 || a.NC > 16 * S1MAXNB)
    return false;
  const int ks = s1x1_ks(a.ach);
  if (ks == 0 || ks * (a.NC / 16) > 32) return false;  // weight image <= 32 KB
  auto al = [](const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; };
  if (!al(a.a, 16) || !al(a.b, 16) || !al(a.out, a.out_f32 ? 16 : 8) ||
      (a.residual != nullptr && !al(a.residual, 8)))
    return false;
  if (a.epilogue == UM_EPI_NONE) return true;
  if (a.epilogue == UM_EPI_RESIDUAL) return !a.out_f32 && a.ldr % 4 == 0 && a.residual != nullptr;
  if (a.epilogue == UM_EPI_STATS)
    return a.stat_slots && a.out_f32 && a.NC <= 16 * S1STATNB && a.stats != nullptr;
  return false;
}

static int small_ks(int ach) {
  const int k = (ach + 31) / 32;
  return k <= 2 ? (k <= 1 ? 1 : 2) : (k <= 4 ? 4 : (k <= 8 ? 8 : (k <= 16 ? 16 : 0)));
}

// the small-M 1x1 path (s1x1_small_kernel): M < 16384 pixels (the streaming
// kernel's lower bound), C <= 512, N a multiple of 16, the same operand and
// epilogue conditions as stream1x1 (igemm's knob s1x1_small, 0 = off)
bool s1x1_small_applicable(int dtype, const IgArgs& a) {
  if (dtype != UM_BF16 || a.R != 1 || a.Rx != 1 || a.stride != 1 || a.pad != 0 ||
      a.padx != 0 || a.cls || a.border || a.pmode != IG_PAD_ZERO || a.oh != a.ah || a.ow != a.aw)
    return false;
  // NC <= 512: wider outputs (the attention's fused 768/1536-channel K/Q/V)
  // re-stage their weights once per 64 pixels and measured slower than the
  // GEMM tiles (tools/conv_table.py, 16 -> 25 us)
  if (a.M >= 16384 || a.M < 256 || a.ach % 8 || a.lda % 8 || a.ld_out % 8 || a.NC % 16 ||
      a.NC > 512)
    return false;
  if (small_ks(a.ach) == 0) return false;
  auto al = [](const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; };
  if (!al(a.a, 16) || !al(a.b, 16) || !al(a.out, a.out_f32 ? 16 : 8) ||
      (a.residual != nullptr && !al(a.residual, 8)))
    return false;
  if (a.epilogue == UM_EPI_NONE) return true;
  if (a.epilogue == UM_EPI_RESIDUAL) return !a.out_f32 && a.ldr % 4 == 0 && a.residual != nullptr;
  if (a.epilogue == UM_EPI_STATS) return a.stat_slots && a.out_f32 && a.stats != nullptr;
  return false;
}

int s1x1_small_run(const IgArgs& a, hipStream_t st) {
  const int ks = small_ks(a.ach);
  const long nstrips = ((long)a.M + 15) / 16;
  const int nb = a.NC / 16;
  // 4 output blocks (64 channels) per workgroup, 2 when that leaves < 256
  // workgroups; strips: one per wave while the grid stays <= 1024 workgroups
  // (KS = 16 keeps two: 16 activation fragments + 4 weight blocks exceed the
  // register file at one wave per SIMD)
  const int ng = (ks < 16 && (long)ceil_div(nstrips, 4) * ceil_div(nb, 4) >= 256) ? 4 : 2;
  const int gy = ceil_div(nb, ng);
  const long gx = std::max<long>(1, std::min<long>(ceil_div(nstrips, 4), std::max<long>(1, 1024 / gy)));
  const size_t lds = (size_t)ks * ng * 16 * 32 * sizeof(bf16_t);
  const bool stats = a.epilogue == UM_EPI_STATS;
#define UM_S1S(KS_, NG_, F32_, ST_)                                                               \
  hipLaunchKernelGGL((s1x1_small_kernel<KS_, NG_, F32_, ST_>), dim3((int)gx, gy), dim3(256), lds, st, \
                     a, nstrips)
#define UM_S1SK(NG_, F32_, ST_)                    \
  switch (ks) {                                    \
    case 1: UM_S1S(1, NG_, F32_, ST_); break;      \
    case 2: UM_S1S(2, NG_, F32_, ST_); break;      \
    case 4: UM_S1S(4, NG_, F32_, ST_); break;      \
    case 8: UM_S1S(8, NG_, F32_, ST_); break;      \
    default: UM_S1S(16, NG_, F32_, ST_); break;    \
  }
#define UM_S1SN(F32_, ST_)              \
  if (ng == 4) { UM_S1SK(4, F32_, ST_) } \
  else { UM_S1SK(2, F32_, ST_) }
  if (stats) {
    UM_S1SN(true, true)
  } else if (a.out_f32) {
    UM_S1SN(true, false)
  } else {
    UM_S1SN(false, false)
  }
#undef UM_S1SN
#undef UM_S1SK
#undef UM_S1S
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int stream1x1_run(const IgArgs& a, hipStream_t st) {
  const int nb = a.NC / 16, ks = s1x1_ks(a.ach);
  const long nstrips = ((long)a.M + 15) / 16;
  const long want = (nstrips + 4 * S1U - 1) / (4 * S1U);
  const int grid = (int)std::min<long>(want, 2048);
  const size_t lds = (size_t)ks * nb * 16 * 32 * sizeof(bf16_t);
  const bool stats = a.epilogue == UM_EPI_STATS;
#define UM_S1(KS_, F32_, ST_)                                                               \
  hipLaunchKernelGGL((stream1x1_kernel<KS_, F32_, ST_>), dim3(grid), dim3(256), lds, st, a, nb, \
                     nstrips)
#define UM_S1K(F32_, ST_)                     \
  switch (ks) {                               \
    case 1: UM_S1(1, F32_, ST_); break;       \
    case 2: UM_S1(2, F32_, ST_); break;       \
    case 4: UM_S1(4, F32_, ST_); break;       \
    default: UM_S1(8, F32_, ST_); break;      \
  }
  if (stats) {
    UM_S1K(true, true)
  } else if (a.out_f32) {
    UM_S1K(true, false)
  } else {
    UM_S1K(false, false)
  }
#undef UM_S1K
#undef UM_S1
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // namespace umamd
