// Training-mode BatchNorm2d + ELU for NHWC activations, split in the phases a
// data-parallel (SyncBN) step needs:
//   forward : conv epilogue partial sums -> um_bn_stats_reduce (f64 per channel)
//             -> [optional all-reduce by the host over RCCL]
//             -> um_bn_coeffs (mean/invstd/scale/shift + running-stat update)
//             -> um_bn_elu_fwd (a = ELU(y*scale + shift)), or fused consumers
//   backward: um_bn_elu_bwd_reduce (sum dz, sum dz*xhat) -> um_bn_stats_reduce
//             -> [all-reduce] -> um_bn_bwd_coeffs (dgamma/dbeta/conv dbias + dx coeffs)
//             -> um_bn_elu_bwd_apply (dy)
// The pre-BN conv output y is always f32 (also in bf16 mode): BN subtracts a
// batch mean that can be much larger than the batch std, so a bf16 y would
// amplify its rounding error by mean/std (measured 4e-2 after one node,
// 40 % after a stage).  a / da / dy use the activation dtype.
// Semantics follow torch.nn.BatchNorm2d (reference model/layers/encoder.py:43,
// model/layers/decoder.py:82): biased variance for normalisation, unbiased
// for running_var, eps 1e-5, momentum 0.1.  ELU alpha = 1 (nn.ELU, reference
// model/layers/encoder.py:44, decoder.py:84).
#include <cstdlib>

#include "common.h"

namespace {

__global__ void coeffs_kernel(const double* __restrict__ st, double count, int C,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              float eps, float momentum, float* running_mean, float* running_var,
                              long long* nbt, float* __restrict__ mean_out,
                              float* __restrict__ invstd_out, float* __restrict__ scale_out,
                              float* __restrict__ shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt != nullptr) *nbt += 1;
  if (c >= C) return;
  // count <= 0: the element count rides in the all-reduced buffer after the
  // C channel pairs (SyncBN with per-rank batch sizes, no host sync)
  if (count <= 0) count = st[2 * C];
  const double mean = st[2 * c] / count;
  double var = st[2 * c + 1] / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  scale_out[c] = g * invstd;
  shift_out[c] = b - (float)mean * g * invstd;
  if (running_mean != nullptr) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
}

// RowMap layout (as the backward kernels): a thread owns 8 channels, keeps
// their scale/shift in registers and walks rows of its block's row chunk.
// pool (optional): per-block channel sums of the stored a, [blocks][C] --
// the SE squeeze of reference decoder.py:124-136 (a block's rows lie in one
// image: rows_per_block divides HW), finished by um_se_mlp_fwd.
// Forward coefficients from the f64 statistics slots (UM_EPI_STAT_SLOTS):
// every workgroup derives scale/shift for all C channels into LDS from the
// same slot sums (so all of them agree bit for bit), workgroup 0 also
// publishes mean/invstd/scale/shift and updates the running statistics --
// the COLRED_BN_FWD finish of reduce.hip without its launch.
struct FwdFin {
  const double* slots;  // null: scale/shift are given
  double count;
  const float *gamma, *beta;
  float eps, momentum;
  float *running_mean, *running_var;
  long long* nbt;
  float *mean, *invstd, *scale, *shift;
};

// s_sc / s_sh hold channels [c0, c0 + n) (this block's slice) at [c - c0]
__device__ __forceinline__ void fwd_fin_coeffs(const FwdFin& f, int C, int c0, int n, float* s_sc,
                                               float* s_sh) {
  const bool pub = blockIdx.x == 0;  // the first row block of every channel slice
  // count <= 0: the element count follows the slots (SyncBN: all-reduced with them)
  const double count = f.count > 0 ? f.count : f.slots[(long)UM_STAT_SLOTS * C * 2];
  stat_slots_finish(f.slots, C, c0, n, [&](int c, double s0, double s1) {
    const double mean = s0 / count;
    double var = s1 / count - mean * mean;
    if (var < 0) var = 0;
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    const float g = f.gamma ? f.gamma[c] : 1.f, b = f.beta ? f.beta[c] : 0.f;
    const float sc = g * invstd, sh = b - (float)mean * g * invstd;
    s_sc[c - c0] = sc;
    s_sh[c - c0] = sh;
    if (pub) {
      f.mean[c] = (float)mean;
      f.invstd[c] = invstd;
      f.scale[c] = sc;
      f.shift[c] = sh;
      const float tmean = (float)mean;
      if (f.running_mean != nullptr) {
        const double unb = count > 1 ? var * count / (count - 1) : var;
        f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * tmean;
        f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unb;
      }
    }
  });
  if (pub && blockIdx.y == 0 && threadIdx.x == 0 && f.nbt != nullptr) *f.nbt += 1;
  __syncthreads();
}

// Optional fused NodeBlock merge of the NEXT graph node (reference
// model/layers/encoder.py:115-124, F3 weight map): when this layer is the
// last-computed predecessor of node s, the apply pass also writes
// out = sum_i sigmoid(w[widx[i]]) * src_i with src_self = the a it just
// stored (bf16-rounded as stored), reading the other predecessors' outputs
// ([M][ld] like a) -- the separate merge launch and its re-read of a go away.
constexpr int FMERGE_MAX = 8;
struct MergeOut {
  int n, self;  // n == 0: no merge
  const void* src[FMERGE_MAX];
  int widx[FMERGE_MAX];
  const float* w;
  void* out;
};

// Channel slices (grid.y): block (x, y) owns rows [x*rows, (x+1)*rows) and
// channels [y*cs, (y+1)*cs).  The small deep layers (M of 1k..16k rows, C of
// 128..512) are sliced so a block finishes only its channels' statistics
// slots (16 KB instead of up to 128 KB per block) and the grid still has a
// few hundred blocks; wide layers keep one slice (cs = C).
// MERGE: the fused-merge instance (its register footprint, ~200 VGPRs with
// up to 8 sources, stays out of the plain instance's ~94)
template <typename T, bool MERGE, typename TY>
__global__ void __launch_bounds__(256) bn_elu_fwd_kernel(
    const TY* __restrict__ y, int ldy, long M, int C, const float* __restrict__ scale,
    const float* __restrict__ shift, T* __restrict__ a, int lda, int apply_elu,
    int rows_per_block, float* __restrict__ pool, FwdFin fin, int cs, MergeOut mo) {
  extern __shared__ float red[];  // [256][8] when pooling, then [2][cs] coefficients (fin)
  const int cb = blockIdx.y * cs;  // this block's channel slice
  const int cg = cs / 8;
  const RowMap rm(cg);
  const long m0 = (long)blockIdx.x * rows_per_block;
  const long m1 = min(M, m0 + rows_per_block);
  int coff = cb;  // index of channel cb in scale / shift
  if (fin.slots != nullptr) {
    float* s_sc = red + (pool ? 256 * 8 : 0);
    fwd_fin_coeffs(fin, C, cb, cs, s_sc, s_sc + cs);
    scale = s_sc;
    shift = s_sc + cs;
    coff = 0;
  }
  float mc[FMERGE_MAX];  // merge coefficients (uniform; unrolled static indices)
#pragma unroll
  for (int i = 0; i < FMERGE_MAX; ++i)
    mc[i] = MERGE && i < mo.n ? sigmoidf_(mo.w[mo.widx[i]]) : 0.f;
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float ps[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && g < cg) {
      const int c = cb + g * 8;
      float sc[8], sh[8];
      load8(scale + coff + g * 8, sc);
      load8(shift + coff + g * 8, sh);
      auto row = [&](long m, float* v) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float z = v[e] * sc[e] + sh[e];
          v[e] = apply_elu ? eluf_(z) : z;
        }
        store8(a + m * lda + c, v);
        if (pool || MERGE) {
          float r[8];
          load8_rounded(v, r, a);
          if (pool)
#pragma unroll
            for (int e = 0; e < 8; ++e) ps[e] += r[e];
          if constexpr (MERGE) {  // the merge in source order, as merge_fwd_kernel
            float acc[8], sv[8];
#pragma unroll
            for (int i = 0; i < FMERGE_MAX; ++i) {
              if (i >= mo.n) break;
              if (i == mo.self) {
#pragma unroll
                for (int e = 0; e < 8; ++e) sv[e] = r[e];
              } else {
                load8(reinterpret_cast<const T*>(mo.src[i]) + m * lda + c, sv);
              }
              if (i == 0) {
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] = sv[e] * mc[0];
              } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] += mc[i] * sv[e];
              }
            }
            store8(reinterpret_cast<T*>(mo.out) + m * lda + c, acc);
          }
        }
      };
      if constexpr (MERGE) {
        for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
          float v[8];
          load8(y + m * ldy + c, v);
          row(m, v);
        }
      } else {
#pragma unroll 4
        for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
          float v[8];
          load8(y + m * ldy + c, v);
          row(m, v);
        }
      }
    }
    if (pool) {
      lane_reduce<8>(red, rm, ps);
      if (rm.lane == 0 && g < cg) store8(pool + (long)blockIdx.x * C + cb + g * 8, ps);
    }
  }
}

// rows per backward block: the row-chunk sizing of common.h (about 512
// blocks, 16..max rows) with the cap as a tuning key (bn_bwd_rows_max,
// default 1024 = rows_per_part)
static int bn_bwd_rows(long M) {
  static const int cap = (int)umamd::tuning_env("bn_bwd_rows_max", 1024);
  const long r = (M + 511) / 512;
  int p = 16;
  while (p < r && p < cap) p <<= 1;
  return p;
}

// rows per forward block: ~2048 blocks over the chip, >= 16 rows each; with
// SE pooling a divisor of HW, so no block straddles two images
inline int fwd_rows(long M, long HW) {
  long r = (M + 2047) / 2048;
  if (r < 16) r = 16;
  if (HW > 0) {
    if (r > HW) r = HW;
    while (HW % r) --r;
  }
  return (int)r;
}

// Backward reduce: dz = (da + add[n][c]) * ELU'(z), z = y*scale + shift,
// xhat = (y - mean) * invstd; partial sums per block [blk][C][2].
template <typename T, typename TY>
__global__ void __launch_bounds__(256) bn_elu_bwd_reduce_kernel(
    const T* __restrict__ da, int ldda, const TY* __restrict__ y, int ldy, long M, int C,
    long HW, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ add_nc, int apply_elu, float* __restrict__ parts,
    int rows_per_block, double* __restrict__ slots, int cs) {
  extern __shared__ float red[];  // [256][16]
  const int cb = blockIdx.y * cs;  // channel slice (see bn_elu_fwd_kernel)
  const int cg = cs / 8;
  const RowMap rm(cg);
  const long m0 = (long)blockIdx.x * rows_per_block;
  const long m1 = min(M, m0 + rows_per_block);
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (rm.active() && g < cg) {
      const int c = cb + g * 8;
      float mu[8], is[8], sc[8], sh[8];
      load8(mean + c, mu);
      load8(invstd + c, is);
      load8(scale + c, sc);
      load8(shift + c, sh);
      // SE layers: add[n][c] (n = m / HW) is one vector for a block inside one
      // image (the row blocks are 16..1024 rows, the images 1k..128k pixels):
      // loaded once, no per-row 64-bit division and table load
      const bool one_img = add_nc && m0 / HW == (m1 - 1) / HW;
      float ad0[8];
      if (one_img) load8(add_nc + (m0 / HW) * C + c, ad0);
      auto row = [&](long m, const float* ad) {
        float dv[8], yv[8];
        load8(da + m * ldda + c, dv);
        load8(y + m * ldy + c, yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = dv[e] + (ad ? ad[e] : 0.f);
          if (apply_elu) {
            const float z = yv[e] * sc[e] + sh[e];
            d = z > 0.f ? d : d * __expf(z);
          }
          acc[e] += d;
          acc[8 + e] += d * (yv[e] - mu[e]) * is[e];
        }
      };
      if (!add_nc || one_img) {
#pragma unroll 4
        for (long m = m0 + rm.lane; m < m1; m += rm.lanes) row(m, add_nc ? ad0 : nullptr);
      } else {
#pragma unroll 2
        for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
          float ad[8];
          load8(add_nc + (m / HW) * C + c, ad);
          row(m, ad);
        }
      }
    }
    lane_reduce<16>(red, rm, acc);
    if (slots != nullptr) {  // stage [8G channels][2] in LDS, then contiguous f64 atomics
      if (g0 == 0) stat_slots_count(slots, C, M);
      if (rm.lane == 0 && g < cg)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[(rm.g * 8 + e) * 2] = acc[e];
          red[(rm.g * 8 + e) * 2 + 1] = acc[8 + e];
        }
      __syncthreads();
      stat_slots_add_row(slots, blockIdx.x, C, cb + g0 * 8, min(rm.G * 8, cs - g0 * 8),
                         [&](int i) { return red[i]; });
      __syncthreads();
    } else if (rm.lane == 0 && g < cg) {
      {
        float* o = parts + ((long)blockIdx.x * C + cb + g * 8) * 2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[2 * e] = acc[e];
          o[2 * e + 1] = acc[8 + e];
        }
      }
    }
  }
}

__global__ void bwd_coeffs_kernel(const double* __restrict__ st, double count, int C,
                                  const float* __restrict__ gamma,
                                  const float* __restrict__ invstd,
                                  const double* __restrict__ st_local, float* dgamma,
                                  float* dbeta, float* dbias, float dbias_scale, int accumulate,
                                  float* __restrict__ k1, float* __restrict__ k2,
                                  float* __restrict__ k3) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (count <= 0) count = st[2 * C];  // all-reduced element count (see coeffs_kernel)
  const double sdz = st[2 * c], sdzx = st[2 * c + 1];
  const float g = gamma ? gamma[c] : 1.f;
  // dx = g*invstd*(dz - sdz/n - xhat*sdzx/n)
  const float a1 = g * invstd[c], a2 = (float)(sdz / count);
  k1[c] = a1;
  k2[c] = a2;
  k3[c] = (float)(sdzx / count);
  // conv-bias gradient: sum_m dy = k1 (sdz - n k2 - k3 sum xhat), sum xhat = 0
  // (global sums; dbias_scale spreads it over the ranks' gradient average)
  if (dbias) dbias[c] = dbias_scale * a1 * (float)(sdz - count * (double)a2);
  // parameter grads use the local (per-rank) sums, like torch SyncBatchNorm
  const double* sl = st_local ? st_local : st;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)sl[2 * c + 1];
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)sl[2 * c];
}

// Backward coefficients from the f64 slots of bn_elu_bwd_reduce (as
// COLRED_BN_BWD in reduce.hip): every workgroup derives k1..k3 into LDS,
// workgroup 0 writes dgamma, dbeta and the closed-form conv-bias gradient.
struct ApplyFin {
  const double* slots;  // null: k1..k3 are given
  double count;         // <= 0: read after the slots (SyncBN)
  const float* gamma;
  float *dgamma, *dbeta, *dbias;
  const double* local;  // SyncBN: this rank's slots before the all-reduce (dgamma/dbeta),
                        // or null: dgamma/dbeta from the global sums x dbias_scale
  float dbias_scale;    // SyncBN: 1/world (DDP averages the ranks' bias gradients)
};

// s_k1..s_k3 hold channels [c0, c0 + n) at [c - c0]
__device__ __forceinline__ void apply_fin_coeffs(const ApplyFin& f, int C, int c0, int n,
                                                 const float* __restrict__ invstd, float* s_k1,
                                                 float* s_k2, float* s_k3) {
  const bool pub = blockIdx.x == 0;  // the first row block of every channel slice
  const double count = f.count > 0 ? f.count : f.slots[(long)UM_STAT_SLOTS * C * 2];
  stat_slots_finish(f.slots, C, c0, n, [&](int c, double s0, double s1) {
    const float g = f.gamma ? f.gamma[c] : 1.f;
    const float a1 = g * invstd[c], a2 = (float)(s0 / count);
    s_k1[c - c0] = a1;
    s_k2[c - c0] = a2;
    s_k3[c - c0] = (float)(s1 / count);
    if (pub) {
      if (f.local == nullptr) {
        // SyncBN without the local copy: the global sums / world.  DDP
        // averages the ranks' gradients, so the result equals the average of
        // the per-rank sums torch SyncBatchNorm uses (dbias_scale = 1 alone)
        if (f.dgamma) f.dgamma[c] = f.dbias_scale * (float)s1;
        if (f.dbeta) f.dbeta[c] = f.dbias_scale * (float)s0;
      }
      // conv-bias gradient sum_m dy = k1 (s0 - n k2 - k3 sum xhat), sum xhat = 0
      // (global sums; dbias_scale spreads it over the ranks' gradient average)
      if (f.dbias) f.dbias[c] = f.dbias_scale * a1 * (float)(s0 - count * (double)a2);
    }
  });
  // parameter grads from this rank's sums, like torch SyncBatchNorm
  if (pub && f.local != nullptr)
    stat_slots_finish(f.local, C, c0, n, [&](int c, double s0, double s1) {
      if (f.dgamma) f.dgamma[c] = (float)s1;
      if (f.dbeta) f.dbeta[c] = (float)s0;
    });
  __syncthreads();
}

// dy = k1*(dz - k2 - xhat*k3); optional per-block partial sums of dy
// ([blk][C], the conv-bias gradient) written to sum_parts.
template <typename T, typename TY>
__global__ void __launch_bounds__(256) bn_elu_bwd_apply_kernel(
    const T* __restrict__ da, int ldda, const TY* __restrict__ y, int ldy, long M, int C,
    long HW, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ add_nc, int apply_elu, const float* __restrict__ k1,
    const float* __restrict__ k2, const float* __restrict__ k3, T* __restrict__ dy, int lddy,
    float* __restrict__ sum_parts, int rows_per_block, ApplyFin fin, int cs) {
  extern __shared__ float red[];  // [256][8], then [3][cs] coefficients (fin)
  const int cb = blockIdx.y * cs;  // channel slice (see bn_elu_fwd_kernel)
  const int cg = cs / 8;
  const RowMap rm(cg);
  const long m0 = (long)blockIdx.x * rows_per_block;
  const long m1 = min(M, m0 + rows_per_block);
  int koff = cb;  // index of channel cb in k1..k3
  if (fin.slots != nullptr) {
    float* s_k = red + 256 * 8;
    apply_fin_coeffs(fin, C, cb, cs, invstd, s_k, s_k + cs, s_k + 2 * cs);
    k1 = s_k;
    k2 = s_k + cs;
    k3 = s_k + 2 * cs;
    koff = 0;
  }
  for (int g0 = 0; g0 < cg; g0 += rm.G) {
    const int g = g0 + rm.g;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rm.active() && g < cg) {
      const int c = cb + g * 8;
      // dy = A*dz + B*y + D  with A = k1, B = -k1*k3*invstd, D = -k1*k2 + k1*k3*mean*invstd
      float sc[8], sh[8], A[8], B[8], D[8];
      {
        float mu[8], is[8], a1[8], a2[8], a3[8];
        load8(mean + c, mu);
        load8(invstd + c, is);
        load8(k1 + koff + g * 8, a1);
        load8(k2 + koff + g * 8, a2);
        load8(k3 + koff + g * 8, a3);
        load8(scale + c, sc);
        load8(shift + c, sh);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          A[e] = a1[e];
          B[e] = -a1[e] * a3[e] * is[e];
          D[e] = -a1[e] * a2[e] + a1[e] * a3[e] * mu[e] * is[e];
        }
      }
      // SE add vector hoisted for a block inside one image (as the reduce)
      const bool one_img = add_nc && m0 / HW == (m1 - 1) / HW;
      float ad0[8];
      if (one_img) load8(add_nc + (m0 / HW) * C + c, ad0);
      auto row = [&](long m, const float* dv, const float* yv) {
        float ad[8], o[8];
        if (one_img) {
#pragma unroll
          for (int e = 0; e < 8; ++e) ad[e] = ad0[e];
        } else if (add_nc) {
          load8(add_nc + (m / HW) * C + c, ad);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = dv[e] + (add_nc ? ad[e] : 0.f);
          if (apply_elu) {
            const float z = yv[e] * sc[e] + sh[e];
            d = z > 0.f ? d : d * __expf(z);
          }
          o[e] = A[e] * d + B[e] * yv[e] + D[e];
        }
        store8(dy + m * lddy + c, o);
        if (sum_parts) {
          float r[8];
          load8_rounded(o, r, dy);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += r[e];
        }
      };
#pragma unroll 4
      for (long m = m0 + rm.lane; m < m1; m += rm.lanes) {
        float dv[8], yv[8];
        load8(da + m * ldda + c, dv);
        load8(y + m * ldy + c, yv);
        row(m, dv, yv);
      }
    }
    if (sum_parts) {
      lane_reduce<8>(red, rm, acc);
      if (rm.lane == 0 && g < cg) store8(sum_parts + (long)blockIdx.x * C + cb + g * 8, acc);
    }
  }
}

}  // namespace

extern "C" {

int um_bn_coeffs(const double* stats, double count, int C, const float* gamma, const float* beta,
                 float eps, float momentum, float* running_mean, float* running_var,
                 long long* num_batches_tracked, float* mean, float* invstd, float* scale,
                 float* shift, hipStream_t st) {
  hipLaunchKernelGGL(coeffs_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, st, stats, count, C,
                     gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked,
                     mean, invstd, scale, shift);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"

namespace {
// Channel-slice plan of the three BN passes: small layers (M * C up to 8M
// elements) with C >= 128 take 64-channel slices (tuning key bn_slice = 0 turns
// it off) and rows such that the grid has ~512 blocks (>= 32 rows: the 32
// row lanes of a 64-channel block).
struct Slices {
  int cs, ns;
};
Slices bn_slices(long M, int C) {
  static const int on = (int)umamd::tuning_env("bn_slice", 1);
  if (!on || C < 128 || C % 64 || M * C > (8l << 20)) return {C, 1};
  return {64, C / 64};
}
int sliced_rows(long M, long HW, int ns) {
  const long target = (512 + ns - 1) / ns;  // row blocks
  long r = (M + target - 1) / target;
  int p = 32;
  while (p < r) p <<= 1;
  long rr = p;
  if (HW > 0) {
    if (rr > HW) rr = HW;
    while (HW % rr) --rr;
  }
  return (int)rr;
}
int fwd_rows_c(long M, long HW, int C) {
  const Slices s = bn_slices(M, C);
  return s.ns > 1 ? sliced_rows(M, HW, s.ns) : fwd_rows(M, HW);
}
int bwd_rows_c(long M, int C) {
  const Slices s = bn_slices(M, C);
  return s.ns > 1 ? sliced_rows(M, 0, s.ns) : bn_bwd_rows(M);
}
}  // namespace

extern "C" {

int um_bn_fwd_pool_parts(long M, long HW) {
  return HW > 0 && M % HW == 0 ? (int)(M / fwd_rows(M, HW)) : 0;
}

int um_bn_fwd_pool_parts_c(long M, long HW, int C) {
  return HW > 0 && M % HW == 0 ? (int)(M / fwd_rows_c(M, HW, C)) : 0;
}

static int bn_fwd_launch(int dtype, long M, int C, const void* y, int ldy, const float* scale,
                         const float* shift, void* a, int lda, int apply_elu, long HW,
                         float* pool_parts, const FwdFin& fin, hipStream_t st,
                         const MergeOut& mo = MergeOut{}) {
  UM_CHECK_ARG(C % 8 == 0 && ldy % 8 == 0 && lda % 8 == 0, "um_bn_elu_fwd: C/ld not multiple of 8");
  UM_CHECK_ARG(pool_parts == nullptr || (HW > 0 && M % HW == 0), "um_bn_elu_fwd: HW");
  const Slices sl = bn_slices(M, C);
  const int rows = fwd_rows_c(M, pool_parts ? HW : 0, C);
  const dim3 g(ceil_div(M, rows), sl.ns);
  const size_t shm = (pool_parts ? 256 * 8 * sizeof(float) : 0) +
                     (fin.slots ? 2 * (size_t)sl.cs * sizeof(float) : 0);
  const bool yact = dtype & UM_Y_ACT;
  dtype &= ~UM_Y_ACT;
#define UM_BN_FWD(T_, MG_, TY_)                                                            \
  hipLaunchKernelGGL((bn_elu_fwd_kernel<T_, MG_, TY_>), g, dim3(256), shm, st, (const TY_*)y, \
                     ldy, M, C, scale, shift, (T_*)a, lda, apply_elu, rows, pool_parts, fin,   \
                     sl.cs, mo)
  if (dtype == UM_BF16 && yact) {
    if (mo.n) UM_BN_FWD(bf16_t, true, bf16_t); else UM_BN_FWD(bf16_t, false, bf16_t);
  } else if (dtype == UM_BF16) {
    if (mo.n) UM_BN_FWD(bf16_t, true, float); else UM_BN_FWD(bf16_t, false, float);
  } else {
    if (mo.n) UM_BN_FWD(float, true, float); else UM_BN_FWD(float, false, float);
  }
#undef UM_BN_FWD
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_bn_elu_fwd(int dtype, long M, int C, const void* y, int ldy, const float* scale,
                  const float* shift, void* a, int lda, int apply_elu, long HW, float* pool_parts,
                  hipStream_t st) {
  FwdFin fin{};
  return bn_fwd_launch(dtype, M, C, y, ldy, scale, shift, a, lda, apply_elu, HW, pool_parts, fin, st);
}

int um_bn_elu_fwd_slots(int dtype, long M, int C, const void* y, int ldy, const double* slots,
                        double count, const float* gamma, const float* beta, float eps,
                        float momentum, float* running_mean, float* running_var,
                        long long* num_batches_tracked, float* mean, float* invstd, float* scale,
                        float* shift, void* a, int lda, int apply_elu, long HW, float* pool_parts,
                        hipStream_t st) {
  UM_CHECK_ARG(slots != nullptr && mean && invstd && scale && shift,
               "um_bn_elu_fwd_slots: slots / coefficient outputs");
  FwdFin fin{};
  fin.slots = slots; fin.count = count; fin.gamma = gamma; fin.beta = beta;
  fin.eps = eps; fin.momentum = momentum;
  fin.running_mean = running_mean; fin.running_var = running_var; fin.nbt = num_batches_tracked;
  fin.mean = mean; fin.invstd = invstd; fin.scale = scale; fin.shift = shift;
  return bn_fwd_launch(dtype, M, C, y, ldy, nullptr, nullptr, a, lda, apply_elu, HW, pool_parts,
                       fin, st);
}

int um_bn_elu_fwd_slots_merge(int dtype, long M, int C, const void* y, int ldy,
                              const double* slots, double count, const float* gamma,
                              const float* beta, float eps, float momentum, float* running_mean,
                              float* running_var, long long* num_batches_tracked, float* mean,
                              float* invstd, float* scale, float* shift, void* a, int lda,
                              int apply_elu, int nsrc, const void* const* srcs, const int* widx,
                              const float* w, int self, void* merged, hipStream_t st) {
  UM_CHECK_ARG(slots != nullptr && mean && invstd && scale && shift,
               "um_bn_elu_fwd_slots_merge: slots / coefficient outputs");
  UM_CHECK_ARG(nsrc >= 2 && nsrc <= FMERGE_MAX && self >= 0 && self < nsrc && srcs && widx &&
                   w && merged,
               "um_bn_elu_fwd_slots_merge: merge sources");
  FwdFin fin{};
  fin.slots = slots; fin.count = count; fin.gamma = gamma; fin.beta = beta;
  fin.eps = eps; fin.momentum = momentum;
  fin.running_mean = running_mean; fin.running_var = running_var; fin.nbt = num_batches_tracked;
  fin.mean = mean; fin.invstd = invstd; fin.scale = scale; fin.shift = shift;
  MergeOut mo{};
  mo.n = nsrc;
  mo.self = self;
  for (int i = 0; i < nsrc; ++i) {
    UM_CHECK_ARG(i == self || srcs[i] != nullptr, "um_bn_elu_fwd_slots_merge: null source");
    mo.src[i] = srcs[i];
    mo.widx[i] = widx[i];
  }
  mo.w = w;
  mo.out = merged;
  return bn_fwd_launch(dtype, M, C, y, ldy, nullptr, nullptr, a, lda, apply_elu, 0, nullptr, fin,
                       st, mo);
}

int um_bn_bwd_parts(long M) { return ceil_div(M, bn_bwd_rows(M)); }

static int bwd_reduce_launch(int dtype, long M, int C, long HW, const void* da, int ldda,
                             const void* y, int ldy, const float* mean, const float* invstd,
                             const float* scale, const float* shift, const float* add_nc,
                             int apply_elu, float* parts, double* slots,
                             hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0, "um_bn_elu_bwd_reduce: C %% 8");
  // channel slices only where the statistics go to slots (the partial rows
  // of the other paths are sized by um_bn_bwd_parts)
  const Slices sl = slots != nullptr ? bn_slices(M, C) : Slices{C, 1};
  const int rows = sl.ns > 1 ? bwd_rows_c(M, C) : bn_bwd_rows(M);
  const dim3 blocks(ceil_div(M, rows), sl.ns);
  const size_t shm = 256 * 16 * sizeof(float);
#define UM_BN_RED(T_, TY_)                                                                   \
  hipLaunchKernelGGL((bn_elu_bwd_reduce_kernel<T_, TY_>), blocks, dim3(256), shm, st,        \
                     (const T_*)da, ldda, (const TY_*)y, ldy, M, C, HW, mean, invstd, scale, \
                     shift, add_nc, apply_elu, parts, rows, slots, sl.cs)
  if (dtype == (UM_BF16 | UM_Y_ACT)) UM_BN_RED(bf16_t, bf16_t);
  else if (dtype == UM_BF16) UM_BN_RED(bf16_t, float);
  else UM_BN_RED(float, float);
#undef UM_BN_RED
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_bn_elu_bwd_reduce(int dtype, long M, int C, long HW, const void* da, int ldda,
                         const void* y, int ldy, const float* mean, const float* invstd,
                         const float* scale, const float* shift, const float* add_nc,
                         int apply_elu, float* parts, hipStream_t st) {
  return bwd_reduce_launch(dtype, M, C, HW, da, ldda, y, ldy, mean, invstd, scale, shift, add_nc,
                           apply_elu, parts, nullptr, st);
}

int um_bn_elu_bwd_reduce_slots(int dtype, long M, int C, long HW, const void* da, int ldda,
                               const void* y, int ldy, const float* mean, const float* invstd,
                               const float* scale, const float* shift, const float* add_nc,
                               int apply_elu, double* slots, hipStream_t st) {
  UM_CHECK_ARG(slots != nullptr, "um_bn_elu_bwd_reduce_slots: slots");
  return bwd_reduce_launch(dtype, M, C, HW, da, ldda, y, ldy, mean, invstd, scale, shift, add_nc,
                           apply_elu, nullptr, slots, st);
}

int um_bn_bwd_coeffs(const double* stats, double count, int C, const float* gamma,
                     const float* invstd, const double* stats_local, float* dgamma, float* dbeta,
                     float* dbias, float dbias_scale, int accumulate, float* k1, float* k2,
                     float* k3, hipStream_t st) {
  hipLaunchKernelGGL(bwd_coeffs_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, st, stats, count, C,
                     gamma, invstd, stats_local, dgamma, dbeta, dbias, dbias_scale, accumulate, k1,
                     k2, k3);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

static int bwd_apply_launch(int dtype, long M, int C, long HW, const void* da, int ldda,
                            const void* y, int ldy, const float* mean, const float* invstd,
                            const float* scale, const float* shift, const float* add_nc,
                            int apply_elu, const float* k1, const float* k2, const float* k3,
                            void* dy, int lddy, float* sum_parts, const ApplyFin& fin,
                            hipStream_t st) {
  UM_CHECK_ARG(C % 8 == 0, "um_bn_elu_bwd_apply: C %% 8");
  const Slices sl = (fin.slots != nullptr && sum_parts == nullptr) ? bn_slices(M, C) : Slices{C, 1};
  const int rows = sl.ns > 1 ? bwd_rows_c(M, C) : bn_bwd_rows(M);
  const dim3 blocks(ceil_div(M, rows), sl.ns);
  const size_t shm = 256 * 8 * sizeof(float) + (fin.slots ? 3 * (size_t)sl.cs * sizeof(float) : 0);
#define UM_BN_APPLY(T_, TY_)                                                                 \
  hipLaunchKernelGGL((bn_elu_bwd_apply_kernel<T_, TY_>), blocks, dim3(256), shm, st,         \
                     (const T_*)da, ldda, (const TY_*)y, ldy, M, C, HW, mean, invstd, scale, \
                     shift, add_nc, apply_elu, k1, k2, k3, (T_*)dy, lddy, sum_parts, rows, fin, \
                     sl.cs)
  if (dtype == (UM_BF16 | UM_Y_ACT)) UM_BN_APPLY(bf16_t, bf16_t);
  else if (dtype == UM_BF16) UM_BN_APPLY(bf16_t, float);
  else UM_BN_APPLY(float, float);
#undef UM_BN_APPLY
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_bn_elu_bwd_apply(int dtype, long M, int C, long HW, const void* da, int ldda,
                        const void* y, int ldy, const float* mean, const float* invstd,
                        const float* scale, const float* shift, const float* add_nc,
                        int apply_elu, const float* k1, const float* k2, const float* k3,
                        void* dy, int lddy, float* sum_parts, hipStream_t st) {
  ApplyFin fin{};
  return bwd_apply_launch(dtype, M, C, HW, da, ldda, y, ldy, mean, invstd, scale, shift, add_nc,
                          apply_elu, k1, k2, k3, dy, lddy, sum_parts, fin, st);
}

int um_bn_elu_bwd_apply_slots(int dtype, long M, int C, long HW, const void* da, int ldda,
                              const void* y, int ldy, const float* mean, const float* invstd,
                              const float* scale, const float* shift, const float* add_nc,
                              int apply_elu, const double* slots, double count,
                              const double* local_slots, const float* gamma, float* dgamma,
                              float* dbeta, float* dbias, float dbias_scale, void* dy, int lddy,
                              hipStream_t st) {
  UM_CHECK_ARG(slots != nullptr, "um_bn_elu_bwd_apply_slots: slots");
  ApplyFin fin{};
  fin.slots = slots; fin.count = count; fin.gamma = gamma; fin.local = local_slots;
  fin.dgamma = dgamma; fin.dbeta = dbeta; fin.dbias = dbias; fin.dbias_scale = dbias_scale;
  return bwd_apply_launch(dtype, M, C, HW, da, ldda, y, ldy, mean, invstd, scale, shift, add_nc,
                          apply_elu, nullptr, nullptr, nullptr, dy, lddy, nullptr, fin, st);
}

}  // extern "C"
