// Efficient (linear) attention core, reference model/layers/attention.py:42-76.
//
// Layout: qkv[m = n*S + s][ld] holds K in columns [0,C), Q in [C,2C), V in
// [2C,3C) (the three 1x1 convs run as one GEMM).  Heads h own channels
// [h*d, (h+1)*d), d = C / heads.
//   Ks  = softmax over pixels s of K[:, c]            (per n, c)   attention.py:63
//   Qs  = softmax over the head's d channels of Q[s]  (per n, s, h) attention.py:64
//   ctx = Ks_h^T V_h   (d x d per n, h)                             attention.py:66
//   att = Qs_h ctx_h   -> written [m][C]                            attention.py:68-71
// The 1x1 reprojection + residual is a conv epilogue (conv.hip).
// Backward recomputes Ks/Qs from qkv and the saved (kmax, ksum).
#include "common.h"

namespace {

constexpr int PT = 64;         // pixels per apply tile

// ---------------------------------------------------------------- k stats --
// pixels per k-stat partial: at most ~64 chunks per image (16..256 pixels),
// so the small bottleneck maps still spread over the chip
static inline int ks_chunk(int S) {
  int c = 16;
  while (c < 256 && (long)c * 64 < S) c <<= 1;
  return c;
}

// grid (chunk, n, 64-channel group): 4 pixel lanes x 64 channels per block
template <typename T>
__global__ void kstats_kernel(const T* __restrict__ qkv, int ld, int S, int C, int chunk_px,
                              float* __restrict__ parts, int nchunks) {
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int s0 = chunk * chunk_px, s1 = min(S, s0 + chunk_px);
  __shared__ float sm[4][64], ss[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = blockIdx.z * 64 + cl;
  float mx = -INFINITY, sum = 0.f;
  if (c < C) {
    for (int s = s0 + pl; s < s1; s += 4) {
      const float v = to_f32(qkv[((long)n * S + s) * ld + c]);
      if (v > mx) {
        sum = sum * __expf(mx - v) + 1.f;
        mx = v;
      } else {
        sum += __expf(v - mx);
      }
    }
  }
  sm[pl][cl] = mx;
  ss[pl][cl] = sum;
  __syncthreads();
  if (pl == 0 && c < C) {
    float M = sm[0][cl];
    for (int r = 1; r < 4; ++r) M = fmaxf(M, sm[r][cl]);
    float t = 0.f;
    for (int r = 0; r < 4; ++r)
      if (sm[r][cl] > -INFINITY) t += ss[r][cl] * __expf(sm[r][cl] - M);
    float* o = parts + (((long)n * nchunks + chunk) * C + c) * 2;
    o[0] = M;
    o[1] = t;
  }
}

// one wave per (n, c); the lanes stride the chunk partials
__global__ void kstats_combine_kernel(const float* __restrict__ parts, int N, int nchunks, int C,
                                      float* __restrict__ kmax, float* __restrict__ ksum) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= N * C) return;  // wave-uniform
  const int n = i / C, c = i % C;
  float M = -INFINITY;
  for (int k = lane; k < nchunks; k += 64)
    M = fmaxf(M, parts[(((long)n * nchunks + k) * C + c) * 2]);
  M = wave_max(M);
  float t = 0.f;
  for (int k = lane; k < nchunks; k += 64) {
    const float* p = parts + (((long)n * nchunks + k) * C + c) * 2;
    if (p[0] > -INFINITY) t += p[1] * __expf(p[0] - M);
  }
  t = wave_sum(t);
  if (lane == 0) {
    kmax[i] = M;
    ksum[i] = t;
  }
}

// ------------------------------------------------------------------- ctx --
// partial ctx over a pixel chunk: parts[n][chunk][h][d][d]
template <typename T>
__global__ void ctx_kernel(const T* __restrict__ qkv, int ld, int S, int C, int heads,
                           const float* __restrict__ kmax, const float* __restrict__ ksum,
                           int chunk_px, int nchunks, float* __restrict__ parts) {
  extern __shared__ float sh[];
  const int d = C / heads;
  const int chunk = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = chunk * chunk_px, s1 = min(S, s0 + chunk_px);
  const int np = s1 - s0;
  float* sK = sh;                  // [chunk_px][d]
  float* sV = sh + chunk_px * d;   // [chunk_px][d]
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    const long row = ((long)n * S + s0 + s) * ld;
    const int ch = h * d + c;
    sK[i] = __expf(to_f32(qkv[row + ch]) - kmax[n * C + ch]) / ksum[n * C + ch];
    sV[i] = to_f32(qkv[row + 2 * C + ch]);
  }
  __syncthreads();
  const int dd = d * d;
  const int lanes = dd >= 256 ? 1 : 256 / dd;
  float* red = sh + 2 * chunk_px * d;  // [256]
  for (int o0 = 0; o0 < dd; o0 += 256 / lanes) {
    const int o = o0 + threadIdx.x % (256 / lanes);
    const int pl = threadIdx.x / (256 / lanes);
    float acc = 0.f;
    if (o < dd && pl < lanes) {
      const int c = o / d, cp = o % d;
      for (int s = pl; s < np; s += lanes) acc += sK[s * d + c] * sV[s * d + cp];
    }
    if (lanes > 1) {
      red[threadIdx.x] = acc;
      __syncthreads();
      if (pl == 0 && o < dd) {
        float t = 0.f;
        for (int r = 0; r < lanes; ++r) t += red[r * (256 / lanes) + threadIdx.x];
        acc = t;
      }
      __syncthreads();
    }
    if (pl == 0 && o < dd)
      parts[(((long)n * nchunks + chunk) * heads + h) * dd + o] = acc;
  }
}

// out[n][j] = sum_b parts[n][b][j]
// out[n][j] = sum_b parts[n][b][j]: block = (jl columns) x (256/jl b-lanes),
// 4 accumulators per thread, lanes combined in LDS; grid (ceil(L/jl), N)
__global__ void __launch_bounds__(256) sum_parts_kernel(const float* __restrict__ parts, int N,
                                                        int B, int L, float* __restrict__ out,
                                                        int jl) {
  __shared__ float red[256];
  const int lanes = 256 / jl;
  const int n = blockIdx.y;
  const int j = blockIdx.x * jl + (threadIdx.x % jl);
  const int lane = threadIdx.x / jl;
  float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
  if (j < L) {
    const float* p = parts + (long)n * B * L + j;
    int b = lane;
    for (; b + 3 * lanes < B; b += 4 * lanes) {
      t0 += p[(long)b * L];
      t1 += p[(long)(b + lanes) * L];
      t2 += p[(long)(b + 2 * lanes) * L];
      t3 += p[(long)(b + 3 * lanes) * L];
    }
    for (; b < B; b += lanes) t0 += p[(long)b * L];
  }
  float t = (t0 + t1) + (t2 + t3);
  red[threadIdx.x] = t;
  __syncthreads();
  if (lane == 0 && j < L) {
    for (int q = 1; q < lanes; ++q) t += red[q * jl + (threadIdx.x % jl)];
    out[(long)n * L + j] = t;
  }
}

inline int sum_parts_cols(int L, int B) {  // columns per block: leave >= 8 b-lanes
  int jl = 64;
  while (jl > 1 && 256 / jl < 8) jl >>= 1;
  while (jl > 1 && (256 / jl) * 4 < B && jl > 16) jl >>= 1;
  return jl;
}

// ----------------------------------------------------------------- apply --
template <typename T>
__global__ void apply_kernel(const T* __restrict__ qkv, int ld, int S, int C, int heads,
                             const float* __restrict__ ctx, T* __restrict__ att, int ldo) {
  extern __shared__ float sh[];
  const int d = C / heads;
  const int tile = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = tile * PT, np = min(PT, S - s0);
  const int dq = d + 1;      // padded rows: per-pixel loops stay bank-conflict free
  float* sC = sh;            // [d][d]
  float* sQ = sh + d * d;    // [PT][d+1]
  const float* cg = ctx + ((long)n * heads + h) * d * d;
  for (int i = threadIdx.x; i < d * d; i += blockDim.x) sC[i] = cg[i];
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    sQ[s * dq + c] = to_f32(qkv[((long)n * S + s0 + s) * ld + C + h * d + c]);
  }
  __syncthreads();
  if (threadIdx.x < np) {
    float* q = sQ + threadIdx.x * dq;
    float mx = -INFINITY;
    for (int c = 0; c < d; ++c) mx = fmaxf(mx, q[c]);
    float sum = 0.f;
    for (int c = 0; c < d; ++c) {
      q[c] = __expf(q[c] - mx);
      sum += q[c];
    }
    const float inv = 1.f / sum;
    for (int c = 0; c < d; ++c) q[c] *= inv;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, cp = i % d;
    float acc = 0.f;
    for (int c = 0; c < d; ++c) acc += sC[c * d + cp] * sQ[s * dq + c];
    att[((long)n * S + s0 + s) * ldo + h * d + cp] = from_f32<T>(acc);
  }
}

// ------------------------------------------------------------ apply bwd --
// dQ (into dqkv Q slot) and partial dctx per tile: parts[n][tile][h][d][d]
template <typename T>
__global__ void apply_bwd_kernel(const T* __restrict__ qkv, int ld, int S, int C, int heads,
                                 const float* __restrict__ ctx, const T* __restrict__ datt,
                                 int ldd, T* __restrict__ dqkv, int ldq, int ntiles,
                                 float* __restrict__ parts) {
  extern __shared__ float sh[];
  const int d = C / heads;
  const int dq = d + 1;  // padded pixel rows (per-pixel loops conflict free)
  const int tile = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = tile * PT, np = min(PT, S - s0);
  float* sCt = sh;                // ctx^T [d][d]: sCt[cp][c] = ctx[c][cp]
  float* sQ = sCt + d * d;        // [PT][d+1]  softmaxed q
  float* sG = sQ + PT * dq;       // [PT][d+1]  datt
  float* sD = sG + PT * dq;       // [PT][d+1]  dQs
  const float* cg = ctx + ((long)n * heads + h) * d * d;
  for (int i = threadIdx.x; i < d * d; i += blockDim.x) sCt[(i % d) * d + i / d] = cg[i];
  for (int i = threadIdx.x; i < PT * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    if (s < np) {
      const long row = (long)n * S + s0 + s;
      sQ[s * dq + c] = to_f32(qkv[row * ld + C + h * d + c]);
      sG[s * dq + c] = to_f32(datt[row * ldd + h * d + c]);
    } else {
      sQ[s * dq + c] = 0.f;
      sG[s * dq + c] = 0.f;
    }
  }
  __syncthreads();
  if (threadIdx.x < np) {
    float* q = sQ + threadIdx.x * dq;
    float mx = -INFINITY;
    for (int c = 0; c < d; ++c) mx = fmaxf(mx, q[c]);
    float sum = 0.f;
    for (int c = 0; c < d; ++c) {
      q[c] = __expf(q[c] - mx);
      sum += q[c];
    }
    const float inv = 1.f / sum;
    for (int c = 0; c < d; ++c) q[c] *= inv;
  }
  __syncthreads();
  // dQs[s][c] = sum_c' ctx[c][c'] * datt[s][c']
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    float acc = 0.f;
    for (int cp = 0; cp < d; ++cp) acc += sCt[cp * d + c] * sG[s * dq + cp];
    sD[s * dq + c] = acc;
  }
  // dctx partial[c][c'] = sum_s qs[s][c] * datt[s][c']
  float* out = parts + (((long)n * ntiles + tile) * heads + h) * d * d;
  for (int o = threadIdx.x; o < d * d; o += blockDim.x) {
    const int c = o / d, cp = o % d;
    float acc = 0.f;
    for (int s = 0; s < np; ++s) acc += sQ[s * dq + c] * sG[s * dq + cp];
    out[o] = acc;
  }
  __syncthreads();
  // dq = qs * (dQs - <qs, dQs>): thread per (pixel, channel)
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    float dot = 0.f;
    for (int k = 0; k < d; ++k) dot += sQ[s * dq + k] * sD[s * dq + k];
    const long row = (long)n * S + s0 + s;
    dqkv[row * ldq + C + h * d + c] = from_f32<T>(sQ[s * dq + c] * (sD[s * dq + c] - dot));
  }
}

// ---------------------------------------------------------------- kv bwd --
// dV (into dqkv V slot), dKs (f32 scratch [m][C]) and partial r[c] = sum_s Ks*dKs
template <typename T>
__global__ void kv_bwd_kernel(const T* __restrict__ qkv, int ld, int S, int C, int heads,
                              const float* __restrict__ kmax, const float* __restrict__ ksum,
                              const float* __restrict__ dctx, T* __restrict__ dqkv, int ldq,
                              float* __restrict__ dks, int ntiles, float* __restrict__ parts) {
  extern __shared__ float sh[];
  const int d = C / heads;
  const int tile = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = tile * PT, np = min(PT, S - s0);
  float* sC = sh;             // dctx [d][d]
  float* sCt = sC + d * d;    // dctx^T [d][d] (conflict-free reads along c)
  float* sK = sCt + d * d;    // Ks [PT][d]
  float* sV = sK + PT * d;    // V  [PT][d]
  float* sP = sV + PT * d;    // Ks * dKs [PT][d]
  const float* cg = dctx + ((long)n * heads + h) * d * d;
  for (int i = threadIdx.x; i < d * d; i += blockDim.x) {
    sC[i] = cg[i];
    sCt[(i % d) * d + i / d] = cg[i];
  }
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    const long row = ((long)n * S + s0 + s) * ld;
    const int ch = h * d + c;
    sK[i] = __expf(to_f32(qkv[row + ch]) - kmax[n * C + ch]) / ksum[n * C + ch];
    sV[i] = to_f32(qkv[row + 2 * C + ch]);
  }
  __syncthreads();
  // each thread handles elements (s, c); accumulate r for its channel
  for (int i = threadIdx.x; i < np * d; i += blockDim.x) {
    const int s = i / d, c = i % d;
    float g = 0.f, dv = 0.f;
    for (int cp = 0; cp < d; ++cp) {
      g += sCt[cp * d + c] * sV[s * d + cp];   // dKs[s][c]
      dv += sK[s * d + cp] * sC[cp * d + c];   // dV[s][c]
    }
    const long row = (long)n * S + s0 + s;
    dks[row * C + h * d + c] = g;
    dqkv[row * ldq + 2 * C + h * d + c] = from_f32<T>(dv);
    sP[i] = sK[i] * g;
  }
  __syncthreads();
  float* out = parts + (((long)n * ntiles + tile) * C) + h * d;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float t = 0.f;
    for (int s = 0; s < np; ++s) t += sP[s * d + c];
    out[c] = t;
  }
}

template <typename T>
__global__ void k_bwd_kernel(const T* __restrict__ qkv, int ld, long M, int S, int C,
                             const float* __restrict__ kmax, const float* __restrict__ ksum,
                             const float* __restrict__ dks, const float* __restrict__ r,
                             T* __restrict__ dqkv, int ldq) {
  const long total = M * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long m = i / C;
    const int c = i % C;
    const int n = m / S;
    const float ks = __expf(to_f32(qkv[m * ld + c]) - kmax[n * C + c]) / ksum[n * C + c];
    dqkv[m * ldq + c] = from_f32<T>(ks * (dks[i] - r[n * C + c]));
  }
}

// ------------------------------------------------ narrow heads (d = 4, 8) --
// The stage-1/2 attention (C = 32/64, 8 heads) has d = 4/8: one head of one
// pixel is 8-16 bytes.  These kernels give each thread one (pixel, head) pair
// in registers -- a block row of H threads covers a pixel's C contiguous
// channels -- and reduce the d x d outer products of the context / its
// gradient across the block with cross-lane shuffles (lanes H apart hold the
// same head) and one LDS pass over the 4 waves.
constexpr int NT_PX = 4;  // pixels per thread in the reducing kernels

template <int D, typename T>
__device__ __forceinline__ void loadD(const T* p, float* v) {
  if constexpr (D == 8) {
    load8(p, v);
  } else if constexpr (sizeof(T) == 2) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    const float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  }
}
template <int D, typename T>
__device__ __forceinline__ void storeD(T* p, const float* v) {
  if constexpr (D == 8) {
    store8(p, v);
  } else if constexpr (sizeof(T) == 2) {
    uint2 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// sum acc[K] over the threads of the block that share a head (t % H) and
// leave each wave's head sums in red[wave][h][K] (4 * H * K floats of LDS);
// the caller adds the 4 wave rows
template <int K>
__device__ __forceinline__ void head_reduce(float (&acc)[K], int H, float* red) {
  for (int o = H; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  const int wave = threadIdx.x >> 6, wl = threadIdx.x & 63;
  if (wl < H)
#pragma unroll
    for (int k = 0; k < K; ++k) red[(wave * H + wl) * K + k] = acc[k];
  __syncthreads();
}

// ctx partial over a chunk: parts[n][chunk][h][D][D]
template <typename T, int D>
__global__ void __launch_bounds__(256) ctx_small_kernel(
    const T* __restrict__ qkv, int ld, int S, int C, int H, const float* __restrict__ kmax,
    const float* __restrict__ ksum, int chunk_px, int nchunks, float* __restrict__ parts) {
  __shared__ float red[4 * 64 * D];  // 4 waves x H x D*D (H*D <= 64)
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int h = threadIdx.x % H, pl = threadIdx.x / H, PL = 256 / H;
  const int s0 = chunk * chunk_px, s1 = min(S, s0 + chunk_px);
  float km[D], kinv[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    km[c] = kmax[n * C + h * D + c];
    kinv[c] = 1.f / ksum[n * C + h * D + c];
  }
  float acc[D * D];
#pragma unroll
  for (int k = 0; k < D * D; ++k) acc[k] = 0.f;
  for (int s = s0 + pl; s < s1; s += PL) {
    const long row = ((long)n * S + s) * ld;
    float k[D], v[D];
    loadD<D>(qkv + row + h * D, k);
    loadD<D>(qkv + row + 2 * C + h * D, v);
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const float ks = __expf(k[c] - km[c]) * kinv[c];
#pragma unroll
      for (int cp = 0; cp < D; ++cp) acc[c * D + cp] += ks * v[cp];
    }
  }
  head_reduce<D * D>(acc, H, red);
  for (int o = threadIdx.x; o < H * D * D; o += 256) {
    const int hh = o / (D * D), r = o - hh * D * D;
    float t = 0.f;
    for (int w = 0; w < 4; ++w) t += red[(w * H + hh) * D * D + r];
    parts[(((long)n * nchunks + chunk) * H + hh) * D * D + r] = t;
  }
}

// att = softmax_d(Q) ctx: one (pixel, head) per thread
template <typename T, int D>
__global__ void __launch_bounds__(256) apply_small_kernel(const T* __restrict__ qkv, int ld,
                                                          int S, int C, int H,
                                                          const float* __restrict__ ctx,
                                                          T* __restrict__ att, int ldo) {
  __shared__ float sC[64 * D];  // H x D x D (C = H*D <= 64)
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < C * D; i += 256) sC[i] = ctx[(long)n * C * D + i];
  __syncthreads();
  const int h = threadIdx.x % H, pl = threadIdx.x / H, PL = 256 / H;
  const int s = blockIdx.x * PL + pl;
  if (s >= S) return;
  const long row = (long)n * S + s;
  float q[D];
  loadD<D>(qkv + row * ld + C + h * D, q);
  float mx = q[0];
#pragma unroll
  for (int c = 1; c < D; ++c) mx = fmaxf(mx, q[c]);
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < D; ++c) {
    q[c] = __expf(q[c] - mx);
    sum += q[c];
  }
  const float inv = 1.f / sum;
  const float* cm = sC + h * D * D;
  float o[D];
#pragma unroll
  for (int cp = 0; cp < D; ++cp) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) a += q[c] * cm[c * D + cp];
    o[cp] = a * inv;
  }
  storeD<D>(att + row * ldo + h * D, o);
}

// dQ and the partial dctx per tile of NT_PX * 256/H pixels
template <typename T, int D>
__global__ void __launch_bounds__(256) apply_bwd_small_kernel(
    const T* __restrict__ qkv, int ld, int S, int C, int H, const float* __restrict__ ctx,
    const T* __restrict__ datt, int ldd, T* __restrict__ dqkv, int ldq, int ntiles,
    float* __restrict__ parts) {
  __shared__ float sC[64 * D];
  __shared__ float red[4 * 64 * D];
  const int n = blockIdx.y, tile = blockIdx.x;
  for (int i = threadIdx.x; i < C * D; i += 256) sC[i] = ctx[(long)n * C * D + i];
  __syncthreads();
  const int h = threadIdx.x % H, pl = threadIdx.x / H, PL = 256 / H;
  const float* cm = sC + h * D * D;
  float acc[D * D];
#pragma unroll
  for (int k = 0; k < D * D; ++k) acc[k] = 0.f;
  for (int it = 0; it < NT_PX; ++it) {
    const int s = (tile * NT_PX + it) * PL + pl;
    if (s >= S) break;
    const long row = (long)n * S + s;
    float q[D], g[D];
    loadD<D>(qkv + row * ld + C + h * D, q);
    loadD<D>(datt + row * ldd + h * D, g);
    float mx = q[0];
#pragma unroll
    for (int c = 1; c < D; ++c) mx = fmaxf(mx, q[c]);
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      q[c] = __expf(q[c] - mx);
      sum += q[c];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int c = 0; c < D; ++c) q[c] *= inv;
    float dqs[D], dot = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      float a = 0.f;
#pragma unroll
      for (int cp = 0; cp < D; ++cp) a += cm[c * D + cp] * g[cp];
      dqs[c] = a;
      dot += q[c] * a;
    }
    float dq[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
      dq[c] = q[c] * (dqs[c] - dot);
#pragma unroll
      for (int cp = 0; cp < D; ++cp) acc[c * D + cp] += q[c] * g[cp];
    }
    storeD<D>(dqkv + row * ldq + C + h * D, dq);
  }
  head_reduce<D * D>(acc, H, red);
  for (int o = threadIdx.x; o < H * D * D; o += 256) {
    const int hh = o / (D * D), r = o - hh * D * D;
    float t = 0.f;
    for (int w = 0; w < 4; ++w) t += red[(w * H + hh) * D * D + r];
    parts[(((long)n * ntiles + tile) * H + hh) * D * D + r] = t;
  }
}

// dV, dKs (f32 [m][C]) and the partial r[c] = sum_s Ks dKs per tile
template <typename T, int D>
__global__ void __launch_bounds__(256) kv_bwd_small_kernel(
    const T* __restrict__ qkv, int ld, int S, int C, int H, const float* __restrict__ kmax,
    const float* __restrict__ ksum, const float* __restrict__ dctx, T* __restrict__ dqkv,
    int ldq, float* __restrict__ dks, int ntiles, float* __restrict__ parts) {
  __shared__ float sC[64 * D];
  __shared__ float red[4 * 64];
  const int n = blockIdx.y, tile = blockIdx.x;
  for (int i = threadIdx.x; i < C * D; i += 256) sC[i] = dctx[(long)n * C * D + i];
  __syncthreads();
  const int h = threadIdx.x % H, pl = threadIdx.x / H, PL = 256 / H;
  const float* cm = sC + h * D * D;
  float km[D], kinv[D], acc[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    km[c] = kmax[n * C + h * D + c];
    kinv[c] = 1.f / ksum[n * C + h * D + c];
    acc[c] = 0.f;
  }
  for (int it = 0; it < NT_PX; ++it) {
    const int s = (tile * NT_PX + it) * PL + pl;
    if (s >= S) break;
    const long row = (long)n * S + s;
    float k[D], v[D];
    loadD<D>(qkv + row * ld + h * D, k);
    loadD<D>(qkv + row * ld + 2 * C + h * D, v);
#pragma unroll
    for (int c = 0; c < D; ++c) k[c] = __expf(k[c] - km[c]) * kinv[c];
    float g[D], dv[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int cp = 0; cp < D; ++cp) {
        a += cm[c * D + cp] * v[cp];  // dKs[c]
        b += k[cp] * cm[cp * D + c];  // dV[c]
      }
      g[c] = a;
      dv[c] = b;
      acc[c] += k[c] * a;
    }
    float* dk = dks + row * C + h * D;
#pragma unroll
    for (int c = 0; c < D; c += 4)
      *reinterpret_cast<float4*>(dk + c) = make_float4(g[c], g[c + 1], g[c + 2], g[c + 3]);
    storeD<D>(dqkv + row * ldq + 2 * C + h * D, dv);
  }
  head_reduce<D>(acc, H, red);
  for (int o = threadIdx.x; o < H * D; o += 256) {
    const int hh = o / D, r = o - hh * D;
    float t = 0.f;
    for (int w = 0; w < 4; ++w) t += red[(w * H + hh) * D + r];
    parts[((long)n * ntiles + tile) * C + o] = t;
  }
}

static inline bool small_heads(int C, int heads) {
  const int d = C / heads;
  return (d == 4 || d == 8) && C <= 64 && 64 % heads == 0;
}

inline int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

inline int ctx_chunk(int d) {  // keeps the ctx kernel's LDS <= 33 KB
  int c = 4096 / d;
  if (c > 1024) c = 1024;
  return c;
}

// the backward for narrow heads: the register kernels, tiles of
// NT_PX * 256/H pixels (never more tiles than um_attn_ws_tiles sizes for)
template <typename T, int D>
int attn_bwd_small_t(int N, int S, int C, int heads, const void* qkv, int ld, const float* kmax,
                     const float* ksum, const float* ctx, const void* datt, int ldd, void* dqkv,
                     int ldq, float* dks_ws, float* ws, float* dctx, float* r, hipStream_t st) {
  const int tp = NT_PX * (256 / heads);
  const int nt = ceil_div(S, tp);
  hipLaunchKernelGGL((apply_bwd_small_kernel<T, D>), dim3(nt, N), dim3(256), 0, st,
                     (const T*)qkv, ld, S, C, heads, ctx, (const T*)datt, ldd, (T*)dqkv, ldq, nt,
                     ws);
  const int L = heads * D * D;
  {
    const int jl = sum_parts_cols(L, nt);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(ceil_div(L, jl), N), dim3(256), 0, st, ws, N, nt, L,
                       dctx, jl);
  }
  hipLaunchKernelGGL((kv_bwd_small_kernel<T, D>), dim3(nt, N), dim3(256), 0, st, (const T*)qkv,
                     ld, S, C, heads, kmax, ksum, dctx, (T*)dqkv, ldq, dks_ws, nt, ws);
  {
    const int jl = sum_parts_cols(C, nt);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(ceil_div(C, jl), N), dim3(256), 0, st, ws, N, nt, C,
                       r, jl);
  }
  const long M = (long)N * S;
  hipLaunchKernelGGL(k_bwd_kernel<T>, dim3(grid_for(M * C)), dim3(256), 0, st, (const T*)qkv, ld,
                     M, S, C, kmax, ksum, dks_ws, r, (T*)dqkv, ldq);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int attn_bwd_small(int dtype, int N, int S, int C, int heads, const void* qkv, int ld,
                   const float* kmax, const float* ksum, const float* ctx, const void* datt,
                   int ldd, void* dqkv, int ldq, float* dks_ws, float* ws, float* dctx, float* r,
                   hipStream_t st) {
  const int d = C / heads;
  if (dtype == UM_BF16)
    return d == 4 ? attn_bwd_small_t<bf16_t, 4>(N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt,
                                                ldd, dqkv, ldq, dks_ws, ws, dctx, r, st)
                  : attn_bwd_small_t<bf16_t, 8>(N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt,
                                                ldd, dqkv, ldq, dks_ws, ws, dctx, r, st);
  return d == 4 ? attn_bwd_small_t<float, 4>(N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt, ldd,
                                             dqkv, ldq, dks_ws, ws, dctx, r, st)
                : attn_bwd_small_t<float, 8>(N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt, ldd,
                                             dqkv, ldq, dks_ws, ws, dctx, r, st);
}

// ------------------------------------------------ MFMA heads (d = 16..64) --
// Stages 3-5 of the encoder (C = 128 / 256 / 512, 8 heads: d = 16 / 32 / 64).
// The d x d products run on v_mfma_f32_16x16x4_f32 from f32 LDS images (f32
// operands: the fp32 build keeps fp32 arithmetic, and at these sizes the
// launches are latency-bound, not MFMA-bound), and the passes are fused:
//   forward : ctx_part_mfma (per pixel chunk: the chunk's own key-softmax
//             max m_b and sum l_b, and ctx_b = exp(K - m_b)^T V) ->
//             apply_mfma (every tile workgroup combines the chunk partials,
//             ctx = sum_b e^(m_b - M) ctx_b / sum_b e^(m_b - M) l_b, in its
//             prologue; tile 0 publishes kmax = M, ksum, ctx for the
//             backward; then att = softmax_c(Q) ctx)
//   backward: apply_bwd_mfma (dQ, dctx partial per tile) -> kv_bwd_mfma
//             (dctx combined in the prologue; dV, dKs, r partial) ->
//             k_bwd_mfma (r combined in the prologue; dK)
// 2 + 3 launches per attention instead of 5 + 5 (kstats, combine, ctx,
// part sums, apply / apply_bwd, part sums, kv_bwd, part sums, k_bwd).
constexpr int MCH = 64;        // pixels per chunk / tile
constexpr int PST = MCH + 16;  // row stride of [channel][pixel] images (floats)

// row stride of [pixel][channel] / [channel][channel] images: 16 banks
// between consecutive rows, so the two 16-lane halves of a ds_read_b32
// group read disjoint banks
template <int D> struct MS { static constexpr int ST = (D % 32 == 0) ? D + 16 : D + 32; };

// acc (one 16x16 block) += A(r, k) B(k, c) over k in [0, K), K % 4 == 0;
// A(r, k) at a[r * ar + k * ak], B(k, c) at b[k * bk + c * bc].  Lane l
// feeds A(l % 16, k + l / 16), B(k + l / 16, l % 16) and holds
// D(4 * (l / 16) + j, l % 16) in acc[j].
__device__ __forceinline__ void mma16(f32x4_t& acc, const float* a, int ar, int ak,
                                      const float* b, int bk, int bc, int K) {
  const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
  for (int k = 0; k < K; k += 4)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i * ar + (k + kk) * ak],
                                                b[(k + kk) * bk + i * bc], acc, 0, 0, 0);
}

// rows [row0, row0 + np) of src (pixel stride ld), channels [col0, col0 + D)
// -> f32 LDS image, zero rows up to MCH.  T_ = true: transposed image
// dst[c * PST + s], else dst[s * ST + c]
template <typename T, int D, bool T_>
__device__ __forceinline__ void load_img(float* dst, const T* __restrict__ src, long row0, int ld,
                                         int col0, int np) {
  constexpr int ST = MS<D>::ST, V = D / 8;
  constexpr int IT = (MCH * V + 255) / 256;  // 1 (D <= 32) or 2
  float v[IT][8];
#pragma unroll
  for (int u = 0; u < IT; ++u) {  // every load issued before the first LDS store
    const int i = threadIdx.x + u * 256, s = i / V, c = (i - s * V) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
    if (i < MCH * V && s < np) load8(src + (row0 + s) * ld + col0 + c, v[u]);
  }
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = threadIdx.x + u * 256, s = i / V, c = (i - s * V) * 8;
    if (i >= MCH * V) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (T_) dst[(c + e) * PST + s] = v[u][e];
      else dst[s * ST + c + e] = v[u][e];
    }
  }
}

// the wave's share of the (D/16)^2 output blocks of a D x D product, or for
// D = 16 the whole block over a quarter of the MCH-deep reduction (wave_k)
template <int D> struct Blocks {
  static constexpr int NB = (D / 16) * (D / 16);
  static constexpr int PER = NB >= 4 ? NB / 4 : 1;
  static constexpr bool KSPLIT = NB < 4;
};

// D x D product over the MCH pixels (A(c, s), B(s, c')), result written by
// `put(c, c', v)`; for D = 16 the four waves' k-quarters are summed in red
// (4 * 256 floats)
template <int D, typename F>
__device__ __forceinline__ void dd_product(const float* a, int ar, int ak, const float* b, int bk,
                                           int bc, float* red, F put) {
  using B = Blocks<D>;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4_t acc[B::PER];
#pragma unroll
  for (int q = 0; q < B::PER; ++q) acc[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if constexpr (B::KSPLIT) {
    const int k0 = w * (MCH / 4);
    mma16(acc[0], a + k0 * ak, ar, ak, b + k0 * bk, bk, bc, MCH / 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) red[w * 256 + (4 * (lane >> 4) + j) * 16 + (lane & 15)] = acc[0][j];
    __syncthreads();
    const int o = threadIdx.x;  // 256 = 16 x 16 outputs
    put(o >> 4, o & 15, red[o] + red[256 + o] + red[512 + o] + red[768 + o]);
  } else {
#pragma unroll
    for (int q = 0; q < B::PER; ++q) {
      const int blk = w * B::PER + q, bi = blk / (D / 16), bj = blk % (D / 16);
      mma16(acc[q], a + 16 * bi * ar, ar, ak, b + 16 * bj * bc, bk, bc, MCH);
#pragma unroll
      for (int j = 0; j < 4; ++j) put(16 * bi + 4 * (lane >> 4) + j, 16 * bj + (lane & 15), acc[q][j]);
    }
  }
}

// forward (1): chunk partials [n][h][b] = {m[D], l[D], ctx[D][D]}
template <typename T, int D>
__global__ void __launch_bounds__(256) ctx_part_mfma(const T* __restrict__ qkv, int ld, int S,
                                                     int C, int heads, int nb,
                                                     float* __restrict__ part) {
  constexpr int ST = MS<D>::ST, G = 256 / D;
  __shared__ float sK[MCH * ST], sV[MCH * ST];
  __shared__ float red[1024];
  const int b = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = b * MCH, np = min(MCH, S - s0);
  const long row0 = (long)n * S + s0;
  load_img<T, D, false>(sK, qkv, row0, ld, h * D, np);
  load_img<T, D, false>(sV, qkv, row0, ld, 2 * C + h * D, np);
  __syncthreads();
  const int c = threadIdx.x % D, g = threadIdx.x / D;
  float mx = -INFINITY;
  for (int s = g; s < np; s += G) mx = fmaxf(mx, sK[s * ST + c]);
  red[threadIdx.x] = mx;
  __syncthreads();
  mx = red[c];
  for (int q = 1; q < G; ++q) mx = fmaxf(mx, red[q * D + c]);
  float sum = 0.f;
  for (int s = g; s < MCH; s += G) {
    float e = 0.f;
    if (s < np) {
      e = __expf(sK[s * ST + c] - mx);
      sum += e;
    }
    sK[s * ST + c] = e;
  }
  __syncthreads();  // every thread has read red (the maxima)
  red[threadIdx.x] = sum;
  __syncthreads();
  float* o = part + (((long)n * heads + h) * nb + b) * (D * D + 2 * D);
  if (g == 0) {
    for (int q = 1; q < G; ++q) sum += red[q * D + c];
    o[c] = mx;
    o[D + c] = sum;
  }
  __syncthreads();  // red is reused by the product (D = 16)
  // ctx_b(c, c') = sum_s sK[s][c] sV[s][c']
  dd_product<D>(sK, 1, ST, sV, ST, 1, red,
                [&](int r, int cc, float v) { o[2 * D + r * D + cc] = v; });
}

// combine the chunk partials of (n, h): M[c], L[c] into sM / sL, and the
// final ctx (D x D) into dst[c * dst_r + c' * dst_c] (every workgroup of
// the pair does the same, bit-identically)
template <int D>
__device__ __forceinline__ void ctx_combine(const float* __restrict__ p, int nb, float* sM,
                                            float* sL, float* red, float* dst, int dst_r,
                                            int dst_c) {
  constexpr int G = 256 / D, PS = D * D + 2 * D;
  const int t = threadIdx.x, c = t % D, g = t / D;
  float M = -INFINITY;
  for (int b = g; b < nb; b += G) M = fmaxf(M, p[(long)b * PS + c]);
  red[t] = M;
  __syncthreads();
  M = red[c];
  for (int q = 1; q < G; ++q) M = fmaxf(M, red[q * D + c]);
  float L = 0.f;
  for (int b = g; b < nb; b += G) {
    const float* q = p + (long)b * PS;
    L += __expf(q[c] - M) * q[D + c];
  }
  __syncthreads();  // every thread has read the maxima
  red[t] = L;
  __syncthreads();
  if (g == 0) {
    for (int q = 1; q < G; ++q) L += red[q * D + c];
    sM[c] = M;
    sL[c] = L;
  }
  __syncthreads();
  // b outer, this thread's outputs inner: their loads are issued together
  constexpr int PER = (D * D + 255) / 256;
  float acc[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) acc[u] = 0.f;
#pragma unroll 2
  for (int b = 0; b < nb; ++b) {
    const float* q = p + (long)b * PS;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int o = t + u * 256;
      if (o < D * D) acc[u] += __expf(q[o / D] - sM[o / D]) * q[2 * D + o];
    }
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int o = t + u * 256;
    if (o < D * D) dst[(o / D) * dst_r + (o % D) * dst_c] = acc[u] / sL[o / D];
  }
}

// softmax over the D channels of each of the MCH pixels of a transposed
// image x[c * PST + s]: wave w takes channels [w D/4, (w+1) D/4) of every
// pixel (lane = pixel), the maxima and sums meet in red (2 x 256 floats)
template <int D>
__device__ __forceinline__ void softmax_cols(float* x, float* red) {
  const int s = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int Q = D / 4;
  float mx = -INFINITY;
#pragma unroll 4
  for (int c = w * Q; c < (w + 1) * Q; ++c) mx = fmaxf(mx, x[c * PST + s]);
  red[w * 64 + s] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[s], red[64 + s]), fmaxf(red[128 + s], red[192 + s]));
  float sum = 0.f;
#pragma unroll 4
  for (int c = w * Q; c < (w + 1) * Q; ++c) {
    const float e = __expf(x[c * PST + s] - mx);
    x[c * PST + s] = e;
    sum += e;
  }
  red[256 + w * 64 + s] = sum;
  __syncthreads();
  const float inv = 1.f / (red[256 + s] + red[320 + s] + red[384 + s] + red[448 + s]);
#pragma unroll 4
  for (int c = w * Q; c < (w + 1) * Q; ++c) x[c * PST + s] *= inv;
}

// forward (2): att = softmax_c(Q) ctx over tiles [blockIdx.x * tpw, ...) of
// MCH pixels (the combine is done once per workgroup)
template <typename T, int D>
__global__ void __launch_bounds__(256) apply_mfma(const T* __restrict__ qkv, int ld, int S, int C,
                                                  int heads, int nb, int tpw,
                                                  const float* __restrict__ part,
                                                  float* __restrict__ kmax,
                                                  float* __restrict__ ksum,
                                                  float* __restrict__ ctxg, T* __restrict__ att,
                                                  int ldo) {
  constexpr int ST = MS<D>::ST;
  __shared__ float sC[D * ST], sQt[D * PST];
  __shared__ float sM[D], sL[D], red[512];
  const int h = blockIdx.y, n = blockIdx.z;
  ctx_combine<D>(part + ((long)n * heads + h) * nb * (D * D + 2 * D), nb, sM, sL, red, sC, ST, 1);
  __syncthreads();
  if (blockIdx.x == 0) {  // the backward's kmax / ksum / ctx
    for (int o = threadIdx.x; o < D * D; o += 256)
      ctxg[((long)n * heads + h) * D * D + o] = sC[(o / D) * ST + o % D];
    if (threadIdx.x < D) {
      kmax[(long)n * C + h * D + threadIdx.x] = sM[threadIdx.x];
      ksum[(long)n * C + h * D + threadIdx.x] = sL[threadIdx.x];
    }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt = (S + MCH - 1) / MCH;
  for (int tile = blockIdx.x * tpw; tile < min(nt, (blockIdx.x + 1) * tpw); ++tile) {
    const int s0 = tile * MCH, np = min(MCH, S - s0);
    const long row0 = (long)n * S + s0;
    __syncthreads();  // the previous tile's products have read sQt
    load_img<T, D, true>(sQt, qkv, row0, ld, C + h * D, np);
    __syncthreads();
    softmax_cols<D>(sQt, red);
    __syncthreads();
    // att(s, c') = sum_c Qs(s, c) ctx(c, c'): wave w takes pixel rows 16w..16w+15
#pragma unroll
    for (int bj = 0; bj < D / 16; ++bj) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      mma16(acc, sQt + 16 * w, 1, PST, sC + 16 * bj, ST, 1, D);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int s = 16 * w + 4 * (lane >> 4) + j;
        if (s < np)
          att[(row0 + s) * ldo + h * D + 16 * bj + (lane & 15)] = from_f32<T>(acc[j]);
      }
    }
  }
}

// backward (1): dQ and the tile's dctx partial ws[n][h][tile][D][D]
//   dQs(s, c) = sum_c' datt(s, c') ctx(c, c'), dQ = Qs (dQs - <Qs, dQs>_c)
//   dctx(c, c') = sum_s Qs(s, c) datt(s, c')
template <typename T, int D>
__global__ void __launch_bounds__(256) apply_bwd_mfma(const T* __restrict__ qkv, int ld, int S,
                                                      int C, int heads,
                                                      const float* __restrict__ ctxg,
                                                      const T* __restrict__ datt, int ldd,
                                                      T* __restrict__ dqkv, int ldq, int nt,
                                                      float* __restrict__ ws) {
  constexpr int ST = MS<D>::ST;
  extern __shared__ float sh[];
  float* sCt = sh;                // ctx^T [c'][c]
  float* sGt = sCt + D * ST;      // datt^T [c'][s]
  float* sG = sGt + D * PST;      // datt [s][c']
  float* sQt = sG + MCH * ST;     // Qs^T [c][s]
  float* sQ = sQt + D * PST;      // Qs [s][c]
  float* red = sQ + MCH * ST;     // [1024]
  const int tile = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = tile * MCH, np = min(MCH, S - s0);
  const long row0 = (long)n * S + s0;
  const float* cg = ctxg + ((long)n * heads + h) * D * D;
  {
    constexpr int PER = (D * D + 255) / 256;
    float v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int o = threadIdx.x + u * 256;
      v[u] = o < D * D ? cg[o] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int o = threadIdx.x + u * 256;
      if (o < D * D) sCt[(o % D) * ST + o / D] = v[u];
    }
  }
  load_img<T, D, true>(sGt, datt, row0, ldd, h * D, np);
  load_img<T, D, false>(sG, datt, row0, ldd, h * D, np);
  load_img<T, D, true>(sQt, qkv, row0, ld, C + h * D, np);
  __syncthreads();
  softmax_cols<D>(sQt, red);
  __syncthreads();
  for (int i = threadIdx.x; i < MCH * D; i += 256) {
    const int s = i / D, c = i - s * D;
    sQ[s * ST + c] = s < np ? sQt[c * PST + s] : 0.f;  // pad pixels add nothing to dctx
  }
  __syncthreads();
  // dctx partial
  float* o = ws + (((long)n * heads + h) * nt + tile) * D * D;
  dd_product<D>(sQ, 1, ST, sG, ST, 1, red,
                [&](int r, int cc, float v) { o[r * D + cc] = v; });
  // dQs for pixel rows 16w..: lane holds (s = 16w + 4(l/16) + j, c = 16 bj + l % 16)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4_t acc[D / 16];
#pragma unroll
  for (int bj = 0; bj < D / 16; ++bj) {
    acc[bj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    mma16(acc[bj], sGt + 16 * w, 1, PST, sCt + 16 * bj, ST, 1, D);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int s = 16 * w + 4 * (lane >> 4) + j;
    float dot = 0.f;
#pragma unroll
    for (int bj = 0; bj < D / 16; ++bj) dot += sQ[s * ST + 16 * bj + (lane & 15)] * acc[bj][j];
    // sum over the 16 lanes of this row group (same lane >> 4)
    dot += __shfl_xor(dot, 1, 64);
    dot += __shfl_xor(dot, 2, 64);
    dot += __shfl_xor(dot, 4, 64);
    dot += __shfl_xor(dot, 8, 64);
    if (s < np) {
#pragma unroll
      for (int bj = 0; bj < D / 16; ++bj) {
        const int c = 16 * bj + (lane & 15);
        dqkv[(row0 + s) * ldq + C + h * D + c] = from_f32<T>(sQ[s * ST + c] * (acc[bj][j] - dot));
      }
    }
  }
}

// backward (2): dctx combined from the tile partials; over tiles
// [blockIdx.x * tpw, ...): dV into dqkv, dKs into dks [M][C] f32, and the
// workgroup's r partial ws_r[n][blockIdx.x][C] = sum_s Ks dKs
//   dKs(s, c) = sum_c' V(s, c') dctx(c, c'), dV(s, c') = sum_c Ks(s, c) dctx(c, c')
template <typename T, int D>
__global__ void __launch_bounds__(256) kv_bwd_mfma(const T* __restrict__ qkv, int ld, int S, int C,
                                                   int heads, const float* __restrict__ kmax,
                                                   const float* __restrict__ ksum, int nt,
                                                   int tpw, const float* __restrict__ ws_dctx,
                                                   T* __restrict__ dqkv, int ldq,
                                                   float* __restrict__ dks,
                                                   float* __restrict__ ws_r) {
  constexpr int ST = MS<D>::ST;
  extern __shared__ float sh[];
  float* sD = sh;               // dctx [c][c']
  float* sDt = sD + D * ST;     // dctx^T [c'][c]
  float* sVt = sDt + D * ST;    // V^T [c'][s]
  float* sKt = sVt + D * PST;   // Ks^T [c][s]
  float* sR = sKt + D * PST;    // [4][D] per-wave r partials
  const int h = blockIdx.y, n = blockIdx.z;
  __shared__ float sKm[D], sKi[D];
  const float* p = ws_dctx + ((long)n * heads + h) * nt * D * D;
  {
    constexpr int PER = (D * D + 255) / 256;
    float acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = 0.f;
#pragma unroll 2
    for (int t = 0; t < nt; ++t)
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int o = threadIdx.x + u * 256;
        if (o < D * D) acc[u] += p[(long)t * D * D + o];
      }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int o = threadIdx.x + u * 256;
      if (o < D * D) {
        const int c = o / D, cc = o - c * D;
        sD[c * ST + cc] = acc[u];
        sDt[cc * ST + c] = acc[u];
      }
    }
  }
  if (threadIdx.x < D) {
    sKm[threadIdx.x] = kmax[(long)n * C + h * D + threadIdx.x];
    sKi[threadIdx.x] = 1.f / ksum[(long)n * C + h * D + threadIdx.x];
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float racc[D / 16];
#pragma unroll
  for (int bj = 0; bj < D / 16; ++bj) racc[bj] = 0.f;
  for (int tile = blockIdx.x * tpw; tile < min(nt, (blockIdx.x + 1) * tpw); ++tile) {
    const int s0 = tile * MCH, np = min(MCH, S - s0);
    const long row0 = (long)n * S + s0;
    __syncthreads();  // the previous tile's products have read sVt / sKt
    load_img<T, D, true>(sVt, qkv, row0, ld, 2 * C + h * D, np);
    load_img<T, D, true>(sKt, qkv, row0, ld, h * D, np);
    __syncthreads();
    for (int i = threadIdx.x; i < D * MCH; i += 256) {
      const int c = i / MCH, s = i - c * MCH;
      sKt[c * PST + s] = s < np ? __expf(sKt[c * PST + s] - sKm[c]) * sKi[c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int bj = 0; bj < D / 16; ++bj) {
      f32x4_t kv = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
      mma16(kv, sVt + 16 * w, 1, PST, sDt + 16 * bj, ST, 1, D);  // dKs, cols c
      mma16(dv, sKt + 16 * w, 1, PST, sD + 16 * bj, ST, 1, D);   // dV, cols c'
      const int c = 16 * bj + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int s = 16 * w + 4 * (lane >> 4) + j;
        if (s < np) {
          dks[(row0 + s) * C + h * D + c] = kv[j];
          dqkv[(row0 + s) * ldq + 2 * C + h * D + c] = from_f32<T>(dv[j]);
          racc[bj] += sKt[c * PST + s] * kv[j];
        }
      }
    }
  }
#pragma unroll
  for (int bj = 0; bj < D / 16; ++bj) {
    float r = racc[bj];
    r += __shfl_xor(r, 16, 64);
    r += __shfl_xor(r, 32, 64);
    if (lane < 16) sR[w * D + 16 * bj + lane] = r;
  }
  __syncthreads();
  if (threadIdx.x < D) {
    const int c = threadIdx.x;
    ws_r[((long)n * gridDim.x + blockIdx.x) * C + h * D + c] =
        sR[c] + sR[D + c] + sR[2 * D + c] + sR[3 * D + c];
  }
}

// backward (3): r combined from the kv workgroups' partials; dK = Ks (dKs - r)
template <typename T, int D>
__global__ void __launch_bounds__(256) k_bwd_mfma(const T* __restrict__ qkv, int ld, int S, int C,
                                                  const float* __restrict__ kmax,
                                                  const float* __restrict__ ksum, int nparts,
                                                  const float* __restrict__ ws_r,
                                                  const float* __restrict__ dks,
                                                  T* __restrict__ dqkv, int ldq) {
  __shared__ float sR[D], sKm[D], sKi[D];
  const int tile = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int s0 = tile * MCH, np = min(MCH, S - s0);
  const long row0 = (long)n * S + s0;
  if (threadIdx.x < D) {
    float r = 0.f;
    for (int t = 0; t < nparts; ++t) r += ws_r[((long)n * nparts + t) * C + h * D + threadIdx.x];
    sR[threadIdx.x] = r;
    sKm[threadIdx.x] = kmax[(long)n * C + h * D + threadIdx.x];
    sKi[threadIdx.x] = 1.f / ksum[(long)n * C + h * D + threadIdx.x];
  }
  __syncthreads();
  constexpr int V = D / 8;
  for (int i = threadIdx.x; i < np * V; i += 256) {
    const int s = i / V, c = (i - s * V) * 8;
    const long m = row0 + s;
    float k[8], g[8], out[8];
    load8(qkv + m * ld + h * D + c, k);
    load8(dks + m * C + h * D + c, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float ks = __expf(k[e] - sKm[c + e]) * sKi[c + e];
      out[e] = ks * (g[e] - sR[c + e]);
    }
    store8(dqkv + m * ldq + h * D + c, out);
  }
}

inline bool mfma_heads(int C, int heads) {
  const int d = C / heads;
  return C % heads == 0 && (d == 16 || d == 32 || d == 64);
}


// tiles per workgroup of the kernels that combine partials in their
// prologue: about 512 workgroups (the combine is read once per workgroup)
inline int tiles_per_wg(int nt, int heads, int N) {
  const long g = (long)nt * heads * N;
  const int t = (int)std::max(1l, g / 512);
  return std::min(t, nt);
}

template <typename T, int D>
int attn_fwd_mfma_t(int N, int S, int C, int heads, const void* qkv, int ld, float* kmax,
                    float* ksum, float* ctx, float* ws, void* att, int ldo, hipStream_t st) {
  const int nb = ceil_div(S, MCH);
  const int tpw = tiles_per_wg(nb, heads, N), nwg = ceil_div(nb, tpw);
  hipLaunchKernelGGL((ctx_part_mfma<T, D>), dim3(nb, heads, N), dim3(256), 0, st,
                     (const T*)qkv, ld, S, C, heads, nb, ws);
  hipLaunchKernelGGL((apply_mfma<T, D>), dim3(nwg, heads, N), dim3(256), 0, st, (const T*)qkv, ld,
                     S, C, heads, nb, tpw, ws, kmax, ksum, ctx, (T*)att, ldo);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

template <typename T, int D>
size_t apply_bwd_mfma_lds() {
  constexpr int ST = MS<D>::ST;
  return (size_t)(D * ST + 2 * D * PST + 2 * MCH * ST + 1024) * sizeof(float);
}
template <int D>
size_t kv_bwd_mfma_lds() {
  constexpr int ST = MS<D>::ST;
  return (size_t)(2 * D * ST + 2 * D * PST + 4 * D) * sizeof(float);
}

template <typename T, int D>
int attn_bwd_mfma_t(int N, int S, int C, int heads, const void* qkv, int ld, const float* kmax,
                    const float* ksum, const float* ctx, const void* datt, int ldd, void* dqkv,
                    int ldq, float* dks_ws, float* ws, hipStream_t st) {
  const int nt = ceil_div(S, MCH);
  float* ws_dctx = ws;
  float* ws_r = ws + (long)N * heads * nt * D * D;
  static bool attr = false;  // d = 64 needs more than the default 64 KB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&apply_bwd_mfma<T, D>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&kv_bwd_mfma<T, D>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    attr = true;
  }
  const dim3 g(nt, heads, N);
  const size_t lds_a = apply_bwd_mfma_lds<T, D>(), lds_k = kv_bwd_mfma_lds<D>();
  hipLaunchKernelGGL((apply_bwd_mfma<T, D>), g, dim3(256), lds_a, st,
                     (const T*)qkv, ld, S, C, heads, ctx, (const T*)datt, ldd, (T*)dqkv, ldq, nt,
                     ws_dctx);
  const int tpw = tiles_per_wg(nt, heads, N), nwg = ceil_div(nt, tpw);
  hipLaunchKernelGGL((kv_bwd_mfma<T, D>), dim3(nwg, heads, N), dim3(256), lds_k, st, (const T*)qkv,
                     ld, S, C, heads, kmax, ksum, nt, tpw, ws_dctx, (T*)dqkv, ldq, dks_ws, ws_r);
  hipLaunchKernelGGL((k_bwd_mfma<T, D>), g, dim3(256), 0, st, (const T*)qkv, ld, S, C, kmax, ksum,
                     nwg, ws_r, dks_ws, (T*)dqkv, ldq);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

#define UM_ATTN_D(FN, T_, d, ...)                              \
  (d == 16 ? FN<T_, 16>(__VA_ARGS__)                           \
           : (d == 32 ? FN<T_, 32>(__VA_ARGS__) : FN<T_, 64>(__VA_ARGS__)))

}  // namespace

extern "C" {

// workspace sizes (floats)
long um_attn_ws_kstats(int N, int S, int C) {
  return (long)N * ceil_div(S, ks_chunk(S)) * C * 2;
}
long um_attn_ws_ctx(int N, int S, int C, int heads) {
  const int d = C / heads;
  if (mfma_heads(C, heads))  // chunk partials {m, l, ctx}
    return (long)N * heads * ceil_div(S, MCH) * (d * d + 2 * d);
  return (long)N * ceil_div(S, ctx_chunk(d)) * heads * d * d;
}
long um_attn_ws_tiles(int N, int S, int C, int heads) {
  const int d = C / heads;
  if (mfma_heads(C, heads))  // dctx partials, then r partials
    return (long)N * ceil_div(S, MCH) * (heads * d * d + C);
  const long a = (long)N * ceil_div(S, PT) * heads * d * d;
  const long b = (long)N * ceil_div(S, PT) * C;
  return a > b ? a : b;
}

int um_attn_fwd(int dtype, int N, int S, int C, int heads, const void* qkv, int ld,
                float* kmax, float* ksum, float* ctx, float* ws, void* att, int ldo,
                hipStream_t st) {
  UM_CHECK_ARG(C % heads == 0, "um_attn_fwd: C %% heads");
  const int d = C / heads;
  UM_CHECK_ARG(d <= 64, "um_attn_fwd: head dim %d > 64", d);
  if (mfma_heads(C, heads) && ld % 8 == 0 && ldo % 8 == 0) {
    if (dtype == UM_BF16)
      return UM_ATTN_D(attn_fwd_mfma_t, bf16_t, d, N, S, C, heads, qkv, ld, kmax, ksum, ctx, ws,
                       att, ldo, st);
    return UM_ATTN_D(attn_fwd_mfma_t, float, d, N, S, C, heads, qkv, ld, kmax, ksum, ctx, ws, att,
                     ldo, st);
  }
  const int kch = ks_chunk(S);
  const int nks = ceil_div(S, kch);
  const int cch = ctx_chunk(d);
  const int nctx = ceil_div(S, cch);
  if (dtype == UM_BF16) {
    hipLaunchKernelGGL(kstats_kernel<bf16_t>, dim3(nks, N, ceil_div(C, 64)), dim3(256), 0, st,
                       (const bf16_t*)qkv, ld, S, C, kch, ws, nks);
  } else {
    hipLaunchKernelGGL(kstats_kernel<float>, dim3(nks, N, ceil_div(C, 64)), dim3(256), 0, st,
                       (const float*)qkv, ld, S, C, kch, ws, nks);
  }
  hipLaunchKernelGGL(kstats_combine_kernel, dim3(ceil_div(N * C, 4)), dim3(256), 0, st, ws, N,
                     nks, C, kmax, ksum);
  const bool small = small_heads(C, heads) && ld % 8 == 0 && ldo % 8 == 0;
  const size_t shm_ctx = (2 * (size_t)cch * d + 256) * sizeof(float);
  if (small) {
#define UM_CTXS(T_, D_)                                                                       \
  hipLaunchKernelGGL((ctx_small_kernel<T_, D_>), dim3(nctx, N), dim3(256), 0, st,             \
                     (const T_*)qkv, ld, S, C, heads, kmax, ksum, cch, nctx, ws)
    if (dtype == UM_BF16) { if (d == 4) UM_CTXS(bf16_t, 4); else UM_CTXS(bf16_t, 8); }
    else { if (d == 4) UM_CTXS(float, 4); else UM_CTXS(float, 8); }
#undef UM_CTXS
  } else if (dtype == UM_BF16)
    hipLaunchKernelGGL(ctx_kernel<bf16_t>, dim3(nctx, heads, N), dim3(256), shm_ctx, st,
                       (const bf16_t*)qkv, ld, S, C, heads, kmax, ksum, cch, nctx, ws);
  else
    hipLaunchKernelGGL(ctx_kernel<float>, dim3(nctx, heads, N), dim3(256), shm_ctx, st,
                       (const float*)qkv, ld, S, C, heads, kmax, ksum, cch, nctx, ws);
  const int L = heads * d * d;
  {
    const int jl = sum_parts_cols(L, nctx);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(ceil_div(L, jl), N), dim3(256), 0, st, ws, N, nctx,
                       L, ctx, jl);
  }
  const size_t shm_ap = ((size_t)d * d + PT * (d + 1)) * sizeof(float);
  const dim3 g(ceil_div(S, PT), heads, N);
  if (small) {
    const dim3 gs(ceil_div(S, 256 / heads), N);
#define UM_APS(T_, D_)                                                                        \
  hipLaunchKernelGGL((apply_small_kernel<T_, D_>), gs, dim3(256), 0, st, (const T_*)qkv, ld, S, \
                     C, heads, ctx, (T_*)att, ldo)
    if (dtype == UM_BF16) { if (d == 4) UM_APS(bf16_t, 4); else UM_APS(bf16_t, 8); }
    else { if (d == 4) UM_APS(float, 4); else UM_APS(float, 8); }
#undef UM_APS
  } else if (dtype == UM_BF16)
    hipLaunchKernelGGL(apply_kernel<bf16_t>, g, dim3(256), shm_ap, st, (const bf16_t*)qkv, ld, S,
                       C, heads, ctx, (bf16_t*)att, ldo);
  else
    hipLaunchKernelGGL(apply_kernel<float>, g, dim3(256), shm_ap, st, (const float*)qkv, ld, S, C,
                       heads, ctx, (float*)att, ldo);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// dqkv [M][3C] is fully written.  dks_ws: f32 [M][C]; ws: um_attn_ws_tiles floats;
// dctx: f32 [N][heads][d][d]; r: f32 [N][C]
int um_attn_bwd(int dtype, int N, int S, int C, int heads, const void* qkv, int ld,
                const float* kmax, const float* ksum, const float* ctx, const void* datt,
                int ldd, void* dqkv, int ldq, float* dks_ws, float* ws, float* dctx, float* r,
                hipStream_t st) {
  const int d = C / heads;
  UM_CHECK_ARG(d <= 64 && C % heads == 0, "um_attn_bwd: head dim");
  if (mfma_heads(C, heads) && ld % 8 == 0 && ldd % 8 == 0 && ldq % 8 == 0 && C % 8 == 0) {
    if (dtype == UM_BF16)
      return UM_ATTN_D(attn_bwd_mfma_t, bf16_t, d, N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt,
                       ldd, dqkv, ldq, dks_ws, ws, st);
    return UM_ATTN_D(attn_bwd_mfma_t, float, d, N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt, ldd,
                     dqkv, ldq, dks_ws, ws, st);
  }
  if (small_heads(C, heads) && ld % 8 == 0 && ldd % 8 == 0 && ldq % 8 == 0)
    return attn_bwd_small(dtype, N, S, C, heads, qkv, ld, kmax, ksum, ctx, datt, ldd, dqkv, ldq,
                          dks_ws, ws, dctx, r, st);
  const int nt = ceil_div(S, PT);
  const dim3 g(nt, heads, N);
  const size_t shm_a = ((size_t)d * d + 3 * PT * (d + 1)) * sizeof(float);
  static bool attr = false;  // d = 64 needs more than the default 64 KB of dynamic LDS
  if (!attr) {
    const void* ks[] = {reinterpret_cast<const void*>(&apply_bwd_kernel<bf16_t>),
                        reinterpret_cast<const void*>(&apply_bwd_kernel<float>),
                        reinterpret_cast<const void*>(&kv_bwd_kernel<bf16_t>),
                        reinterpret_cast<const void*>(&kv_bwd_kernel<float>)};
    for (const void* k : ks)
      hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(apply_bwd_kernel<bf16_t>, g, dim3(256), shm_a, st, (const bf16_t*)qkv, ld,
                       S, C, heads, ctx, (const bf16_t*)datt, ldd, (bf16_t*)dqkv, ldq, nt, ws);
  else
    hipLaunchKernelGGL(apply_bwd_kernel<float>, g, dim3(256), shm_a, st, (const float*)qkv, ld, S,
                       C, heads, ctx, (const float*)datt, ldd, (float*)dqkv, ldq, nt, ws);
  const int L = heads * d * d;
  {
    const int jl = sum_parts_cols(L, nt);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(ceil_div(L, jl), N), dim3(256), 0, st, ws, N, nt, L,
                       dctx, jl);
  }
  const size_t shm_k = ((size_t)2 * d * d + 3 * PT * d) * sizeof(float);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(kv_bwd_kernel<bf16_t>, g, dim3(256), shm_k, st, (const bf16_t*)qkv, ld, S,
                       C, heads, kmax, ksum, dctx, (bf16_t*)dqkv, ldq, dks_ws, nt, ws);
  else
    hipLaunchKernelGGL(kv_bwd_kernel<float>, g, dim3(256), shm_k, st, (const float*)qkv, ld, S, C,
                       heads, kmax, ksum, dctx, (float*)dqkv, ldq, dks_ws, nt, ws);
  {
    const int jl = sum_parts_cols(C, nt);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(ceil_div(C, jl), N), dim3(256), 0, st, ws, N, nt, C,
                       r, jl);
  }
  const long M = (long)N * S;
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(k_bwd_kernel<bf16_t>, dim3(grid_for(M * C)), dim3(256), 0, st,
                       (const bf16_t*)qkv, ld, M, S, C, kmax, ksum, dks_ws, r, (bf16_t*)dqkv, ldq);
  else
    hipLaunchKernelGGL(k_bwd_kernel<float>, dim3(grid_for(M * C)), dim3(256), 0, st,
                       (const float*)qkv, ld, M, S, C, kmax, ksum, dks_ws, r, (float*)dqkv, ldq);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
