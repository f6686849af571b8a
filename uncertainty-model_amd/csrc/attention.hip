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

}  // namespace

extern "C" {

// workspace sizes (floats)
long um_attn_ws_kstats(int N, int S, int C) {
  return (long)N * ceil_div(S, ks_chunk(S)) * C * 2;
}
long um_attn_ws_ctx(int N, int S, int C, int heads) {
  const int d = C / heads;
  return (long)N * ceil_div(S, ctx_chunk(d)) * heads * d * d;
}
long um_attn_ws_tiles(int N, int S, int C, int heads) {
  const int d = C / heads;
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
