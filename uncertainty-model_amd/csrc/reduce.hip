// Column reductions of per-block partial rows, finished in the same launch.
//
// Many producers (conv epilogue BN statistics, BN backward sums, bias
// gradients) leave partial rows parts[p][c][v] (v < NV values per channel).
// One launch sums them: each workgroup reduces a chunk of rows for all
// channels into an f64 slab row ws[b][c][v] (fixed order, so the result is
// deterministic), then the LAST workgroup to arrive (agent-scope ticket,
// MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility")
// sums the slab rows and applies the finishing step:
//   COLRED_SUMS      : f64 sums to st[c][v] (SyncBN: the host all-reduces them)
//   COLRED_BN_FWD    : BatchNorm2d train coefficients + running statistics
//                      (reference model/layers/encoder.py:43, decoder.py:82)
//   COLRED_BN_BWD    : BatchNorm2d backward coefficients + dgamma/dbeta
//   COLRED_ROWS      : out[c] (+)= sum (f32; conv-bias gradients)
// This replaces the former two launches (reduce kernel + coefficient kernel)
// per BN layer and per direction.  The ticket counters are static device
// words reset by the last workgroup, so launches of one entry must be
// stream-ordered (one stream per process, as everywhere in umamd).
#include <cstdlib>

#include <cstring>

#include "common.h"
#include "reduce.h"

namespace {

__device__ unsigned int g_ticket[umamd::COLRED_NMODES];

__device__ __forceinline__ void finish(const umamd::ColRed& a, int c, double s0, double s1) {
  switch (a.mode) {
    case umamd::COLRED_SUMS:
      a.st[2 * c] = s0;
      a.st[2 * c + 1] = s1;
      break;
    case umamd::COLRED_BN_FWD: {
      const double mean = s0 / a.count;
      double var = s1 / a.count - mean * mean;
      if (var < 0) var = 0;
      const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
      const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
      a.mean[c] = (float)mean;
      a.invstd[c] = invstd;
      a.scale[c] = g * invstd;
      a.shift[c] = b - (float)mean * g * invstd;
      if (a.running_mean != nullptr) {
        const double unb = a.count > 1 ? var * a.count / (a.count - 1) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * (float)mean;
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * (float)unb;
      }
      break;
    }
    case umamd::COLRED_BN_BWD: {
      // dx = g*invstd*(dz - sdz/n - xhat*sdzx/n); dgamma = sum dz*xhat, dbeta = sum dz
      const float g = a.gamma ? a.gamma[c] : 1.f;
      const float k1 = g * a.invstd_in[c], k2 = (float)(s0 / a.count);
      a.k1[c] = k1;
      a.k2[c] = k2;
      a.k3[c] = (float)(s1 / a.count);
      if (a.dgamma) a.dgamma[c] = (float)s1;
      if (a.dbeta) a.dbeta[c] = (float)s0;
      // conv-bias gradient sum_m dy = k1 (s0 - n k2 - k3 sum xhat), sum xhat = 0
      if (a.dbias) a.dbias[c] = k1 * (float)(s0 - a.count * (double)k2);
      break;
    }
    default:  // COLRED_ROWS
      a.out[c] = a.accumulate ? a.out[c] + (float)s0 : (float)s0;
  }
}

// publish this workgroup's slab row; the last arriver sums the slab rows
// and finishes
template <int NV>
__device__ __forceinline__ void publish_finish(const umamd::ColRed& a) {
  __shared__ int last;
  const int C = a.C;
  const int NT = blockDim.x;
  if (gridDim.x > 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&g_ticket[a.mode], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      last = (t == gridDim.x - 1);
      if (last) {
        __hip_atomic_store(&g_ticket[a.mode], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!last) return;
  } else {
    __syncthreads();
  }
  if (threadIdx.x == 0 && a.mode == umamd::COLRED_BN_FWD && a.nbt != nullptr) *a.nbt += 1;
  for (int c = threadIdx.x; c < C; c += NT) {
    double s0 = 0.0, s1 = 0.0;
    for (int b = 0; b < (int)gridDim.x; ++b) {
      s0 += a.ws[((long)b * C + c) * NV];
      if (NV == 2) s1 += a.ws[((long)b * C + c) * NV + 1];
    }
    finish(a, c, s0, s1);
  }
}


template <int NV>
__global__ void __launch_bounds__(1024) colred_kernel(umamd::ColRed a) {
  __shared__ double red[1024 * NV];
  const int C = a.C;
  const int NT = blockDim.x;
  const int CU = C < NT ? C : NT;
  const int L = NT / CU;
  const int u = threadIdx.x % CU, l = threadIdx.x / CU;
  const long p0 = (long)blockIdx.x * a.rows_per_block;
  const long p1 = min((long)a.nparts, p0 + a.rows_per_block);
  for (int c0 = 0; c0 < C; c0 += CU) {
    const int c = c0 + u;
    double s[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) s[v] = 0.0;
    if (l < L && c < C) {
      const float* q = a.parts + (long)c * NV;
      long p = p0 + l;
      for (; p + 3 * L < p1; p += 4 * L) {  // four rows in flight per lane
        float t[4][NV];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int v = 0; v < NV; ++v) t[k][v] = q[(p + k * L) * a.rowstride + v];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int v = 0; v < NV; ++v) s[v] += (double)t[k][v];
      }
      for (; p < p1; p += L)
#pragma unroll
        for (int v = 0; v < NV; ++v) s[v] += (double)q[p * a.rowstride + v];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) red[threadIdx.x * NV + v] = s[v];
    __syncthreads();
    if (l == 0 && c < C) {
      for (int r = 1; r < L; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) s[v] += red[(r * CU + u) * NV + v];
#pragma unroll
      for (int v = 0; v < NV; ++v) a.ws[((long)blockIdx.x * C + c) * NV + v] = s[v];
    }
    __syncthreads();
  }
  publish_finish<NV>(a);
}

// Vector form of colred_kernel for rows whose C*NV floats are 16-byte
// aligned: a lane sums one float4 (2 channels x (sum, sumsq) for NV = 2) of a
// row and keeps 8 rows in flight, so a 1024-thread workgroup has 4x the bytes
// in flight of the scalar form -- these reductions are latency-bound (a
// single workgroup over <= 512 KB of partials, ~125 launches per step).
template <int NV>
__global__ void __launch_bounds__(1024) colred_vec_kernel(umamd::ColRed a) {
  __shared__ double red[1024 * 4];
  const int F4 = a.C * NV / 4;  // float4 per row
  const int NT = blockDim.x;
  const int CU = F4 < NT ? F4 : NT;
  const int L = NT / CU;
  const int u = threadIdx.x % CU, l = threadIdx.x / CU;
  const long p0 = (long)blockIdx.x * a.rows_per_block;
  const long p1 = min((long)a.nparts, p0 + a.rows_per_block);
  const long rs4 = a.rowstride / 4;
  const float4* q0 = reinterpret_cast<const float4*>(a.parts);
  for (int f0 = 0; f0 < F4; f0 += CU) {
    const int f = f0 + u;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    if (l < L && f < F4) {
      const float4* q = q0 + f;
      long p = p0 + l;
      for (; p + 7 * L < p1; p += 8 * L) {
        float4 t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = q[(p + k * L) * rs4];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s[0] += (double)t[k].x; s[1] += (double)t[k].y;
          s[2] += (double)t[k].z; s[3] += (double)t[k].w;
        }
      }
      for (; p < p1; p += L) {
        const float4 t = q[p * rs4];
        s[0] += (double)t.x; s[1] += (double)t.y; s[2] += (double)t.z; s[3] += (double)t.w;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = s[j];
    __syncthreads();
    if (l == 0 && f < F4) {
      for (int r = 1; r < L; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += red[(r * CU + u) * 4 + j];
      // flat index 4f + j = c * NV + v: the [b][c][v] slab row layout
#pragma unroll
      for (int j = 0; j < 4; ++j) a.ws[(long)blockIdx.x * a.C * NV + 4 * f + j] = s[j];
    }
    __syncthreads();
  }
  publish_finish<NV>(a);
}

}  // namespace

namespace umamd {

// Up to 128K values: ONE 1024-thread workgroup (no ticket, no fences: the
// agent-scope release/acquire pair costs about as much as a kernel boundary,
// MI355X_MICROARCH.md price list).  Larger: 256-thread workgroups of >= 16K
// values each and the last-arriver finish.
// (UMAMD_TUNING colred_single / colred_per override the two sizes for sweeps)
long tuning_env(const char* key, long dflt) {
  const char* v = getenv("UMAMD_TUNING");
  if (v == nullptr) return dflt;
  const size_t n = strlen(key);
  for (const char* p = v; *p;) {
    if (!strncmp(p, key, n) && p[n] == '=') return atol(p + n + 1);
    p = strchr(p, ',');
    if (p == nullptr) break;
    ++p;
  }
  return dflt;
}

int colred_blocks(int nparts, int C, int NV) {
  static const long single = tuning_env("colred_single", 128 * 1024);
  static const long per = tuning_env("colred_per", 16384);
  const long work = (long)nparts * C * NV;
  if (work <= single) return 1;
  long b = (work + per - 1) / per;  // >= `per` values per workgroup
  if (b > 128) b = 128;
  if (b > nparts) b = nparts;
  if (b < 1) b = 1;
  return (int)b;
}

long colred_ws_bytes(int nparts, int C, int NV) {
  return (long)colred_blocks(nparts, C, NV) * C * NV * sizeof(double);
}

int colred_run(ColRed a, int NV, hipStream_t st) {
  if (a.nparts <= 0 || a.C <= 0) return UM_OK;
  const int nb = colred_blocks(a.nparts, a.C, NV);
  a.rows_per_block = ceil_div(a.nparts, nb);
  const int blocks = ceil_div(a.nparts, a.rows_per_block);
  const int threads = blocks == 1 ? 1024 : 256;
  const bool vec = (a.C * NV) % 4 == 0 && a.rowstride % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.parts) & 15) == 0;
  // measured per step on MI355X: NV = 2 (BN statistics) 9.0 -> 8.5 us per
  // launch with the vector form; NV = 1 (bias sums over narrow rows) slower
  // (8.0 -> 9.8 us), so it keeps the scalar form
  if (vec && NV == 2)
    hipLaunchKernelGGL(colred_vec_kernel<2>, dim3(blocks), dim3(threads), 0, st, a);
  else if (NV == 2)
    hipLaunchKernelGGL(colred_kernel<2>, dim3(blocks), dim3(threads), 0, st, a);
  else
    hipLaunchKernelGGL(colred_kernel<1>, dim3(blocks), dim3(threads), 0, st, a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // namespace umamd

extern "C" {

long um_colred_ws(int nparts, int C, int nv) {
  return umamd::colred_ws_bytes(nparts, C, nv == 2 ? 2 : 1);
}

int um_bn_stats_coeffs(const float* parts, int nparts, int C, double* ws, double count,
                       const float* gamma, const float* beta, float eps, float momentum,
                       float* running_mean, float* running_var, long long* num_batches_tracked,
                       float* mean, float* invstd, float* scale, float* shift, hipStream_t st) {
  UM_CHECK_ARG(ws != nullptr && count > 0, "um_bn_stats_coeffs: ws / count");
  umamd::ColRed a{};
  a.parts = parts; a.nparts = nparts; a.C = C; a.rowstride = (long)C * 2; a.ws = ws;
  a.mode = umamd::COLRED_BN_FWD;
  a.count = count; a.gamma = gamma; a.beta = beta; a.eps = eps; a.momentum = momentum;
  a.running_mean = running_mean; a.running_var = running_var; a.nbt = num_batches_tracked;
  a.mean = mean; a.invstd = invstd; a.scale = scale; a.shift = shift;
  return umamd::colred_run(a, 2, st);
}

int um_bn_bwd_stats_coeffs(const float* parts, int nparts, int C, double* ws, double count,
                           const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                           float* dbias, float* k1, float* k2, float* k3, hipStream_t st) {
  UM_CHECK_ARG(ws != nullptr && count > 0, "um_bn_bwd_stats_coeffs: ws / count");
  umamd::ColRed a{};
  a.parts = parts; a.nparts = nparts; a.C = C; a.rowstride = (long)C * 2; a.ws = ws;
  a.mode = umamd::COLRED_BN_BWD;
  a.count = count; a.gamma = gamma; a.invstd_in = invstd; a.dgamma = dgamma; a.dbeta = dbeta;
  a.dbias = dbias; a.k1 = k1; a.k2 = k2; a.k3 = k3;
  return umamd::colred_run(a, 2, st);
}

int um_reduce_rows(const float* partials, int parts, int C, int stride, float* out,
                   int accumulate, double* ws, hipStream_t st) {
  UM_CHECK_ARG(ws != nullptr && stride >= C, "um_reduce_rows: ws / stride");
  umamd::ColRed a{};
  a.parts = partials; a.nparts = parts; a.C = C; a.rowstride = stride; a.ws = ws;
  a.mode = umamd::COLRED_ROWS;
  a.out = out; a.accumulate = accumulate;
  return umamd::colred_run(a, 1, st);
}

int um_bn_stats_reduce(const float* parts, int nparts, int C, double* out, double* ws,
                       hipStream_t st) {
  UM_CHECK_ARG(ws != nullptr, "um_bn_stats_reduce: ws");
  umamd::ColRed a{};
  a.parts = parts; a.nparts = nparts; a.C = C; a.rowstride = (long)C * 2; a.ws = ws;
  a.mode = umamd::COLRED_SUMS;
  a.st = out;
  return umamd::colred_run(a, 2, st);
}

}  // extern "C"
