// Common device/host helpers for the umamd HIP library (gfx950 / CDNA4 only).
//
// Activations are NHWC ("channels-last") with an explicit pixel stride `ld`
// (elements between consecutive pixels) so producers can write straight into
// a channel slice of a wider buffer.  Element storage type is either f32 or
// bf16 (UM_F32 / UM_BF16); all arithmetic is f32.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <string.h>

#include "../../include/umamd.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __hip_bfloat16 bf16_t;

// ------------------------------------------------------------ error state --
namespace umamd {
void set_error(const char* fmt, ...);
// Tuning values for sweeps: the ONE environment variable UMAMD_TUNING holds
// "key=value,key=value" (keys as um_set_tuning's); a key not listed there
// gives ``dflt``.  Read once per key by each caller (static initialisers).
long tuning_env(const char* key, long dflt);
}  // namespace umamd

#define UM_CHECK_ARG(cond, ...)                    \
  do {                                             \
    if (!(cond)) {                                 \
      umamd::set_error(__VA_ARGS__);               \
      return UM_ERR_ARG;                           \
    }                                              \
  } while (0)

#define UM_LAUNCH_CHECK()                                               \
  do {                                                                  \
    hipError_t _e = hipGetLastError();                                  \
    if (_e != hipSuccess) {                                             \
      umamd::set_error("%s: %s", __func__, hipGetErrorString(_e));      \
      return UM_ERR_HIP;                                                \
    }                                                                   \
  } while (0)

// ------------------------------------------------------------ conversions --
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return __bfloat162float(x); }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float x) {
  return __float2bfloat16(x);
}

// 8-element vector load/store (16 B for bf16, 32 B for f32) -> f32[8]
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  // round-to-nearest-even via the compiler's cvt (keeps NaN a NaN)
  bf16_t x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) |
         ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}
__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
  uint4 u;
  u.x = pack_bf16x2(v[0], v[1]);
  u.y = pack_bf16x2(v[2], v[3]);
  u.z = pack_bf16x2(v[4], v[5]);
  u.w = pack_bf16x2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

// 4-element vector stores (8 B for bf16, 16 B for f32)
__device__ __forceinline__ void store4(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void store4(bf16_t* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

// the values of v as they are stored in a T tensor (bf16 rounding)
__device__ __forceinline__ void load8_rounded(const float* v, float* r, const float*) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = v[i];
}
__device__ __forceinline__ void load8_rounded(const float* v, float* r, const bf16_t*) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = __bfloat162float(__float2bfloat16(v[i]));
}

// raw 8-element copies (no conversion) used for LDS staging
template <typename T> struct Raw8;
template <> struct Raw8<bf16_t> { uint4 v; };
template <> struct Raw8<float> { uint4 a, b; };
__device__ __forceinline__ void raw_load8(const bf16_t* p, Raw8<bf16_t>& r) {
  r.v = *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void raw_load8(const float* p, Raw8<float>& r) {
  r.a = *reinterpret_cast<const uint4*>(p);
  r.b = *reinterpret_cast<const uint4*>(p + 4);
}
__device__ __forceinline__ void raw_zero(Raw8<bf16_t>& r) { r.v = make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ void raw_zero(Raw8<float>& r) {
  r.a = make_uint4(0, 0, 0, 0);
  r.b = r.a;
}
__device__ __forceinline__ void raw_store8(bf16_t* p, const Raw8<bf16_t>& r) {
  *reinterpret_cast<uint4*>(p) = r.v;
}
__device__ __forceinline__ void raw_store8(float* p, const Raw8<float>& r) {
  *reinterpret_cast<uint4*>(p) = r.a;
  *reinterpret_cast<uint4*>(p + 4) = r.b;
}

// ---------------------------------------------------------- wave helpers --
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Row-chunk x channel-group block mapping shared by the backward kernels:
// thread t owns 8 channels g = t % G (G = min(C/8, 256)) and row lane
// t / G; a block covers BWD_ROWS rows and all channel groups (looped when
// C/8 > 256).  Per-channel results are reduced across row lanes in LDS.
struct RowMap {
  int G, lanes, g, lane;
  __device__ RowMap(int cg) {
    G = cg < 256 ? cg : 256;
    lanes = 256 / G;
    g = threadIdx.x % G;
    lane = threadIdx.x / G;
  }
  __device__ bool active() const { return lane < lanes; }
};

// reduce red[lanes][G][NV] over lanes into thread (lane==0) registers.
// G | 64 (C = 32..256 channels): the lanes of one channel group inside a
// wave are combined with a butterfly of cross-lane shuffles (offsets G..32)
// and only the four wave sums meet in LDS -- no serial 64-lane LDS walk.
template <int NV>
__device__ __forceinline__ void lane_reduce(float* red, const RowMap& rm, float* v) {
  if (rm.G < 64 && (64 % rm.G) == 0) {
    for (int o = rm.G; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < NV; ++e) v[e] += __shfl_xor(v[e], o, 64);
    const int wave = threadIdx.x >> 6, wl = threadIdx.x & 63;
    if (wl < rm.G)
#pragma unroll
      for (int e = 0; e < NV; ++e) red[(wave * rm.G + wl) * NV + e] = v[e];
    __syncthreads();
    if (rm.lane == 0)  // wave 0, wl == g
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
#pragma unroll
        for (int e = 0; e < NV; ++e) v[e] += red[(w * rm.G + rm.g) * NV + e];
    __syncthreads();
    return;
  }
  if (rm.active())
#pragma unroll
    for (int e = 0; e < NV; ++e) red[(rm.lane * rm.G + rm.g) * NV + e] = v[e];
  __syncthreads();
  if (rm.lane == 0) {
    for (int r = 1; r < rm.lanes; ++r)
#pragma unroll
      for (int e = 0; e < NV; ++e) v[e] += red[(r * rm.G + rm.g) * NV + e];
  }
  __syncthreads();
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float eluf_(float x) { return x > 0.f ? x : expm1f(x); }

// reflect index for padding (|pad| < n), torch 'reflect' semantics
__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Arrival on an agent-scope counter shared by `expected` workgroups (the
// producer/consumer recipe of MI355X_MICROARCH.md "Workgroup dispatch":
// every wave drains its stores, the workgroup barrier, lane 0 releases, then
// the relaxed add).  Returns true in the workgroup that arrived last, after
// its acquire, so it may read what the others stored; that workgroup resets
// the counter to 0 for the next use.  `flag`: an LDS int.
__device__ __forceinline__ bool ticket_last(unsigned int* ctr, unsigned int expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == expected - 1;
    if (*flag) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return *flag != 0;
}

// ------------------------------------------------- BN statistics slots --
// Per-channel (sum, sum of squares) accumulated straight into f64 "slots"
// [UM_STAT_SLOTS][C][2] (zeroed by the caller) by no-return f64 atomics: the
// producer of row block b adds into slot b % UM_STAT_SLOTS, so at most
// blocks/16 adders meet on one address (the atomics run at the memory side,
// MI355X_MICROARCH.md "Global float atomics"), and the consumer sums the 16
// slots -- no partial-row array and no separate reduction launch.
__device__ __forceinline__ void stat_slot_add(double* slots, long row_block, int C, int c,
                                              float s0, float s1) {
  double* p = slots + ((row_block % UM_STAT_SLOTS) * C + c) * 2;
  unsafeAtomicAdd(p, (double)s0);
  unsafeAtomicAdd(p + 1, (double)s1);
}

// Block-wide form: the sums of channels [c0, c0 + ncols) of one row block,
// val(i) = value i = 2*col + v (v = 0 sum, 1 sum of squares), one atomic per
// thread on consecutive doubles -- a wave covers 512 contiguous bytes instead
// of one scattered 8-byte request per lane.
template <class F>
__device__ __forceinline__ void stat_slots_add_row(double* slots, long row_block, int C, int c0,
                                                   int ncols, F val) {
  double* p = slots + ((row_block % UM_STAT_SLOTS) * C + c0) * 2;
  for (int i = threadIdx.x; i < 2 * ncols; i += blockDim.x) unsafeAtomicAdd(p + i, (double)val(i));
}

// the element count after the slots (read by the consumers when the host
// passes count <= 0, i.e. after a SyncBN all-reduce of slots + count): one
// plain store by the launch's first workgroup
__device__ __forceinline__ void stat_slots_count(double* slots, int C, long count) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    slots[(long)UM_STAT_SLOTS * C * 2] = (double)count;
}

// Block-wide finish over all C channels: fin(c, s0, s1) is called once per
// channel with the f64 slot sums.  SPL lanes share a channel (each sums every
// SPL-th slot with 16-byte loads, all issued before the first add, then a
// shuffle tree), so a block reads the 16 x C x 16 bytes in one round trip
// for C <= 256; the fixed order makes every block's sums identical.  Must be
// reached by all threads of the block.
// Channel range [c0, c0 + n) only (a block that owns a channel slice).
template <int SPL, class F>
__device__ __forceinline__ void stat_slots_finish_t(const double* __restrict__ slots, int C, int c0,
                                                    int n, F fin) {
  constexpr int PER = UM_STAT_SLOTS / SPL;
  const int total = n * SPL;
  for (int base = 0; base < total; base += blockDim.x) {
    const int idx = base + threadIdx.x;
    const int c = c0 + idx / SPL, part = idx % SPL;
    const bool in = c < c0 + n;
    double2 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k)
      v[k] = in ? *reinterpret_cast<const double2*>(slots + ((long)(part + k * SPL) * C + c) * 2)
                : make_double2(0.0, 0.0);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      s0 += v[k].x;
      s1 += v[k].y;
    }
#pragma unroll
    for (int o = SPL >> 1; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    if (in && part == 0) fin(c, s0, s1);
  }
}

template <class F>
__device__ __forceinline__ void stat_slots_finish(const double* __restrict__ slots, int C, int c0,
                                                  int n, F fin) {
  const int nt = blockDim.x;
  if (16 * n <= nt) stat_slots_finish_t<16>(slots, C, c0, n, fin);
  else if (8 * n <= nt) stat_slots_finish_t<8>(slots, C, c0, n, fin);
  else if (4 * n <= nt) stat_slots_finish_t<4>(slots, C, c0, n, fin);
  else stat_slots_finish_t<2>(slots, C, c0, n, fin);
}

template <class F>
__device__ __forceinline__ void stat_slots_finish(const double* __restrict__ slots, int C, F fin) {
  stat_slots_finish(slots, C, 0, C, fin);
}

// rows per block of the row-chunk reductions (RowMap kernels): aim at about
// 512 blocks (16..1024 rows): small deep layers still fill the chip and the
// full-resolution layers do not write thousands of partial rows
static inline int rows_per_part(long M) {
  const long r = (M + 511) / 512;
  int p = 16;
  while (p < r && p < 1024) p <<= 1;
  return p;
}
static inline int parts_for(long M) { return (int)((M + rows_per_part(M) - 1) / rows_per_part(M)); }
