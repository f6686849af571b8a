// SyncBN statistics exchange without RCCL: device-side, over IPC-mapped
// per-rank arenas (reference parallel_main.py:156-158, torch SyncBatchNorm's
// per-layer all-reduce of (sum, sum of squares, count) in forward and
// (sum dz, sum dz*xhat) in backward).
//
// Every rank owns one arena (uncached device memory, hipExtMallocWithFlags
// hipDeviceMallocUncached: coherent across processes and devices without
// cache maintenance) that the other ranks map with hipIpcOpenMemHandle:
//
//   [0, 256)             header: u64 epoch counter, u32 timeout flag
//   [256 + s*stride ...) slot s: u64 flag at +0, 2C + 1 doubles at +64
//
// um_bnx_allreduce (ONE 256-thread workgroup, stream-ordered like the RCCL
// call it replaces, so it is capturable in a HIP graph):
//   1. e = ++epoch (every rank runs the same sequence of exchanges, so the
//      epochs agree: identical on all ranks by construction);
//   2. the 16 local statistics slots (UM_STAT_SLOTS) summed in slot order
//      into the rank's own arena slot s, plus its element count;
//   3. release (system scope) -> flag_s = e;
//   4. one thread per peer polls the peer's flag_s until it reaches e
//      (bounded: after ~2^24 polls it sets the timeout flag and goes on, so
//      no wave can hang the device; um_bnx_status reports it);
//   5. acquire, then every rank sums the ranks' values in RANK ORDER (the
//      same f64 result on every rank) and writes them back as slot 0 of its
//      statistics buffer, slots 1..15 zero, the global count after them --
//      the layout the BN consumers read after an in-place all-reduce.
// A slot is reused only in the next step, after every rank has passed this
// step's later exchanges, each of which waited for every peer: a peer can
// no longer be reading it.
#include "common.h"

namespace {

constexpr long BNX_HDR = 256;
constexpr int BNX_LIMIT_LOG2 = 24;

__device__ __forceinline__ long bnx_stride(int max_c) {
  return ((64 + (2L * max_c + 1) * 8) + 255) / 256 * 256;
}

__global__ void __launch_bounds__(256) bnx_allreduce_kernel(double* __restrict__ stats, int C,
                                                            const unsigned long long* __restrict__ table,
                                                            int world, int rank, int slot,
                                                            int max_c) {
  __shared__ unsigned long long s_epoch;
  __shared__ int s_timeout;
  const int tid = threadIdx.x;
  const long stride = bnx_stride(max_c);
  char* mine = reinterpret_cast<char*>(table[rank]);
  unsigned long long* ctr = reinterpret_cast<unsigned long long*>(mine);
  if (tid == 0) {
    const unsigned long long e =
        __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
    __hip_atomic_store(ctr, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_epoch = e;
    s_timeout = 0;
  }
  __syncthreads();
  const unsigned long long e = s_epoch;
  const int n = 2 * C;
  double* my_data = reinterpret_cast<double*>(mine + BNX_HDR + slot * stride + 64);
  // 2. this rank's sums over its 16 slots (slot order), and its count
  for (int i = tid; i < n; i += blockDim.x) {
    double v = 0.0;
#pragma unroll
    for (int s = 0; s < UM_STAT_SLOTS; ++s) v += stats[(long)s * n + i];
    __hip_atomic_store(&my_data[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid == 0)
    __hip_atomic_store(&my_data[n], stats[(long)UM_STAT_SLOTS * n], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. publish: every storing wave drained, then one release + flag store
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long* flag = reinterpret_cast<unsigned long long*>(mine + BNX_HDR + slot * stride);
    __hip_atomic_store(flag, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 4. wait for every peer's flag of this slot (bounded)
  if (tid < world && tid != rank) {
    const unsigned long long* pf = reinterpret_cast<const unsigned long long*>(
        reinterpret_cast<const char*>(table[tid]) + BNX_HDR + slot * stride);
    unsigned int spins = 0;
    while (__hip_atomic_load(pf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (++spins >> BNX_LIMIT_LOG2) {
        s_timeout = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (s_timeout)
      __hip_atomic_store(reinterpret_cast<unsigned int*>(mine + 8), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  // 5. the ranks' values summed in rank order -> slot 0 of stats, zeros after
  for (int i = tid; i <= n; i += blockDim.x) {
    double v = 0.0;
    for (int r = 0; r < world; ++r) {
      const double* d = reinterpret_cast<const double*>(
          reinterpret_cast<const char*>(table[r]) + BNX_HDR + slot * stride + 64);
      v += __hip_atomic_load(&d[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (i < n) stats[i] = v;
    else stats[(long)UM_STAT_SLOTS * n] = v;
  }
  for (long i = n + tid; i < (long)UM_STAT_SLOTS * n; i += blockDim.x) stats[i] = 0.0;
}

}  // namespace

extern "C" {

long um_bnx_bytes(int nslots, int max_c) {
  return BNX_HDR + (long)nslots * (((64 + (2L * max_c + 1) * 8) + 255) / 256 * 256);
}

int um_bnx_alloc(long bytes, void** base, void* handle64) {
  UM_CHECK_ARG(bytes > 0 && base && handle64, "um_bnx_alloc: arguments");
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    umamd::set_error("um_bnx_alloc: hipExtMallocWithFlags(uncached) failed: %s",
                     hipGetErrorString(hipGetLastError()));
    return UM_ERR_HIP;
  }
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    umamd::set_error("um_bnx_alloc: zeroing failed");
    (void)hipFree(p);
    return UM_ERR_HIP;
  }
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
    umamd::set_error("um_bnx_alloc: hipIpcGetMemHandle failed: %s",
                     hipGetErrorString(hipGetLastError()));
    (void)hipFree(p);
    return UM_ERR_HIP;
  }
  memcpy(handle64, &h, sizeof(h));
  *base = p;
  return UM_OK;
}

int um_bnx_open(const void* handle64, void** ptr) {
  UM_CHECK_ARG(handle64 && ptr, "um_bnx_open: arguments");
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  if (hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    umamd::set_error("um_bnx_open: hipIpcOpenMemHandle failed: %s",
                     hipGetErrorString(hipGetLastError()));
    return UM_ERR_HIP;
  }
  return UM_OK;
}

int um_bnx_close(void* ptr) {
  return hipIpcCloseMemHandle(ptr) == hipSuccess ? UM_OK : UM_ERR_HIP;
}

int um_bnx_free(void* base) { return hipFree(base) == hipSuccess ? UM_OK : UM_ERR_HIP; }

// the timeout flag of this rank's arena (0: every exchange completed)
int um_bnx_status(const void* base) {
  unsigned int v = 0;
  if (hipMemcpy(&v, reinterpret_cast<const char*>(base) + 8, sizeof(v), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return -1;
  return (int)v;
}

int um_bnx_allreduce(double* stats, int C, const unsigned long long* table, int world, int rank,
                     int slot, int nslots, int max_c, hipStream_t st) {
  UM_CHECK_ARG(stats && table && world >= 1 && world <= 256 && rank >= 0 && rank < world &&
                   slot >= 0 && slot < nslots && C > 0 && C <= max_c,
               "um_bnx_allreduce: arguments (C %d, slot %d)", C, slot);
  hipLaunchKernelGGL(bnx_allreduce_kernel, dim3(1), dim3(256), 0, st, stats, C, table, world, rank,
                     slot, max_c);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
