// The disparity / uncertainty heads as VALU kernels: reference
// model/layers/decoder.py:244-247, disp = scale * sigmoid(Conv3x3(
// ReflectionPad2d(1)(x))) with 4 output channels (left/right disparity,
// left/right uncertainty), at every decoder scale (C = 32..256 input
// channels, 256x512 .. 32x64 at B=8).
//
// A 4-output conv is a GEMM with N = 4: an MFMA tile computes 16 (or more)
// output columns, so 3/4 of every MFMA and of the tile's LDS staging is
// padding, and the implicit-GEMM / halo kernels built for wide outputs ran
// these convs at 7-57 TFLOP/s (forward 42 us and data gradient 86 us at
// 256x512; ~0.35 ms per step for the four heads, profiles/r03/w_counters.json).
// Here a thread owns one output pixel (forward) or one input pixel and 8
// channels (data gradient) and runs the 3x3xC (or 3x3x4) reduction in f32
// registers; the f32 weights sit in LDS as float4 (w0..w3)[tap][c], read by
// whole waves at one address (broadcast).  So the heads also compute with
// the f32 weights (the bf16 MFMA path needed the split-bf16 pack for that).
#include <algorithm>

#include "common.h"

namespace {

__device__ __forceinline__ int reflect1(int i, int n) {
  // ReflectionPad2d(1) index map for i in [-1, n]
  return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

// sw[t * Cp + c] = (w[0][c][t], w[1][c][t], w[2][c][t], w[3][c][t]), zero
// for c >= Creal; w is the reference layout [4][Creal][3][3] (f32)
__device__ __forceinline__ void stage_head_weights(float4* sw, const float* __restrict__ w,
                                                   int Creal, int Cp) {
  for (int i = threadIdx.x; i < 9 * Cp; i += blockDim.x) {
    const int t = i / Cp, c = i - t * Cp;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < Creal) {
      v.x = w[(0 * Creal + c) * 9 + t];
      v.y = w[(1 * Creal + c) * 9 + t];
      v.z = w[(2 * Creal + c) * 9 + t];
      v.w = w[(3 * Creal + c) * 9 + t];
    }
    sw[i] = v;
  }
  __syncthreads();
}

// forward: a block owns 64 output pixels (one per lane) and its 4 waves
// split the input channels in quarters (Cp % 32 == 0: so the small deep
// heads, 16k pixels at C = 256, still fill the chip); the partial sums meet
// in LDS and wave 0 writes d[m][0..3] = scale * sigmoid(sum + bias)
template <typename T>
__global__ void __launch_bounds__(256) head_fwd_kernel(const T* __restrict__ x, int ldx, int N,
                                                        int H, int W, int Creal, int Cp,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        float scale, float* __restrict__ d) {
  extern __shared__ float4 sw[];  // [9][Cp] weights, then [4 waves][64] partial sums
  stage_head_weights(sw, w, Creal, Cp);
  float4* part = sw + 9 * Cp;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cq = Cp / 4, c0 = wave * cq;
  const float b0 = bias ? bias[0] : 0.f, b1 = bias ? bias[1] : 0.f;
  const float b2 = bias ? bias[2] : 0.f, b3 = bias ? bias[3] : 0.f;
  const long M = (long)N * H * W;
  for (long m0 = (long)blockIdx.x * 64; m0 < M; m0 += (long)gridDim.x * 64) {
    const long m = m0 + lane;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (m < M) {
      const int xo = (int)(m % W);
      const long r = m / W;
      const int yo = (int)(r % H);
      const long nbase = (r / H) * H;
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        const long row = (nbase + reflect1(yo + ty - 1, H)) * W;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          const T* px = x + (row + reflect1(xo + tx - 1, W)) * ldx;
          const float4* wt = sw + (ty * 3 + tx) * Cp;
          for (int c8 = c0; c8 < c0 + cq; c8 += 8) {
            float v[8];
            load8(px + c8, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float4 q = wt[c8 + e];
              a0 = fmaf(v[e], q.x, a0);
              a1 = fmaf(v[e], q.y, a1);
              a2 = fmaf(v[e], q.z, a2);
              a3 = fmaf(v[e], q.w, a3);
            }
          }
        }
      }
    }
    part[wave * 64 + lane] = make_float4(a0, a1, a2, a3);
    __syncthreads();
    if (wave == 0 && m < M) {
      float4 s = part[lane];
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float4 u = part[k * 64 + lane];
        s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
      }
      *reinterpret_cast<float4*>(d + m * 4) =
          make_float4(scale * sigmoidf_(s.x + b0), scale * sigmoidf_(s.y + b1),
                      scale * sigmoidf_(s.z + b2), scale * sigmoidf_(s.w + b3));
    }
    __syncthreads();
  }
}

// the (q, tap) pairs of one axis that reach input index p through
// ReflectionPad2d(1) + a 3-tap window: q + t - 1 == p, plus the reflected
// reads q + t - 1 == -1 (-> 1) and == n (-> n - 2)
__device__ __forceinline__ int taps_of(int p, int n, int* q, int* t) {
  int k = 0;
#pragma unroll
  for (int tt = 0; tt < 3; ++tt) {
    const int qq = p - tt + 1;
    if (qq >= 0 && qq < n) { q[k] = qq; t[k] = tt; ++k; }
  }
  if (p == 1) { q[k] = 0; t[k] = 0; ++k; }
  if (p == n - 2) { q[k] = n - 1; t[k] = 2; ++k; }
  return k;
}

// data gradient: thread = (input pixel m, channel group g of 8); dx[m][g*8..]
// (+)= sum over the (q, t) pairs of dl[q][k] * w[k][c][t].  Items are ordered
// g-major so a wave's lanes share g (broadcast weight reads).
template <typename T>
__global__ void __launch_bounds__(256) head_dgrad_kernel(const T* __restrict__ dl, int ldl,
                                                          int N, int H, int W, int Creal, int Cp,
                                                          const float* __restrict__ w,
                                                          T* __restrict__ dx, int ldx,
                                                          int accumulate) {
  extern __shared__ float4 sw[];
  stage_head_weights(sw, w, Creal, Cp);
  const long M = (long)N * H * W;
  const int G = Cp / 8;
  const long items = M * G;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < items;
       it += (long)gridDim.x * blockDim.x) {
    const int g = (int)(it / M);
    const long m = it - (long)g * M;
    const int xi = (int)(m % W);
    const long r = m / W;
    const int yi = (int)(r % H);
    const long nbase = (r / H) * H;
    int qy[5], ty[5], qx[5], tx[5];  // 3 direct taps + 2 reflected (both at n == 3)
    const int ny = taps_of(yi, H, qy, ty), nx = taps_of(xi, W, qx, tx);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int a = 0; a < ny; ++a) {
      const long row = (nbase + qy[a]) * W;
      for (int b = 0; b < nx; ++b) {
        float l[8];
        load8(dl + (row + qx[b]) * ldl, l);  // channels 0..3 are the four outputs
        const float4* wt = sw + (ty[a] * 3 + tx[b]) * Cp + g * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float4 q = wt[e];
          acc[e] = fmaf(l[0], q.x, fmaf(l[1], q.y, fmaf(l[2], q.z, fmaf(l[3], q.w, acc[e]))));
        }
      }
    }
    T* o = dx + m * ldx + g * 8;
    if (accumulate) {
      float prev[8];
      load8(o, prev);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += prev[e];
    }
    store8(o, acc);
  }
}

// weight (and bias) gradient: dW[k][c][t] = sum_q dl[q][k] x[reflect(q + t)][c],
// db[k] = sum_q dl[q][k].  A block walks 8 x 32 output tiles (persistent over
// tiles, grid.y = 32-channel chunks): the reflect-padded 10 x 34 input tile of
// its 32 channels and the tile's dl (float4 per pixel) are staged in LDS;
// thread = (channel pair cp, pixel subset ps of 16 pixels) keeps the 2 x 9 x 4
// partial sums in registers over all its tiles; at the end the 16 subsets are
// reduced (wave shuffles, then LDS over the 4 waves) and added into the
// zeroed f32 dW / db with one atomic per value and block.
constexpr int WTY = 8, WTX = 32, WCC = 32;  // tile rows, cols, channels per chunk

__device__ __forceinline__ void load2(const bf16_t* p, float& a, float& b) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  a = __uint_as_float(u << 16);
  b = __uint_as_float(u & 0xffff0000u);
}
__device__ __forceinline__ void load2(const float* p, float& a, float& b) {
  const float2 u = *reinterpret_cast<const float2*>(p);
  a = u.x;
  b = u.y;
}
template <typename T>
__global__ void __launch_bounds__(256) head_wgrad_kernel(const T* __restrict__ x, int ldx,
                                                          const T* __restrict__ dl, int ldl,
                                                          int N, int H, int W, int Creal,
                                                          float* __restrict__ dw,
                                                          float* __restrict__ db) {
  __shared__ T sx[WTY + 2][WTX + 2][WCC];
  __shared__ float4 sdl[WTY][WTX];
  __shared__ float red[4][16][73];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cp = tid & 15, ps = tid >> 4;        // channel pair, pixel subset
  // subset ps: row ps >> 1, columns (ps & 1) + 2j: the 4 subsets of a wave
  // read 4 distinct LDS bank groups (pixels 64 B apart, rows 34 pixels apart)
  const int prow = ps >> 1, pcol0 = ps & 1;
  const int c0 = blockIdx.y * WCC;
  const int tiles_x = (W + WTX - 1) / WTX, tiles_y = (H + WTY - 1) / WTY;
  const int ntiles = N * tiles_x * tiles_y;
  float acc[2][9][4];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[e][t][k] = 0.f;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / (tiles_x * tiles_y), rem = tile - n * tiles_x * tiles_y;
    const int y0 = (rem / tiles_x) * WTY, x0 = (rem % tiles_x) * WTX;
    // the input tile: padded rows y0-1 .. y0+WTY, cols x0-1 .. x0+WTX
    for (int i = tid; i < (WTY + 2) * (WTX + 2) * (WCC / 8); i += 256) {
      const int c8 = i % (WCC / 8), px = i / (WCC / 8);
      const int ry = px / (WTX + 2), rx = px - ry * (WTX + 2);
      const int yy = reflect1(min(y0 - 1 + ry, H), H), xx = reflect1(min(x0 - 1 + rx, W), W);
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int c = c0 + c8 * 8;  // c < Creal: c + 8 <= ceil8(Creal) <= ldx
      if (c < Creal) load8(x + (((long)n * H + yy) * W + xx) * ldx + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (c + e < Creal) ? v[e] : 0.f;
      store8(&sx[ry][rx][c8 * 8], v);
    }
    {
      const int ly = tid / WTX, lx = tid % WTX;
      const int yy = y0 + ly, xx = x0 + lx;
      float4 l = make_float4(0.f, 0.f, 0.f, 0.f);
      if (yy < H && xx < W) {
        float v[8];
        load8(dl + (((long)n * H + yy) * W + xx) * ldl, v);
        l = make_float4(v[0], v[1], v[2], v[3]);
      }
      sdl[ly][lx] = l;
      if (blockIdx.y == 0) {
        bsum[0] += l.x; bsum[1] += l.y; bsum[2] += l.z; bsum[3] += l.w;
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < 16; ++j) {
      const int col = pcol0 + 2 * j;
      const float4 l = sdl[prow][col];
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          float xa, xb;
          load2(&sx[prow + ty][col + tx][2 * cp], xa, xb);
          const int t = ty * 3 + tx;
          acc[0][t][0] = fmaf(xa, l.x, acc[0][t][0]);
          acc[0][t][1] = fmaf(xa, l.y, acc[0][t][1]);
          acc[0][t][2] = fmaf(xa, l.z, acc[0][t][2]);
          acc[0][t][3] = fmaf(xa, l.w, acc[0][t][3]);
          acc[1][t][0] = fmaf(xb, l.x, acc[1][t][0]);
          acc[1][t][1] = fmaf(xb, l.y, acc[1][t][1]);
          acc[1][t][2] = fmaf(xb, l.z, acc[1][t][2]);
          acc[1][t][3] = fmaf(xb, l.w, acc[1][t][3]);
        }
    }
    __syncthreads();
  }
  // reduce over the pixel subsets: lanes cp, cp+16, cp+32, cp+48 of a wave,
  // then the 4 waves through LDS
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = acc[e][t][k];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        acc[e][t][k] = v;
      }
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) red[wave][lane][(e * 9 + t) * 4 + k] = acc[e][t][k];
  }
  __syncthreads();
  for (int i = tid; i < 16 * 72; i += 256) {
    const int cpi = i / 72, r = i - cpi * 72;
    const int e = r / 36, t = (r / 4) % 9, k = r % 4;
    const int c = c0 + 2 * cpi + e;
    if (c >= Creal) continue;
    const float v = red[0][cpi][r] + red[1][cpi][r] + red[2][cpi][r] + red[3][cpi][r];
    atomicAdd(dw + ((long)k * Creal + c) * 9 + t, v);
  }
  if (db != nullptr && blockIdx.y == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = bsum[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      bsum[k] = v;
    }
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) red[0][wave][k] = bsum[k];
    __syncthreads();
    if (tid < 4) atomicAdd(db + tid, red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid]);
  }
}

int grid_of(long items) {
  const long b = (items + 255) / 256;
  return (int)std::min<long>(b, 4096);
}

}  // namespace

extern "C" {

int um_head_fwd(int dtype, int N, int H, int W, int Creal, int Cp, int ldx, const void* x,
                const float* w, const float* bias, float scale, float* d, hipStream_t st) {
  UM_CHECK_ARG(Cp % 8 == 0 && ldx % 8 == 0 && Cp >= Creal && ldx >= Cp && H >= 2 && W >= 2,
               "um_head_fwd: channels / strides (C %d Cp %d ldx %d, %dx%d)", Creal, Cp, ldx, H,
               W);
  UM_CHECK_ARG(x && w && d, "um_head_fwd: null pointer");
  UM_CHECK_ARG(Cp % 32 == 0, "um_head_fwd: Cp %d not a multiple of 32", Cp);
  const long M = (long)N * H * W;
  const size_t shm = (9 * (size_t)Cp + 256) * sizeof(float4);
  UM_CHECK_ARG(shm <= 64 * 1024, "um_head_fwd: C %d too large", Cp);
  const int grid = (int)std::min<long>((M + 63) / 64, 8192);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, dim3(grid), dim3(256), shm, st,
                       (const bf16_t*)x, ldx, N, H, W, Creal, Cp, w, bias, scale, d);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(grid), dim3(256), shm, st,
                       (const float*)x, ldx, N, H, W, Creal, Cp, w, bias, scale, d);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_head_dgrad(int dtype, int N, int H, int W, int Creal, int Cp, const void* dl, int ldl,
                  const float* w, void* dx, int ldx, int accumulate, hipStream_t st) {
  UM_CHECK_ARG(Cp % 8 == 0 && ldx % 8 == 0 && ldl % 8 == 0 && Cp >= Creal && ldx >= Cp &&
                   H >= 2 && W >= 2,
               "um_head_dgrad: channels / strides (C %d Cp %d ldx %d ldl %d, %dx%d)", Creal, Cp,
               ldx, ldl, H, W);
  UM_CHECK_ARG(dl && w && dx, "um_head_dgrad: null pointer");
  const long items = (long)N * H * W * (Cp / 8);
  const size_t shm = 9 * (size_t)Cp * sizeof(float4);
  UM_CHECK_ARG(shm <= 64 * 1024, "um_head_dgrad: C %d too large", Cp);
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(head_dgrad_kernel<bf16_t>, dim3(grid_of(items)), dim3(256), shm, st,
                       (const bf16_t*)dl, ldl, N, H, W, Creal, Cp, w, (bf16_t*)dx, ldx,
                       accumulate);
  else
    hipLaunchKernelGGL(head_dgrad_kernel<float>, dim3(grid_of(items)), dim3(256), shm, st,
                       (const float*)dl, ldl, N, H, W, Creal, Cp, w, (float*)dx, ldx, accumulate);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

int um_head_wgrad(int dtype, int N, int H, int W, int Creal, int ldx, const void* x,
                  const void* dl, int ldl, float* dw, float* db, hipStream_t st) {
  UM_CHECK_ARG(ldx % 8 == 0 && ldl % 8 == 0 && ldl >= 4 && H >= 2 && W >= 2 &&
                   ldx >= (Creal + 7) / 8 * 8,
               "um_head_wgrad: channels / strides (C %d ldx %d ldl %d, %dx%d)", Creal, ldx, ldl,
               H, W);
  UM_CHECK_ARG(x && dl && dw, "um_head_wgrad: null pointer");
  const int chunks = (Creal + WCC - 1) / WCC;
  const int ntiles = N * ((H + WTY - 1) / WTY) * ((W + WTX - 1) / WTX);
  // persistent over tiles: ~2 blocks per CU in total over the chunks
  const int gx = std::max(1, std::min(ntiles, 512 / chunks));
  if (dtype == UM_BF16)
    hipLaunchKernelGGL(head_wgrad_kernel<bf16_t>, dim3(gx, chunks), dim3(256), 0, st,
                       (const bf16_t*)x, ldx, (const bf16_t*)dl, ldl, N, H, W, Creal, dw, db);
  else
    hipLaunchKernelGGL(head_wgrad_kernel<float>, dim3(gx, chunks), dim3(256), 0, st,
                       (const float*)x, ldx, (const float*)dl, ldl, N, H, W, Creal, dw, db);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

}  // extern "C"
