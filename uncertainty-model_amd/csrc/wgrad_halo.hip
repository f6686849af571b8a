// Halo-tiled weight gradient for small-channel spatial convolutions (gfx950).
//
//   dW[k][r][s][c] = sum_{n,p,q} DY[n,p,q,k] * X[n, p*st-pad+r, q*st-pad+s, c]
//
// The implicit-GEMM weight gradient re-gathers X once per tap; for the
// high-resolution 32..64-channel layers (encoder stages 1-2 with 7x7 / 5x5
// taps, decoder 3x3 convs at 1/2 and full resolution) that gather, not the
// MFMA, bounds it.  Here a block stages one output-pixel tile of DY and the
// matching X halo ONCE into LDS, in their natural NHWC order, and every tap
// reads its shifted window from that image:
//   - MFMA v_mfma_f32_16x16x32_bf16 with the reduction over 32 pixels;
//     A = DY^T (16 output channels x 32 pixels), B = X_shift (32 pixels x 16
//     input channels), both fragments read transposed from the pixel-major
//     images with ds_read_b64_tr_b16 (per 16-lane group: 4 pixel rows x 16
//     channels -> lane i gets channel i of the 4 pixels);
//   - the images swizzle 16-channel (32-B) chunks by a parity function of
//     the pixel index, chosen per (channel chunks, stride) by exhaustive
//     search over the gfx950 32-lane bank groups (conflict-free for the
//     stride-1 layers);
//   - 8 waves; wave w owns taps w, w+8, ... of the block's tap group and all
//     (16 x 16) output tiles of those taps, so one A fragment feeds every
//     tap and one B fragment every output-channel tile;
//   - blocks stride over pixel tiles and write one f32 partial slab each
//     ([split][K][R*R*C], the layout of the generic kernel), summed by
//     wgrad_reduce_kernel.
// Replaces the weight-gradient half of the nn.Conv2d backward of reference
// model/layers/encoder.py:36-41 and model/layers/decoder.py:37-41.
#include <algorithm>

#include <map>
#include <mutex>

#include "common.h"
#include "wgrad_halo.h"

namespace {

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

struct HwArgs {
  const bf16_t* x;
  const bf16_t* dy;
  float* slabs;
  int N, H, W, C, ldx;   // input
  int P, Q, K, ldy;      // output-gradient
  int R, stride, pad, reflect;
  int cimg, kimg;        // image channel strides (16 * power of two)
  int xm0, xm1, xm2;     // X image swizzle bit positions (31 = unused)
  int ym0, ym1, ym2;     // DY image swizzle bit positions
  int cshift, kshift;    // log2(cimg), log2(kimg)
  int TH, TW, HH, HWd;   // pixel tile; halo rows and row stride (pixels, % 32 == 0)
  int HWr, twshift;      // real halo row length, log2(TW)
  int tiles_x, tiles_y, ntiles;
  int taps_per_group;
};

// swizzle of 32-B channel chunks: bits (pix >> s_i) & 1 (masks are single
// bits; unused entries shift by 31, which reads 0 for any pixel index)
__device__ __forceinline__ int swz(int pix, int s0, int s1, int s2) {
  return ((pix >> s0) & 1) | (((pix >> s1) & 1) << 1) | (((pix >> s2) & 1) << 2);
}

// element offset of 8-channel chunk c8 of pixel pix in a swizzled image
__device__ __forceinline__ int img_off(int pix, int c8, int cimg, int m0, int m1, int m2) {
  const int c16 = (c8 >> 1) ^ swz(pix, m0, m1, m2);
  return pix * cimg + (c16 << 4) + ((c8 & 1) << 3);
}

__device__ __forceinline__ bf16x4_t tr_read(const bf16_t* img, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (__attribute__((address_space(3))) bf16x4_t*)(img + off));
}

template <int KT, int CT, int TPW>
__global__ void __launch_bounds__(512) hwgrad_kernel(HwArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* sY = smem;                              // [TH*TW][kimg]
  bf16_t* sX = smem + a.TH * a.TW * a.kimg;       // [HH][HWd][cimg], HWd % 32 == 0

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int RR = a.R * a.R;
  const int tap0 = blockIdx.y * a.taps_per_group;
  const int tap1 = min(RR, tap0 + a.taps_per_group);
  const int st = a.stride;

  // LDS element offsets of this lane's transposed reads relative to a
  // chunk's base pixel.  Chunk bases are multiples of 32 pixels (tile rows
  // of 32/64 and halo rows padded to HWd % 32 == 0), so the swizzle of the
  // lane's pixel, which uses bits 0..4 only, is the same in every chunk:
  // precompute it once per (tap, channel tile, read).
  int xo[TPW][CT][2];
  bool my_ok[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = tap0 + wave + 8 * i;
    my_ok[i] = t < tap1;
    const int tt = my_ok[i] ? t : tap0;  // unused slots read a valid tap, never stored
    const int r = tt / a.R, s = tt - (tt / a.R) * a.R;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pix = r * a.HWd + s + (8 * g + q + 4 * h) * st;
      const int sw = swz(pix, a.xm0, a.xm1, a.xm2);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) xo[i][ct][h] = (pix << a.cshift) + 4 * p + ((ct ^ sw) << 4);
    }
  }
  int yo[KT][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pix = 8 * g + q + 4 * h;
    const int sw = swz(pix, a.ym0, a.ym1, a.ym2);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) yo[kt][h] = (pix << a.kshift) + 4 * p + ((kt ^ sw) << 4);
  }
  bool any = false;
#pragma unroll
  for (int i = 0; i < TPW; ++i) any |= my_ok[i];

  f32x4_t acc[TPW][KT][CT];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[i][kt][ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int tpi = a.tiles_x * a.tiles_y;
  const int kc8s = a.kshift - 3, cc8s = a.cshift - 3;  // log2 of 8-channel chunks per pixel
  const int tile_pix = a.TH * a.TW;
  const int chunks_per_row = a.TW >> 5;
  const int ny = tile_pix << kc8s;          // DY elements (16 B each)
  const int nxr = a.HWr << cc8s;            // X elements per halo row
  const int nx = a.HH * nxr;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int n = tile / tpi;
    const int tr = tile - n * tpi;
    const int py0 = (tr / a.tiles_x) * a.TH;
    const int qx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * a.TW;
    const int iy0 = py0 * st - a.pad, ix0 = qx0 * st - a.pad;
    // ---- stage DY tile and X halo: 4 loads in flight per thread before the
    // LDS stores; index decode by shifts (power-of-two widths) and one
    // division by the halo row length
    for (int i0 = tid; i0 < ny + nx; i0 += 4 * 512) {
      uint4 v[4];
      int off[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 512;
        v[u] = make_uint4(0, 0, 0, 0);
        off[u] = -1;
        if (i < ny) {
          const int pix = i >> kc8s, c8 = i & ((1 << kc8s) - 1);
          const int py = py0 + (pix >> a.twshift), qx = qx0 + (pix & (a.TW - 1));
          off[u] = img_off(pix, c8, a.kimg, a.ym0, a.ym1, a.ym2);
          if (py < a.P && qx < a.Q && c8 * 8 < a.K)
            v[u] = *reinterpret_cast<const uint4*>(
                a.dy + ((long)(n * a.P + py) * a.Q + qx) * a.ldy + c8 * 8);
        } else if (i < ny + nx) {
          const int j = i - ny;
          const int hr = j / nxr;
          const int jr = j - hr * nxr;
          const int hc = jr >> cc8s, c8 = jr & ((1 << cc8s) - 1);
          int iy = iy0 + hr, ix = ix0 + hc;
          if (a.reflect) {
            iy = reflect_idx(iy, a.H);
            ix = reflect_idx(ix, a.W);
          }
          off[u] = a.TH * a.TW * a.kimg + img_off(hr * a.HWd + hc, c8, a.cimg, a.xm0, a.xm1, a.xm2);
          if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W && c8 * 8 < a.C)
            v[u] = *reinterpret_cast<const uint4*>(
                a.x + ((long)(n * a.H + iy) * a.W + ix) * a.ldx + c8 * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (off[u] >= 0) *reinterpret_cast<uint4*>(smem + off[u]) = v[u];
    }
    __syncthreads();
    if (any) {
      for (int ch = 0; ch < tile_pix / 32; ++ch) {
        const int ty = ch / chunks_per_row, tx0 = (ch - ty * chunks_per_row) * 32;
        const bf16_t* yb = sY + ((ty * a.TW + tx0) << a.kshift);
        const bf16_t* xb = sX + ((ty * st * a.HWd + tx0 * st) << a.cshift);
        bf16x8_t fa[KT];
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const bf16x4_t lo = tr_read(yb, yo[kt][0]), hi = tr_read(yb, yo[kt][1]);
          fa[kt] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        bf16x8_t fb[TPW][CT];
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const bf16x4_t lo = tr_read(xb, xo[i][ct][0]), hi = tr_read(xb, xo[i][ct][1]);
            fb[i][ct] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int kt = 0; kt < KT; ++kt)
              acc[i][kt][ct] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kt], fb[i][ct], acc[i][kt][ct], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- partial slab [split][K][R][R][C]
  float* out = a.slabs + (long)blockIdx.x * a.K * RR * a.C;
  const long rrc = (long)RR * a.C;
  const int col = lane & 15, row4 = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (!my_ok[i]) continue;
    const int tap = tap0 + wave + 8 * i;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int c = ct * 16 + col;
        if (c >= a.C) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = kt * 16 + row4 + e;
          if (k < a.K) out[(long)k * rrc + (long)tap * a.C + c] = acc[i][kt][ct][e];
        }
      }
  }
}

int pow2_chunks(int ch) {  // 16-channel chunks rounded up to a power of two
  int n = (ch + 15) / 16, p = 1;
  while (p < n) p <<= 1;
  return p;
}

// bank-conflict-minimising swizzle (exhaustive search over parity masks,
// see file header; the winners are single bits): bit positions, 31 = unused
void masks_for(int nch, int stride, int* m) {
  m[0] = m[1] = m[2] = 31;
  if (nch == 2) m[0] = stride == 1 ? 3 : 2;
  if (nch == 4) { m[0] = 1; m[1] = stride == 1 ? 3 : 2; }
  if (nch == 8) {
    if (stride == 1) { m[0] = 0; m[1] = 1; m[2] = 3; }
    else { m[0] = 1; m[1] = 2; m[2] = 4; }
  }
}

int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return r;
}

struct HwPlan {
  bool ok;
  int KT, CT, TPW, groups, splits;
  HwArgs a;
  size_t lds;
};

int blocks_per_cu(const HwPlan& h);
int cu_count();

HwPlan plan(int N, int H, int W, int C, int ldx, int K, int R, int stride, int pad, int reflect,
            int P, int Q, int ldy) {
  HwPlan h{};
  h.ok = false;
  if (R < 3 || Q < 32 || (stride != 1 && stride != 2)) return h;
  const int nct = pow2_chunks(C), nkt = pow2_chunks(K);
  if (nct > 8 || nkt > 8) return h;
  const int tiles_per_tap = nct * nkt;
  if (tiles_per_tap > 32) return h;
  int tpw = 32 / tiles_per_tap;
  const int RR = R * R;
  tpw = std::min(tpw, (RR + 7) / 8);
  // template instances available: TPW in {1, 2, 4, 7}
  if (tpw >= 7) tpw = 7;
  else if (tpw >= 4) tpw = 4;
  else if (tpw >= 2) tpw = 2;
  else tpw = 1;
  h.KT = nkt;
  h.CT = nct;
  h.TPW = tpw;
  h.groups = (RR + 8 * tpw - 1) / (8 * tpw);
  HwArgs& a = h.a;
  a.N = N; a.H = H; a.W = W; a.C = C; a.ldx = ldx;
  a.P = P; a.Q = Q; a.K = K; a.ldy = ldy;
  a.R = R; a.stride = stride; a.pad = pad; a.reflect = reflect;
  a.cimg = 16 * nct;
  a.kimg = 16 * nkt;
  a.cshift = ilog2(a.cimg);
  a.kshift = ilog2(a.kimg);
  int m[3];
  masks_for(nct, stride, m);
  a.xm0 = m[0]; a.xm1 = m[1]; a.xm2 = m[2];
  masks_for(nkt, 1, m);
  a.ym0 = m[0]; a.ym1 = m[1]; a.ym2 = m[2];
  // pixel tile: 256 or 128 pixels, 64 or 32 wide; keep LDS <= 76 KB (2 blocks/CU)
  for (int tp : {256, 128}) {
    a.TW = Q >= 64 ? 64 : 32;
    a.TH = tp / a.TW;
    a.HH = (a.TH - 1) * stride + R;
    a.HWr = (a.TW - 1) * stride + R;
    a.HWd = (a.HWr + 31) / 32 * 32;
    a.twshift = ilog2(a.TW);
    h.lds = (size_t)2 * (a.TH * a.TW * a.kimg + a.HH * a.HWd * a.cimg);
    if (h.lds <= 80 * 1024) break;
  }
  if (h.lds > 150 * 1024) return h;
  a.tiles_x = (Q + a.TW - 1) / a.TW;
  a.tiles_y = (P + a.TH - 1) / a.TH;
  a.ntiles = N * a.tiles_x * a.tiles_y;
  a.taps_per_group = 8 * tpw;
  // splits: ONE round of resident workgroups (occupancy x CUs; the wide
  // instances hold ~200 VGPRs, one workgroup per CU: 327 workgroups of the
  // 128x256 7x7 layer ran as 1.3 rounds), >= 2 tiles per block, <= 64 MB of
  // slabs
  const long slab = (long)K * RR * C * 4;
  const long resident = (long)std::max(1, blocks_per_cu(h)) * cu_count();
  long sp = std::max<long>(1, resident / h.groups);
  sp = std::min<long>(sp, (a.ntiles + 1) / 2);
  sp = std::min<long>(sp, std::max<long>(1, (64l << 20) / slab));
  h.splits = (int)std::max<long>(1, sp);
  h.ok = true;
  return h;
}

template <int KT, int CT, int TPW>
int launch_hw(const HwPlan& h, float* slabs, hipStream_t st) {
  HwArgs a = h.a;
  a.slabs = slabs;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&hwgrad_kernel<KT, CT, TPW>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((hwgrad_kernel<KT, CT, TPW>), dim3(h.splits, h.groups), dim3(512), h.lds, st,
                     a);
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// (KT, CT, TPW) instances: KT*CT*TPW <= 32, TPW snapped to {1, 2, 4, 7}
#define HW_INSTANCES(X)                                                     \
  X(1, 1, 2) X(1, 1, 4) X(1, 1, 7) X(1, 2, 2) X(1, 2, 4) X(1, 2, 7)         \
  X(2, 1, 2) X(2, 1, 4) X(2, 1, 7) X(1, 4, 2) X(1, 4, 4) X(1, 4, 7)         \
  X(4, 1, 2) X(4, 1, 4) X(4, 1, 7) X(2, 2, 2) X(2, 2, 4) X(2, 2, 7)         \
  X(2, 4, 2) X(2, 4, 4) X(4, 2, 2) X(4, 2, 4) X(1, 8, 2) X(1, 8, 4)         \
  X(8, 1, 2) X(8, 1, 4) X(4, 4, 1) X(4, 4, 2) X(2, 8, 1) X(2, 8, 2)         \
  X(8, 2, 1) X(8, 2, 2) X(4, 8, 1) X(8, 4, 1)

#define HW_LAUNCH(kt, ct, tpw) \
  if (h.KT == kt && h.CT == ct && h.TPW == tpw) return launch_hw<kt, ct, tpw>(h, slabs, st);
#define HW_EXISTS(kt, ct, tpw) \
  if (h.KT == kt && h.CT == ct && h.TPW == tpw) return true;

int dispatch(const HwPlan& h, float* slabs, hipStream_t st) {
  HW_INSTANCES(HW_LAUNCH)
  return -1;
}
bool exists(const HwPlan& h) {
  HW_INSTANCES(HW_EXISTS)
  return false;
}

// cached per (instance, dynamic LDS): plan() runs several times per conv on
// every eager step, the runtime queries only once
template <int KT, int CT, int TPW>
int occupancy_hw(size_t lds) {
  static std::mutex mu;
  static std::map<size_t, int> cache;
  std::lock_guard<std::mutex> g(mu);
  const auto it = cache.find(lds);
  if (it != cache.end()) return it->second;
  const void* f = reinterpret_cast<const void*>(&hwgrad_kernel<KT, CT, TPW>);
  (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 512, lds) != hipSuccess) {
    (void)hipGetLastError();
    n = 1;
  }
  cache[lds] = n;
  return n;
}

#define HW_OCC(kt, ct, tpw) \
  if (h.KT == kt && h.CT == ct && h.TPW == tpw) return occupancy_hw<kt, ct, tpw>(h.lds);

// resident 512-thread workgroups per CU of the plan's instance (VGPRs, LDS)
int blocks_per_cu(const HwPlan& h) {
  HW_INSTANCES(HW_OCC)
  return 1;
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        v > 0)
      n = v;
    else
      n = 256;
    (void)hipGetLastError();
  }
  return n;
}

}  // namespace

namespace umamd {

int hwgrad_splits(int N, int H, int W, int C, int ldx, int K, int R, int stride, int pad,
                  int reflect, int P, int Q, int ldy) {
  const HwPlan h = plan(N, H, W, C, ldx, K, R, stride, pad, reflect, P, Q, ldy);
  return (h.ok && exists(h)) ? h.splits : 0;
}

int hwgrad_run(const void* x, int N, int H, int W, int C, int ldx, int K, int R, int stride,
               int pad, int reflect, int P, int Q, const void* dy, int ldy, float* slabs,
               int splits, hipStream_t st) {
  HwPlan h = plan(N, H, W, C, ldx, K, R, stride, pad, reflect, P, Q, ldy);
  if (!h.ok || !exists(h) || h.splits != splits) return -1;
  h.a.x = reinterpret_cast<const bf16_t*>(x);
  h.a.dy = reinterpret_cast<const bf16_t*>(dy);
  return dispatch(h, slabs, st);
}

}  // namespace umamd
