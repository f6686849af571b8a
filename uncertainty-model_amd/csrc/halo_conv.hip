// Halo-tiled direct convolution on MFMA (gfx950) for the small-channel,
// high-resolution 3x3 / 5x5 / 7x7 layers: forward (zero or reflect padding)
// and the stride-1 data gradient of zero-padded convs (a forward conv of dy
// with the flipped, transposed weights).
//
// The tap-major implicit GEMM (igemm.hip) re-gathers the input pixels from
// L2 for every tap: R*R times the activation bytes, which for 32..64 output
// channels is more than the MFMAs can consume (the 7x7 32->32 layers reached
// ~290 TFLOP/s).  Here a workgroup owns an 8 x 32 output-pixel tile of one
// image and up to 64 output channels, stages the (8+R-1) x (32+R-1) input
// halo of one 32-channel chunk ONCE in LDS and runs all R*R taps from it
// (wider outputs: a grid column of such blocks per 64/96/128 channels):
//   - A fragments (16 pixels x 32 channels) are ds_read_b128 of 16
//     consecutive halo pixels; the 16-byte channel chunks of a pixel are
//     XOR-swizzled by bits 2-3 of the pixel index, so any 16 consecutive
//     pixels cover the 64 LDS banks exactly once (conflict-free);
//   - the weights of one tap row (R taps x BN output channels x 32 channels)
//     are staged in a double-buffered LDS image with the same swizzle (the
//     next row is loaded to registers during the current row's MFMAs), so B
//     fragments are ds_read_b128 too and the 4 waves share one copy;
//   - the next chunk's halo is loaded to registers while the current one is
//     computed; v_mfma_f32_16x16x32_bf16, f32 accumulation.
// Epilogue as igemm's: bias, optional residual / sigmoid-scale / accumulate,
// f32 or bf16 output, and the BN partial statistics (two 128-pixel rows per
// tile, so um_conv_stats_parts counts them like the GEMM's).
// Replaces nn.Conv2d forward / input-gradient of reference
// model/layers/encoder.py:36-42 (7x7, 5x5, 3x3 zero padded) and
// model/layers/decoder.py:30-52 (3x3 reflection padded, forward).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "halo_conv.h"

namespace {

using umamd::IgArgs;

constexpr int TH = 8, TW = 32, CK = 32;

// element offset of 8-channel chunk c (0..3) of halo pixel p.  A fragment read
// (ds_read_b128) takes 16 consecutive pixels from ANY start pixel p0 (tap
// offsets), lane l -> pixel p0 + (l & 15), chunk l >> 4, serviced in the lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32).  With chunk ^ 2*bit2(p)
// each group covers the 64 banks exactly once for every p0 (the former
// chunk ^ ((p >> 2) & 3) was 2-way in every group: SQ_LDS_BANK_CONFLICT 0.4)
__device__ __forceinline__ int himg(int p, int c) { return p * CK + ((c ^ ((p >> 1) & 2)) << 3); }

// PF2: weight tap rows are loaded two rows ahead into two register sets
// (rows r+1 and r+2 in flight while row r computes) instead of one: a tap
// row of MFMAs (~0.4-0.8 us) is shorter than an L2 round trip under load
//
// Persistent tiles: workgroup b takes output tiles b, b + gridDim.x, ... of
// its column block, and the halo of the NEXT (tile, chunk) is loaded into
// registers while the current one computes and stores -- for a one-chunk
// layer (32 input channels) the following tile's halo, so its load latency
// hides behind this tile's MFMAs and epilogue instead of opening every
// workgroup's life (grid = ntiles: one tile per workgroup, as before).
//
// WM (weight mode): 0 = tap rows streamed through a double-buffered LDS row
// image (the next row loaded to registers during the current row), 1 = PF2,
// 2 = RESIDENT: every chunk's R*R tap weights of the column block are loaded
// into (dynamic) LDS once per workgroup and reused by all its tiles -- no
// weight load, register set or barrier inside the tap loop (3x3 layers whose
// weights fit, umamd::halo_run).
// staged epilogue switch (tuning key halo_staged, read on the host into the
// launch's argument block)
#define umamd_halo_staged (a.staged)
template <int R, int BN, bool FLIP, bool REFLECT, int WM>
__global__ void __launch_bounds__(256) halo_conv_kernel(IgArgs a, int tiles_x, int tiles_y,
                                                        int ntiles) {
  constexpr bool PF2 = WM == 1, RES = WM == 2;
  constexpr int HH = TH + R - 1, HWd = TW + R - 1, HP = HH * HWd;
  constexpr int PIECES = HP * 4;                 // 16-byte pieces per chunk
  constexpr int NP = (PIECES + 255) / 256;       // per thread
  constexpr int TN = BN / 16;
  constexpr int TM = 4;                          // 4 x 16 pixels per wave (2 tile rows)
  constexpr int RR = R * R;
  constexpr int WP = R * BN * 4;              // 16-byte weight pieces per tap row
  constexpr int NW = (WP + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t sH[HP * CK];
  __shared__ __attribute__((aligned(16))) bf16_t sW[RES ? 1 : 2][RES ? 8 : R * BN * CK];
  __shared__ float sStat[4][BN][2];
  extern __shared__ __attribute__((aligned(16))) bf16_t sWr[];  // RES: [chunk][tap][BN] rows

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bn = blockIdx.y * BN;
  const bf16_t* __restrict__ src = reinterpret_cast<const bf16_t*>(a.a);
  const bf16_t* __restrict__ wsrc = reinterpret_cast<const bf16_t*>(a.b);
  struct Geo {
    int ty0, tx0, nimg;
  };
  auto geo = [&](int t) {
    Geo g;
    const int bx = t % tiles_x;
    t /= tiles_x;
    g.ty0 = (t % tiles_y) * TH;
    g.tx0 = bx * TW;
    g.nimg = t / tiles_y;
    return g;
  };

  uint4 hv[NP];
  auto load_halo = [&](const Geo& g, int c0) {
    const int iy0 = g.ty0 - a.pad, ix0 = g.tx0 - a.pad;
    const long img_base = (long)g.nimg * a.ah * a.aw * a.lda;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = tid + k * 256;
      hv[k] = make_uint4(0, 0, 0, 0);
      if (i < PIECES) {
        const int p = i >> 2, c = i & 3;
        const int hy = p / HWd, hx = p - (p / HWd) * HWd;
        int y = iy0 + hy, x = ix0 + hx;
        const int ch = c0 + c * 8;
        bool ok = ch < a.ach;
        if (REFLECT) {
          y = reflect_idx(y, a.ah);
          x = reflect_idx(x, a.aw);
        } else {
          ok = ok && y >= 0 && y < a.ah && x >= 0 && x < a.aw;
        }
        if (ok)
          hv[k] = *reinterpret_cast<const uint4*>(src + img_base + ((long)y * a.aw + x) * a.lda + ch);
      }
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = tid + k * 256;
      if (i < PIECES) *reinterpret_cast<uint4*>(&sH[himg(i >> 2, i & 3)]) = hv[k];
    }
  };

  // weight tap row r of chunk c0 -> registers: piece i = (s, n, c) of tap (r, s),
  // output channel bn + n, reduction channels c0 + 8c .. + 8
  const int ncol = lane & 15, kq = lane >> 4;
  uint4 wv[NW], wv2[NW];
  auto load_wset = [&](uint4 (&w)[NW], int r, int c0) {
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int i = tid + k * 256;
      w[k] = make_uint4(0, 0, 0, 0);
      if (i < WP) {
        const int c = i & 3, nn = (i >> 2) % BN, ss = (i >> 2) / BN;
        const int n = bn + nn, ch = c0 + c * 8;
        const int tap = r * R + ss;
        const int btap = FLIP ? RR - 1 - tap : tap;
        if (n < a.NC && ch < a.ach)
          w[k] = *reinterpret_cast<const uint4*>(wsrc + (long)n * a.ldb + (long)btap * a.ach + ch);
      }
    }
  };
  auto store_wset = [&](const uint4 (&w)[NW], int buf) {
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int i = tid + k * 256;
      if (i < WP) {
        const int c = i & 3, row = i >> 2;  // row = ss * BN + nn
        *reinterpret_cast<uint4*>(&sW[buf][himg(row, c)]) = w[k];
      }
    }
  };
  auto load_wrow = [&](int r, int c0) { load_wset(wv, r, c0); };
  auto store_wrow = [&](int buf) { store_wset(wv, buf); };
  bool nok[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) nok[j] = bn + j * 16 + ncol < a.NC;

  // A fragment base pixel of fragment i: tile row 2*wave + (i >> 1), column (i & 1)*16 + row
  int pbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) pbase[i] = (2 * wave + (i >> 1)) * HWd + (i & 1) * 16 + ncol;

  const int nchunk = (a.ach + CK - 1) / CK;
  // the R taps of tap row r from LDS weight buffer buf (RES: buf = chunk).
  // pb / bq / kk: per-tile opaque copies of pbase / ncol / kq (see the tile
  // loop)
  int pb[TM], bq = ncol, kk = kq;
  auto taps = [&](f32x4_t (&acc)[TM][TN], int r, int buf, bool zero = false) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8_t*>(&sH[himg(pb[i] + r * HWd + s, kk)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = RES ? *reinterpret_cast<const bf16x8_t*>(
                          &sWr[himg((buf * RR + r * R + s) * BN + j * 16 + bq, kk)])
                    : *reinterpret_cast<const bf16x8_t*>(&sW[buf][himg(s * BN + j * 16 + bq, kk)]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              fa[i], fb[j], (zero && s == 0) ? f32x4_t{0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
    }
  };
  int t = blockIdx.x;
  if (t >= ntiles) return;
  load_halo(geo(t), 0);
  if constexpr (RES) {
    // all weights of this column block: rows (chunk * RR + tap) * BN + n, in
    // batches of 8 pieces per thread with every load issued before its stores
    const int total = nchunk * RR * BN * 4;
    for (int b0 = 0; b0 < total; b0 += 8 * 256) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = b0 + k * 256 + tid;
        v[k] = make_uint4(0, 0, 0, 0);
        if (i < total) {
          const int c = i & 3, row = i >> 2;
          const int nn = row % BN, ct = row / BN;
          const int tap = ct % RR, ch = (ct / RR) * CK + c * 8;
          const int n = bn + nn, btap = FLIP ? RR - 1 - tap : tap;
          if (n < a.NC && ch < a.ach)
            v[k] = *reinterpret_cast<const uint4*>(wsrc + (long)n * a.ldb + (long)btap * a.ach + ch);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = b0 + k * 256 + tid;
        if (i < total) *reinterpret_cast<uint4*>(&sWr[himg(i >> 2, i & 3)]) = v[k];
      }
    }
  }
  const int row_g = (lane >> 4) * 4;
  // persistent tiles (RES only: the streamed modes keep one tile per
  // workgroup, whose straight-line code needs fewer registers)
  constexpr bool LOOP = RES;
  for (;;) {
    const Geo cur = geo(t);
    // the halo after chunk ch: the next chunk of this tile, else the next
    // tile's first chunk (if any); one load site, so one copy of its code
    auto prefetch = [&](int ch) {
      const bool same = ch + 1 < nchunk;
      if constexpr (LOOP) {
        const int pt = same ? t : t + (int)gridDim.x;
        if (pt < ntiles) load_halo(same ? cur : geo(pt), same ? (ch + 1) * CK : 0);
      } else {
        if (same) load_halo(cur, (ch + 1) * CK);
      }
    };
    // the fragment address bases re-derived per tile: the compiler would
    // otherwise keep every tap's LDS address of the whole loop live across
    // the epilogue (~70 VGPRs at 64 columns)
#pragma unroll
    for (int i = 0; i < TM; ++i) pb[i] = pbase[i];
    bq = ncol;
    kk = kq;
    if constexpr (LOOP) {
      asm volatile("" : "+v"(bq), "+v"(kk));
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(pb[i]));
    }
    f32x4_t acc[TM][TN];
    if constexpr (RES) {
      // chunk 0 peeled: its first tap starts the accumulators from zero (an
      // accumulator zeroed before the chunk loop costs a second AGPR set)
      auto chunk = [&](int ch, bool first) {
        __syncthreads();  // the previous chunk's fragment reads are done (and sWr stored)
        store_halo();
        prefetch(ch);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) taps(acc, r, ch, first && r == 0);
      };
      chunk(0, true);
      for (int ch = 1; ch < nchunk; ++ch) chunk(ch, false);
    } else if constexpr (PF2) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      for (int ch = 0; ch < nchunk; ++ch) {
        const int c0 = ch * CK;
        load_wset(wv, 0, c0);
        if (R > 1) load_wset(wv2, 1, c0);
        __syncthreads();  // the previous chunk's fragment reads are done
        store_halo();
        prefetch(ch);
        store_wset(wv, 0);
        __syncthreads();
        // row r: set `nxt` holds row r+1 (loaded a row ago), `fre` is free and
        // takes row r+2; the sets alternate, so the pair loop keeps every
        // register-array index static
        auto row = [&](int r, uint4 (&nxw)[NW], uint4 (&fre)[NW]) {
          if (r + 2 < R) load_wset(fre, r + 2, c0);
          taps(acc, r, r & 1);
          if (r + 1 < R) store_wset(nxw, (r + 1) & 1);  // that buffer was last read in row r-1
          __syncthreads();
        };
#pragma unroll 1
        for (int r = 0; r < R; r += 2) {
          row(r, wv2, wv);
          if (r + 1 < R) row(r + 1, wv, wv2);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      for (int ch = 0; ch < nchunk; ++ch) {
        const int c0 = ch * CK;
        __syncthreads();  // the previous chunk's fragment reads are done
        store_halo();
        __syncthreads();
        load_wrow(0, c0);
        prefetch(ch);
        store_wrow(0);
        __syncthreads();
#pragma unroll 1
        for (int r = 0; r < R; ++r) {
          const int buf = r & 1;
          if (r + 1 < R) load_wrow(r + 1, c0);
          taps(acc, r, buf);
          if (r + 1 < R) store_wrow(buf ^ 1);  // that buffer was last read in row r-1
          __syncthreads();
        }
      }
    }

    // -------------------------------------------------------------- epilogue --
    const int ty0 = cur.ty0, tx0 = cur.tx0, nimg = cur.nimg;
    // lane coordinates made opaque per tile: otherwise the compiler hoists
    // the tile-invariant part of all TM*TN*4 64-bit output offsets out of the
    // tile loop (+100 VGPRs, half the occupancy)
    int rg = row_g, nc = ncol;
    if constexpr (LOOP) asm volatile("" : "+v"(rg), "+v"(nc));
    float csum[TN], csq[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
    // STAGED (bf16 output written once, no residual / sigmoid): the tile's
    // values go through the (now free) halo LDS as [pixel][JP*16 columns],
    // JP column blocks per pass, and leave as 16-byte rows of 8 channels --
    // instead of 2-byte stores of one column at 4 pixels per lane
    constexpr int JP = TN % 2 == 0 ? 2 : 1;
    static_assert(TH * TW * JP * 16 <= HP * CK, "staged epilogue tile exceeds the halo LDS");
    // not where the staging registers would cost a wave per SIMD (3x3 at 96
    // columns streamed, 7x7 at 64 columns)
    constexpr bool STG = !(R == 3 && BN == 96) && !(R == 7 && BN == 64);
    const bool staged = STG && umamd_halo_staged && !a.out_f32 && !a.accumulate &&
                        a.epilogue != UM_EPI_RESIDUAL && a.epilogue != UM_EPI_SIGMOID_SCALE &&
                        a.NC % 8 == 0 && a.ld_out % 8 == 0 &&
                        (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
    bf16_t* sE = sH;
    if (staged) __syncthreads();  // every wave's fragment reads of sH are done
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = bn + j * 16 + nc;
      if (nok[j]) {
      const float bv = a.bias != nullptr ? a.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ty = 2 * wave + (i >> 1);
        const int oxb = tx0 + (i & 1) * 16 + rg;
        // partial tiles at the bottom / right edge (output sizes not multiples
        // of the 8 x 32 tile: the padded-domain reflect data gradient)
        const bool yok = ty0 + ty < a.oh;
        const long mrow = ((long)nimg * a.oh + ty0 + ty) * a.ow + oxb;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (!yok || oxb + q >= a.ow) continue;
          const long m = mrow + q;
          float v = acc[i][j][q] + bv;
          const long off = m * a.ld_out + n;
          if (a.epilogue == UM_EPI_RESIDUAL)
            v += to_f32(reinterpret_cast<const bf16_t*>(a.residual)[m * a.ldr + n]);
          if (a.epilogue == UM_EPI_SIGMOID_SCALE) v = a.epi_scale * sigmoidf_(v);
          if (staged) {
            sE[(((2 * wave + (i >> 1)) * TW + (i & 1) * 16 + rg + q) * JP + j % JP) * 16 + nc] =
                from_f32<bf16_t>(v);
          } else if (a.out_f32) {
            float* o = reinterpret_cast<float*>(a.out) + off;
            if (a.accumulate) v += *o;
            *o = v;
          } else {
            bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + off;
            if (a.accumulate) v += to_f32(*o);
            *o = from_f32<bf16_t>(v);
          }
          csum[j] += v;
          csq[j] += v * v;
        }
      }
      }
      if (staged && j % JP == JP - 1) {
        __syncthreads();
        constexpr int GP = JP * 2;  // 8-channel groups per pixel in a pass
#pragma unroll
        for (int it = tid; it < TH * TW * GP; it += 256) {
          const int pix = it / GP, g = it % GP;
          const int py = ty0 + pix / TW, px = tx0 + pix % TW;
          const int n0 = bn + (j / JP) * JP * 16 + g * 8;
          if (py < a.oh && px < a.ow && n0 < a.NC) {
            const long m = ((long)nimg * a.oh + py) * a.ow + px;
            *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.out) + m * a.ld_out + n0) =
                *reinterpret_cast<const uint4*>(&sE[(pix * JP) * 16 + g * 8]);
          }
        }
        __syncthreads();  // the pass's LDS reads are done (next pass / next tile's halo)
      }
    }
    if (a.epilogue == UM_EPI_STATS) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float sm = csum[j], sq = csq[j];
        sm += __shfl_xor(sm, 16, 64);
        sm += __shfl_xor(sm, 32, 64);
        sq += __shfl_xor(sq, 16, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (lane < 16) {
          sStat[wave][j * 16 + lane][0] = sm;
          sStat[wave][j * 16 + lane][1] = sq;
        }
      }
      __syncthreads();
      // two partial rows per tile: waves {0,1} (tile rows 0-3) and {2,3} (rows 4-7)
      if (a.stat_slots) {
        stat_slots_count(reinterpret_cast<double*>(a.stats), a.NC, a.M);
        for (int half = 0; half < 2; ++half)
          stat_slots_add_row(reinterpret_cast<double*>(a.stats), 2 * t + half, a.NC, bn,
                             min(BN, a.NC - bn), [&](int i) {
                               return sStat[2 * half][i >> 1][i & 1] + sStat[2 * half + 1][i >> 1][i & 1];
                             });
      } else {
        for (int c = tid; c < 2 * BN; c += 256) {
          const int col = c % BN, half = c / BN;
          const int n = bn + col;
          if (n >= a.NC) continue;
          const float sm = sStat[2 * half][col][0] + sStat[2 * half + 1][col][0];
          const float sq = sStat[2 * half][col][1] + sStat[2 * half + 1][col][1];
          float* o = a.stats + ((long)(2 * t + half) * a.NC + n) * 2;
          o[0] = sm;
          o[1] = sq;
        }
      }
      __syncthreads();  // sStat is rewritten by the next tile
    }
    if constexpr (!LOOP) break;
    t += gridDim.x;
    if (t >= ntiles) break;
  }
}

// workgroups of one column block: every tile (knob halo_persist 0), or the
// resident count (occupancy x CUs, over the column blocks) x halo_persist,
// or (tests) at most knob halo_grid
template <typename K>
int persist_grid(K kernel, int ntiles, int col_blocks, size_t shm) {
  const int mult = umamd::igemm_halo_persist(), cap = umamd::igemm_halo_grid();
  if (cap > 0) return std::max(1, std::min(ntiles, cap));
  if (mult <= 0) return ntiles;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 256, shm) != hipSuccess || occ < 1)
    occ = 1;
  const long res = (long)occ * cus * mult / std::max(1, col_blocks);
  return (int)std::max(1l, std::min((long)ntiles, res));
}

// resident-weight LDS bytes of a 3x3 launch (0: the weights do not fit the
// knob's budget, stream the tap rows)
// One-chunk layers only (ach <= 32): there the next tile's halo is the
// prefetch target.  Micro-benchmark on MI355X (tools/halo_micro.sh r04w2):
// 8x256x512 C32->K32 fwd 74.5 -> 66.5 us, dgrad 75.1 -> 65.9; a two-chunk
// layer (C48 -> K32, reflect) went 94 -> 106 us forward, so it streams.
size_t res_bytes(const IgArgs& a, int bn) {
  const int kb = umamd::igemm_halo_res_kb();
  if (kb <= 0 || a.R != 3 || a.ach > CK || umamd::igemm_halo_pf2()) return 0;
  const size_t b = (size_t)9 * bn * CK * sizeof(bf16_t);
  return b <= (size_t)kb * 1024 ? b : 0;
}

template <int R, int BN, int WM>
void launch_rp(const IgArgs& a, int ncb, int tiles_x, int tiles_y, size_t shm, hipStream_t st) {
  const int ntiles = a.on * tiles_y * tiles_x;
  auto go = [&](auto kernel) {
    const dim3 grid(WM == 2 ? persist_grid(kernel, ntiles, ncb, shm) : ntiles, ncb);
    hipLaunchKernelGGL(kernel, grid, dim3(256), shm, st, a, tiles_x, tiles_y, ntiles);
  };
  if (a.flip) go(halo_conv_kernel<R, BN, true, false, WM>);
  else if (a.pmode == umamd::IG_PAD_REFLECT) go(halo_conv_kernel<R, BN, false, true, WM>);
  else go(halo_conv_kernel<R, BN, false, false, WM>);
}

template <int R, int BN>
int launch_r(const IgArgs& a, hipStream_t st) {
  const int tiles_x = (a.ow + TW - 1) / TW, tiles_y = (a.oh + TH - 1) / TH;
  const int ncb = (a.NC + BN - 1) / BN;
  // PF2 only where the second register set keeps the instance <= 256 VGPRs
  // (2 waves per SIMD): BN 16/32, and BN 64 at R = 3 (R = 5, 7 at BN 64 would
  // reach 270-320 VGPRs and one wave per SIMD)
  if constexpr (R == 3) {
    const size_t shm = res_bytes(a, BN);
    if (shm > 0) {
      launch_rp<R, BN, 2>(a, ncb, tiles_x, tiles_y, shm, st);
      UM_LAUNCH_CHECK();
      return UM_OK;
    }
  }
  if constexpr (BN <= 32 || (R == 3 && BN <= 64)) {
    if (umamd::igemm_halo_pf2()) launch_rp<R, BN, 1>(a, ncb, tiles_x, tiles_y, 0, st);
    else launch_rp<R, BN, 0>(a, ncb, tiles_x, tiles_y, 0, st);
  } else {
    launch_rp<R, BN, 0>(a, ncb, tiles_x, tiles_y, 0, st);
  }
  UM_LAUNCH_CHECK();
  return UM_OK;
}

// Output-column block width: up to 64 columns one block; wider outputs (the
// decoder's 88/128/168-channel convs and data gradients) take column blocks of
// 64, 96 or 128 (3x3 only: the double-buffered tap-row weights of a 128-wide
// 5x5/7x7 block would not fit LDS), whichever pads the fewest columns (ties:
// the wider block, fewer re-reads of the halo).
template <int R>
int launch_bn(const IgArgs& a, hipStream_t st) {
  if (a.NC <= 16) return launch_r<R, 16>(a, st);
  if (a.NC <= 32) return launch_r<R, 32>(a, st);
  if (a.NC <= 64) return launch_r<R, 64>(a, st);
  if constexpr (R == 3) {
    auto padded = [&](int bn) { return (a.NC + bn - 1) / bn * bn; };
    int bn = 128;
    if (padded(96) < padded(bn)) bn = 96;
    if (padded(64) < padded(bn)) bn = 64;
    if (bn == 128) return launch_r<R, 128>(a, st);
    if (bn == 96) return launch_r<R, 96>(a, st);
  }
  return launch_r<R, 64>(a, st);
}

}  // namespace

namespace umamd {

bool halo_applicable(int dtype, const IgArgs& a, int min_tiles, int max_nc) {
  if (dtype != UM_BF16 || a.stride != 1 || a.cls) return false;
  if (a.R != 3 && a.R != 5 && a.R != 7) return false;
  if (a.pmode == IG_FOLD) return false;                         // reflect transpose: igemm
  if (a.flip && a.pmode != IG_PAD_ZERO) return false;
  // "same" conv, or the zero-pad transposed conv onto the reflect-padded
  // input (output (H+2p) x (W+2p) from a P x Q dy with pad R-1: the padded
  // form of the reflect data gradient, umamd::pad_dgrad in conv.hip);
  // partial edge tiles are masked in the epilogue
  const bool same = a.oh == a.ah && a.ow == a.aw && a.pad == (a.R - 1) / 2;
  const bool grown = a.flip && a.pad == a.R - 1 && a.oh == a.ah + a.R - 1 && a.ow == a.aw + a.R - 1;
  if (!same && !grown) return false;
  if (!same && (a.epilogue == UM_EPI_STATS)) return false;
  if (a.ow < TW / 2) return false;  // mostly-empty column tiles: the GEMM
  if (a.NC > max_nc || a.ach % 8 || a.lda % 8) return false;
  // 8-channel operands fill a quarter of each 32-channel chunk: past one
  // 64-column block the tap-packed GEMM is faster (disp-head data gradient
  // 64x128 C128 K8: 35 us tap-packed vs 49 us on 128-wide halo blocks)
  if (a.ach < 32 && a.NC > 64) return false;
  // partial-row statistics follow the GEMM's 128-row layout; the f64 slots
  // (stat_slots) take any tiling
  if (a.epilogue == UM_EPI_STATS && !a.stat_slots && a.stats_rows != 128) return false;
  // enough tiles to fill the chip
  return (long)a.on * ((a.oh + TH - 1) / TH) * ((a.ow + TW - 1) / TW) >= min_tiles;
}

int halo_run(const IgArgs& a0, hipStream_t st) {
  IgArgs a = a0;
  a.staged = igemm_halo_staged();
  if (a.R == 3) return launch_bn<3>(a, st);
  if (a.R == 5) return launch_bn<5>(a, st);
  return launch_bn<7>(a, st);
}

}  // namespace umamd
