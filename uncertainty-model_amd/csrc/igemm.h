// Internal interface of the tap-major implicit-GEMM convolution (igemm.hip),
// used by the C-ABI conv entries in conv.hip.
#pragma once

#include <hip/hip_runtime.h>

namespace umamd {

enum { IG_PAD_ZERO = 0, IG_PAD_REFLECT = 1, IG_FOLD = 2 };

struct IgArgs {
  // gathered operand ("A"): NHWC image [on][ah][aw][ach], pixel stride lda
  const void* a;
  int ah, aw, ach, lda;
  // output pixels: GEMM row m = (n, oy, ox) over [on][oh][ow]
  int on, oh, ow;
  // tap geometry: source row = oy*stride - pad + tsign*r, column ox*stride -
  // padx + tsign*s, taps r < R, s < Rx (flipped weight taps for dgrad)
  int R, stride, pad, pmode, fold_pad, flip;
  int Rx, padx, tsign;
  // parity-class mode (stride-2 data gradient): weight tap (r0y + 2r, r0x + 2s)
  // of the wR x wR kernel; output row (n, i', j') -> pixel (2i'+ay, 2j'+ax) of
  // an outH x outW image
  int cls, wR, r0y, r0x, ay, ax, outH, outW;
  // border-list mode (with IG_FOLD, reflect data gradient): GEMM row m is the
  // m-th pixel of [on] x {pixels of an oh x ow image whose row is in rr[] or
  // whose column is in rc[]} -- the pixels a reflect pad folds into -- and the
  // gather sums only the folded sources (the zero-pad part comes from a plain
  // same-size data gradient launched before it)
  int border, nrr, nrc, rr[4], rc[4];
  // weights ("B"): row n (output channel) at b + n*ldb, element tap*ach + c
  const void* b;
  long ldb;
  int NC, M;
  // epilogue
  const float* bias;
  void* out;
  int ld_out, out_f32, epilogue, accumulate;
  float epi_scale;
  const void* residual;
  int ldr;
  float* stats;     // [parts][NC][2] f32 partial rows, or (stat_slots) f64 slots
  int stats_rows;   // set by igemm_run (igemm_stats_rows)
  int stat_slots;   // UM_EPI_STAT_SLOTS: stats is double[UM_STAT_SLOTS][NC][2]
  int staged;       // halo conv: LDS-staged 16-byte output rows (set by halo_run)
  int colmajor;     // tile order, set by igemm_run (knob xcd_col)
  int tappack;      // 4 taps x 8 channels per k-step (ach == 8), set by igemm_run
};

__device__ __forceinline__ int pick4(const int (&v)[4], int i) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : (i == 2 ? v[2] : v[3]));
}

// border-list mode: listed pixel m -> (n, y, x); rows rr[] (ascending) are
// listed whole, the other rows at the columns rc[]
__device__ __forceinline__ void border_pixel(const IgArgs& a, int m, int& n, int& y, int& x) {
  const int W = a.ow, full = a.nrr * W;
  const int per = full + (a.oh - a.nrr) * a.nrc;
  n = m / per;
  int k = m - n * per;
  if (k < full) {
    const int i = k / W;
    y = pick4(a.rr, i);
    x = k - i * W;
    return;
  }
  k -= full;
  const int idx = k / a.nrc;
  x = pick4(a.rc, k - idx * a.nrc);
  y = idx;  // the idx-th row not in rr[]
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < a.nrr && pick4(a.rr, j) <= y) ++y;
}

// rows per BN partial-statistics row of a stats epilogue (M, NC of the GEMM)
int igemm_stats_rows(int M, int NC);

// workspace bytes the split-K heuristic wants for this shape (0: no split)
long igemm_ws_bytes(int dtype, int M, int NC, int taps, int ach);
long igemm_border_ws_bytes(int dtype, int M, int NC, int taps, int ach);
// launch; ws may be null (then no split)
int igemm_run(int dtype, const IgArgs& a, float* ws, long ws_bytes, hipStream_t st);

// the four parity classes of a stride-2 data gradient in one launch: 1 =
// launched, 0 = not eligible (launch them one by one), < 0 = -error code
int igemm_run_cls4(int dtype, IgArgs (&as)[4], float* ws, long ws_bytes, hipStream_t st);
// workspace of the 4-class LDS-DMA form (0 when it does not apply or needs none)
long igemm_cls4_ws_bytes(int dtype, const int (&M)[4], const int (&taps)[4], int NC, int ach);

// reflect data gradients with more input channels than this run as one fold
// pass, the others as a zero-pad pass + the border-list pass (knob
// "fold_split_nc")
int igemm_fold_split_nc();
bool igemm_halo_dgrad(int dtype, int N, int H, int W, int C, int R);

// reflect data gradients in the padded form (knob pad_dgrad): 0 off, 1 for
// dx wider than fold_split_nc, 2 all
int igemm_pad_dgrad();

// halo conv weight rows two rows ahead (tuning key "halo_pf2")
int igemm_halo_pf2();
// halo conv grid: persistent workgroups per resident slot (knob
// "halo_persist", 0 = one tile per workgroup) and a grid cap ("halo_grid")
int igemm_halo_persist();
int igemm_halo_grid();
// resident-weight LDS budget (KB) of the 3x3 halo convs ("halo_res_kb", 0 = off)
int igemm_halo_res_kb();
// halo conv bf16 outputs staged through LDS as 16-byte rows ("halo_staged")
int igemm_halo_staged();
// reflect fold of the split-form data gradient as a VALU pass ("border_valu")
int igemm_border_valu();

// fill the border-list fields of a (oh, ow, fold_pad set) and return the
// number of listed pixels per image
int igemm_border_list(IgArgs& a);

}  // namespace umamd
