// Shared definitions of the k = 7 stride-1 single-channel-side kernels (conv_k7.hip: fp32 VALU,
// conv_k7_mfma.hip: bf16 MFMA).
#pragma once
#include "common.h"

namespace cg {

constexpr int K7 = 7, KT7 = 343;
constexpr int TD = 4, TH = 8, TW = 32;
constexpr int HD = TD + 6, HH = TH + 6, HWD = TW + 6, HWP = 40;  // halo dims, padded row
constexpr int HALO = HD * HH * HWP;

struct K7Args {
  int n, di, hi, wi, do_, ho, wo;
  int P;          // src = o + t - P
  int reflect;    // mirror out-of-range source (else zero)
  int flip;       // use W[c, 342 - t]
  long long wc;   // weight stride of the wide channel (tap stride 1)
  int tiles_d, tiles_h, tiles_w;
  int probe;      // phase probes (common.h CG_PROBE)
};

// mode-2 BatchNorm statistics of the reflect-folded output (cgan3d_epilogue.bn_fold): the input-grad
// of the generator's last conv lands on the padded grid, dy = fold(out) on the unpadded one, and
// sum_v dy(v) a(v) = sum_q out(q) a(refl(q - P)) for the pair weights a = act' (1, xhat) — so the
// statistics come straight from this kernel's outputs and z at the reflected voxel (no fold pass)
struct K7Fold {
  const float* z;   // BatchNorm input on the unpadded grid [n][zd][zh][zw][16]
  const float* ss;  // [scale | shift]
  const float* mi;  // [mean | invstd]
  float* part;      // mode-2 slab, slot = block
  double* acc;      // or fp64 accumulators (cgan3d_bn_fuse acc_mode 4): replica block % reps
  int reps;
  int act;
  float slope;
  int P, zd, zh, zw;
};

// streamed-plane 1 -> 16 kernel (conv_k7p.hip): 1 if it took the launch (k7m_n2w otherwise)
int k7p_n2w_try(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, const float* x, const float* w,
                float* y, const K7Fold* fold, const BnFuse* fz, bool out16, hipStream_t s);

// streamed-plane weight gradient (conv_k7p.hip): 1 if it took the launch (k7m_wg otherwise); its
// partial rows (blocks x 16 x 343 floats) are summed by colsum_kernel (common.h colsum_launch)
int k7p_wgrad_try(const cgan3d_conv_geom* g, bool wide_in, long long wc, const float* x, const float* go, float* dw,
                  float* ws, hipStream_t s, const __bf16* wide16);
long long k7p_wg_blocks(const cgan3d_conv_geom* g, bool wide_in);

__device__ __forceinline__ void k7_tile(const K7Args& a, int bid, int* n, int* d0, int* h0, int* w0) {
  int tw = bid % a.tiles_w; bid /= a.tiles_w;
  int th = bid % a.tiles_h; bid /= a.tiles_h;
  int td = bid % a.tiles_d; *n = bid / a.tiles_d;
  *d0 = td * TD; *h0 = th * TH; *w0 = tw * TW;
}

__device__ __forceinline__ int k7_src(int i, int n, int reflect) {
  if (reflect) i = reflect_idx(i, n);  // halo cells past a partial tile may still fall outside
  return (i >= 0 && i < n) ? i : -1;
}

}  // namespace cg
