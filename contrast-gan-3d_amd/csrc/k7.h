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
