// BatchNorm statistics from fp64 accumulator replicas (cgan3d_bn_fuse acc_mode 3 / 4) — shared by the
// elementwise passes of bn.hip and the ResNet-block conv's staging prologue (conv_k3m.hip, round 5):
// the replica sum, the per-channel finalize and the elementwise maps, written once so both give the
// same bits (model/blocks.py:50-53, torch.nn.BatchNorm3d in training mode).
#pragma once
#include "common.h"

namespace cg {

__device__ __forceinline__ float act_f(float v, int act, float slope) {
  if (act == CGAN3D_ACT_RELU) return fmaxf(v, 0.f);
  if (act == CGAN3D_ACT_LRELU) return v > 0.f ? v : v * slope;
  return v;
}

// sums[q * C + c] = sum over replicas of acc[(r * 2 + q) * C + c]: the 256 threads split the pairs
// (j = q * C + c, 2C <= 128 of them) and the replicas (T = 256 / 2C threads per pair), eight loads
// in flight per thread — one round trip for reps <= 8T (the atomics left the values at the memory
// side: each round trip is long) — then the T partial sums of a pair are added through LDS (`part`,
// 256 doubles).  `prefetch` runs between issuing the first round of loads and using them: the caller
// issues its own first loads there, so the two round trips overlap instead of adding up.  Ends with
// sums[] written by threads < 2C (the caller barriers before reading it).
template <class F>
__device__ __forceinline__ void acc_sums(const double* __restrict__ acc, int reps, int C, double* sums, double* part,
                                         F&& prefetch) {
  const int tid = threadIdx.x, P = 2 * C, T = 256 / P, j = tid % P, h = tid / P;
  // unconditional loads (clamped replica, value masked after): a load under a branch gets its own
  // wait before the branch joins, which serialised the first round trip
  double v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = acc[(long long)min(h + u * T, reps - 1) * P + j];
  prefetch();
  __builtin_amdgcn_sched_barrier(0);  // keep the sums below every load issued above
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += h + u * T < reps ? v[u] : 0.0;
  for (int r0 = h + 8 * T; r0 < reps; r0 += 8 * T) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + u * T;
      v[u] = r < reps ? acc[(long long)r * P + j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  part[tid] = s;
  lds_barrier();
  if (tid < P) {
    double t = 0.0;
    for (int k = 0; k < T; ++k) t += part[k * P + tid];
    sums[tid] = t;
  }
}

// Forward finalize of channel c from the (sum, sum of squares) replicas' totals: scale / shift of
// act(z * scale + shift); `publish` (one block of the launch) writes the layer's scale / shift, mean /
// invstd (read by the backward) and the running buffers (momentum update, unbiased variance).
// gamma[c] / beta[c] loaded by the caller ahead of the replica combine (bn_acc_fwd_coeffs loads them)
__device__ __forceinline__ void bn_acc_fwd_coeffs_pre(const double* sums, int c, int C, double nvox, float gamma_c,
                                                      float beta_c, float eps, float* sc_out, float* sh_out,
                                                      bool publish, float* scale_shift, float* mean_invstd, float* rmean,
                                                      float* rvar, long long* nbt, float momentum) {
  const double mean = sums[c] / nvox, var = fmax(sums[C + c] / nvox - mean * mean, 0.0);
  const double invstd = 1.0 / sqrt(var + (double)eps);
  const double sc = (double)gamma_c * invstd;
  *sc_out = (float)sc;
  *sh_out = (float)((double)beta_c - mean * sc);
  if (publish) {
    scale_shift[c] = *sc_out;
    scale_shift[C + c] = *sh_out;
    mean_invstd[c] = (float)mean;
    mean_invstd[C + c] = (float)invstd;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * nvox / (nvox > 1 ? nvox - 1 : 1));
    if (nbt && c == 0) *nbt += 1;
  }
}

__device__ __forceinline__ void bn_acc_fwd_coeffs(const double* sums, int c, int C, double nvox, const float* gamma,
                                                  const float* beta, float eps, float* sc_out, float* sh_out,
                                                  bool publish, float* scale_shift, float* mean_invstd, float* rmean,
                                                  float* rvar, long long* nbt, float momentum) {
  bn_acc_fwd_coeffs_pre(sums, c, C, nvox, gamma[c], beta[c], eps, sc_out, sh_out, publish, scale_shift, mean_invstd,
                        rmean, rvar, nbt, momentum);
}

// Backward finalize of channel c from the (sum g, sum g * xhat) totals: the coefficients of
// bn_bwd_map (k0 = gamma * invstd, k1 = mean g, k2 = mean g * xhat); `publish` writes dbeta = sum g,
// dgamma = sum g * xhat (added when `accumulate`).
__device__ __forceinline__ void bn_acc_bwd_coeffs(const double* sums, int c, int C, double nvox, const float* gamma,
                                                  const float* mi, float* k0, float* k1, float* k2, bool publish,
                                                  float* dgamma, float* dbeta, int accumulate) {
  *k0 = gamma[c] * mi[C + c];
  *k1 = (float)(sums[c] / nvox);
  *k2 = (float)(sums[C + c] / nvox);
  if (publish) {
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)sums[c] : (float)sums[c];
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)sums[C + c] : (float)sums[C + c];
  }
}

// bn_acc_bwd_coeffs with gamma[c] and invstd[c] loaded by the caller ahead of the replica combine
// (loaded here, they were one more round trip between the block's two barriers); same arithmetic
__device__ __forceinline__ void bn_acc_bwd_coeffs_pre(const double* sums, int c, int C, double nvox, float gamma_c,
                                                      float invstd_c, float* k0, float* k1, float* k2, bool publish,
                                                      float* dgamma, float* dbeta, int accumulate) {
  *k0 = gamma_c * invstd_c;
  *k1 = (float)(sums[c] / nvox);
  *k2 = (float)(sums[C + c] / nvox);
  if (publish) {
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)sums[c] : (float)sums[c];
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)sums[C + c] : (float)sums[C + c];
  }
}

// dz of one element: g = dy * act'(z * scale + shift), xhat = (z - mean) * invstd,
// dz = k0 * (g - k1 - xhat * k2).  (A three-FMA form a * g + (b * z + c) was measured as well: it
// moves the bf16 step's chaotic last bits — test_batchnorm_accumulators_match_slab_path's critic bias
// tensors over their bar — for nothing measurable in these HBM-bound passes; kept the original.)
__device__ __forceinline__ float bn_bwd_map(float dy, float z, float sc, float sf, float mean, float inv, float k0,
                                            float k1, float k2, int act, float slope) {
  const float g = dy * act_grad(z * sc + sf, act, slope);
  const float xh = (z - mean) * inv;
  return k0 * (g - k1 - xh * k2);
}

}  // namespace cg
