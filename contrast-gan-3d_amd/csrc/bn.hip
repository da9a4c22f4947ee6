// Training-mode BatchNorm3d (+ ReLU / Identity / LeakyReLU) for gfx950, channels-last fp32.
//
// Replaces aten native_batch_norm / native_batch_norm_backward + relu / threshold_backward of
// ConvBlock (contrast_gan_3D/model/blocks.py:26-27,45-53): per-channel batch statistics over
// N*D*H*W, biased variance to normalise, unbiased variance into running_var, eps 1e-5,
// momentum 0.1 (torch.nn.BatchNorm3d defaults).
//
// Forward statistics come from the producing conv's epilogue as per-block (sum, M2, count)
// partials (conv.hip) combined here with Chan's formula in fp64, so the activation tensor is not
// re-read for statistics.  Backward is a two-pass reduction (sum dy, sum dy*xhat per channel,
// per-block partials -> fp64 combine) followed by one elementwise pass.
#include "bn_acc.h"

namespace cg {

// Chan's pairwise combine of (count, mean, M2) triples
__device__ __forceinline__ void chan_merge(double& n, double& m, double& q, double nb, double mb, double qb) {
  const double t = n + nb;
  if (t <= 0.0) return;
  const double d = mb - m;
  m += d * (nb / t);
  q += qb + d * d * (n * nb / t);
  n = t;
}

// one block per channel; single pass over the per-block (sum, M2, count) partials, each thread
// folding its partials with Chan's formula, then a shuffle / LDS tree of the same combine (fp64)
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ stats, long long nblk, int C,
                                                          const float* gamma, const float* beta, float* rmean,
                                                          float* rvar, long long* nbt, float momentum, float eps,
                                                          float* scale_shift, float* mean_invstd) {
  __shared__ double red[3][4];
  const int c = blockIdx.x, tid = threadIdx.x;
  const long long stride = 2LL * C + 1;
  double n = 0.0, m = 0.0, q = 0.0;
  for (long long b0 = tid; b0 < nblk; b0 += 4 * blockDim.x) {
    float sv[4], qv[4], nv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // four partials in flight
      const long long b = b0 + k * blockDim.x;
      const long long o = (b < nblk ? b : 0) * stride;
      sv[k] = stats[o + c]; qv[k] = stats[o + C + c]; nv[k] = b < nblk ? stats[o + 2 * C] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (nv[k] > 0.f) chan_merge(n, m, q, nv[k], (double)sv[k] / nv[k], qv[k]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double nb = __shfl_xor(n, off, 64), mb = __shfl_xor(m, off, 64), qb = __shfl_xor(q, off, 64);
    chan_merge(n, m, q, nb, mb, qb);
  }
  if ((tid & 63) == 0) { red[0][tid >> 6] = n; red[1][tid >> 6] = m; red[2][tid >> 6] = q; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) chan_merge(n, m, q, red[0][w], red[1][w], red[2][w]);
    const double N = n, mean = m;
    const double var = q / N;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * invstd;
    scale_shift[c] = (float)sc;
    scale_shift[C + c] = (float)((double)beta[c] - mean * sc);
    mean_invstd[c] = (float)mean;
    mean_invstd[C + c] = (float)invstd;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * N / (N > 1 ? N - 1 : 1));
    if (nbt && c == 0) *nbt += 1;
  }
}

// optional bf16 shadow of an output (read by the ResNet-block conv's halo staging)
typedef __bf16 bf16x4_n __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store16(__bf16* o16, long long i, f32x4 v) {
  bf16x4_n h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  reinterpret_cast<bf16x4_n*>(o16)[i] = h;
}

// float4 i of a tensor kept in fp32 or (B16, round 4: the generator's 64^3 16-channel tensors) in bf16
template <bool B16>
__device__ __forceinline__ f32x4 load4(const void* __restrict__ p, long long i) {
  if constexpr (B16) {
    const bf16x4_n h = reinterpret_cast<const bf16x4_n*>(p)[i];
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  } else {
    return reinterpret_cast<const f32x4*>(p)[i];
  }
}

// y = act(z*scale + shift) (+ residual); C % 4 == 0, float4 vectorised grid-stride.  With
// 256 % (C/4) == 0 the grid stride is a multiple of C/4, so a thread keeps its 4 channels (and
// their scale/shift in registers) for the whole loop.
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, long long n4, int C,
                                                       const float* __restrict__ ss, int act, float slope,
                                                       const float* __restrict__ res, float* __restrict__ y,
                                                       __bf16* __restrict__ y16) {
  const int C4 = C >> 2;
  const int c = (threadIdx.x % C4) * 4;
  f32x4 sc, sf;
#pragma unroll
  for (int e = 0; e < 4; ++e) { sc[e] = ss[c + e]; sf[e] = ss[C + c + e]; }
  const f32x4* z4 = reinterpret_cast<const f32x4*>(z);
  const f32x4* r4 = reinterpret_cast<const f32x4*>(res);
  f32x4* y4 = reinterpret_cast<f32x4*>(y);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 v = z4[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_f(v[e] * sc[e] + sf[e], act, slope);
    if (res) v += r4[i];
    if (y) y4[i] = v;  // (null: only the bf16 copy is read downstream)
    if (y16) store16(y16, i, v);
  }
}

// per-block partials of sum(dyh) and sum(dyh * xhat), float4 per thread (4 channels fixed per
// thread: 256 % (C/4) == 0)
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ dy, const float* __restrict__ z,
                                                            long long n4, int C, const float* __restrict__ ss,
                                                            const float* __restrict__ mi, int act, float slope,
                                                            float* part) {
  __shared__ f32x4 r0[256], r1[256];
  const int tid = threadIdx.x, C4 = C >> 2;
  const int c = (tid % C4) * 4;
  f32x4 sc, sf, mean, inv;
#pragma unroll
  for (int e = 0; e < 4; ++e) { sc[e] = ss[c + e]; sf[e] = ss[C + c + e]; mean[e] = mi[c + e]; inv[e] = mi[C + c + e]; }
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  const f32x4* z4 = reinterpret_cast<const f32x4*>(z);
  const f32x4* d4 = reinterpret_cast<const f32x4*>(dy);
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const f32x4 zz = z4[i], dd = d4[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g = dd[e] * act_grad(zz[e] * sc[e] + sf[e], act, slope);
      a0[e] += g;
      a1[e] += g * (zz[e] - mean[e]) * inv[e];
    }
  }
  r0[tid] = a0;
  r1[tid] = a1;
  __syncthreads();
  if (tid < C4) {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = tid; k < 256; k += C4) { s0 += r0[k]; s1 += r1[k]; }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      part[(long long)blockIdx.x * 2 * C + 4 * tid + e] = s0[e];
      part[(long long)blockIdx.x * 2 * C + C + 4 * tid + e] = s1[e];
    }
  }
}

// fp64 combine of the partials -> dgamma, dbeta and the apply coefficients (one block per channel)
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                              long long nvox, const float* __restrict__ gamma,
                                                              const float* __restrict__ mi, float* dgamma,
                                                              float* dbeta, float* coef, int accumulate) {
  __shared__ double red[2][4];
  const int c = blockIdx.x, tid = threadIdx.x;
  double s0 = 0.0, s1 = 0.0;
  for (int b = tid; b < nblk; b += blockDim.x) {
    s0 += part[(long long)b * 2 * C + c];
    s1 += part[(long long)b * 2 * C + C + c];
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  if ((tid & 63) == 0) { red[0][tid >> 6] = s0; red[1][tid >> 6] = s1; }
  __syncthreads();
  if (tid == 0) {
    s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)s0 : (float)s0;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)s1 : (float)s1;
    coef[c] = gamma[c] * mi[C + c];
    coef[C + c] = (float)(s0 / (double)nvox);
    coef[2 * C + c] = (float)(s1 / (double)nvox);
  }
}

// dz = gamma*invstd*(dyh - mean(dyh) - xhat*mean(dyh*xhat)), float4, channels fixed per thread
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ z,
                                                           long long n4, int C, const float* __restrict__ ss,
                                                           const float* __restrict__ mi, int act, float slope,
                                                           const float* __restrict__ coef, float* dz,
                                                           __bf16* __restrict__ dz16) {
  const int C4 = C >> 2;
  const int c = (threadIdx.x % C4) * 4;
  f32x4 sc, sf, mean, inv, k0, k1, k2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = ss[c + e]; sf[e] = ss[C + c + e]; mean[e] = mi[c + e]; inv[e] = mi[C + c + e];
    k0[e] = coef[c + e]; k1[e] = coef[C + c + e]; k2[e] = coef[2 * C + c + e];
  }

  const f32x4* z4 = reinterpret_cast<const f32x4*>(z);
  const f32x4* d4 = reinterpret_cast<const f32x4*>(dy);
  f32x4* o4 = reinterpret_cast<f32x4*>(dz);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const f32x4 zz = z4[i], dd = d4[i];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = bn_bwd_map(dd[e], zz[e], sc[e], sf[e], mean[e], inv[e], k0[e], k1[e], k2[e], act, slope);
    if (dz) o4[i] = o;
    if (dz16) store16(dz16, i, o);
  }
}

// bn_bwd_apply_kernel with dy = reflect_fold(padded) gathered on the fly: per voxel the 1..8
// padded sources that mirror onto it (fold_src), float4 of channels per thread, channels fixed per
// thread (256 % (C/4) == 0); the bf16 copy (and the fp32 dz when asked) as bn_bwd_apply_kernel.
struct NoPrefetch {
  __device__ void operator()() const {}
};

// coef == NULL: the coefficients from fp64 accumulators (cgan3d_bn_backward_acc_fold): every block
// combines the replicas, block 0 publishes dgamma / dbeta and zeroes `zero`
template <bool B16>  // padded and z in bf16
__global__ __launch_bounds__(256) void bn_bwd_apply_fold_kernel(const void* __restrict__ padded,
                                                                const void* __restrict__ z, int n, int D, int H, int W,
                                                                int P, int C, const float* __restrict__ ss,
                                                                const float* __restrict__ mi, int act, float slope,
                                                                const float* __restrict__ coef, float* dz,
                                                                __bf16* __restrict__ dz16, const double* __restrict__ acc,
                                                                int reps, double nvox, const float* __restrict__ gamma,
                                                                float* dgamma, float* dbeta, int accumulate,
                                                                double* zero, int zero_n) {
  __shared__ double sums[2 * 256], part[256];
  __shared__ float co[3 * 256];
  if (!coef) {
    const int tid = threadIdx.x;
    if (blockIdx.x == 0)
      for (int j = tid; j < zero_n; j += blockDim.x) zero[j] = 0.0;
    acc_sums(acc, reps, C, sums, part, NoPrefetch());
    __syncthreads();
    for (int c = tid; c < C; c += blockDim.x)
      bn_acc_bwd_coeffs(sums, c, C, nvox, gamma, mi, &co[c], &co[C + c], &co[2 * C + c], blockIdx.x == 0, dgamma,
                        dbeta, accumulate);
    __syncthreads();
    coef = co;
  }
  const int C4 = C >> 2;
  const int c = (threadIdx.x % C4) * 4;
  f32x4 sc, sf, mean, inv, k0, k1, k2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = ss[c + e]; sf[e] = ss[C + c + e]; mean[e] = mi[c + e]; inv[e] = mi[C + c + e];
    k0[e] = coef[c + e]; k1[e] = coef[C + c + e]; k2[e] = coef[2 * C + c + e];
  }

  const int Dp = D + 2 * P, Hp = H + 2 * P, Wp = W + 2 * P;
  const long long n4 = (long long)n * D * H * W * C4;
  f32x4* o4 = reinterpret_cast<f32x4*>(dz);
  // 32-bit index math: C/4 a power of two (C divides 256), the padded volume below 2^31 float4
  // (checked by the callers); four 64-bit divides per float4 made this pass VALU-bound
  const int c4s = __builtin_ctz(C4);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)n4; i += gridDim.x * blockDim.x) {
    const unsigned v0 = i >> c4s;
    const int c4 = (int)(i & (C4 - 1));
    const unsigned v1 = v0 / (unsigned)W, v2 = v1 / (unsigned)H, v3 = v2 / (unsigned)D;
    const int w = (int)(v0 - v1 * W), h = (int)(v1 - v2 * H), d = (int)(v2 - v3 * D), nb = (int)v3;
    int qd[2], qh[2], qw[2];
    const int nd = fold_src(d, D, P, qd), nh = fold_src(h, H, P, qh), nw = fold_src(w, W, P, qw);
    const f32x4 zz = load4<B16>(z, i);
    f32x4 dd = load4<B16>(padded, ((((nb * Dp + qd[0]) * Hp + qh[0]) * Wp + qw[0]) << c4s) + c4);
    if (nd * nh * nw > 1) {  // boundary voxel: its mirrored sources
      for (int a = 0; a < nd; ++a)
        for (int b = 0; b < nh; ++b)
          for (int e = 0; e < nw; ++e)
            if (a | b | e) dd += load4<B16>(padded, ((((nb * Dp + qd[a]) * Hp + qh[b]) * Wp + qw[e]) << c4s) + c4);
    }
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = bn_bwd_map(dd[e], zz[e], sc[e], sf[e], mean[e], inv[e], k0[e], k1[e], k2[e], act, slope);
    if (dz) o4[i] = o;
    if (dz16) store16(dz16, i, o);
  }
}

// bn_bwd_apply_fold_kernel<true> by rows (round 5c): block (h chunk, nb * D + d), a row of W voxels
// x C channels read as 16-byte granules of 8 bf16 channels (RW = W C / 8 threads per row, a power of
// two dividing 256), FOLD_U rows per thread.  No per-element divides (the grid-stride form spent 3
// runtime divides per 8 bytes), the interior loads of all FOLD_U rows in flight while the replicas
// are combined, 16-byte accesses, the boundary rows' mirror loads issued together: 38.3 -> 25.3 us at 64^3 B = 4
// (bench_ops bn_fold64; a bf16 add over the same bytes takes 15.4).  Sums the mirrored sources
// in the grid-stride kernel's order, so the two are bit-identical.
typedef __bf16 bf16x8_n __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_n __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void bf8_set(float* d, u32x4_n r) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    d[2 * e] = __uint_as_float(r[e] << 16);
    d[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}

__device__ __forceinline__ void bf8_add(float* d, u32x4_n r) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    d[2 * e] += __uint_as_float(r[e] << 16);
    d[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
  }
}

template <int FOLD_U>
__global__ __launch_bounds__(256) void bn_bwd_fold_rows_kernel(const __bf16* __restrict__ padded,
                                                               const __bf16* __restrict__ z, int D, int H, int W,
                                                               int P, int C, int lrw, int lc8,
                                                               const float* __restrict__ ss,
                                                               const float* __restrict__ mi, int act, float slope,
                                                               float* dz, __bf16* __restrict__ dz16,
                                                               const double* __restrict__ acc, int reps, double nvox,
                                                               const float* __restrict__ gamma, float* dgamma,
                                                               float* dbeta, int accumulate, double* zero,
                                                               int zero_n, unsigned pbytes, int probe) {
  __shared__ double sums[2 * 256], part[256];
  __shared__ float co[7 * 128];  // k0, k1, k2, scale, shift, mean, invstd (C <= 128): in LDS, not 56 VGPRs
  const int tid = threadIdx.x;
  const int RP = 256 >> lrw;  // rows per pass
  const int rl = tid >> lrw, g = tid & ((1 << lrw) - 1);
  const int w = g >> lc8, c = (g & ((1 << lc8) - 1)) * 8;
  // planes dispatched boundary first (D >= 2P + 2): the 2P planes with a d-mirror have every row on
  // the slower path, started first they finish under the interior planes instead of after them
  int nb, d;
  {
    const int y = blockIdx.y, nbd = 2 * P, nbat = gridDim.y / D;
    if (D < 2 * P + 2) {
      nb = y / D; d = y - nb * D;
    } else if (y < nbat * nbd) {
      nb = y / nbd;
      const int k = y - nb * nbd;
      d = k < P ? 1 + k : D - 1 - P + (k - P);
    } else {
      const int y2 = y - nbat * nbd, ni = D - nbd;
      nb = y2 / ni;
      const int k = y2 - nb * ni;
      d = k == 0 ? 0 : (k <= D - 2 - 2 * P ? k + P : D - 1);
    }
  }
  const int nd_ = nb * D + d;
  const int h0 = blockIdx.x * (FOLD_U * RP) + rl;
  const int Dp = D + 2 * P, Hp = H + 2 * P, Wp = W + 2 * P;
  const bool pub = blockIdx.x == 0 && blockIdx.y == 0;
  if (pub)
    for (int j = tid; j < zero_n; j += blockDim.x) zero[j] = 0.0;
  // interior source, its w-mirror (per lane; the interior again where there is none) and z of this
  // thread's FOLD_U rows, raw bits: every lane's common sources in flight before the first use — a
  // mirror load issued inside the row loop waited for all earlier stores (vmcnt counts both) and made
  // the pass 2x the HBM time
  int qd[2], qw[2];
  const int nd = fold_src(d, D, P, qd), nw = fold_src(w, W, P, qw);
  const int wsrc = nw > 1 ? qw[1] : qw[0];
  u32x4_n zr[FOLD_U], pr[FOLD_U], pw[FOLD_U];
  // mirror sources through a buffer descriptor: a lane without one gets an offset past the end, which
  // the range check drops (zeros, no memory request) — most lanes of every wave have none
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void*)padded, (short)0, (int)pbytes, 0x00020000);
  constexpr unsigned OOB = 0xfffffff0u;
  float tss, tmi, gc, ic;
  auto pf = [&] {  // the layer's scale / shift / mean / invstd first: loaded after the data, their wait
                   // covered every row's loads
    tss = ss[min(tid, 2 * C - 1)];
    tmi = mi[min(tid, 2 * C - 1)];
    gc = gamma[min(tid, C - 1)];
    ic = mi[C + min(tid, C - 1)];
#pragma unroll
    for (int u = 0; u < FOLD_U; ++u) {
      const int h = min(h0 + u * RP, H - 1);
      const __bf16* prow = padded + ((long long)((nb * Dp + d + P) * Hp + h + P) * Wp) * C + c;
      zr[u] = CG_PROBE(probe, 8) ? u32x4_n{} : *reinterpret_cast<const u32x4_n*>(z + ((long long)(nd_ * H + h) * W + w) * C + c);
      pr[u] = CG_PROBE(probe, 2) ? u32x4_n{} : *reinterpret_cast<const u32x4_n*>(prow + (w + P) * C);
      const unsigned wo = 2u * (unsigned)((((nb * Dp + d + P) * Hp + h + P) * Wp + wsrc) * C + c);
      pw[u] = CG_PROBE(probe, 2) ? u32x4_n{} : __builtin_amdgcn_raw_buffer_load_b128(prs, nw > 1 ? wo : OOB, 0, 0);
    }
  };
  if (CG_PROBE(probe, 1)) {
    pf();
    if (tid < 2 * C) sums[tid] = 1.0;
  } else {
    acc_sums(acc, reps, C, sums, part, pf);
  }
  if (tid < 2 * C) {
    co[3 * C + tid] = tss;
    co[5 * C + tid] = tmi;
  }
  lds_barrier();
  if (tid < C)  // C <= 128 (the launcher's check)
    bn_acc_bwd_coeffs_pre(sums, tid, C, nvox, gc, ic, &co[tid], &co[C + tid], &co[2 * C + tid], pub, dgamma, dbeta,
                          accumulate);
  lds_barrier();
  const float* cq = co + c;
  auto finish = [&](int u, int h, const float* dd) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zz = __uint_as_float((e & 1) ? (zr[u][e >> 1] & 0xffff0000u) : (zr[u][e >> 1] << 16));
      o[e] = bn_bwd_map(dd[e], zz, cq[3 * C + e], cq[4 * C + e], cq[5 * C + e], cq[6 * C + e], cq[e], cq[C + e],
                        cq[2 * C + e], act, slope);
    }
    const long long i = ((long long)(nd_ * H + h) * W + w) * C + c;
    if (CG_PROBE(probe, 4)) return;
    if (dz) {
      reinterpret_cast<f32x4*>(dz + i)[0] = f32x4{o[0], o[1], o[2], o[3]};
      reinterpret_cast<f32x4*>(dz + i)[1] = f32x4{o[4], o[5], o[6], o[7]};
    }
    if (dz16) {
      bf16x8_n v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)o[e];
      *reinterpret_cast<bf16x8_n*>(dz16 + i) = v;
    }
  };
  // rows off the d / h boundary first (at most the prefetched w-mirror) ...
#pragma unroll
  for (int u = 0; u < FOLD_U; ++u) {
    const int h = h0 + u * RP;
    if (h >= H) break;
    int qh[2];
    if (nd * fold_src(h, H, P, qh) != 1) continue;  // (wave-uniform at RW >= 64)
    float dd[8];
    bf8_set(dd, pr[u]);
    if (nw > 1) bf8_add(dd, pw[u]);
    finish(u, h, dd);
  }
  // ... then the d / h boundary rows, whose further sources are loaded here (a load under the branch
  // above made every row wait for all loads and stores in flight)
  if (CG_PROBE(probe, 2)) return;
#pragma unroll
  for (int u = 0; u < FOLD_U; ++u) {
    const int h = h0 + u * RP;
    if (h >= H) break;
    int qh[2];
    const int nh = fold_src(h, H, P, qh);
    if (nd * nh == 1) continue;
    // all 6 further candidates loaded at once (the preimage itself where one does not exist), then the
    // existing ones summed in (a, b, e) order: loaded one by one, each waited for the last, and the
    // boundary blocks set the kernel's length (33.8 us at 64^3, against 15.4 for a bf16 add)
    u32x4_n m[8];
#pragma unroll
    for (int j = 2; j < 8; ++j) {
      const int a = j >> 2, b = (j >> 1) & 1, e = j & 1;
      const int sd = a < nd ? qd[a] : qd[0], sh = b < nh ? qh[b] : qh[0], sw = e < nw ? qw[e] : qw[0];
      const unsigned mo = 2u * (unsigned)((((nb * Dp + sd) * Hp + sh) * Wp + sw) * C + c);
      m[j] = __builtin_amdgcn_raw_buffer_load_b128(prs, (a < nd && b < nh && e < nw) ? mo : OOB, 0, 0);
    }
    m[1] = pw[u];
    float dd[8];
    bf8_set(dd, pr[u]);
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if ((j >> 2) < nd && ((j >> 1) & 1) < nh && (j & 1) < nw) bf8_add(dd, m[j]);
    finish(u, h, dd);
  }
}

// ---- fused-statistics path: per-block partials written by the producing kernel's epilogue into
// a channel-major slab part[(q * C + c) * nslots + b] (no atomics); one block per channel reads its
// contiguous rows (coalesced) and combines them in fp64.
__device__ __forceinline__ void slab_sums(const float* __restrict__ part, int nslots, int C, int c, double* s0,
                                          double* s1) {
  __shared__ double red[2][4];
  const int tid = threadIdx.x;
  const float* r0 = part + (long long)c * nslots;
  const float* r1 = part + (long long)(C + c) * nslots;
  double a0 = 0.0, a1 = 0.0;
  for (int b0 = tid; b0 < nslots; b0 += 4 * blockDim.x) {
    float v0[4], v1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // four slots in flight
      const int b = b0 + k * blockDim.x, bb = b < nslots ? b : 0;
      v0[k] = b < nslots ? r0[bb] : 0.f;
      v1[k] = b < nslots ? r1[bb] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) { a0 += v0[k]; a1 += v1[k]; }
  }
  a0 = wave_sum_d(a0);
  a1 = wave_sum_d(a1);
  if ((tid & 63) == 0) { red[0][tid >> 6] = a0; red[1][tid >> 6] = a1; }
  __syncthreads();
  *s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  *s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
}

// forward slab rows: sum (c), M2 about the block mean (C + c), block count (2C); Chan's combine
// in fp64, read coalesced (one block per channel, threads striding the slots).
__device__ __forceinline__ void finalize_slab_channel(int c, const float* __restrict__ part, int nslots, int C,
                                                      double nvox, const float* gamma, const float* beta,
                                                      float* rmean, float* rvar, long long* nbt, float momentum,
                                                      float eps, float* scale_shift, float* mean_invstd) {
  __shared__ double red[3][4];
  const int tid = threadIdx.x;
  const float* rs = part + (long long)c * nslots;
  const float* rq = part + (long long)(C + c) * nslots;
  const float* rn = part + (long long)2 * C * nslots;
  double n = 0.0, m = 0.0, q = 0.0;
  for (int b0 = tid; b0 < nslots; b0 += 4 * blockDim.x) {
    float sv[4], qv[4], nv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // four slots in flight
      const int b = b0 + k * blockDim.x, bb = b < nslots ? b : 0;
      sv[k] = rs[bb]; qv[k] = rq[bb]; nv[k] = b < nslots ? rn[bb] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (nv[k] > 0.f) chan_merge(n, m, q, nv[k], (double)sv[k] / nv[k], qv[k]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double nb = __shfl_xor(n, off, 64), mb = __shfl_xor(m, off, 64), qb = __shfl_xor(q, off, 64);
    chan_merge(n, m, q, nb, mb, qb);
  }
  if ((tid & 63) == 0) { red[0][tid >> 6] = n; red[1][tid >> 6] = m; red[2][tid >> 6] = q; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) chan_merge(n, m, q, red[0][w], red[1][w], red[2][w]);
    const double mean = m, var = q / n;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * invstd;
    scale_shift[c] = (float)sc;
    scale_shift[C + c] = (float)((double)beta[c] - mean * sc);
    mean_invstd[c] = (float)mean;
    mean_invstd[C + c] = (float)invstd;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * nvox / (nvox > 1 ? nvox - 1 : 1));
    if (nbt && c == 0) *nbt += 1;
  }
}

__global__ __launch_bounds__(256) void bn_finalize_slab_kernel(const float* __restrict__ part, int nslots, int C,
                                                               double nvox, const float* gamma, const float* beta,
                                                               float* rmean, float* rvar, long long* nbt,
                                                               float momentum, float eps, float* scale_shift,
                                                               float* mean_invstd) {
  finalize_slab_channel(blockIdx.x, part, nslots, C, nvox, gamma, beta, rmean, rvar, nbt, momentum, eps, scale_shift,
                        mean_invstd);
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_slab_kernel(const float* __restrict__ part, int nslots, int C,
                                                                   double nvox, const float* __restrict__ gamma,
                                                                   const float* __restrict__ mi, float* dgamma,
                                                                   float* dbeta, float* coef, int accumulate) {
  const int c = blockIdx.x;
  double s0, s1;
  slab_sums(part, nslots, C, c, &s0, &s1);
  if (threadIdx.x == 0) {
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)s0 : (float)s0;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)s1 : (float)s1;
    coef[c] = gamma[c] * mi[C + c];
    coef[C + c] = (float)(s0 / nvox);
    coef[2 * C + c] = (float)(s1 / nvox);
  }
}

__global__ __launch_bounds__(256) void channel_sum_kernel(const float* __restrict__ x, long long total, int C,
                                                          float* part) {
  __shared__ float r0[256];
  const int tid = threadIdx.x;
  float a0 = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < total; i += (long long)gridDim.x * blockDim.x)
    a0 += x[i];
  r0[tid] = a0;
  __syncthreads();
  if (tid < C) {
    float s0 = 0.f;
    for (int k = tid; k < 256; k += C) s0 += r0[k];
    part[(long long)blockIdx.x * C + tid] = s0;
  }
}

__global__ __launch_bounds__(256) void channel_sum_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                                   float* out) {
  __shared__ double red[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  double s = 0.0;
  for (int b = tid; b < nblk; b += blockDim.x) s += part[(long long)b * C + c];
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) out[c] = (float)(red[0] + red[1] + red[2] + red[3]);
}

// ---- several channel sums in two launches (the critic's bias gradients, one tensor per layer):
// grid (nblk, n) of fp64 partial sums into each descriptor's workspace, then one block per
// descriptor combines its nblk partials per channel (wave per channel).  fp64 throughout: a bias
// gradient is often a near-cancelling sum (the critic's last bias: -1/n per real logit, +1/n per
// fake one, exactly 0 in real arithmetic).
__global__ __launch_bounds__(256) void channel_sum_multi_kernel(const cgan3d_csum_desc* __restrict__ descs) {
  __shared__ double r0[256];
  const cgan3d_csum_desc e = descs[blockIdx.y];
  const int tid = threadIdx.x, C = e.c;
  const long long total = (long long)e.nvox * C;
  double a0 = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < total; i += (long long)gridDim.x * blockDim.x)
    a0 += (double)e.x[i];
  r0[tid] = a0;
  __syncthreads();
  for (int w = 128; w >= C; w >>= 1) {  // tree over the 256 / C threads of each channel
    if (tid < w) r0[tid] += r0[tid + w];
    __syncthreads();
  }
  if (tid < C) e.ws[(long long)blockIdx.x * C + tid] = r0[tid];
}

// block (channel, descriptor): 256 threads over the nblk partials, fp64 tree
__global__ __launch_bounds__(256) void channel_sum_multi_finalize_kernel(const cgan3d_csum_desc* __restrict__ descs,
                                                                         int nblk) {
  __shared__ double red[4];
  const cgan3d_csum_desc e = descs[blockIdx.y];
  const int c = blockIdx.x, tid = threadIdx.x;
  if (c >= e.c) return;
  double s = 0.0;
  for (int b = tid; b < nblk; b += 256) s += e.ws[(long long)b * e.c + c];
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    const double t = (red[0] + red[1]) + (red[2] + red[3]);
    e.out[c] = e.accumulate ? e.out[c] + (float)t : (float)t;
  }
}

// ---- finalize fused into the elementwise pass (small slabs): every block combines the whole slab
// itself (G = 256 / C threads per channel, Chan in fp64, group shuffles), block 0 publishes the
// statistics / running buffers / parameter gradients; no separate finalize launch.  Only for small
// slabs (<= 24 KB per block, e.g. 32^3 patches): at 64^3 the 16^3 x 64-channel layers' 196 KB slab
// read by every block made the fused launch slower than finalize + apply.
__device__ __forceinline__ void slab_chan(const float* __restrict__ part, int nslots, int C, int c, int j, int G,
                                          double* n, double* m, double* q) {
  const float* rs = part + (long long)c * nslots;
  const float* rq = part + (long long)(C + c) * nslots;
  const float* rn = part + (long long)2 * C * nslots;
  double nn = 0.0, mm = 0.0, qq = 0.0;
  for (int b0 = j; b0 < nslots; b0 += 4 * G) {
    float sv[4], qv[4], nv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = b0 + k * G, bb = b < nslots ? b : 0;
      sv[k] = rs[bb]; qv[k] = rq[bb]; nv[k] = b < nslots ? rn[bb] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (nv[k] > 0.f) chan_merge(nn, mm, qq, nv[k], (double)sv[k] / nv[k], qv[k]);
  }
  for (int off = G >> 1; off > 0; off >>= 1) {
    const double nb = __shfl_xor(nn, off, 64), mb = __shfl_xor(mm, off, 64), qb = __shfl_xor(qq, off, 64);
    chan_merge(nn, mm, qq, nb, mb, qb);
  }
  *n = nn; *m = mm; *q = qq;
}

__global__ __launch_bounds__(256) void bn_apply_slab_kernel(const float* __restrict__ part, int nslots, int C,
                                                            double nvox, const float* gamma, const float* beta,
                                                            float* rmean, float* rvar, long long* nbt, float momentum,
                                                            float eps, float* scale_shift, float* mean_invstd,
                                                            const float* __restrict__ z, long long n4, int act,
                                                            float slope, const float* __restrict__ res,
                                                            float* __restrict__ y, __bf16* __restrict__ y16) {
  __shared__ float ssh[2 * 256];
  const int tid = threadIdx.x, G = 256 / C, c = tid / G, j = tid - c * G;
  double n, m, q;
  slab_chan(part, nslots, C, c, j, G, &n, &m, &q);
  if (j == 0) {
    const double mean = m, var = q / n;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * invstd;
    ssh[c] = (float)sc;
    ssh[C + c] = (float)((double)beta[c] - mean * sc);
    if (blockIdx.x == 0) {
      scale_shift[c] = ssh[c];
      scale_shift[C + c] = ssh[C + c];
      mean_invstd[c] = (float)mean;
      mean_invstd[C + c] = (float)invstd;
      if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
      if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * nvox / (nvox > 1 ? nvox - 1 : 1));
      if (nbt && c == 0) *nbt += 1;
    }
  }
  __syncthreads();
  const int C4 = C >> 2, cc = (tid % C4) * 4;
  f32x4 sc4, sf4;
#pragma unroll
  for (int e = 0; e < 4; ++e) { sc4[e] = ssh[cc + e]; sf4[e] = ssh[C + cc + e]; }
  const f32x4* z4 = reinterpret_cast<const f32x4*>(z);
  const f32x4* r4 = reinterpret_cast<const f32x4*>(res);
  f32x4* y4 = reinterpret_cast<f32x4*>(y);
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 v = z4[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_f(v[e] * sc4[e] + sf4[e], act, slope);
    if (res) v += r4[i];
    if (y) y4[i] = v;  // (null: only the bf16 copy is read downstream)
    if (y16) store16(y16, i, v);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_slab_kernel(const float* __restrict__ part, int nslots, int C,
                                                                double nvox, const float* __restrict__ gamma,
                                                                const float* __restrict__ mi, float* dgamma,
                                                                float* dbeta, int accumulate,
                                                                const float* __restrict__ dy,
                                                                const float* __restrict__ z, long long n4,
                                                                const float* __restrict__ ss, int act, float slope,
                                                                float* __restrict__ dz, __bf16* __restrict__ dz16) {
  __shared__ float co[3 * 256];
  const int tid = threadIdx.x, G = 256 / C, c = tid / G, j = tid - c * G;
  {
    const float* r0 = part + (long long)c * nslots;
    const float* r1 = part + (long long)(C + c) * nslots;
    double a0 = 0.0, a1 = 0.0;
    for (int b0 = j; b0 < nslots; b0 += 4 * G) {
      float v0[4], v1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int b = b0 + k * G, bb = b < nslots ? b : 0;
        v0[k] = b < nslots ? r0[bb] : 0.f;
        v1[k] = b < nslots ? r1[bb] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) { a0 += v0[k]; a1 += v1[k]; }
    }
    for (int off = G >> 1; off > 0; off >>= 1) {
      a0 += __shfl_xor(a0, off, 64);
      a1 += __shfl_xor(a1, off, 64);
    }
    if (j == 0) {
      co[c] = gamma[c] * mi[C + c];
      co[C + c] = (float)(a0 / nvox);
      co[2 * C + c] = (float)(a1 / nvox);
      if (blockIdx.x == 0) {
        if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)a0 : (float)a0;
        if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)a1 : (float)a1;
      }
    }
  }
  __syncthreads();
  const int C4 = C >> 2, cc = (tid % C4) * 4;
  f32x4 sc, sf, mean, inv, k0, k1, k2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = ss[cc + e]; sf[e] = ss[C + cc + e]; mean[e] = mi[cc + e]; inv[e] = mi[C + cc + e];
    k0[e] = co[cc + e]; k1[e] = co[C + cc + e]; k2[e] = co[2 * C + cc + e];
  }

  const f32x4* z4 = reinterpret_cast<const f32x4*>(z);
  const f32x4* d4 = reinterpret_cast<const f32x4*>(dy);
  f32x4* o4 = reinterpret_cast<f32x4*>(dz);
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const f32x4 zz = z4[i], dd = d4[i];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = bn_bwd_map(dd[e], zz[e], sc[e], sf[e], mean[e], inv[e], k0[e], k1[e], k2[e], act, slope);
    if (dz) o4[i] = o;
    if (dz16) store16(dz16, i, o);
  }
}

// ---- statistics from fp64 accumulators (cgan3d_bn_fuse acc_mode 3 / 4: the producing conv added its
// per-block pairs into `reps` replicas acc[r][2][C]); finalize folded into the elementwise pass: every
// block combines the replicas itself (16 KB at reps 16, C 64: all loads in flight), block 0 publishes
// statistics / running buffers / parameter gradients and zeroes an accumulator the stream is done
// with (the caller rotates them, so none needs a memset launch).
// float4 per thread loaded before the statistics are known (acc_pass_blocks sizes the grid at ~2)
constexpr int ACC_PF = 2;

// RES: residual added (a load under `if (res)` made the compiler wait for every load in flight); Z16: z in bf16
template <bool RES, bool Z16>
__global__ __launch_bounds__(256) void bn_apply_acc_kernel(const double* __restrict__ acc, int reps, int C, double nvox,
                                                           const float* gamma, const float* beta, float* rmean,
                                                           float* rvar, long long* nbt, float momentum, float eps,
                                                           float* scale_shift, float* mean_invstd,
                                                           const void* __restrict__ z, long long n4, int act,
                                                           float slope, const float* __restrict__ res,
                                                           float* __restrict__ y, __bf16* __restrict__ y16,
                                                           double* zero, int zero_n) {
  __shared__ double sums[2 * 256], part[256];
  __shared__ float ssh[2 * 256];
  const int tid = threadIdx.x;
  if (blockIdx.x == 0)
    for (int j = tid; j < zero_n; j += blockDim.x) zero[j] = 0.0;
  // the first ACC_PF float4 of this thread's elementwise range are loaded while the replicas are in flight
  const f32x4* r4 = reinterpret_cast<const f32x4*>(res);
  const long long i0 = (long long)blockIdx.x * blockDim.x + tid, stride = (long long)gridDim.x * blockDim.x;
  f32x4 zp[ACC_PF], rp[ACC_PF];
  acc_sums(acc, reps, C, sums, part, [&] {
#pragma unroll
    for (int u = 0; u < ACC_PF; ++u) {
      const long long i = min(i0 + u * stride, n4 - 1);
      zp[u] = load4<Z16>(z, i);
      if (RES) rp[u] = r4[i];
    }
  });
  lds_barrier();
  for (int c = tid; c < C; c += blockDim.x)
    bn_acc_fwd_coeffs(sums, c, C, nvox, gamma, beta, eps, &ssh[c], &ssh[C + c], blockIdx.x == 0, scale_shift,
                      mean_invstd, rmean, rvar, nbt, momentum);
  lds_barrier();
  const int C4 = C >> 2, cc = (tid % C4) * 4;
  f32x4 sc4, sf4;
#pragma unroll
  for (int e = 0; e < 4; ++e) { sc4[e] = ssh[cc + e]; sf4[e] = ssh[C + cc + e]; }
  f32x4* y4 = reinterpret_cast<f32x4*>(y);
  auto apply = [&](long long i, f32x4 v, const f32x4& r) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_f(v[e] * sc4[e] + sf4[e], act, slope);
    if (RES) v += r;
    if (y) y4[i] = v;
    if (y16) store16(y16, i, v);
  };
#pragma unroll
  for (int u = 0; u < ACC_PF; ++u)
    if (i0 + u * stride < n4) apply(i0 + u * stride, zp[u], rp[u]);
  for (long long i = i0 + ACC_PF * stride; i < n4; i += stride) apply(i, load4<Z16>(z, i), RES ? r4[i] : f32x4{});
}

template <bool B16>  // dy and z in bf16
__global__ __launch_bounds__(256) void bn_bwd_apply_acc_kernel(const double* __restrict__ acc, int reps, int C,
                                                               double nvox, const float* __restrict__ gamma,
                                                               const float* __restrict__ mi, float* dgamma,
                                                               float* dbeta, int accumulate,
                                                               const void* __restrict__ dy,
                                                               const void* __restrict__ z, long long n4,
                                                               const float* __restrict__ ss, int act, float slope,
                                                               float* __restrict__ dz, __bf16* __restrict__ dz16,
                                                               double* zero, int zero_n) {
  __shared__ double sums[2 * 256], part[256];
  __shared__ float co[3 * 256];
  const int tid = threadIdx.x;
  if (blockIdx.x == 0)
    for (int j = tid; j < zero_n; j += blockDim.x) zero[j] = 0.0;
  const long long i0 = (long long)blockIdx.x * blockDim.x + tid, stride = (long long)gridDim.x * blockDim.x;
  f32x4 zp[ACC_PF], dp[ACC_PF];
  acc_sums(acc, reps, C, sums, part, [&] {
#pragma unroll
    for (int u = 0; u < ACC_PF; ++u) {
      const long long i = min(i0 + u * stride, n4 - 1);
      zp[u] = load4<B16>(z, i);
      dp[u] = load4<B16>(dy, i);
    }
  });
  lds_barrier();
  for (int c = tid; c < C; c += blockDim.x)
    bn_acc_bwd_coeffs(sums, c, C, nvox, gamma, mi, &co[c], &co[C + c], &co[2 * C + c], blockIdx.x == 0, dgamma, dbeta,
                      accumulate);
  lds_barrier();
  const int C4 = C >> 2, cc = (tid % C4) * 4;
  f32x4 sc, sf, mean, inv, k0, k1, k2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = ss[cc + e]; sf[e] = ss[C + cc + e]; mean[e] = mi[cc + e]; inv[e] = mi[C + cc + e];
    k0[e] = co[cc + e]; k1[e] = co[C + cc + e]; k2[e] = co[2 * C + cc + e];
  }

  f32x4* o4 = reinterpret_cast<f32x4*>(dz);
  auto apply = [&](long long i, const f32x4& zz, const f32x4& dd) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = bn_bwd_map(dd[e], zz[e], sc[e], sf[e], mean[e], inv[e], k0[e], k1[e], k2[e], act, slope);
    if (dz) o4[i] = o;
    if (dz16) store16(dz16, i, o);
  };
#pragma unroll
  for (int u = 0; u < ACC_PF; ++u)
    if (i0 + u * stride < n4) apply(i0 + u * stride, zp[u], dp[u]);
  for (long long i = i0 + ACC_PF * stride; i < n4; i += stride) apply(i, load4<B16>(z, i), load4<B16>(dy, i));
}

// blocks of the accumulator passes: ~2 float4 per thread, at most `cap` blocks — each block reads the
// replicas once (reps x 2C doubles, 4-16 KB, values the atomics left at the memory side): measured at
// 64^3 B=4, the 16-channel passes took 19.5 / 28 us with 4096 blocks against 13.9 / 15.4 with 1024,
// the reflect-folded backward (a gather) 46 us with 4096 against 60 with 1024; the whole step with
// 1 / 2 / 3 / 4 / 8 float4 per thread (round 3): 1.629 / 1.613 / 1.617 / 1.626 / 1.677 ms
static int acc_pass_blocks(long long n4, long long cap = 1024) {
  return (int)std::max(1LL, std::min((n4 + 511) / 512, cap));
}

// blocks of the fused finalize + elementwise launch, or 0 when the slab is too large to be read by
// every block (then: separate finalize launch)
static int slab_fused_blocks(int nslots, int C, int rows, long long n4) {
  if (C < 4 || C > 256 || 256 % C) return 0;
  long long b = (n4 + 256 * 16 - 1) / (256 * 16);  // ~16 float4 per thread
  b = std::max(1LL, std::min(b, 256LL));
  const long long per_block = (long long)nslots * C * rows * 4;  // read by every block, latency-bound:
  return per_block <= 24 * 1024 && per_block * b <= (16LL << 20) ? (int)b : 0;  // measured: 196 KB/block is 3x slower
}

static int reduce_blocks(long long total) {
  long long b = (total + 256 * 8 - 1) / (256 * 8);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace cg

using namespace cg;

extern "C" int cgan3d_bn_finalize(const float* stats, int64_t nblk, int32_t c, const float* gamma, const float* beta,
                                  float* running_mean, float* running_var, int64_t* num_batches_tracked,
                                  float momentum, float eps, float* scale_shift, float* mean_invstd, void* stream) {
  CG_CHECK_ARG(stats && gamma && beta && scale_shift && mean_invstd, "cgan3d_bn_finalize: null pointer");
  CG_CHECK_ARG(nblk > 0 && c > 0 && c <= 1024, "cgan3d_bn_finalize: bad sizes");
  ::cg::launch(bn_finalize_kernel, dim3(c), dim3(256), 0, (hipStream_t)stream, stats, (long long)nblk, c, gamma,
                     beta, running_mean, running_var, (long long*)num_batches_tracked, momentum, eps, scale_shift,
                     mean_invstd);
  CG_LAUNCH_CHECK("bn_finalize_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_apply(const float* z, int64_t nvox, int32_t c, const float* scale_shift, int32_t act,
                               float slope, const float* residual, float* y, void* y_bf16, void* stream) {
  CG_CHECK_ARG(z && scale_shift && (y || y_bf16), "cgan3d_bn_apply: null pointer");
  CG_CHECK_ARG(nvox > 0 && c > 0 && c % 4 == 0 && 256 % (c / 4) == 0,
               "cgan3d_bn_apply: channels must be a multiple of 4 dividing 1024");
  const long long n4 = (long long)nvox * c / 4;
  int blocks = (int)std::min<long long>((n4 + 255) / 256, 4096);
  ::cg::launch(bn_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, z, n4, c, scale_shift, act,
                     slope, residual, y, reinterpret_cast<__bf16*>(y_bf16));
  CG_LAUNCH_CHECK("bn_apply_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_finalize_slab(const float* part, int32_t nslots, int32_t c, int64_t nvox, const float* gamma,
                                       const float* beta, float* running_mean, float* running_var,
                                       int64_t* num_batches_tracked, float momentum, float eps, float* scale_shift,
                                       float* mean_invstd, void* stream) {
  CG_CHECK_ARG(part && gamma && beta && scale_shift && mean_invstd, "cgan3d_bn_finalize_slab: null pointer");
  CG_CHECK_ARG(nslots > 0 && c > 0 && c <= 1024 && nvox > 0, "cgan3d_bn_finalize_slab: bad sizes");
  ::cg::launch(bn_finalize_slab_kernel, dim3(c), dim3(256), 0, (hipStream_t)stream, part, nslots, c, (double)nvox,
                     gamma, beta, running_mean, running_var, (long long*)num_batches_tracked, momentum, eps,
                     scale_shift, mean_invstd);
  CG_LAUNCH_CHECK("bn_finalize_slab_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_backward_slab(const float* dy, const float* z, int64_t nvox, int32_t c, const float* part,
                                       int32_t nslots, const float* scale_shift, const float* mean_invstd,
                                       const float* gamma, int32_t act, float slope, float* dgamma, float* dbeta,
                                       float* dz, int32_t accumulate, float* ws, void* dz_bf16, void* stream) {
  CG_CHECK_ARG(dy && z && part && scale_shift && mean_invstd && gamma && (dz || dz_bf16) && ws,
               "cgan3d_bn_backward_slab: null pointer");
  CG_CHECK_ARG(nvox > 1 && nslots > 0 && c >= 4 && c <= 256 && 256 % c == 0,
               "cgan3d_bn_backward_slab: channels must divide 256 and be >= 4");
  hipStream_t s = (hipStream_t)stream;
  if (const int fb = slab_fused_blocks(nslots, c, 2, (long long)nvox * c / 4)) {
    ::cg::launch(bn_bwd_apply_slab_kernel, dim3(fb), dim3(256), 0, s, part, nslots, c, (double)nvox, gamma,
                 mean_invstd, dgamma, dbeta, (int)accumulate, dy, z, (long long)nvox * c / 4, scale_shift, act, slope,
                 dz, reinterpret_cast<__bf16*>(dz_bf16));
    CG_LAUNCH_CHECK("bn_bwd_apply_slab_kernel");
    return CGAN3D_OK;
  }
  ::cg::launch(bn_bwd_finalize_slab_kernel, dim3(c), dim3(256), 0, s, part, nslots, c, (double)nvox, gamma,
                     mean_invstd, dgamma, dbeta, ws, accumulate);
  CG_LAUNCH_CHECK("bn_bwd_finalize_slab_kernel");
  const long long n4 = (long long)nvox * c / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 4096);
  ::cg::launch(bn_bwd_apply_kernel, dim3(blocks), dim3(256), 0, s, dy, z, n4, c, scale_shift, mean_invstd, act,
                     slope, ws, dz, reinterpret_cast<__bf16*>(dz_bf16));
  CG_LAUNCH_CHECK("bn_bwd_apply_kernel");
  return CGAN3D_OK;
}

extern "C" int64_t cgan3d_bn_backward_ws_floats(int64_t nvox, int32_t c) {
  return (int64_t)reduce_blocks((long long)nvox * c) * 2 * c + 3 * c;
}

extern "C" int cgan3d_bn_backward(const float* dy, const float* z, int64_t nvox, int32_t c, const float* scale_shift,
                                  const float* mean_invstd, const float* gamma, int32_t act, float slope, float* dgamma,
                                  float* dbeta, float* dz, int32_t accumulate, float* ws, void* stream) {
  CG_CHECK_ARG(dy && z && scale_shift && mean_invstd && gamma && dz && ws, "cgan3d_bn_backward: null pointer");
  CG_CHECK_ARG(nvox > 1 && c >= 4 && c <= 256 && 256 % c == 0,
               "cgan3d_bn_backward: channels must divide 256 and be >= 4");
  hipStream_t s = (hipStream_t)stream;
  const long long total = (long long)nvox * c, n4 = total / 4;
  const int nblk = reduce_blocks(total);
  float* part = ws;
  float* coef = ws + (long long)nblk * 2 * c;
  ::cg::launch(bn_bwd_reduce_kernel, dim3(nblk), dim3(256), 0, s, dy, z, n4, c, scale_shift, mean_invstd,
                     act, slope, part);
  CG_LAUNCH_CHECK("bn_bwd_reduce_kernel");
  ::cg::launch(bn_bwd_finalize_kernel, dim3(c), dim3(256), 0, s, part, nblk, c, (long long)nvox, gamma,
                     mean_invstd, dgamma, dbeta, coef, accumulate);
  CG_LAUNCH_CHECK("bn_bwd_finalize_kernel");
  int blocks = (int)std::min<long long>((n4 + 255) / 256, 4096);
  ::cg::launch(bn_bwd_apply_kernel, dim3(blocks), dim3(256), 0, s, dy, z, n4, c, scale_shift, mean_invstd,
                     act, slope, coef, dz, nullptr);
  CG_LAUNCH_CHECK("bn_bwd_apply_kernel");
  return CGAN3D_OK;
}

extern "C" int64_t cgan3d_channel_sum_ws_floats(int64_t nvox, int32_t c) {
  return (int64_t)reduce_blocks((long long)nvox * c) * c;
}

extern "C" int cgan3d_channel_sum(const float* x, int64_t nvox, int32_t c, float* out, float* ws, void* stream) {
  CG_CHECK_ARG(x && out && ws, "cgan3d_channel_sum: null pointer");
  CG_CHECK_ARG(nvox > 0 && c > 0 && c <= 256 && 256 % c == 0, "cgan3d_channel_sum: channels must divide 256");
  hipStream_t s = (hipStream_t)stream;
  const long long total = (long long)nvox * c;
  const int nblk = reduce_blocks(total);
  ::cg::launch(channel_sum_kernel, dim3(nblk), dim3(256), 0, s, x, total, c, ws);
  CG_LAUNCH_CHECK("channel_sum_kernel");
  ::cg::launch(channel_sum_finalize_kernel, dim3(c), dim3(256), 0, s, ws, nblk, c, out);
  CG_LAUNCH_CHECK("channel_sum_finalize_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_apply_slab(const float* part, int32_t nslots, int32_t c, int64_t nvox, const float* gamma,
                                    const float* beta, float* running_mean, float* running_var,
                                    int64_t* num_batches_tracked, float momentum, float eps, float* scale_shift,
                                    float* mean_invstd, const float* z, int32_t act, float slope,
                                    const float* residual, float* y, void* y_bf16, void* stream) {
  CG_CHECK_ARG(part && gamma && beta && scale_shift && mean_invstd && z && (y || y_bf16),
               "cgan3d_bn_apply_slab: null pointer");
  CG_CHECK_ARG(nslots > 0 && nvox > 0 && c >= 4 && c % 4 == 0 && 256 % c == 0,
               "cgan3d_bn_apply_slab: channels must be a multiple of 4 dividing 256");
  const long long n4 = (long long)nvox * c / 4;
  if (const int fb = slab_fused_blocks(nslots, c, 3, n4)) {
    ::cg::launch(bn_apply_slab_kernel, dim3(fb), dim3(256), 0, (hipStream_t)stream, part, nslots, c, (double)nvox,
                 gamma, beta, running_mean, running_var, (long long*)num_batches_tracked, momentum, eps, scale_shift,
                 mean_invstd, z, n4, act, slope, residual, y, reinterpret_cast<__bf16*>(y_bf16));
    CG_LAUNCH_CHECK("bn_apply_slab_kernel");
    return CGAN3D_OK;
  }
  int rc = cgan3d_bn_finalize_slab(part, nslots, c, nvox, gamma, beta, running_mean, running_var, num_batches_tracked,
                                   momentum, eps, scale_shift, mean_invstd, stream);
  return rc ? rc : cgan3d_bn_apply(z, nvox, c, scale_shift, act, slope, residual, y, y_bf16, stream);
}

extern "C" int cgan3d_channel_sum_multi(const cgan3d_csum_desc* descs, int32_t n, int32_t nblk, int32_t cmax,
                                        void* stream) {
  CG_CHECK_ARG(descs && n > 0 && n <= 65535 && nblk > 0 && nblk <= 4096 && cmax > 0 && cmax <= 256,
               "cgan3d_channel_sum_multi: need a device descriptor array, 0 < n <= 65535, 0 < nblk <= 4096, "
               "0 < cmax <= 256 (the largest channel count)");
  hipStream_t s = (hipStream_t)stream;
  ::cg::launch(channel_sum_multi_kernel, dim3(nblk, n), dim3(256), 0, s, descs);
  CG_LAUNCH_CHECK("channel_sum_multi_kernel");
  ::cg::launch(channel_sum_multi_finalize_kernel, dim3(cmax, n), dim3(256), 0, s, descs, (int)nblk);
  CG_LAUNCH_CHECK("channel_sum_multi_finalize_kernel");
  return CGAN3D_OK;
}


extern "C" int cgan3d_bn_backward_slab_fold(const float* padded, const float* z, int32_t n, int32_t d, int32_t h,
                                            int32_t w, int32_t c, int32_t pad, const float* part, int32_t nslots,
                                            const float* scale_shift, const float* mean_invstd, const float* gamma,
                                            int32_t act, float slope, float* dgamma, float* dbeta, float* dz,
                                            int32_t accumulate, float* ws, void* dz_bf16, void* stream) {
  CG_CHECK_ARG(padded && z && part && scale_shift && mean_invstd && gamma && (dz || dz_bf16) && ws,
               "cgan3d_bn_backward_slab_fold: null pointer");
  CG_CHECK_ARG(n > 0 && nslots > 0 && c >= 4 && c <= 256 && 256 % c == 0 && pad >= 0 && d > 2 * pad && h > 2 * pad &&
                   w > 2 * pad,
               "cgan3d_bn_backward_slab_fold: channels must divide 256 (>= 4), dims must exceed 2*pad");
  const long long nvox = (long long)n * d * h * w;
  CG_CHECK_ARG(nvox > 1, "cgan3d_bn_backward_slab_fold: need more than one voxel");
  CG_CHECK_ARG((long long)n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * (c / 4) < (1LL << 31),
               "cgan3d_bn_backward_slab_fold: padded volume exceeds 32-bit float4 indexing");
  hipStream_t s = (hipStream_t)stream;
  ::cg::launch(bn_bwd_finalize_slab_kernel, dim3(c), dim3(256), 0, s, part, nslots, c, (double)nvox, gamma,
               mean_invstd, dgamma, dbeta, ws, accumulate);
  CG_LAUNCH_CHECK("bn_bwd_finalize_slab_kernel");
  const long long n4 = nvox * c / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 4096);
  ::cg::launch(bn_bwd_apply_fold_kernel<false>, dim3(blocks), dim3(256), 0, s, (const void*)padded, (const void*)z, n, d, h, w, pad, c, scale_shift,
               mean_invstd, act, slope, (const float*)ws, dz, reinterpret_cast<__bf16*>(dz_bf16), (const double*)nullptr, 1,
               0.0, (const float*)nullptr, (float*)nullptr, (float*)nullptr, 0, (double*)nullptr, 0);
  CG_LAUNCH_CHECK("bn_bwd_apply_fold_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_apply_acc(const double* acc, int32_t reps, int32_t c, int64_t nvox, const float* gamma,
                                   const float* beta, float* running_mean, float* running_var,
                                   int64_t* num_batches_tracked, float momentum, float eps, float* scale_shift,
                                   float* mean_invstd, const void* z, int32_t act, float slope, const float* residual,
                                   float* y, void* y_bf16, double* zero, int32_t zero_n, int32_t in_bf16,
                                   void* stream) {
  CG_CHECK_ARG(acc && gamma && beta && scale_shift && mean_invstd && z && (y || y_bf16),
               "cgan3d_bn_apply_acc: null pointer");
  CG_CHECK_ARG(reps > 0 && reps <= 64 && nvox > 0 && c >= 4 && c <= 128 && 256 % c == 0 && zero_n >= 0 &&
                   (zero || !zero_n),
               "cgan3d_bn_apply_acc: channels must divide 256 (4..128), reps 1..64");
  const long long n4 = (long long)nvox * c / 4;
  auto* kern = residual ? (in_bf16 ? bn_apply_acc_kernel<true, true> : bn_apply_acc_kernel<true, false>)
                        : (in_bf16 ? bn_apply_acc_kernel<false, true> : bn_apply_acc_kernel<false, false>);
  ::cg::launch(kern, dim3(acc_pass_blocks(n4)), dim3(256),
               0, (hipStream_t)stream, acc, (int)reps, (int)c,
               (double)nvox, gamma, beta, running_mean, running_var, (long long*)num_batches_tracked, momentum, eps,
               scale_shift, mean_invstd, z, n4, act, slope, residual, y, reinterpret_cast<__bf16*>(y_bf16), zero,
               (int)zero_n);
  CG_LAUNCH_CHECK("bn_apply_acc_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_backward_acc(const void* dy, const void* z, int64_t nvox, int32_t c, const double* acc,
                                      int32_t reps, const float* scale_shift, const float* mean_invstd,
                                      const float* gamma, int32_t act, float slope, float* dgamma, float* dbeta,
                                      float* dz, int32_t accumulate, void* dz_bf16, double* zero, int32_t zero_n,
                                      int32_t in_bf16, void* stream) {
  CG_CHECK_ARG(dy && z && acc && scale_shift && mean_invstd && gamma && (dz || dz_bf16),
               "cgan3d_bn_backward_acc: null pointer");
  CG_CHECK_ARG(reps > 0 && reps <= 64 && nvox > 1 && c >= 4 && c <= 128 && 256 % c == 0 && zero_n >= 0 &&
                   (zero || !zero_n),
               "cgan3d_bn_backward_acc: channels must divide 256 (4..128), reps 1..64");
  const long long n4 = (long long)nvox * c / 4;
  ::cg::launch(in_bf16 ? bn_bwd_apply_acc_kernel<true> : bn_bwd_apply_acc_kernel<false>, dim3(acc_pass_blocks(n4)),
               dim3(256), 0, (hipStream_t)stream, acc, (int)reps,
               (int)c, (double)nvox, gamma, mean_invstd, dgamma, dbeta, (int)accumulate, dy, z, n4, scale_shift, act,
               slope, dz, reinterpret_cast<__bf16*>(dz_bf16), zero, (int)zero_n);
  CG_LAUNCH_CHECK("bn_bwd_apply_acc_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_bn_backward_acc_fold(const void* padded, const void* z, int32_t n, int32_t d, int32_t h,
                                           int32_t w, int32_t c, int32_t pad, const double* acc, int32_t reps,
                                           const float* scale_shift, const float* mean_invstd, const float* gamma,
                                           int32_t act, float slope, float* dgamma, float* dbeta, float* dz,
                                           int32_t accumulate, void* dz_bf16, double* zero, int32_t zero_n,
                                           int32_t in_bf16, void* stream) {
  CG_CHECK_ARG(padded && z && acc && scale_shift && mean_invstd && gamma && (dz || dz_bf16),
               "cgan3d_bn_backward_acc_fold: null pointer");
  CG_CHECK_ARG(n > 0 && reps > 0 && reps <= 64 && c >= 4 && c <= 128 && 256 % c == 0 && pad >= 0 && d > 2 * pad &&
                   h > 2 * pad && w > 2 * pad && zero_n >= 0 && (zero || !zero_n),
               "cgan3d_bn_backward_acc_fold: channels must divide 256 (4..128), dims must exceed 2*pad, reps 1..64");
  const long long nvox = (long long)n * d * h * w;
  CG_CHECK_ARG(nvox > 1, "cgan3d_bn_backward_acc_fold: need more than one voxel");
  CG_CHECK_ARG((long long)n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * (c / 4) < (1LL << 31),
               "cgan3d_bn_backward_acc_fold: padded volume exceeds 32-bit float4 indexing");
  const long long n4 = nvox * c / 4;
  const long long rw = (long long)w * c / 8;  // 16-byte granules per row
  if (in_bf16 && c % 8 == 0 && rw <= 256 && (rw & (rw - 1)) == 0 && (long long)n * d <= 65535 &&
      (long long)n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * c * 2 < (1LL << 31)) {
#ifdef CGAN3D_PROBES
    const int fu = (g_probe & 64) ? 2 : 4;
#else
    const int fu = 4;
#endif
    const int lrw = __builtin_ctzll(rw), hpb = fu * (256 >> lrw);
    ::cg::launch(fu == 2 ? bn_bwd_fold_rows_kernel<2> : bn_bwd_fold_rows_kernel<4>, dim3((h + hpb - 1) / hpb, n * d), dim3(256), 0, (hipStream_t)stream,
                 (const __bf16*)padded, (const __bf16*)z, d, h, w, pad, c, lrw, __builtin_ctz(c / 8), scale_shift,
                 mean_invstd, act, slope, dz, reinterpret_cast<__bf16*>(dz_bf16), acc, (int)reps, (double)nvox, gamma,
                 dgamma, dbeta, (int)accumulate, zero, (int)zero_n,
                 (unsigned)((long long)n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * c * 2),
#ifdef CGAN3D_PROBES
                 g_probe
#else
                 0
#endif
    );
    CG_LAUNCH_CHECK("bn_bwd_fold_rows_kernel");
    return CGAN3D_OK;
  }
  ::cg::launch(in_bf16 ? bn_bwd_apply_fold_kernel<true> : bn_bwd_apply_fold_kernel<false>, dim3(acc_pass_blocks(n4, 4096)),
               dim3(256), 0, (hipStream_t)stream, padded, z, n, d,
               h, w, pad, c, scale_shift, mean_invstd, act, slope, (const float*)nullptr, dz,
               reinterpret_cast<__bf16*>(dz_bf16), acc, (int)reps, (double)nvox, gamma, dgamma, dbeta, (int)accumulate,
               zero, (int)zero_n);
  CG_LAUNCH_CHECK("bn_bwd_apply_fold_kernel");
  return CGAN3D_OK;
}
