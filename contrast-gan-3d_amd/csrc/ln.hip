// LayerNorm critic of the gp_layernorm conf (experiments/gp_layernorm.py:9-11; model/blocks.py:40-45):
// every middle ConvBlock normalises its conv output per sample over (C, D, H, W), no affine
// parameters, eps 1e-5, then LeakyReLU.  In NDHWC a sample's C*D*H*W values are one contiguous run
// of L floats, so every operation here is "per-sample sums, then an elementwise pass":
//
//   cgan3d_ln_reduce — grid (chunks, n): two fp64 sums per (sample, chunk) of a mode's quantities
//                      into a partial array [n][chunks][2];
//   cgan3d_ln_apply  — grid (blocks, n): every block first combines its sample's partials (fixed
//                      order, so every block holds the same per-sample constants), then the
//                      elementwise formula of the mode.
//
// With x^ = (z - mu) * r (r = 1/sqrt(var + eps), biased var) and m = LeakyReLU'(x^):
//   forward     a = lrelu(x^)                                     sums (z, z^2)
//   backward    rho = m*da;  dz = r*(rho - <rho> - x^ <rho x^>)     sums (rho, rho x^)
//   tangent     (forward-mode along the GP direction, model/utils.py:34-39 differentiated):
//               adot = m * r*(zdot - <zdot> - x^ <zdot x^>)          sums (zdot, zdot x^)
//   sigma seed  sum rho * udot = sum da * adot                      sums (da adot, -)
//   adjoint     the primal adjoint the tangent injects (reverse-over-forward of the penalty):
//               xbar = m*abar - r*(c rho + zdot q),  c = <zdot x^>, q = <rho x^>
//               zbar = r*(xbar - <xbar> - x^ <xbar x^>) + sbar x^ / L,  sbar = -r * sum rho udot
//                                                                    sums (xbar, xbar x^)
// (<.> = mean over the sample).  DESIGN.md §3.6 derives the penalty gradient from these.
#include "common.h"

namespace cg {

struct LnArgs {
  long long L;       // elements per sample (C * D * H * W)
  int chunks;        // partial sums per sample
  int mode;
  float slope, eps;
  const float* z;     // conv output (pre-norm)
  const float* da;    // dL/da (the conv input-grad of the next layer)
  const float* zdot;  // tangent conv output
  const float* adot;  // tangent activation
  const float* abar;  // primal adjoint of the activation (NULL: zero)
  const double* p_stats;  // partials (sum z, sum z^2)
  const double* p_bwd;    // partials (sum rho, sum rho x^)
  const double* p_jvp;    // partials (sum zdot, sum zdot x^)
  const double* p_sig;    // partials (sum da adot, -)
  const double* p_adj;    // partials (sum xbar, sum xbar x^)
  double* part;           // reduce output [n][chunks][2]
  float* out;             // apply output
};

// the sample's two sums from its `chunks` partials (sequential, identical in every block)
__device__ __forceinline__ void ln_sums(const double* __restrict__ p, int b, int chunks, double* s0, double* s1) {
  double a0 = 0.0, a1 = 0.0;
  const double* q = p + (long long)b * chunks * 2;
  for (int c = 0; c < chunks; ++c) {
    a0 += q[2 * c];
    a1 += q[2 * c + 1];
  }
  *s0 = a0;
  *s1 = a1;
}

struct LnConst {
  float mu, r, invL;
  float k0, k1;  // mode constants (means of the reduced quantities)
  float c, q, sbar;
};

// per-sample constants: mean / rstd always; the adjoint's c, q; and, for the elementwise pass
// (apply), the means of the mode's own reduced quantities
__device__ __forceinline__ LnConst ln_consts(const LnArgs& a, int b, bool apply) {
  LnConst k{};
  const double L = (double)a.L;
  double s0, s1;
  ln_sums(a.p_stats, b, a.chunks, &s0, &s1);
  const double mu = s0 / L;
  double var = s1 / L - mu * mu;
  var = var > 0.0 ? var : 0.0;
  k.mu = (float)mu;
  k.r = (float)(1.0 / sqrt(var + (double)a.eps));
  k.invL = (float)(1.0 / L);
  if (a.mode == CGAN3D_LN_BWD && apply) {
    ln_sums(a.p_bwd, b, a.chunks, &s0, &s1);
    k.k0 = (float)(s0 / L); k.k1 = (float)(s1 / L);
  } else if (a.mode == CGAN3D_LN_JVP && apply) {
    ln_sums(a.p_jvp, b, a.chunks, &s0, &s1);
    k.k0 = (float)(s0 / L); k.k1 = (float)(s1 / L);
  } else if (a.mode == CGAN3D_LN_ADJ) {
    ln_sums(a.p_jvp, b, a.chunks, &s0, &s1);
    k.c = (float)(s1 / L);
    ln_sums(a.p_bwd, b, a.chunks, &s0, &s1);
    k.q = (float)(s1 / L);
    if (apply) {
      ln_sums(a.p_adj, b, a.chunks, &s0, &s1);
      k.k0 = (float)(s0 / L); k.k1 = (float)(s1 / L);
      ln_sums(a.p_sig, b, a.chunks, &s0, &s1);
      k.sbar = -k.r * (float)s0;
    }
  }
  return k;
}

// xbar of the adjoint mode at element i of sample b (abar may be NULL)
__device__ __forceinline__ float ln_xbar(const LnArgs& a, const LnConst& k, long long i, float xh, float m) {
  const float rho = m * a.da[i];
  const float ab = a.abar ? a.abar[i] : 0.f;
  return m * ab - k.r * (k.c * rho + a.zdot[i] * k.q);
}

__global__ __launch_bounds__(256) void ln_reduce_kernel(LnArgs a) {
  __shared__ double red[2][4];
  const int b = blockIdx.y, tid = threadIdx.x;
  const long long base = (long long)b * a.L;
  const long long per = (a.L + a.chunks - 1) / a.chunks;
  const long long beg = per * blockIdx.x, end = beg + per < a.L ? beg + per : a.L;
  LnConst k{};
  if (a.mode != CGAN3D_LN_STATS) k = ln_consts(a, b, false);
  double s0 = 0.0, s1 = 0.0;
  for (long long j = beg + tid; j < end; j += blockDim.x) {
    const long long i = base + j;
    const float z = a.z[i];
    if (a.mode == CGAN3D_LN_STATS) {
      s0 += (double)z;
      s1 += (double)z * (double)z;
      continue;
    }
    const float xh = (z - k.mu) * k.r;
    const float m = xh > 0.f ? 1.f : a.slope;
    if (a.mode == CGAN3D_LN_BWD) {
      const float rho = m * a.da[i];
      s0 += (double)rho;
      s1 += (double)(rho * xh);
    } else if (a.mode == CGAN3D_LN_JVP) {
      const float zd = a.zdot[i];
      s0 += (double)zd;
      s1 += (double)(zd * xh);
    } else if (a.mode == CGAN3D_LN_SIG) {
      s0 += (double)(a.da[i] * a.adot[i]);
    } else {  // ADJ
      const float xb = ln_xbar(a, k, i, xh, m);
      s0 += (double)xb;
      s1 += (double)(xb * xh);
    }
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  if ((tid & 63) == 0) { red[0][tid >> 6] = s0; red[1][tid >> 6] = s1; }
  __syncthreads();
  if (tid == 0) {
    double* o = a.part + ((long long)b * a.chunks + blockIdx.x) * 2;
    o[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    o[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ __launch_bounds__(256) void ln_apply_kernel(LnArgs a) {
  const int b = blockIdx.y;
  const LnConst k = ln_consts(a, b, true);
  const long long base = (long long)b * a.L;
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < a.L; j += (long long)gridDim.x * blockDim.x) {
    const long long i = base + j;
    const float xh = (a.z[i] - k.mu) * k.r;
    const float m = xh > 0.f ? 1.f : a.slope;
    float v;
    if (a.mode == CGAN3D_LN_STATS) {
      v = xh * m;  // LeakyReLU(x^)
    } else if (a.mode == CGAN3D_LN_BWD) {
      const float rho = m * a.da[i];
      v = k.r * (rho - k.k0 - xh * k.k1);
    } else if (a.mode == CGAN3D_LN_JVP) {
      v = m * k.r * (a.zdot[i] - k.k0 - xh * k.k1);
    } else {  // ADJ
      const float xb = ln_xbar(a, k, i, xh, m);
      v = k.r * (xb - k.k0 - xh * k.k1) + k.sbar * xh * k.invL;
    }
    a.out[i] = v;
  }
}

static int ln_chunks(long long L) {
  long long c = (L + 4095) / 4096;
  return (int)std::max(1LL, std::min(c, 64LL));
}

static int ln_check(const cgan3d_ln_args* p, const char* who) {
  if (!p || p->n <= 0 || p->L <= 0 || p->mode < 0 || p->mode > CGAN3D_LN_ADJ || !p->z || !p->p_stats) {
    set_error("%s: bad args (need n > 0, L > 0, a mode, z and the statistics partials)", who);
    return CGAN3D_EINVAL;
  }
  const int m = p->mode;
  const bool ok = (m != CGAN3D_LN_BWD || p->da) && (m != CGAN3D_LN_JVP || p->zdot) &&
                  (m != CGAN3D_LN_SIG || (p->da && p->adot)) &&
                  (m != CGAN3D_LN_ADJ || (p->da && p->zdot && p->p_bwd && p->p_jvp));
  if (!ok) {
    set_error("%s: mode %d misses an operand", who, m);
    return CGAN3D_EINVAL;
  }
  return CGAN3D_OK;
}

static LnArgs ln_args(const cgan3d_ln_args* p) {
  LnArgs a;
  a.L = p->L; a.chunks = ln_chunks(p->L); a.mode = p->mode; a.slope = p->slope; a.eps = p->eps;
  a.z = p->z; a.da = p->da; a.zdot = p->zdot; a.adot = p->adot; a.abar = p->abar;
  a.p_stats = p->p_stats; a.p_bwd = p->p_bwd; a.p_jvp = p->p_jvp; a.p_sig = p->p_sig; a.p_adj = p->p_adj;
  a.part = nullptr; a.out = nullptr;
  return a;
}

}  // namespace cg

using namespace cg;

extern "C" int64_t cgan3d_ln_partial_doubles(int32_t n, int64_t L) { return (int64_t)n * ln_chunks(L) * 2; }

extern "C" int cgan3d_ln_reduce(const cgan3d_ln_args* p, double* part, void* stream) {
  if (int rc = ln_check(p, "cgan3d_ln_reduce")) return rc;
  CG_CHECK_ARG(part != nullptr, "cgan3d_ln_reduce: null partials");
  LnArgs a = ln_args(p);
  a.part = part;
  ::cg::launch(ln_reduce_kernel, dim3(a.chunks, p->n), dim3(256), 0, (hipStream_t)stream, a);
  CG_LAUNCH_CHECK("ln_reduce_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_ln_apply(const cgan3d_ln_args* p, float* out, void* stream) {
  if (int rc = ln_check(p, "cgan3d_ln_apply")) return rc;
  CG_CHECK_ARG(out != nullptr, "cgan3d_ln_apply: null output");
  LnArgs a = ln_args(p);
  CG_CHECK_ARG(a.mode != CGAN3D_LN_BWD || a.p_bwd, "cgan3d_ln_apply: backward needs its partials");
  CG_CHECK_ARG(a.mode != CGAN3D_LN_JVP || a.p_jvp, "cgan3d_ln_apply: tangent needs its partials");
  CG_CHECK_ARG(a.mode != CGAN3D_LN_SIG, "cgan3d_ln_apply: the sigma seed mode only reduces");
  CG_CHECK_ARG(a.mode != CGAN3D_LN_ADJ || (a.p_adj && a.p_sig), "cgan3d_ln_apply: adjoint needs its partials");
  a.out = out;
  const long long blocks = std::max(1LL, std::min((a.L + 2047) / 2048, 256LL));
  ::cg::launch(ln_apply_kernel, dim3((unsigned)blocks, p->n), dim3(256), 0, (hipStream_t)stream, a);
  CG_LAUNCH_CHECK("ln_apply_kernel");
  return CGAN3D_OK;
}
