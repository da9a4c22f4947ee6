// Loss reductions and their gradients for the G+D step (gfx950).
//
//  * Wasserstein critic/generator terms   — model/loss.py:74-80, Trainer.py:119-121,151
//  * WGAN gradient penalty                — model/utils.py:12-41 (lambda * mean_b (||g_b||-1)^2)
//  * ZNCC with the StableStd custom grad  — model/loss.py:11-41 (batch-global, 1e-6 / 1e-8 eps)
//  * masked HU-range loss                 — model/loss.py:44-71
//  * opt_hat = subopt - tanh(.) backward  — Trainer.py:170-171, generator.py:85
//
// Reductions accumulate per-block partials in fp64 and combine them in a single block, so no
// atomics and bit-reproducible results.  Loss values are written to a device array (no host
// sync); the Trainer reads them only on logging iterations, as the reference does.
#include "common.h"

namespace cg {

enum { L_D = 0, L_WD = 1, L_GP = 2, L_G = 3, L_SIM = 4, L_HU = 5, L_GFULL = 6 };

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// dlogits layout [real | fake | gp] (samples x per_sample)
__global__ __launch_bounds__(256) void critic_logits_kernel(const float* __restrict__ logits, int nr, int nf, int ng,
                                                            int ps, float gan_w, float* dl, float* losses) {
  __shared__ double red[4];
  double sr = 0.0, sf = 0.0;
  const long long er = (long long)nr * ps, ef = (long long)nf * ps, eg = (long long)ng * ps;
  for (long long i = threadIdx.x; i < er; i += blockDim.x) sr += logits[i];
  for (long long i = threadIdx.x; i < ef; i += blockDim.x) sf += logits[er + i];
  sr = block_sum_d(sr, red);
  sf = block_sum_d(sf, red);
  const float gr = -gan_w / (float)er, gf = gan_w / (float)ef;
  for (long long i = threadIdx.x; i < er; i += blockDim.x) dl[i] = gr;
  for (long long i = threadIdx.x; i < ef; i += blockDim.x) dl[er + i] = gf;
  for (long long i = threadIdx.x; i < eg; i += blockDim.x) dl[er + ef + i] = 1.f;
  if (threadIdx.x == 0) {
    const float wd = (float)(gan_w * (sf / ef - sr / er));
    losses[L_WD] = wd;
    losses[L_D] = wd;
    losses[L_GP] = 0.f;
  }
}

__global__ __launch_bounds__(256) void gen_logits_kernel(const float* __restrict__ logits, int n, float gan_w,
                                                         float* dl, float* losses) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += logits[i];
  s = block_sum_d(s, red);
  if (dl)
    for (int i = threadIdx.x; i < n; i += blockDim.x) dl[i] = -gan_w / (float)n;
  if (threadIdx.x == 0) {
    losses[L_G] = (float)(-gan_w * s / n);
    // the full generator loss, when the similarity / HU terms were computed first (beside the
    // critic update); cgan3d_generator_output_grad writes it again when it runs after this
    losses[L_GFULL] = losses[L_G] + losses[L_SIM] + losses[L_HU];
  }
}

// --- gradient penalty -------------------------------------------------------------------
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long long ps, int chunks, float* part) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const long long per = (ps + chunks - 1) / chunks;
  const long long beg = per * blockIdx.x, end = beg + per < ps ? beg + per : ps;
  double s = 0.0;
  for (long long i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const double v = g[(long long)b * ps + i];
    s += v * v;
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) part[(long long)b * chunks + blockIdx.x] = (float)s;
}

// Finalize folded into the scaling pass: every block combines the B x chunks partial sums itself
// (same order in every block, so every block holds the same coefficients); block 0 writes the loss.
// lg (optional): the critic's logits [real nr x lps | fake nf x lps | ...] — block 0 also computes the
// Wasserstein term (critic_logits_kernel's losses) so no separate launch sits on the step's path
__global__ __launch_bounds__(256) void gp_scale_kernel(const float* __restrict__ part, int B, int chunks,
                                                       float lambda_, float* losses, const float* __restrict__ g,
                                                       long long ps, long long total, float* out,
                                                       const float* __restrict__ lg, int nr, int nf, int lps,
                                                       float gan_w, float* zero, long long zero_n) {
  __shared__ double red[4];
  __shared__ float coef[1024];
  // the critic's gradient arena zeroed here (optimizer_D.zero_grad) instead of in a fill launch
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += (long long)gridDim.x * blockDim.x)
    zero[i] = 0.f;
  double acc = 0.0;
  if (chunks >= 64 && B <= 8) {  // many partials, few samples: every sample's sum in one pass (all
                                  // samples' loads in flight), one block-level reduction round
    __shared__ double wred[8][4];
    double ss[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) ss[b] = 0.0;
    for (int c = threadIdx.x; c < chunks; c += blockDim.x) {
      // unconditional loads (a clamped sample for b >= B, masked after): a load under `if (b < B)`
      // waited for its own round trip
      float v[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) v[b] = part[(long long)min(b, B - 1) * chunks + c];
#pragma unroll
      for (int b = 0; b < 8; ++b) ss[b] += b < B ? (double)v[b] : 0.0;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b >= B) break;
      const double w = wave_sum_d(ss[b]);
      if ((threadIdx.x & 63) == 0) wred[b][threadIdx.x >> 6] = w;
    }
    __syncthreads();
    if (threadIdx.x < B) {
      const int b = threadIdx.x;
      const double t = wred[b][0] + wred[b][1] + wred[b][2] + wred[b][3];
      const double nrm = sqrt(t);
      acc = (nrm - 1.0) * (nrm - 1.0);
      coef[b] = nrm > 0.0 ? (float)(lambda_ * 2.0 / B * (nrm - 1.0) / nrm) : 0.f;
    }
  } else if (chunks >= 64) {  // many partials per sample: the block sums each sample's together
    for (int b = 0; b < B; ++b) {
      double ss = 0.0;
      for (int c = threadIdx.x; c < chunks; c += blockDim.x) ss += part[(long long)b * chunks + c];
      ss = block_sum_d(ss, red);
      if (threadIdx.x == 0) {
        const double nrm = sqrt(ss);
        acc += (nrm - 1.0) * (nrm - 1.0);
        coef[b] = nrm > 0.0 ? (float)(lambda_ * 2.0 / B * (nrm - 1.0) / nrm) : 0.f;
      }
    }
  } else {
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
      double ss = 0.0;
      for (int c = 0; c < chunks; ++c) ss += part[(long long)b * chunks + c];
      const double nrm = sqrt(ss);
      acc += (nrm - 1.0) * (nrm - 1.0);
      // d/dg_b of lambda*mean((||g_b||-1)^2) = lambda * 2/B * (||g_b||-1) * g_b/||g_b||  (0 at ||g_b||=0)
      coef[b] = nrm > 0.0 ? (float)(lambda_ * 2.0 / B * (nrm - 1.0) / nrm) : 0.f;
    }
  }
  acc = block_sum_d(acc, red);  // (its barriers also publish coef)
  float wd = 0.f;
  if (lg && blockIdx.x == 0) {  // as critic_logits_kernel
    const long long er = (long long)nr * lps, ef = (long long)nf * lps;
    double sr = 0.0, sf = 0.0;
    for (long long i = threadIdx.x; i < er; i += blockDim.x) sr += lg[i];
    for (long long i = threadIdx.x; i < ef; i += blockDim.x) sf += lg[er + i];
    sr = block_sum_d(sr, red);
    sf = block_sum_d(sf, red);
    wd = (float)(gan_w * (sf / ef - sr / er));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float gp = (float)(lambda_ * acc / B);
    if (lg) losses[L_WD] = wd;
    losses[L_GP] = gp;
    losses[L_D] = (lg ? wd : losses[L_WD]) + gp;
  }
  if ((ps & 3) == 0 && total < (1LL << 32) && !(((uintptr_t)g | (uintptr_t)out) & 15)) {  // float4 with 32-bit index math (no 64-bit divide per element)
    const unsigned n4 = (unsigned)(total >> 2), ps4 = (unsigned)(ps >> 2);
    const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
    f32x4* o4 = reinterpret_cast<f32x4*>(out);
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) o4[i] = coef[i / ps4] * g4[i];
  } else {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
      out[i] = coef[i / ps] * g[i];
  }
}

// --- generator losses ---------------------------------------------------------------------
// One reduction pass: raw fp64 sums of s, t, s^2, t^2, s*t (every product of two fp32 values is exact
// in fp64, so the centred moments E[st] - E[s]E[t] lose nothing that matters: |s|, |t| <= a few),
// the mask count and the HU penalty sum; per-block partials part[b * 8 + q].
__global__ __launch_bounds__(256) void gen_pass1_kernel(const float* __restrict__ s, const float* __restrict__ t,
                                                        const uint8_t* __restrict__ m, long long n, float lo, float hi,
                                                        double* part) {
  __shared__ double red[4];
  double a[7] = {0, 0, 0, 0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const double x = s[i], y = t[i];
    a[0] += x;
    a[1] += y;
    a[2] += x * x;
    a[3] += y * y;
    a[4] += x * y;
    if (m[i]) {
      const float xf = s[i];
      const float lb = fminf(xf, lo) - lo, ub = fmaxf(xf, hi) - hi;
      a[5] += 1.0;
      a[6] += (double)(lb * lb + ub * ub);
    }
  }
#pragma unroll
  for (int q = 0; q < 7; ++q) a[q] = block_sum_d(a[q], red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) part[blockIdx.x * 8 + q] = a[q];
}

// the nblk x 8 partials combined in a fixed order (identical in every block that calls it)
__device__ __forceinline__ void gen_combine(const double* __restrict__ part, int nblk, double* red, double (&a)[7]) {
  for (int q = 0; q < 7; ++q) a[q] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x)
    for (int q = 0; q < 7; ++q) a[q] += part[b * 8 + q];
  for (int q = 0; q < 7; ++q) a[q] = block_sum_d(a[q], red);
}

// dz_last = d(opt_hat)/d(z) chain: opt_hat = subopt - tanh(z)  =>  dz = -dL/dopt_hat * (1 - att^2).
// The reduction's finalize folded in: every block combines the partials into the losses and the
// gradient coefficients A (w coef), Bc (u coef), w_mean, hu_scale; block 0 writes the losses.
__global__ __launch_bounds__(256) void gen_grad_kernel(const float* __restrict__ s, const float* __restrict__ t,
                                                       const float* __restrict__ att, const uint8_t* __restrict__ m,
                                                       const float* __restrict__ dcrit, long long n, float lo, float hi,
                                                       const double* __restrict__ part, int nblk, float sim_w,
                                                       float hu_w, float* losses, float* dz) {
  __shared__ double red[4];
  double a[7];
  gen_combine(part, nblk, red, a);
  const double nn = (double)n;
  const double smd = a[0] / nn, tmd = a[1] / nn;
  const double suw = a[4] - nn * smd * tmd, suu = fmax(a[2] - nn * smd * smd, 0.0), sww = fmax(a[3] - nn * tmd * tmd, 0.0);
  const double cc = suw / nn;
  const double ss = sqrt(suu / (nn - 1.0)), st = sqrt(sww / (nn - 1.0));  // torch.std (unbiased)
  const double D = ss * st + 1e-8;
  const float sm = (float)smd, tm = (float)tmd;
  // dL/ds_j = -(1/D) (w_j - mean w)/n  +  cc*st/D^2 * 2/(n-1) * (s_j - s_mean)/(2 ss + 1e-6), with
  // w_j = t_j - tm in fp32: mean w = mean t - tm exactly
  const float A = (float)(sim_w * (-1.0 / (D * nn)));
  const float Bc = (float)(sim_w * (cc * st / (D * D)) * (2.0 / (nn - 1.0)) / (2.0 * ss + 1e-6));
  const float wm = (float)(tmd - (double)tm), hs = (float)(hu_w * 2.0 / (a[5] + 1e-8));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const double zncc = -cc / D, hu = a[6] / (a[5] + 1e-8);
    losses[L_SIM] = (float)(sim_w * zncc);
    losses[L_HU] = (float)(hu_w * hu);
    losses[L_GFULL] = losses[L_G] + (float)(sim_w * zncc) + (float)(hu_w * hu);
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float x = s[i];
    float g = A * ((t[i] - tm) - wm) + Bc * (x - sm);
    if (m[i]) g += hs * ((fminf(x, lo) - lo) + (fmaxf(x, hi) - hi));
    if (dcrit) g += dcrit[i];
    const float at = att[i];
    dz[i] = -g * (1.f - at * at);
  }
}

static int red_blocks(long long n) {
  long long b = (n + 2047) / 2048;
  if (b > 512) b = 512;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace cg

using namespace cg;

extern "C" int64_t cgan3d_loss_ws_floats(int64_t n) {
  // generator losses: 512 x 8 partial doubles; GP: b x (<=64 chunks) floats, b <= 1024
  (void)n;
  return 2 * (2 * 512 * 4 + 8) + 65 * 1024;
}

extern "C" int cgan3d_critic_logits_grad(const float* logits, int32_t n_real, int32_t n_fake, int32_t n_gp,
                                         int32_t per_sample, float gan_w, float* dlogits, float* losses,
                                         void* stream) {
  CG_CHECK_ARG(logits && dlogits && losses, "cgan3d_critic_logits_grad: null pointer");
  CG_CHECK_ARG(n_real > 0 && n_fake > 0 && n_gp >= 0 && per_sample > 0, "cgan3d_critic_logits_grad: bad sizes");
  ::cg::launch(critic_logits_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, n_real, n_fake, n_gp,
                     per_sample, gan_w, dlogits, losses);
  CG_LAUNCH_CHECK("critic_logits_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_generator_logits_grad(const float* logits, int32_t n, float gan_w, float* dlogits, float* losses,
                                            void* stream) {
  CG_CHECK_ARG(logits && losses && n > 0, "cgan3d_generator_logits_grad: bad args");
  ::cg::launch(gen_logits_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, n, gan_w, dlogits, losses);
  CG_LAUNCH_CHECK("gen_logits_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_gradient_penalty(const float* grad, int32_t b, int64_t per_sample, float lambda_,
                                       float* gamma_out, float* losses, float* ws, void* stream) {
  CG_CHECK_ARG(grad && gamma_out && losses && ws, "cgan3d_gradient_penalty: null pointer");
  CG_CHECK_ARG(b > 0 && b <= 1024 && per_sample > 0, "cgan3d_gradient_penalty: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  int chunks = (int)((per_sample + 8191) / 8192);
  if (chunks > 64) chunks = 64;
  float* part = ws;
  ::cg::launch(sumsq_kernel, dim3(chunks, b), dim3(256), 0, s, grad, (long long)per_sample, chunks, part);
  CG_LAUNCH_CHECK("sumsq_kernel");
  const long long total = (long long)b * per_sample;
  int blocks = (int)std::min<long long>((total + 255) / 256, 1024);
  ::cg::launch(gp_scale_kernel, dim3(blocks), dim3(256), 0, s, part, b, chunks, lambda_, losses, grad,
               (long long)per_sample, total, gamma_out, (const float*)nullptr, 0, 0, 0, 0.f, (float*)nullptr, 0LL);
  CG_LAUNCH_CHECK("gp_scale_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_gradient_penalty_part(const float* grad, const float* part, int32_t b, int32_t chunks,
                                            int64_t per_sample, float lambda_, float* gamma_out, float* losses,
                                            const float* logits, int32_t n_real, int32_t n_fake, int32_t logit_ps,
                                            float gan_w, float* zero, int64_t zero_n, void* stream) {
  CG_CHECK_ARG(grad && part && gamma_out && losses, "cgan3d_gradient_penalty_part: null pointer");
  CG_CHECK_ARG(zero_n >= 0 && (zero || !zero_n), "cgan3d_gradient_penalty_part: zero range");
  CG_CHECK_ARG(b > 0 && b <= 1024 && chunks > 0 && per_sample > 0, "cgan3d_gradient_penalty_part: bad sizes");
  CG_CHECK_ARG(!logits || (n_real > 0 && n_fake > 0 && logit_ps > 0), "cgan3d_gradient_penalty_part: bad logit sizes");
  const long long total = (long long)b * per_sample;
  // every block sums the b x chunks partials itself: fewer, longer blocks when there are many
  int blocks = (int)std::min<long long>((total + 255) / 256, chunks >= 64 ? 256 : 1024);
  ::cg::launch(gp_scale_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, part, b, chunks, lambda_, losses, grad,
               (long long)per_sample, total, gamma_out, logits, n_real, n_fake, logit_ps, gan_w, zero, (long long)zero_n);
  CG_LAUNCH_CHECK("gp_scale_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_generator_output_grad(const float* opt_hat, const float* subopt, const float* att,
                                            const uint8_t* mask, const float* d_critic, int64_t n, float lo, float hi,
                                            float sim_w, float hu_w, float* dz_last, float* losses, float* ws,
                                            void* stream) {
  CG_CHECK_ARG(opt_hat && subopt && att && mask && dz_last && losses && ws, "cgan3d_generator_output_grad: null");
  CG_CHECK_ARG(n > 1, "cgan3d_generator_output_grad: need n > 1");
  CG_CHECK_ARG(((uintptr_t)ws & 7) == 0, "cgan3d_generator_output_grad: workspace must be 8-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  const int nblk = red_blocks(n);
  ::cg::launch(gen_pass1_kernel, dim3(nblk), dim3(256), 0, s, opt_hat, subopt, mask, (long long)n, lo, hi, part);
  CG_LAUNCH_CHECK("gen_pass1_kernel");
  int blocks = (int)std::min<long long>((n + 255) / 256, 512);
  ::cg::launch(gen_grad_kernel, dim3(blocks), dim3(256), 0, s, opt_hat, subopt, att, mask, d_critic,
                     (long long)n, lo, hi, part, nblk, sim_w, hu_w, losses, dz_last);
  CG_LAUNCH_CHECK("gen_grad_kernel");
  return CGAN3D_OK;
}
