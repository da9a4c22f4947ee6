// Generator first / last convolutions: k = 7, stride 1, one side single-channel (fp32 VALU).
//
// model/generator.py:31-38 (first: reflect-pad 3, Conv3d 1 -> C, no bias, BatchNorm follows) and
// generator.py:78-85 (last: reflect-pad 3, Conv3d C -> 1 with bias, tanh; Trainer.py:171 opt_hat =
// subopt - tanh(.)).  These two convs are 37 % of the generator's forward FLOPs, and with one
// operand single-channel an MFMA tile wastes 15/16 of its columns (SURVEY.md §7 hard part iii),
// so they get register-blocked direct kernels instead:
//
//  * n2w  (1 -> C):  out[v, c]  = sum_t x[src(v,t)] * W[c, t]         first fwd; last input-grad
//  * w2n  (C -> 1):  out[v]     = sum_t,c x[src(v,t), c] * W[c, t]     last fwd (+bias, tanh, opt_hat)
//  * wg_w2n:         dW[c, t]   = sum_v x[src(v,t), c] * g[v]          last weight-grad
//  * wg_n2w:         dW[c, t]   = sum_v x[src(v,t)] * g[v, c]          first weight-grad
//
// Block = 4 x 8 x 32 output voxels (a 10 x 14 x 38 input halo in LDS, rows padded to 40 floats so
// each thread's 10-voxel row window is two b128 + one b64 read); thread = 4 consecutive voxels
// along W.  Weights live in LDS and are read as broadcast b128.  The last conv's input-grad is the
// same n2w kernel with the taps flipped over the zero-padded grid (folded by cgan3d_reflect_fold).
#include "k7.h"

namespace cg {

// halo of a single-channel volume, or of channels [c0, c0+CC) of a C-channel volume ([cc][halo])
template <int C, int CC>
__device__ __forceinline__ void k7_load_halo(const K7Args& a, const float* __restrict__ x, float* xs, int n, int d0,
                                             int h0, int w0, int c0) {
  for (int i = threadIdx.x; i < HD * HH * HWD; i += blockDim.x) {
    const int hw = i % HWD, r = i / HWD, hh = r % HH, hd = r / HH;
    const int id = k7_src(d0 + hd - a.P, a.di, a.reflect);
    const int ih = k7_src(h0 + hh - a.P, a.hi, a.reflect);
    const int iw = k7_src(w0 + hw - a.P, a.wi, a.reflect);
    const int o = (hd * HH + hh) * HWP + hw;
    if ((id | ih | iw) >= 0) {
      const long long v = ((long long)(n * a.di + id) * a.hi + ih) * a.wi + iw;
#pragma unroll
      for (int cc = 0; cc < CC; ++cc) xs[cc * HALO + o] = x[v * C + c0 + cc];
    } else {
#pragma unroll
      for (int cc = 0; cc < CC; ++cc) xs[cc * HALO + o] = 0.f;
    }
  }
}

__device__ __forceinline__ void k7_row(const float* xs, float (&xr)[10]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(xs);
  const f32x4 b = *reinterpret_cast<const f32x4*>(xs + 4);
  const float2 c = *reinterpret_cast<const float2*>(xs + 8);
  xr[0] = a[0]; xr[1] = a[1]; xr[2] = a[2]; xr[3] = a[3];
  xr[4] = b[0]; xr[5] = b[1]; xr[6] = b[2]; xr[7] = b[3];
  xr[8] = c.x; xr[9] = c.y;
}

// ------------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void k7_n2w_kernel(K7Args a, const float* __restrict__ x, const float* __restrict__ w,
                                                     float* __restrict__ y, float* stats, float* bn_part) {
  __shared__ __attribute__((aligned(16))) float xs[HALO];
  __shared__ __attribute__((aligned(16))) float ws[KT7 * C];  // [t][c]
  const int tid = threadIdx.x;
  int n, d0, h0, w0;
  k7_tile(a, blockIdx.x, &n, &d0, &h0, &w0);
  for (int i = tid; i < KT7 * C; i += 256) {
    const int t = i / C, c = i - t * C;
    ws[i] = w[(long long)c * a.wc + (a.flip ? KT7 - 1 - t : t)];
  }
  k7_load_halo<1, 1>(a, x, xs, n, d0, h0, w0, 0);
  __syncthreads();
  const int d = tid >> 6, h = (tid >> 3) & 7, wq = (tid & 7) * 4;
  float acc[C][4];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[c][j] = 0.f;
  for (int td = 0; td < K7; ++td) {
    for (int th = 0; th < K7; ++th) {
      float xr[10];
      k7_row(&xs[((d + td) * HH + (h + th)) * HWP + wq], xr);
      const float* wr = &ws[(td * K7 + th) * K7 * C];
#pragma unroll
      for (int tw = 0; tw < K7; ++tw) {
#pragma unroll
        for (int c4 = 0; c4 < C / 4; ++c4) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + tw * C + 4 * c4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[4 * c4 + e][j] = fmaf(xr[j + tw], wv[e], acc[4 * c4 + e][j]);
        }
      }
    }
  }
  const int od = d0 + d, oh = h0 + h;
  bool valid[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ow = w0 + wq + j;
    valid[j] = od < a.do_ && oh < a.ho && ow < a.wo;
    if (valid[j]) {
      float* yp = y + (((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow) * C;
#pragma unroll
      for (int c4 = 0; c4 < C / 4; ++c4)
        *reinterpret_cast<f32x4*>(yp + 4 * c4) =
            f32x4{acc[4 * c4][j], acc[4 * c4 + 1][j], acc[4 * c4 + 2][j], acc[4 * c4 + 3][j]};
    }
  }
  if (stats || bn_part) {  // per-block BatchNorm partials (sum, M2, count): block-major, or slab
    __syncthreads();
    float* red = xs;  // [256][C] fits in the halo buffer (C <= 16)
    __shared__ float bmean[C];
    int cnt = 0;
    {
      const int vd = min(TD, a.do_ - d0), vh = min(TH, a.ho - h0), vw = min(TW, a.wo - w0);
      cnt = vd * vh * vw;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += valid[j] ? acc[c][j] : 0.f;
      red[tid * C + c] = s;
    }
    __syncthreads();
    if (tid < C) {
      double S = 0.0;
      for (int k = 0; k < 256; ++k) S += red[k * C + tid];
      bmean[tid] = (float)(S / cnt);
      if (stats) stats[(long long)blockIdx.x * (2 * C + 1) + tid] = (float)S;
      else bn_part[(long long)tid * gridDim.x + blockIdx.x] = (float)S;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float q = 0.f;
      const float m = bmean[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float dv = valid[j] ? acc[c][j] - m : 0.f;
        q += dv * dv;
      }
      red[tid * C + c] = q;
    }
    __syncthreads();
    if (tid < C) {
      double Q = 0.0;
      for (int k = 0; k < 256; ++k) Q += red[k * C + tid];
      if (stats) stats[(long long)blockIdx.x * (2 * C + 1) + C + tid] = (float)Q;
      else bn_part[(long long)(C + tid) * gridDim.x + blockIdx.x] = (float)Q;
    }
    if (tid == 0) {
      if (stats) stats[(long long)blockIdx.x * (2 * C + 1) + 2 * C] = (float)cnt;
      else bn_part[(long long)2 * C * gridDim.x + blockIdx.x] = (float)cnt;
    }
  }
}

// ------------------------------------------------------------------------------------------
template <int C, int CC>
__global__ __launch_bounds__(256) void k7_w2n_kernel(K7Args a, const float* __restrict__ x, const float* __restrict__ w,
                                                     float* __restrict__ y, const float* __restrict__ bias, int act,
                                                     const float* __restrict__ minuend, float* __restrict__ out2) {
  __shared__ __attribute__((aligned(16))) float xs[CC * HALO];
  __shared__ __attribute__((aligned(16))) float ws[C * 49 * 8];  // [c][td][th][tw padded to 8]
  const int tid = threadIdx.x;
  int n, d0, h0, w0;
  k7_tile(a, blockIdx.x, &n, &d0, &h0, &w0);
  for (int i = tid; i < C * 49 * 8; i += 256) {
    const int tw = i & 7, r = i >> 3, c = r / 49, tdh = r - c * 49;
    ws[i] = tw < K7 ? w[(long long)c * a.wc + tdh * K7 + tw] : 0.f;
  }
  const int d = tid >> 6, h = (tid >> 3) & 7, wq = (tid & 7) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < C; c0 += CC) {
    __syncthreads();
    k7_load_halo<C, CC>(a, x, xs, n, d0, h0, w0, c0);
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < CC; ++cc) {
      for (int td = 0; td < K7; ++td) {
#pragma unroll
        for (int th = 0; th < K7; ++th) {
          float xr[10];
          k7_row(&xs[cc * HALO + ((d + td) * HH + (h + th)) * HWP + wq], xr);
          const float* wr = &ws[((c0 + cc) * 49 + td * K7 + th) * 8];
          const f32x4 wa = *reinterpret_cast<const f32x4*>(wr);
          const f32x4 wb = *reinterpret_cast<const f32x4*>(wr + 4);
          const float wt[7] = {wa[0], wa[1], wa[2], wa[3], wb[0], wb[1], wb[2]};
#pragma unroll
          for (int tw = 0; tw < K7; ++tw)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = fmaf(xr[j + tw], wt[tw], acc[j]);
        }
      }
    }
  }
  const int od = d0 + d, oh = h0 + h;
  const float b = bias ? bias[0] : 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ow = w0 + wq + j;
    if (od < a.do_ && oh < a.ho && ow < a.wo) {
      const long long o = ((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow;
      float v = acc[j] + b;
      if (act == CGAN3D_ACT_TANH) v = tanhf(v);
      y[o] = v;
      if (out2) out2[o] = minuend[o] - v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// dW[c, t] += sum_v x[src(v,t), c] * g[v]   (x: C channels, g: one channel on the output grid)
template <int C, int CC>
__global__ __launch_bounds__(256) void k7_wg_w2n_kernel(K7Args a, const float* __restrict__ x,
                                                        const float* __restrict__ g, float* dw) {
  __shared__ __attribute__((aligned(16))) float xs[CC * HALO];
  __shared__ __attribute__((aligned(16))) float gs[TD * TH * TW];
  const int tid = threadIdx.x;
  int n, d0, h0, w0;
  k7_tile(a, blockIdx.x / (C / CC), &n, &d0, &h0, &w0);
  const int c0 = (blockIdx.x % (C / CC)) * CC;
  k7_load_halo<C, CC>(a, x, xs, n, d0, h0, w0, c0);
  for (int i = tid; i < TD * TH * TW; i += 256) {
    const int ww = i % TW, r = i / TW, hh = r % TH, dd = r / TH;
    const int od = d0 + dd, oh = h0 + hh, ow = w0 + ww;
    gs[i] = (od < a.do_ && oh < a.ho && ow < a.wo) ? g[((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow] : 0.f;
  }
  __syncthreads();
  // thread -> (row half, channel, td, th); 2 * CC * 49 <= 256 busy threads
  const int half = tid / (CC * 49), rem = tid - half * CC * 49;
  const int cc = rem / 49, tdh = rem - cc * 49, td = tdh / K7, th = tdh - td * K7;
  float acc[K7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (half < 2) {
    for (int row = half; row < TD * TH; row += 2) {
      const int dd = row / TH, hh = row - dd * TH;
      const float* xrow = &xs[cc * HALO + ((dd + td) * HH + (hh + th)) * HWP];
      const float* grow = &gs[row * TW];
#pragma unroll
      for (int w4 = 0; w4 < TW; w4 += 4) {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(grow + w4);
        float xr[10];
        k7_row(xrow + w4, xr);
#pragma unroll
        for (int tw = 0; tw < K7; ++tw)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[tw] = fmaf(xr[j + tw], gv[j], acc[tw]);
      }
    }
  }
  __syncthreads();
  float* red = gs;  // combine the two row halves: [CC*49][7]
  if (half == 1)
    for (int tw = 0; tw < K7; ++tw) red[rem * K7 + tw] = acc[tw];
  __syncthreads();
  if (half == 0) {
    for (int tw = 0; tw < K7; ++tw)
      atomicAdd(dw + (long long)(c0 + cc) * a.wc + tdh * K7 + tw, acc[tw] + red[rem * K7 + tw]);
  }
}

// dW[c, t] += sum_v x[src(v,t)] * g[v, c]   (x: one channel, g: C channels on the output grid)
template <int C, int CC>
__global__ __launch_bounds__(256) void k7_wg_n2w_kernel(K7Args a, const float* __restrict__ x,
                                                        const float* __restrict__ g, float* dw) {
  __shared__ __attribute__((aligned(16))) float xs[HALO];
  __shared__ __attribute__((aligned(16))) float gs[CC * TD * TH * TW];  // [cc][row][w]
  const int tid = threadIdx.x;
  int n, d0, h0, w0;
  k7_tile(a, blockIdx.x / (C / CC), &n, &d0, &h0, &w0);
  const int c0 = (blockIdx.x % (C / CC)) * CC;
  k7_load_halo<1, 1>(a, x, xs, n, d0, h0, w0, 0);
  for (int i = tid; i < TD * TH * TW; i += 256) {
    const int ww = i % TW, r = i / TW, hh = r % TH, dd = r / TH;
    const int od = d0 + dd, oh = h0 + hh, ow = w0 + ww;
    const bool ok = od < a.do_ && oh < a.ho && ow < a.wo;
    const long long v = ((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow;
#pragma unroll
    for (int cc = 0; cc < CC; ++cc) gs[cc * TD * TH * TW + i] = ok ? g[v * C + c0 + cc] : 0.f;
  }
  __syncthreads();
  const int half = tid / (CC * 49), rem = tid - half * CC * 49;
  const int cc = rem / 49, tdh = rem - cc * 49, td = tdh / K7, th = tdh - td * K7;
  float acc[K7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (half < 2) {
    for (int row = half; row < TD * TH; row += 2) {
      const int dd = row / TH, hh = row - dd * TH;
      const float* xrow = &xs[((dd + td) * HH + (hh + th)) * HWP];
      const float* grow = &gs[cc * TD * TH * TW + row * TW];
#pragma unroll
      for (int w4 = 0; w4 < TW; w4 += 4) {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(grow + w4);
        float xr[10];
        k7_row(xrow + w4, xr);
#pragma unroll
        for (int tw = 0; tw < K7; ++tw)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[tw] = fmaf(xr[j + tw], gv[j], acc[tw]);
      }
    }
  }
  __syncthreads();
  float* red = gs;
  if (half == 1)
    for (int tw = 0; tw < K7; ++tw) red[rem * K7 + tw] = acc[tw];
  __syncthreads();
  if (half == 0) {
    for (int tw = 0; tw < K7; ++tw)
      atomicAdd(dw + (long long)(c0 + cc) * a.wc + tdh * K7 + tw, acc[tw] + red[rem * K7 + tw]);
  }
}

static K7Args k7_args(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc) {
  K7Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.P = P; a.reflect = reflect; a.flip = flip; a.wc = wc;
  a.tiles_d = (g->do_ + TD - 1) / TD; a.tiles_h = (g->ho + TH - 1) / TH; a.tiles_w = (g->wo + TW - 1) / TW;
  return a;
}

static int k7_blocks(const K7Args& a) { return a.n * a.tiles_d * a.tiles_h * a.tiles_w; }

// Which shapes the k7 kernels take (wide side C in {8, 16}); everything else -> generic kernels.
static bool k7_wide_ok(int c) { return c == 8 || c == 16; }
// bf16 MFMA variants (conv_k7_mfma.hip): 16-channel wide side, CGAN3D_PREC_BF16 geometries
// bf16 MFMA kernels (conv_k7_mfma.hip); their element indices are 32-bit
static bool k7m_ok(const cgan3d_conv_geom* g, int wide) {
  const long long vi = (long long)g->n * g->di * g->hi * g->wi, vo = (long long)g->n * g->do_ * g->ho * g->wo;
  return g->prec == CGAN3D_PREC_BF16 && wide == 16 && std::max(vi, vo) * 16 < (1LL << 31);
}

// number of blocks the n2w kernel uses for this geometry (0 if the k7 path does not apply);
// sizes the BatchNorm partial-statistics buffer (cgan3d_conv3d_stats_floats)
long long k7_wgrad_ws_floats(const cgan3d_conv_geom* g) {
  if (g->k != 7 || g->stride != 1 || g->transposed) return 0;
  if ((g->cout == 1 && k7m_ok(g, g->cin)) || (g->cin == 1 && k7m_ok(g, g->cout))) return k7m_wgrad_ws_floats(g);
  return 0;
}

long long k7_n2w_blocks(const cgan3d_conv_geom* g) {
  if (g->k != 7 || g->stride != 1 || g->cin != 1 || !k7_wide_ok(g->cout)) return 0;
  if (k7m_ok(g, g->cout)) return k7m_n2w_blocks(g);
  return k7_blocks(k7_args(g, 0, 0, 0, 0));
}

// Forward-style launch; returns 1 if handled.
int k7_try_fwd(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e,
               hipStream_t s) {
  if (g->k != 7 || g->stride != 1) return 0;
  // statistics mode: slab (bn_mode) or fp64 accumulators (cgan3d_bn_fuse acc_mode 3 / 4)
  const int smode = e.fz.acc_mode == 3 ? 1 : e.fz.acc_mode == 4 ? 2 : e.bn_mode;
  const bool fold = smode == 2 && e.bn_fold > 0;  // folded mode-2 statistics (k7m input-grad only)
  if (g->cin == 1 && k7_wide_ok(g->cout) && !e.bias && !e.residual && !e.mask_src && !e.out2 &&
      (smode != 2 || (fold && g->transposed && k7m_ok(g, g->cout))) && e.act == CGAN3D_ACT_NONE) {
    if (k7m_ok(g, g->cout)) {
      float* bp = e.bn_mode == 1 ? e.bn_part : nullptr;
      if (!g->transposed)
        k7m_n2w_launch(g, g->pad, g->reflect, 0, g->w_sb, x, w, y, e.stats, bp, s, nullptr, &e.fz, e.out16);
      else k7m_n2w_launch(g, g->k - 1 - g->pad, 0, 1, g->w_sb, x, w, y, e.stats, bp, s, fold ? &e : nullptr, nullptr,
                          e.out16);
      return 1;
    }
    K7Args a;
    if (!g->transposed) a = k7_args(g, g->pad, g->reflect, 0, g->w_sb);
    else a = k7_args(g, g->k - 1 - g->pad, 0, 1, g->w_sb);  // input-grad: flipped taps, zero pad
    float* bp = e.bn_mode == 1 ? e.bn_part : nullptr;
    if (g->cout == 16)
      ::cg::launch((k7_n2w_kernel<16>), dim3(k7_blocks(a)), dim3(256), 0, s, a, x, w, y, e.stats, bp);
    else ::cg::launch((k7_n2w_kernel<8>), dim3(k7_blocks(a)), dim3(256), 0, s, a, x, w, y, e.stats, bp);
    return 1;
  }
  if (g->cout == 1 && k7_wide_ok(g->cin) && !g->transposed && !e.residual && !e.mask_src && !e.stats &&
      (e.act == CGAN3D_ACT_NONE || e.act == CGAN3D_ACT_TANH)) {
    if (k7m_ok(g, g->cin)) {
      k7m_w2n_launch(g, g->pad, g->reflect, g->w_sa, x, w, y, e, s);
      return 1;
    }
    K7Args a = k7_args(g, g->pad, g->reflect, 0, g->w_sa);
    if (g->cin == 16)
      ::cg::launch((k7_w2n_kernel<16, 2>), dim3(k7_blocks(a)), dim3(256), 0, s, a, x, w, y, e.bias, e.act,
                         e.minuend, e.out2);
    else
      ::cg::launch((k7_w2n_kernel<8, 2>), dim3(k7_blocks(a)), dim3(256), 0, s, a, x, w, y, e.bias, e.act,
                         e.minuend, e.out2);
    return 1;
  }
  return 0;
}

// 1 if the forward of a 16 -> 1 k7 conv takes a bf16 MFMA kernel (k7s_w2n / k7m_w2n): given the bf16
// shadow of its input it reads only that
int k7m_w2n_taken(const cgan3d_conv_geom* g) {
  return g->k == 7 && g->stride == 1 && !g->transposed && g->cout == 1 && k7m_ok(g, g->cin);
}

// 1 if the geometry's forward takes the k7m n2w kernel as an input-grad (folded mode-2 statistics)
// the 1 -> 16 MFMA kernel (k7m_n2w_kernel) takes this forward / input-grad launch
int k7m_n2w_ok(const cgan3d_conv_geom* g) {
  return g->k == 7 && g->stride == 1 && g->cin == 1 && k7_wide_ok(g->cout) && k7m_ok(g, g->cout);
}

int k7m_fold_ok(const cgan3d_conv_geom* g) {
  return g->k == 7 && g->stride == 1 && g->transposed && g->cin == 1 && k7m_ok(g, g->cout);
}

// 1 if k7_try_wgrad takes a bf16 MFMA kernel (k7m_wg_kernel) for the geometry: it then reads the
// multi-channel operand from its bf16 shadow alone when one is given
int k7m_wgrad_taken(const cgan3d_conv_geom* g) {
  if (g->k != 7 || g->stride != 1 || g->transposed) return 0;
  return (g->cout == 1 && k7m_ok(g, g->cin)) || (g->cin == 1 && k7m_ok(g, g->cout));
}

// 1 if k7_try_wgrad handles the geometry (same conditions)
int k7_wgrad_handles(const cgan3d_conv_geom* g) {
  if (g->k != 7 || g->stride != 1 || g->transposed) return 0;
  return (g->cout == 1 && (k7m_ok(g, g->cin) || k7_wide_ok(g->cin))) ||
         (g->cin == 1 && (k7m_ok(g, g->cout) || k7_wide_ok(g->cout)));
}

// Weight-grad launch (dw zeroed by the caller unless accumulating); returns 1 if handled.
// wide16: optional bf16 shadow of the multi-channel operand (read instead of its fp32 tensor by
// the MFMA kernel, which rounds it to bf16 anyway: same bits)
int k7_try_wgrad(const cgan3d_conv_geom* g, const float* x, const float* go, float* dw, float* ws, hipStream_t s,
                 const __bf16* wide16) {
  if (g->k != 7 || g->stride != 1 || g->transposed) return 0;
  if (g->cout == 1 && k7m_ok(g, g->cin)) {
    k7m_wgrad_launch(g, true, g->w_sa, x, go, dw, ws, s, g->prec == CGAN3D_PREC_BF16 ? wide16 : nullptr);
    return 1;
  }
  if (g->cin == 1 && k7m_ok(g, g->cout)) {
    k7m_wgrad_launch(g, false, g->w_sb, x, go, dw, ws, s, g->prec == CGAN3D_PREC_BF16 ? wide16 : nullptr);
    return 1;
  }
  if (g->cout == 1 && k7_wide_ok(g->cin)) {
    K7Args a = k7_args(g, g->pad, g->reflect, 0, g->w_sa);
    const int C = g->cin;
    if (C == 16) ::cg::launch((k7_wg_w2n_kernel<16, 2>), dim3(k7_blocks(a) * 8), dim3(256), 0, s, a, x, go, dw);
    else ::cg::launch((k7_wg_w2n_kernel<8, 2>), dim3(k7_blocks(a) * 4), dim3(256), 0, s, a, x, go, dw);
    return 1;
  }
  if (g->cin == 1 && k7_wide_ok(g->cout)) {
    K7Args a = k7_args(g, g->pad, g->reflect, 0, g->w_sb);
    const int C = g->cout;
    if (C == 16) ::cg::launch((k7_wg_n2w_kernel<16, 2>), dim3(k7_blocks(a) * 8), dim3(256), 0, s, a, x, go, dw);
    else ::cg::launch((k7_wg_n2w_kernel<8, 2>), dim3(k7_blocks(a) * 4), dim3(256), 0, s, a, x, go, dw);
    return 1;
  }
  return 0;
}

}  // namespace cg
