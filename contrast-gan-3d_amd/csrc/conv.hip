// Implicit-GEMM 3-D convolutions for gfx950 (fp32, exact-f32 MFMA v_mfma_f32_16x16x4_f32).
//
// Replaces the aten convolution / convolution_backward calls the reference's hot path makes:
// Conv3d and ConvTranspose3d in ConvBlock (contrast_gan_3D/model/blocks.py:29-38), the
// generator's reflect-padded k7 first/last convs (model/generator.py:31-35,78-84) and the
// critic's k4 s2 pyramid (model/discriminator.py:24-80), forward, input-grad and weight-grad.
//
// One gather formulation covers every case (see include/cgan3d.h): a tap t links output
// voxel o and gathered voxel i either as i = o*s - p + t ("forward") or o = i*s - p + t
// ("transposed").  Transposed launches are split into s^3 parity classes so every voxel of a
// 64-voxel tile has the same valid tap list (no wasted MFMA work on the 7/8 invalid taps of a
// stride-2 ConvTranspose3d).  The reduction index K = (valid tap, channel) is walked in chunks
// of 32 staged through LDS; each wave owns 16 output voxels x up to 64 output channels.
#include "common.h"

namespace cg {

struct ConvArgs {
  int n, di, hi, wi, do_, ho, wo, cin, cout, k, s, p, transposed, reflect;
  int kd, sd, pd;          // depth-axis kernel / stride / pad: (k, s, p), or (1, 1, 0) for planar (2-D)
  long long sa, sb;
  int cd, ch, cw;          // grid walked by the tiles: output grid, or one parity class
  long long class_vox;     // voxels per class (or all output voxels)
  int tiles_per_class;
  int nclass;
};

static bool make_args(const cgan3d_conv_geom* g, ConvArgs* a, int bm) {
  a->n = g->n; a->di = g->di; a->hi = g->hi; a->wi = g->wi;
  a->do_ = g->do_; a->ho = g->ho; a->wo = g->wo; a->cin = g->cin; a->cout = g->cout;
  a->k = g->k; a->s = g->stride; a->p = g->pad; a->transposed = g->transposed; a->reflect = g->reflect;
  a->sa = g->w_sa; a->sb = g->w_sb;
  a->kd = geom_kd(g); a->sd = geom_sd(g); a->pd = geom_pd(g);
  if (g->transposed && g->stride > 1) {  // ceil-sized parity-class grids (odd output dims masked)
    const int s = g->stride;
    a->cd = (g->do_ + a->sd - 1) / a->sd; a->ch = (g->ho + s - 1) / s; a->cw = (g->wo + s - 1) / s;
    a->nclass = a->sd * s * s;
  } else {
    a->cd = g->do_; a->ch = g->ho; a->cw = g->wo; a->nclass = 1;
  }
  a->class_vox = (long long)g->n * a->cd * a->ch * a->cw;
  a->tiles_per_class = (int)((a->class_vox + bm - 1) / bm);
  return true;
}

static int validate(const cgan3d_conv_geom* g, const char* who) {
  CG_CHECK_ARG(g != nullptr, "%s: null geometry", who);
  CG_CHECK_ARG(g->n > 0 && g->di > 0 && g->hi > 0 && g->wi > 0 && g->do_ > 0 && g->ho > 0 && g->wo > 0,
               "%s: non-positive dims", who);
  CG_CHECK_ARG(g->cin > 0 && g->cout > 0 && (g->cout <= 64 || g->planar), "%s: channels cin=%d cout=%d (cout<=64)",
               who, g->cin, g->cout);
  CG_CHECK_ARG(!g->planar || (g->di == 1 && g->do_ == 1 && g->prec == CGAN3D_PREC_F32 && g->w_packed <= 1),
               "%s: planar (2-D) geometries have di == do_ == 1 and run in f32 with w_packed 0 or 1", who);
  CG_CHECK_ARG(g->k > 0 && g->k <= 7 && g->stride >= 1 && g->stride <= 2 && g->pad >= 0 && g->pad < g->k,
               "%s: kernel k=%d s=%d p=%d unsupported", who, g->k, g->stride, g->pad);
  CG_CHECK_ARG(!(g->reflect && g->transposed), "%s: reflect padding only in forward mapping", who);
  CG_CHECK_ARG(!g->reflect || ((g->planar || g->pad < g->di) && g->pad < g->hi && g->pad < g->wi),
               "%s: reflect pad %d >= dim", who, g->pad);
  if (!g->transposed && !g->planar) {
    CG_CHECK_ARG((long long)(g->do_ - 1) * g->stride - g->pad + g->k - 1 < (long long)g->di + g->pad &&
                 (long long)(g->ho - 1) * g->stride - g->pad + g->k - 1 < (long long)g->hi + g->pad &&
                 (long long)(g->wo - 1) * g->stride - g->pad + g->k - 1 < (long long)g->wi + g->pad,
                 "%s: output dims exceed padded input", who);
  }
  CG_CHECK_ARG((long long)g->n * g->do_ * g->ho * g->wo < (1LL << 31) &&
               (long long)g->n * g->di * g->hi * g->wi < (1LL << 31), "%s: voxel count exceeds int32", who);
  return CGAN3D_OK;
}

// Per-dimension valid tap list of a parity class: taps t = first + step*m, m < count.
__device__ __forceinline__ void class_taps(int r, int k, int s, int p, int transposed, int* first, int* step,
                                           int* count) {
  if (transposed) {
    int f = (r + p) % s;
    *first = f;
    *step = s;
    *count = f < k ? (k - f + s - 1) / s : 0;
  } else {
    *first = 0;
    *step = 1;
    *count = k;
  }
}

// gathered coordinate along one dim (returns -1 when the tap contributes zero)
__device__ __forceinline__ int gcoord(int base, int off, int n, int reflect) {
  int i = base + off;
  if (reflect) return reflect_idx(i, n);
  return (i >= 0 && i < n) ? i : -1;
}

// ------------------------------------------------------------------------------------------
// cout == 1 forward / input-grad (VALU): one thread per output voxel, weights in LDS.
// Used by the critic's first-layer input-grad (8 -> 1 channel, transposed s2) and, when the
// output is large, its last layer.
//
// conv_cout1_wave_kernel: the same contraction with one wave per output voxel and the
// (tap, channel) reduction spread over the 64 lanes — for the critic's last layer, whose output
// is only N x 3^3 voxels but each voxel reduces 64 taps x 64 channels (forward mapping only).
__global__ __launch_bounds__(256) void conv_cout1_wave_kernel(ConvArgs a, const float* __restrict__ x,
                                                              const float* __restrict__ w, float* y, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [T][cin]
  const int T = a.kd * a.k * a.k;
  // weights staged in source order (ci major, taps contiguous when sa == T: coalesced), 8 loads in
  // flight per thread, transposed into [t][cin] on the LDS side
  for (int i0 = threadIdx.x; i0 < T * a.cin; i0 += 8 * blockDim.x) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * blockDim.x, ci = i / T, t = i - ci * T;
      v[u] = i < T * a.cin ? w[(long long)ci * a.sa + t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * blockDim.x, ci = i / T, t = i - ci * T;
      if (i < T * a.cin) Ws[t * a.cin + ci] = v[u];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long long lin = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (lin >= a.class_vox) return;  // wave-uniform
  int ow = (int)(lin % a.wo); long long tt = lin / a.wo;
  int oh = (int)(tt % a.ho); tt /= a.ho;
  int od = (int)(tt % a.do_); int nb = (int)(tt / a.do_);
  const int bd = od * a.sd - a.pd, bh = oh * a.s - a.p, bw = ow * a.s - a.p;
  const int C4 = a.cin >> 2, R4 = T * C4;
  float acc = 0.f;
#pragma unroll 4
  for (int r4 = lane; r4 < R4; r4 += 64) {
    const int t = r4 / C4, c = (r4 - t * C4) * 4;
    const int td = t / (a.k * a.k), th = (t / a.k) % a.k, tw = t % a.k;
    const int id = gcoord(bd, td, a.di, a.reflect), ih = gcoord(bh, th, a.hi, a.reflect), iw = gcoord(bw, tw, a.wi, a.reflect);
    if ((id | ih | iw) >= 0) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + ((long long)((nb * a.di + id) * a.hi + ih) * a.wi + iw) * a.cin + c);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(Ws + t * a.cin + c);
      acc += xv[0] * wv[0] + xv[1] * wv[1] + xv[2] * wv[2] + xv[3] * wv[3];
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    float v = acc + (ep.bias ? ep.bias[0] : 0.f);
    if (ep.act == CGAN3D_ACT_RELU) v = fmaxf(v, 0.f);
    else if (ep.act == CGAN3D_ACT_LRELU) v = v > 0.f ? v : v * ep.slope;
    else if (ep.act == CGAN3D_ACT_TANH) v = tanhf(v);
    if (ep.mask_src) v = ep.mask_src[lin] > 0.f ? v : v * ep.slope;
    if (ep.residual) v += ep.residual[lin];
    y[lin] = v;
    if (ep.out2) ep.out2[lin] = ep.minuend[lin] - v;
  }
}

// The same contraction with the whole block (4 waves) on one output voxel: for the critic's last
// layer at small batches the wave-per-voxel grid is a few dozen blocks whose lanes each walk 16
// dependent float4 loads; here every voxel's 1024 float4 of (tap, channel) are split over 256
// threads (4 loads each) and reduced through LDS.
__global__ __launch_bounds__(256) void conv_cout1_block_kernel(ConvArgs a, const float* __restrict__ x,
                                                               const float* __restrict__ w, float* y, Epi ep) {
  __shared__ float red[4];
  const int T = a.kd * a.k * a.k;
  // Every load below is unconditional from a clamped, valid address (a dead one masked to zero
  // afterwards by an integer mask): a load under a branch gets a wait of its own.  Round 4: each
  // thread reads the weights of its own (tap, 4 channels) items straight from L2, in flight with its
  // x loads — no LDS staging pass and barrier in front of the dot product (12.8 us for the critic's
  // 324-voxel last layer with them).
  const long long lin = blockIdx.x;
  int ow = (int)(lin % a.wo); long long tt = lin / a.wo;
  int oh = (int)(tt % a.ho); tt /= a.ho;
  int od = (int)(tt % a.do_); int nb = (int)(tt / a.do_);
  const int bd = od * a.sd - a.pd, bh = oh * a.s - a.p, bw = ow * a.s - a.p;
  const int C4 = a.cin >> 2, R4 = T * C4;
  constexpr int MAXR = 8;  // float4 per thread (R4 <= 2048)
  f32x4 xv[MAXR], wv[MAXR];
  unsigned okm = 0;
#pragma unroll
  for (int u = 0; u < MAXR; ++u) {
    const int r4 = threadIdx.x + 256 * u;
    const int t = min(r4, R4 - 1) / C4, c = (min(r4, R4 - 1) - t * C4) * 4;
    const int td = t / (a.k * a.k), th = (t / a.k) % a.k, tw = t % a.k;
    const int id = gcoord(bd, td, a.di, a.reflect), ih = gcoord(bh, th, a.hi, a.reflect),
              iw = gcoord(bw, tw, a.wi, a.reflect);
    const bool ok = r4 < R4 && (id | ih | iw) >= 0;
    xv[u] = *reinterpret_cast<const f32x4*>(
        x + (ok ? ((long long)((nb * a.di + id) * a.hi + ih) * a.wi + iw) * a.cin + c : 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[u][j] = w[(long long)(c + j) * a.sa + t];
    okm |= ok ? 1u << u : 0u;
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < MAXR; ++u) {
    const bool ok = (okm >> u) & 1u;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += keep_if(ok, xv[u][j]) * wv[u][j];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = red[0] + red[1] + red[2] + red[3] + (ep.bias ? ep.bias[0] : 0.f);
    if (ep.act == CGAN3D_ACT_RELU) v = fmaxf(v, 0.f);
    else if (ep.act == CGAN3D_ACT_LRELU) v = v > 0.f ? v : v * ep.slope;
    else if (ep.act == CGAN3D_ACT_TANH) v = tanhf(v);
    if (ep.mask_src) v = ep.mask_src[lin] > 0.f ? v : v * ep.slope;
    if (ep.residual) v += ep.residual[lin];
    y[lin] = v;
    if (ep.out2) ep.out2[lin] = ep.minuend[lin] - v;
  }
}

// ------------------------------------------------------------------------------------------
// cin == 1, stride-1 transposed launches (the critic's last-layer input-grad, discriminator.py:
// Conv3d 64 -> 1 k4 s1 p1 run as 1 -> 64): exact fp32, a thread per (output voxel, channel) —
// the 64 lanes of a wave are the 64 channels of one voxel, so the per-tap validity is wave-uniform —
// the block's sample input and the weights staged once in LDS.  Round 4: the implicit GEMM took
// 12.7 us for these 49k outputs (a 64-long K on 16 x 64 tiles of a mostly empty grid).
constexpr int CIN1T_MAXV = 512, CIN1T_MAXW = 64 * 64;
bool cin1t_ok(const cgan3d_conv_geom* g) {
  return g->transposed && !g->planar && !g->reflect && g->stride == 1 && g->cin == 1 && g->cout >= 2 &&
         g->cout <= 64 && g->k * g->k * g->k * g->cout <= CIN1T_MAXW && g->di * g->hi * g->wi <= CIN1T_MAXV &&
         (long long)g->n * g->do_ * g->ho * g->wo * g->cout < (1LL << 31);
}

__global__ __launch_bounds__(256) void conv_cin1t_kernel(ConvArgs a, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* y, Epi ep,
                                                         int blocks_per_sample) {
  __shared__ float xs[CIN1T_MAXV];
  __shared__ float wsm[CIN1T_MAXW];  // [t][c]
  const int nb = blockIdx.x / blocks_per_sample, part = blockIdx.x - nb * blocks_per_sample;
  const int T = a.k * a.k * a.k, C = a.cout;
  const int nin = a.di * a.hi * a.wi, nout = a.do_ * a.ho * a.wo;
  for (int i = threadIdx.x; i < nin; i += 256) xs[i] = x[(long long)nb * nin + i];
  for (int i = threadIdx.x; i < T * C; i += 256) {
    const int t = i / C, c = i - t * C;
    wsm[i] = w[(long long)c * a.sb + t];
  }
  __syncthreads();
  const int per = (nout * C + blocks_per_sample - 1) / blocks_per_sample;
  const int o0 = part * per, o1 = min(nout * C, o0 + per);
  for (int o = o0 + (int)threadIdx.x; o < o1; o += 256) {
    const int c = o % C, v = o / C;
    const int ow = v % a.wo, oh = (v / a.wo) % a.ho, od = v / (a.wo * a.ho);
    float acc = 0.f;
    for (int td = 0; td < a.k; ++td) {
      const int id = od + a.p - td;
      if ((unsigned)id >= (unsigned)a.di) continue;
      for (int th = 0; th < a.k; ++th) {
        const int ih = oh + a.p - th;
        if ((unsigned)ih >= (unsigned)a.hi) continue;
        for (int tw = 0; tw < a.k; ++tw) {
          const int iw = ow + a.p - tw;
          if ((unsigned)iw >= (unsigned)a.wi) continue;
          acc = fmaf(xs[(id * a.hi + ih) * a.wi + iw], wsm[((td * a.k + th) * a.k + tw) * C + c], acc);
        }
      }
    }
    const long long oi = ((long long)nb * nout + v) * C + c;
    float r = acc + (ep.bias ? ep.bias[c] : 0.f);
    if (ep.act == CGAN3D_ACT_RELU) r = fmaxf(r, 0.f);
    else if (ep.act == CGAN3D_ACT_LRELU) r = r > 0.f ? r : r * ep.slope;
    if (ep.mask_src) r = ep.mask_src[oi] > 0.f ? r : r * ep.slope;
    if (ep.residual) r += ep.residual[oi];
    y[oi] = r;
  }
}

// One thread per output voxel, weights in LDS.
__global__ __launch_bounds__(256) void conv_cout1_kernel(ConvArgs a, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* y, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [T][cin]
  const int T = a.kd * a.k * a.k;
  for (int i = threadIdx.x; i < T * a.cin; i += blockDim.x) {
    int t = i / a.cin, ci = i - t * a.cin;
    Ws[i] = w[(long long)ci * a.sa + t];
  }
  __syncthreads();
  const int cls = blockIdx.x / a.tiles_per_class;
  const int tile = blockIdx.x - cls * a.tiles_per_class;
  const long long lin = (long long)tile * blockDim.x + threadIdx.x;
  if (lin >= a.class_vox) return;
  const int s = a.s, k = a.k, p = a.p;
  int rd = 0, rh = 0, rw = 0;
  if (a.transposed) { rd = cls / (s * s); rh = (cls / s) % s; rw = cls % s; }
  int fd, sd, nd, fh, sh, nh, fw, sw, nw;
  class_taps(rd, a.kd, a.sd, a.pd, a.transposed, &fd, &sd, &nd);
  class_taps(rh, k, s, p, a.transposed, &fh, &sh, &nh);
  class_taps(rw, k, s, p, a.transposed, &fw, &sw, &nw);
  int jw, jh, jd, nb;
  unflatten4(lin, a.cw, a.ch, a.cd, jw, jh, jd, nb);
  int od, oh, ow, bd, bh, bw;
  if (a.transposed) { od = jd * a.sd + rd; oh = jh * s + rh; ow = jw * s + rw; bd = jd; bh = jh; bw = jw; }
  else { od = jd; oh = jh; ow = jw; bd = jd * a.sd - a.pd; bh = jh * s - p; bw = jw * s - p; }
  if (od >= a.do_ || oh >= a.ho || ow >= a.wo) return;  // past the end of a ceil-sized class grid
  float acc = 0.f;
  for (int md = 0; md < nd; ++md) {
    const int td = fd + sd * md;
    const int id = gcoord(bd, a.transposed ? (rd + a.pd - td) / a.sd : td, a.di, a.reflect);
    if (id < 0) continue;
    for (int mh = 0; mh < nh; ++mh) {
      const int th = fh + sh * mh;
      const int ih = gcoord(bh, a.transposed ? (rh + p - th) / s : th, a.hi, a.reflect);
      if (ih < 0) continue;
      for (int mw = 0; mw < nw; ++mw) {
        const int tw = fw + sw * mw;
        const int iw = gcoord(bw, a.transposed ? (rw + p - tw) / s : tw, a.wi, a.reflect);
        if (iw < 0) continue;
        const float* xp = x + ((long long)((nb * a.di + id) * a.hi + ih) * a.wi + iw) * a.cin;
        const float* wp = Ws + ((td * k + th) * k + tw) * a.cin;
        if ((a.cin & 3) == 0) {
          for (int ci = 0; ci < a.cin; ci += 4) {
            f32x4 xv = *reinterpret_cast<const f32x4*>(xp + ci);
            f32x4 wv = *reinterpret_cast<const f32x4*>(wp + ci);
            acc += xv[0] * wv[0] + xv[1] * wv[1] + xv[2] * wv[2] + xv[3] * wv[3];
          }
        } else {
          for (int ci = 0; ci < a.cin; ++ci) acc += xp[ci] * wp[ci];
        }
      }
    }
  }
  float v = acc + (ep.bias ? ep.bias[0] : 0.f);
  if (ep.act == CGAN3D_ACT_RELU) v = fmaxf(v, 0.f);
  else if (ep.act == CGAN3D_ACT_LRELU) v = v > 0.f ? v : v * ep.slope;
  else if (ep.act == CGAN3D_ACT_TANH) v = tanhf(v);
  const long long o = ((long long)(nb * a.do_ + od) * a.ho + oh) * a.wo + ow;
  if (ep.mask_src) v = ep.mask_src[o] > 0.f ? v : v * ep.slope;
  if (ep.residual) v += ep.residual[o];
  y[o] = v;
  if (ep.out2) ep.out2[o] = ep.minuend[o] - v;
}

// ------------------------------------------------------------------------------------------
// Weight gradient (cout >= 2): dwp[(t*cin + a)*cout + b] += sum_o gathered(o, t, a) * aligned(o, b)
// Forward mapping i = o*s - p + t (reflect optional).  Block = 64 (t,a) rows x all cout columns
// over a chunk of output voxels; 32 voxels per LDS stage.
template <int VEC, int NB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a, const float* __restrict__ gx,
                                                         const float* __restrict__ go, float* dwp, long long vpb) {
  constexpr int KV = 32, LD = 80;
  __shared__ __attribute__((aligned(16))) float As[KV * LD];  // [voxel][r]
  __shared__ __attribute__((aligned(16))) float Gs[KV * LD];  // [voxel][b]
  __shared__ int rtab[4][64];                                  // td, th, tw, a   (td = -1: pad row)
  __shared__ int vtab[5][KV];                                  // n*di, bd, bh, bw, aligned voxel

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = a.kd * a.k * a.k * a.cin;
  const int r0 = blockIdx.x * 64;
  const int co0 = blockIdx.z * 64;  // output-channel block (cout > 64: the 2-D critic's 128 channels)
  if (tid < 64) {
    int r = r0 + tid;
    if (r < R) {
      int t = r / a.cin, ci = r - t * a.cin;
      rtab[0][tid] = t / (a.k * a.k); rtab[1][tid] = (t / a.k) % a.k; rtab[2][tid] = t % a.k; rtab[3][tid] = ci;
    } else {
      rtab[0][tid] = -1; rtab[1][tid] = rtab[2][tid] = rtab[3][tid] = 0;
    }
  }
  const long long V = (long long)a.n * a.do_ * a.ho * a.wo;
  const long long vbeg = (long long)blockIdx.y * vpb;
  const long long vend = vbeg + vpb < V ? vbeg + vpb : V;

  f32x4 acc[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;

  for (long long vb = vbeg; vb < vend; vb += KV) {
    if (tid < KV) {
      long long lin = vb + tid;
      if (lin < vend) {
        int ow, oh, od, nb;
        unflatten4(lin, a.wo, a.ho, a.do_, ow, oh, od, nb);
        vtab[0][tid] = nb * a.di; vtab[1][tid] = od * a.sd - a.pd; vtab[2][tid] = oh * a.s - a.p;
        vtab[3][tid] = ow * a.s - a.p; vtab[4][tid] = (int)lin;
      } else {
        vtab[0][tid] = -1; vtab[4][tid] = -1;
      }
    }
    __syncthreads();
    if (VEC == 4) {
      const int r4 = tid & 15;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int v = (tid >> 4) + 16 * i;
        f32x4 val = {0.f, 0.f, 0.f, 0.f};
        const int nb = vtab[0][v], rr = 4 * r4;
        if (nb >= 0 && rtab[0][rr] >= 0) {
          int id = gcoord(vtab[1][v], rtab[0][rr], a.di, a.reflect);
          int ih = gcoord(vtab[2][v], rtab[1][rr], a.hi, a.reflect);
          int iw = gcoord(vtab[3][v], rtab[2][rr], a.wi, a.reflect);
          if ((id | ih | iw) >= 0)
            val = *reinterpret_cast<const f32x4*>(gx + ((long long)((nb + id) * a.hi + ih) * a.wi + iw) * a.cin + rtab[3][rr]);
        }
        *reinterpret_cast<f32x4*>(&As[v * LD + rr]) = val;
      }
    } else {
      const int rr = tid & 63;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int v = (tid >> 6) + 4 * i;
        float val = 0.f;
        const int nb = vtab[0][v];
        if (nb >= 0 && rtab[0][rr] >= 0) {
          int id = gcoord(vtab[1][v], rtab[0][rr], a.di, a.reflect);
          int ih = gcoord(vtab[2][v], rtab[1][rr], a.hi, a.reflect);
          int iw = gcoord(vtab[3][v], rtab[2][rr], a.wi, a.reflect);
          if ((id | ih | iw) >= 0) val = gx[((long long)((nb + id) * a.hi + ih) * a.wi + iw) * a.cin + rtab[3][rr]];
        }
        As[v * LD + rr] = val;
      }
    }
    {
      const int c4 = tid & 15;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int v = (tid >> 4) + 16 * i;
        f32x4 val = {0.f, 0.f, 0.f, 0.f};
        const int ov = vtab[4][v];
        if (ov >= 0 && co0 + 4 * c4 < a.cout)
          val = *reinterpret_cast<const f32x4*>(go + (long long)ov * a.cout + co0 + 4 * c4);
        *reinterpret_cast<f32x4*>(&Gs[v * LD + 4 * c4]) = val;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KV; kk += 4) {
      const float av = As[(kk + g) * LD + 16 * wave + r16];
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float bv = Gs[(kk + g) * LD + 16 * n + r16];
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[n], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // D[row = 4g + j][col = r16]: row -> r = r0 + 16*wave + 4g + j, col -> b = 16n + r16
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = co0 + 16 * n + r16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + 16 * wave + 4 * g + j;
      if (r < R && b < a.cout) atomicAdd(dwp + (long long)r * a.cout + b, acc[n][j]);
    }
  }
}

// cout == 1 weight gradient (VALU): dwp[t*cin + a] += sum_o gathered(o,t,a) * aligned(o)
template <int MAXJ>
__global__ __launch_bounds__(256) void conv_wgrad_cout1_kernel(ConvArgs a, const float* __restrict__ gx,
                                                               const float* __restrict__ go, float* dwp,
                                                               long long vpb) {
  constexpr int VB = 64;
  __shared__ int vtab[5][VB];
  __shared__ float gv[VB];
  const int tid = threadIdx.x;
  const int R4 = a.kd * a.k * a.k * a.cin / 4;
  int td[MAXJ], th[MAXJ], tw[MAXJ], ca[MAXJ];
  f32x4 acc[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    int r4 = tid + 256 * (j + MAXJ * (int)blockIdx.y);
    acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (r4 < R4) {
      int r = 4 * r4, t = r / a.cin;
      ca[j] = r - t * a.cin; td[j] = t / (a.k * a.k); th[j] = (t / a.k) % a.k; tw[j] = t % a.k;
    } else {
      td[j] = -1; th[j] = tw[j] = ca[j] = 0;
    }
  }
  const long long V = (long long)a.n * a.do_ * a.ho * a.wo;
  const long long vbeg = (long long)blockIdx.x * vpb;
  const long long vend = vbeg + vpb < V ? vbeg + vpb : V;
  for (long long vb = vbeg; vb < vend; vb += VB) {
    __syncthreads();
    if (tid < VB) {
      long long lin = vb + tid;
      if (lin < vend) {
        int ow, oh, od, nb;
        unflatten4(lin, a.wo, a.ho, a.do_, ow, oh, od, nb);
        vtab[0][tid] = nb * a.di; vtab[1][tid] = od * a.sd - a.pd; vtab[2][tid] = oh * a.s - a.p;
        vtab[3][tid] = ow * a.s - a.p;
        gv[tid] = go[lin];
      } else {
        vtab[0][tid] = -1; gv[tid] = 0.f;
      }
    }
    __syncthreads();
    const int nv = (int)((vend - vb) < VB ? (vend - vb) : VB);
    for (int v = 0; v < nv; ++v) {
      const int nb = vtab[0][v];
      const float gval = gv[v];
      const int bd = vtab[1][v], bh = vtab[2][v], bw = vtab[3][v];
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        if (td[j] < 0) continue;
        int id = gcoord(bd, td[j], a.di, a.reflect);
        int ih = gcoord(bh, th[j], a.hi, a.reflect);
        int iw = gcoord(bw, tw[j], a.wi, a.reflect);
        if ((id | ih | iw) >= 0) {
          f32x4 xv = *reinterpret_cast<const f32x4*>(gx + ((long long)((nb + id) * a.hi + ih) * a.wi + iw) * a.cin + ca[j]);
          acc[j] += xv * gval;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (td[j] < 0) continue;
    int r = 4 * (tid + 256 * (j + MAXJ * (int)blockIdx.y));
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(dwp + r + e, acc[j][e]);
  }
}

// dw[a*sa + b*sb + t] (+)= dwp[(t*cin + a)*cout + b]; clean: dwp is left zeroed for its next user
__global__ void wgrad_unpack_kernel(float* __restrict__ dwp, float* dw, int T, int cin, int cout, long long sa,
                                    long long sb, int accumulate, int clean) {
  // 32-bit index math (weights are far below 2^31 elements)
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)T * cin * cout) return;
  const unsigned r = i / (unsigned)cout, t = r / (unsigned)cin;
  const int b = (int)(i - r * cout), ca = (int)(r - t * cin);
  float* d = dw + ca * sa + b * sb + (int)t;
  const float v = dwp[i];
  *d = accumulate ? *d + v : v;
  if (clean) dwp[i] = 0.f;
}

// the same for several weight gradients in one launch (blockIdx.y = descriptor); always clean
__global__ __launch_bounds__(256) void wgrad_unpack_multi_kernel(const cgan3d_unpack_desc* __restrict__ descs) {
  const cgan3d_unpack_desc d = descs[blockIdx.y];
  const unsigned total = (unsigned)d.taps * d.cin * d.cout;  // 32-bit index math (small weights)
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const unsigned r = i / (unsigned)d.cout, t = r / (unsigned)d.cin;
    const int b = (int)(i - r * d.cout), ca = (int)(r - t * d.cin);
    float* o = d.dw + ca * d.sa + b * d.sb + (int)t;
    const float v = d.ws[i];
    *o = d.accumulate ? *o + v : v;
    d.ws[i] = 0.f;
  }
}

}  // namespace cg

using namespace cg;

namespace cg {
}  // namespace cg

static Epi to_epi(const cgan3d_epilogue* ep) {
  Epi e{};
  if (ep) {
    e.bias = ep->bias; e.residual = ep->residual; e.mask_src = ep->mask_src; e.minuend = ep->minuend;
    e.out2 = ep->out2; e.stats = ep->stats; e.act = ep->act; e.slope = ep->slope;
    e.bn_part = ep->bn_mode ? ep->bn_part : nullptr; e.bn_mode = ep->bn_part ? ep->bn_mode : 0;
    e.bn_slots = ep->bn_slots; e.bn_z = ep->bn_z; e.bn_ss = ep->bn_ss; e.bn_mi = ep->bn_mi;
    e.bn_act = ep->bn_act; e.bn_slope = ep->bn_slope;
    e.x16 = reinterpret_cast<const __bf16*>(ep->x_bf16);
    e.bn_fold = ep->bn_fold;
    if (const cgan3d_bn_fuse* f = ep->fuse) {
      e.fz.acc_out = f->acc_out; e.fz.acc_mode = f->acc_mode; e.fz.reps = f->reps;
    }
    e.out16 = ep->out_bf16 & 1;
    e.res16 = (ep->out_bf16 >> 1) & 1;
    if (const cgan3d_bn_pre* p = ep->pre) {
      BnPre& q = e.pre;
      q.mode = p->mode; q.z = reinterpret_cast<const __bf16*>(p->z); q.acc = p->acc; q.reps = p->reps;
      q.nvox = (double)p->nvox; q.gamma = p->gamma; q.beta = p->beta; q.rmean = p->running_mean;
      q.rvar = p->running_var; q.nbt = (long long*)p->num_batches_tracked; q.momentum = p->momentum; q.eps = p->eps;
      q.ss = p->scale_shift; q.mi = p->mean_invstd; q.dgamma = p->dgamma; q.dbeta = p->dbeta;
      q.accumulate = p->accumulate; q.act = p->act; q.slope = p->slope; q.out16 = reinterpret_cast<__bf16*>(p->out_bf16);
      q.zero = p->zero; q.zero_n = p->zero_n;
    }
  }
  return e;
}

extern "C" int32_t cgan3d_conv3d_bn_pre_ok(const cgan3d_conv_geom* g) {
  if (!g || validate(g, "cgan3d_conv3d_bn_pre_ok") || g->planar) return 0;
  return k3m_route(g) ? 1 : 0;
}

// the input-BatchNorm prologue (cgan3d_bn_pre): argument checks; routes only to conv_k3m
static int check_pre(const cgan3d_conv_geom* g, const Epi& e) {
  const BnPre& p = e.pre;
  if (!p.mode) return CGAN3D_OK;
  CG_CHECK_ARG(p.mode == 1 || p.mode == 2, "cgan3d_bn_pre: mode must be 1 or 2");
  CG_CHECK_ARG(k3m_route(g) && k3m_ok(g, e), "cgan3d_bn_pre: only the ResNet-block kernel (cgan3d_conv3d_bn_pre_ok)");
  CG_CHECK_ARG((p.mode == 1) == !g->transposed, "cgan3d_bn_pre: mode 1 on the forward, mode 2 on the input-grad");
  CG_CHECK_ARG(p.acc && p.reps >= 1 && p.reps <= 64 && p.nvox > 1 && p.gamma && p.ss && p.mi && p.out16 &&
                   (p.zero || !p.zero_n) && p.zero_n >= 0,
               "cgan3d_bn_pre: acc, reps 1..64, nvox > 1, gamma, scale_shift, mean_invstd, out_bf16 required");
  CG_CHECK_ARG(p.mode == 2 || p.beta, "cgan3d_bn_pre: mode 1 needs beta");
  CG_CHECK_ARG(p.mode == 1 || p.z, "cgan3d_bn_pre: mode 2 needs z");
  CG_CHECK_ARG(p.act == CGAN3D_ACT_NONE || p.act == CGAN3D_ACT_RELU || p.act == CGAN3D_ACT_LRELU,
               "cgan3d_bn_pre: act none, relu or leaky relu");
  return CGAN3D_OK;
}

// the launches that honour cgan3d_epilogue.out_bf16 (their dispatch conditions: the S2T kernel from
// halo_launch, the 1 -> 16 k7 MFMA kernel from k7_try_fwd, the ResNet-block kernel conv_k3m)
extern "C" int32_t cgan3d_conv3d_out_bf16_ok(const cgan3d_conv_geom* g) {
  if (!g || validate(g, "cgan3d_conv3d_out_bf16_ok") || g->planar) return 0;
  if (g->w_packed == 2 && s2_kind(g) == 2) return 1;
  if (k3m_route(g) || t64_geom_ok(g) || f64_geom_ok(g)) return 1;
  return g->w_packed == 0 && k7m_n2w_ok(g) ? 1 : 0;
}

extern "C" int64_t cgan3d_conv3d_sumsq_blocks(const cgan3d_conv_geom* g) { return g ? c1_dgrad_blocks(g) : 0; }

extern "C" int32_t cgan3d_conv3d_neg_dtanh_ok(const cgan3d_conv_geom* g) {
  return g && !g->planar && c1_dgrad_ok(g) ? 1 : 0;
}

extern "C" int32_t cgan3d_bn_fuse_ok(const cgan3d_conv_geom* g) {
  if (!g || validate(g, "cgan3d_bn_fuse_ok")) return 0;
  // the halo-tiled family (halo_epilogue, the stride-2 16 <-> 32 kernels) and the generator's
  // 1 -> 16 k7 MFMA kernel (first conv forward, last conv input-grad with bn_fold)
  if (g->w_packed == 2 && halo_ok(g)) return 1;
  return g->w_packed == 0 && k7m_n2w_ok(g) ? 1 : 0;
}

// host checks of a cgan3d_bn_fuse against the launch it rides on
static int check_fuse(const cgan3d_conv_geom* g, const Epi& e) {
  const BnFuse& f = e.fz;
  if (!f.acc_mode) return CGAN3D_OK;
  CG_CHECK_ARG(cgan3d_bn_fuse_ok(g), "bn_fuse: geometry does not produce accumulators");
  CG_CHECK_ARG(f.acc_mode == 3 || f.acc_mode == 4, "bn_fuse: acc_mode must be 3 or 4");
  CG_CHECK_ARG(f.reps >= 1 && f.reps <= 64, "bn_fuse: reps must be 1..64");
  CG_CHECK_ARG(f.acc_out && !e.bn_mode && !e.stats, "bn_fuse: needs acc_out and no slab");
  CG_CHECK_ARG(f.acc_mode != 4 || (e.bn_z && e.bn_ss && e.bn_mi), "bn_fuse: acc_mode 4 needs bn_z, bn_ss, bn_mi");
  return CGAN3D_OK;
}

extern "C" int64_t cgan3d_conv3d_bn_slots(const cgan3d_conv_geom* g) {
  if (!g || g->cout == 1) return 0;
  const int64_t f = cgan3d_conv3d_stats_floats(g);
  return f > 0 ? f / (2 * g->cout + 1) : 0;
}

extern "C" int64_t cgan3d_conv3d_stats_floats(const cgan3d_conv_geom* g) {
  if (!g) return -1;
  if (g->planar) {  // 2-D variants: the implicit GEMM (cout >= 2) only
    long long mb = 0;
    if (g->cout < 2 || gemm_blocks(g, &mb)) return g->cout < 2 ? 0 : -1;
    return (int64_t)mb * (2 * g->cout + 1);
  }
  if (long long kb = k7_n2w_blocks(g)) return (int64_t)kb * (2 * g->cout + 1);
  if (sk_ok(g)) return (int64_t)sk_blocks(g) * (2 * g->cout + 1);
  if (halo_ok(g)) return (int64_t)halo_mblocks(g) * (2 * g->cout + 1);
  long long mb = 0;
  if (gemm_blocks(g, &mb)) return -1;
  return (int64_t)mb * (2 * g->cout + 1);
}

extern "C" int cgan3d_conv3d_fwd(const cgan3d_conv_geom* g, const float* x, const float* w, float* y,
                                 const cgan3d_epilogue* ep, void* stream) {
  int st = validate(g, "cgan3d_conv3d_fwd");
  if (st) return st;
  CG_CHECK_ARG(x && w && y, "cgan3d_conv3d_fwd: null pointer");
  Epi e = to_epi(ep);
  if (int rc = check_fuse(g, e)) return rc;
  if (int rc = check_pre(g, e)) return rc;
  CG_CHECK_ARG(!ep || (ep->out_bf16 >= 0 && ep->out_bf16 <= 3), "cgan3d_conv3d_fwd: out_bf16 must be 0..3");
  CG_CHECK_ARG(!(e.out16 || e.res16) || cgan3d_conv3d_out_bf16_ok(g),
               "cgan3d_conv3d_fwd: out_bf16 not taken by this launch");
  if (k3m_route(g)) {  // the ResNet-block kernel: any of its epilogues, bf16 input shadow
    CG_CHECK_ARG(!(e.out16 || e.res16) || k3m_ok(g, e),
                 "cgan3d_conv3d_fwd: out_bf16 on the ResNet-block geometry needs the conv_k3m epilogue (x_bf16, "
                 "fused statistics or none)");
    CG_CHECK_ARG(!e.res16 || e.residual, "cgan3d_conv3d_fwd: out_bf16 bit 1 without a residual");
  } else {
    CG_CHECK_ARG(!e.res16, "cgan3d_conv3d_fwd: a bf16 residual only on the ResNet-block kernel");
    CG_CHECK_ARG(!e.out16 || (!e.bias && !e.residual && !e.mask_src && !e.minuend && !e.out2 && !e.stats &&
                              !e.bn_mode && e.act == CGAN3D_ACT_NONE),
                 "cgan3d_conv3d_fwd: out_bf16 with a plain epilogue and accumulator statistics only");
  }
  CG_CHECK_ARG(!(e.out2 && (!e.minuend || g->cout != 1)), "cgan3d_conv3d_fwd: out2 needs minuend and cout==1");
  CG_CHECK_ARG(e.bn_mode >= 0 && e.bn_mode <= 2, "cgan3d_conv3d_fwd: bn_mode must be 0, 1 or 2");
  CG_CHECK_ARG(e.bn_mode != 2 || (e.bn_z && e.bn_ss && e.bn_mi), "cgan3d_conv3d_fwd: bn_mode 2 needs bn_z, bn_ss, bn_mi");
  if (e.bn_mode) {
    const long long slots = cgan3d_conv3d_bn_slots(g);
    CG_CHECK_ARG(slots > 0 && slots == e.bn_slots, "cgan3d_conv3d_fwd: bn_slots %d, the launch has %lld", e.bn_slots,
                 slots);
  }
  {  // mode-2 statistics (slab or accumulators) on the k7 path: only folded, on the bf16 input-grad kernel
    const bool m2 = e.bn_mode == 2 || e.fz.acc_mode == 4;
    CG_CHECK_ARG(!(m2 && g->k == 7 && g->cin == 1) || (e.bn_fold > 0 && k7m_fold_ok(g)),
                 "cgan3d_conv3d_fwd: bn_mode 2 on the k7 path only folded (bn_fold) on the bf16 input-grad kernel");
    CG_CHECK_ARG(e.bn_fold == 0 || (m2 && k7m_fold_ok(g) && g->do_ > 4 * e.bn_fold && g->ho > 4 * e.bn_fold &&
                                    g->wo > 4 * e.bn_fold),
                 "cgan3d_conv3d_fwd: bn_fold needs bn_mode 2 on a k7 bf16 input-grad geometry");
  }
  hipStream_t s = (hipStream_t)stream;
  CG_CHECK_ARG(!g->w_packed || (g->cout > 1 && (g->planar || !(g->k == 7 && g->stride == 1 && g->cin == 1))),
               "cgan3d_conv3d_fwd: packed weights only for the implicit-GEMM path");
  if (g->planar && g->cout > 1) {  // 2-D variants: the generic implicit GEMM for every cout >= 2 role
    CG_CHECK_ARG(!e.out2 && !e.x16 && !e.bn_fold, "cgan3d_conv3d_fwd: planar geometry epilogue");
    int rc = gemm_launch(g, x, w, y, e, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("conv_gemm_kernel");
    return CGAN3D_OK;
  }
  if (g->planar) goto cout1;  // cout == 1: the VALU kernels below
  CG_CHECK_ARG(e.act != CGAN3D_ACT_NEG_DTANH || (!g->planar && c1_dgrad_ok(g)),
               "cgan3d_conv3d_fwd: CGAN3D_ACT_NEG_DTANH only on the critic's first-layer input-grad");
  if (c1_fwd_ok(g) || c1_dgrad_ok(g)) {  // critic first layer (conv_c1.hip)
    CG_CHECK_ARG(!e.bn_mode, "cgan3d_conv3d_fwd: no BatchNorm statistics on the single-channel critic layer");
    CG_CHECK_ARG(!e.stats || c1_dgrad_blocks(g), "cgan3d_conv3d_fwd: stats on the critic's first layer: input-grad only");
    const int rc = g->transposed ? c1_dgrad_launch(g, x, w, y, e, s) : c1_fwd_launch(g, x, w, y, e, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("conv_c1");
    return CGAN3D_OK;
  }
  if (k7_try_fwd(g, x, w, y, e, s)) {
    CG_LAUNCH_CHECK("k7 conv");
    return CGAN3D_OK;
  }
cout1:
  if (g->cout == 1) {
    CG_CHECK_ARG(!e.stats && !e.bn_mode, "cgan3d_conv3d_fwd: stats unsupported for cout==1");
    ConvArgs a;
    CG_CHECK_ARG(make_args(g, &a, 256), "cgan3d_conv3d_fwd: transposed output dims must divide stride");
    size_t lds = (size_t)geom_taps(g) * g->cin * sizeof(float);
    CG_CHECK_ARG(lds <= 64 * 1024, "cgan3d_conv3d_fwd: cout==1 weights exceed LDS");
    const long long r4 = (long long)geom_taps(g) * g->cin / 4;
    if (!g->transposed && g->cin % 4 == 0 && a.class_vox <= 4096 && r4 <= 2048) {
      // very few outputs, long reductions: a block per output voxel
      ::cg::launch(conv_cout1_block_kernel, dim3((unsigned)a.class_vox), dim3(256), 0, s, a, x, w, y, e);
      CG_LAUNCH_CHECK("conv_cout1_block_kernel");
      return CGAN3D_OK;
    }
    if (!g->transposed && g->cin % 4 == 0 && a.class_vox <= 16384) {  // few outputs, long reductions
      ::cg::launch(conv_cout1_wave_kernel, dim3(cg::ceil_div(a.class_vox, 4)), dim3(256), lds, s, a, x, w, y, e);
      CG_LAUNCH_CHECK("conv_cout1_wave_kernel");
      return CGAN3D_OK;
    }
    ::cg::launch(conv_cout1_kernel, dim3(a.nclass * a.tiles_per_class), dim3(256), lds, s, a, x, w, y, e);
    CG_LAUNCH_CHECK("conv_cout1_kernel");
    return CGAN3D_OK;
  }
  if (g->w_packed == 3) {
    CG_CHECK_ARG(sk_ok(g), "cgan3d_conv3d_fwd: w_packed 3 on a geometry conv_sk does not take");
    int rc = sk_launch(g, x, reinterpret_cast<const __bf16*>(w), y, e, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("conv_sk_kernel");
    return CGAN3D_OK;
  }
  if (g->w_packed == 2) {
    CG_CHECK_ARG(halo_ok(g), "cgan3d_conv3d_fwd: w_packed 2 on a geometry the halo kernel does not take");
    CG_CHECK_ARG(!e.out2 && !e.minuend, "cgan3d_conv3d_fwd: halo kernel has no out2 epilogue");
    int rc = halo_launch(g, x, w, y, e, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("conv_halo_kernel");
    return CGAN3D_OK;
  }
  if (!g->w_packed && cin1t_ok(g)) {  // the critic's last-layer input-grad
    CG_CHECK_ARG(!e.stats && !e.bn_mode && !e.out2 && !e.minuend && !e.x16 && !e.fz.acc_mode,
                 "cgan3d_conv3d_fwd: cin == 1 transposed launch: bias / activation / mask / residual epilogue only");
    ConvArgs a;
    CG_CHECK_ARG(make_args(g, &a, 256), "cgan3d_conv3d_fwd: bad transposed geometry");
    const int nout = g->do_ * g->ho * g->wo * g->cout;
    const int bps = std::max(1, std::min(64, (nout + 255) / 256));
    ::cg::launch(conv_cin1t_kernel, dim3((unsigned)(g->n * bps)), dim3(256), 0, s, a, x, w, y, e, bps);
    CG_LAUNCH_CHECK("conv_cin1t_kernel");
    return CGAN3D_OK;
  }
  int rc = gemm_launch(g, x, w, y, e, s);
  if (rc) return rc;
  CG_LAUNCH_CHECK("conv_gemm_kernel");
  return CGAN3D_OK;
}

extern "C" int32_t cgan3d_conv3d_cin1t(const cgan3d_conv_geom* g) {
  return g && !validate(g, "cgan3d_conv3d_cin1t") && cin1t_ok(g) ? 1 : 0;
}

static long long wgrad_vpb(long long V, int gx_blocks) {
  // enough blocks to fill the chip (>= ~1024), but >= 256 voxels per block to bound atomics
  long long target = 2048 / (gx_blocks > 0 ? gx_blocks : 1);
  if (target < 1) target = 1;
  long long vpb = (V + target - 1) / target;
  if (vpb < 256) vpb = 256;
  return (vpb + 63) / 64 * 64;
}

// the generic bf16 weight grad as one deterministic launch pair (wgrad_bf16_launch); the shapes the
// dedicated kernels take are dispatched before it
static bool wgrad_bf16d_ok(const cgan3d_conv_geom* g) {
  return !g->planar && g->cout != 1 && wgrad_bf16_ok(g) && !(g->k == 7 && g->stride == 1 && (g->cin == 1 || g->cout == 1)) &&
         !c1_wgrad_ok(g) && !wgrad_c1_ok(g) && !wgrad_s2_ok(g) && !wgrad_k3_ok(g);
}

extern "C" int64_t cgan3d_conv3d_wgrad_ws_floats(const cgan3d_conv_geom* g) {
  if (!g) return -1;
  if (g->planar) return (int64_t)geom_taps(g) * g->cin * g->cout;
  if (wgrad_bf16d_ok(g)) return std::max<int64_t>(wgrad_bf16_ws_floats(g), (int64_t)g->k * g->k * g->k * g->cin * g->cout);
  return std::max<int64_t>(std::max<int64_t>((int64_t)g->k * g->k * g->k * g->cin * g->cout, k7_wgrad_ws_floats(g)),
                           std::max<int64_t>(std::max<int64_t>(wgrad_k3_ws_floats(g), wgrad_s2_ws_floats(g)),
                                             c1_wgrad_ws_floats(g)));
}

extern "C" int cgan3d_conv3d_wgrad(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw,
                                   int32_t accumulate, float* ws, void* stream) {
  return cgan3d_conv3d_wgrad_ex(g, gathered, aligned, dw, accumulate, ws, nullptr, nullptr, stream);
}

// 1 if the weight gradient of `g` sums into the workspace by atomics (then zeroed by a memset,
// or kept clean under CGAN3D_WGRAD_WS_CLEAN), 0 if it needs no zeroed workspace
static int wgrad_ws_atomic(const cgan3d_conv_geom* g) {
  if (g->planar) return 1;
  return !k7_wgrad_handles(g) && !c1_wgrad_ok(g) && !wgrad_c1_ok(g) && !wgrad_s2_ok(g) && !wgrad_k3_ok(g) &&
         !wgrad_bf16d_ok(g);
}

extern "C" int cgan3d_conv3d_wgrad_ws_mode(const cgan3d_conv_geom* g) {
  if (validate(g, "cgan3d_conv3d_wgrad_ws_mode")) return -1;
  return wgrad_ws_atomic(g);
}

extern "C" int32_t cgan3d_conv3d_bn_fold_ok(const cgan3d_conv_geom* g) {
  return g && !validate(g, "cgan3d_conv3d_bn_fold_ok") && !g->planar && k7m_fold_ok(g) ? 1 : 0;
}

extern "C" int32_t cgan3d_conv3d_shadow_only(const cgan3d_conv_geom* g, int32_t role) {
  if (!g || validate(g, "cgan3d_conv3d_shadow_only") || g->planar) return 0;
  if (role == 0)  // stride-2 16 <-> 32 kernels (conv_s2.hip), the 16 -> 1 k7 forward (conv_k7_mfma.hip), the
                  // ResNet-block kernel (conv_k3m.hip: its halo only ever comes from x_bf16)
    return (g->w_packed == 2 && s2_kind(g) != 0) || k7m_w2n_taken(g) || k3m_route(g) ? 1 : 0;
  if (role != 1 || g->transposed) return 0;
  if (g->k == 7 && g->stride == 1 && (g->cin == 1 || g->cout == 1)) return k7m_wgrad_taken(g);
  if (c1_wgrad_ok(g) || wgrad_c1_ok(g)) return 0;
  return wgrad_s2_ok(g) || wgrad_k3_ok(g) ? 1 : 0;
}

extern "C" int cgan3d_conv3d_wgrad_ex(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw,
                                      int32_t accumulate, float* ws, const void* gathered_bf16,
                                      const void* aligned_bf16, void* stream) {
  int st = validate(g, "cgan3d_conv3d_wgrad");
  if (st) return st;
  CG_CHECK_ARG((accumulate & ~15) == 0,
               "cgan3d_conv3d_wgrad: flags are CGAN3D_WGRAD_ACCUMULATE | CGAN3D_WGRAD_WS_CLEAN | "
               "CGAN3D_WGRAD_DEFER_UNPACK | CGAN3D_WGRAD_DEFER_REDUCE");
  const bool ws_clean = (accumulate & CGAN3D_WGRAD_WS_CLEAN) != 0;
  const bool defer = (accumulate & CGAN3D_WGRAD_DEFER_UNPACK) != 0;
  const bool defer_reduce = (accumulate & CGAN3D_WGRAD_DEFER_REDUCE) != 0;
  CG_CHECK_ARG(!defer_reduce || (!g->planar && wgrad_k3_partials(g) > 0),
               "cgan3d_conv3d_wgrad: CGAN3D_WGRAD_DEFER_REDUCE on a geometry without partials (cgan3d_conv3d_wgrad_partials)");
  CG_CHECK_ARG(!defer || (ws_clean && wgrad_ws_atomic(g)),
               "cgan3d_conv3d_wgrad: CGAN3D_WGRAD_DEFER_UNPACK needs CGAN3D_WGRAD_WS_CLEAN on an atomic-workspace "
               "geometry");
  accumulate &= CGAN3D_WGRAD_ACCUMULATE;
  CG_CHECK_ARG(!ws_clean || wgrad_ws_atomic(g),
               "cgan3d_conv3d_wgrad: CGAN3D_WGRAD_WS_CLEAN on a geometry whose workspace is not atomic "
               "(cgan3d_conv3d_wgrad_ws_mode() == 0)");
  CG_CHECK_ARG(!g->transposed, "cgan3d_conv3d_wgrad: use the forward mapping (see header)");
  CG_CHECK_ARG(gathered && aligned && dw && ws, "cgan3d_conv3d_wgrad: null pointer");
  CG_CHECK_ARG(g->cout == 1 || g->cout % 4 == 0, "cgan3d_conv3d_wgrad: cout must be 1 or a multiple of 4");
  hipStream_t s = (hipStream_t)stream;
  ConvArgs a;
  make_args(g, &a, 64);
  const int T = geom_taps(g);
  const long long R = (long long)T * g->cin;
  const long long V = (long long)g->n * g->do_ * g->ho * g->wo;
  if (g->planar) goto generic;  // 2-D variants: the generic f32 weight-gradient kernels below
  if (g->k == 7 && g->stride == 1 && (g->cin == 1 || g->cout == 1)) {
    if (!accumulate && ::cg::memset_async(dw, 0, R * g->cout * sizeof(float), s) != hipSuccess) {
      set_error("cgan3d_conv3d_wgrad: memset failed");
      return CGAN3D_EHIP;
    }
    // the 16-channel side may come from its bf16 shadow (gathered for a 16 -> 1 conv, aligned for 1 -> 16)
    const __bf16* w16 = reinterpret_cast<const __bf16*>(g->cout == 1 ? gathered_bf16 : aligned_bf16);
    if (k7_try_wgrad(g, gathered, aligned, dw, ws, s, w16)) {
      CG_LAUNCH_CHECK("k7 wgrad");
      return CGAN3D_OK;
    }
    CG_CHECK_ARG(!accumulate, "cgan3d_conv3d_wgrad: internal dispatch error");
  }
  if (c1_wgrad_ok(g)) {  // critic first layer: LDS-window kernel, per-block partials in ws, summed in order
    if (!accumulate && ::cg::memset_async(dw, 0, R * g->cout * sizeof(float), s) != hipSuccess) {
      set_error("cgan3d_conv3d_wgrad: memset failed");
      return CGAN3D_EHIP;
    }
    const int rc = c1_wgrad_launch(g, gathered, aligned, dw, ws, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("c1_wgrad_kernel");
    return CGAN3D_OK;
  }
  if (wgrad_c1_ok(g)) {  // single-channel input: straight into dW, no workspace
    if (!accumulate && ::cg::memset_async(dw, 0, R * g->cout * sizeof(float), s) != hipSuccess) {
      set_error("cgan3d_conv3d_wgrad: memset failed");
      return CGAN3D_EHIP;
    }
    wgrad_c1_launch(g, gathered, aligned, dw, s);
    CG_LAUNCH_CHECK("conv_wgrad_c1_kernel");
    return CGAN3D_OK;
  }
  if (wgrad_s2_ok(g)) {  // stride-2 16 <-> 32 levels: per-block partials + reduce, no memset
    int rc = wgrad_s2_launch(g, gathered, aligned, reinterpret_cast<const __bf16*>(gathered_bf16),
                             reinterpret_cast<const __bf16*>(aligned_bf16), dw, accumulate, ws, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("wgrad_s2_kernel");
    return CGAN3D_OK;
  }
  if (wgrad_k3_ok(g)) {  // ResNet-block shape: per-block partials + reduce, no memset
    int rc = wgrad_k3_launch(g, gathered, aligned, reinterpret_cast<const __bf16*>(gathered_bf16),
                             reinterpret_cast<const __bf16*>(aligned_bf16), dw, accumulate, ws, s, defer_reduce);
    if (rc) return rc;
    CG_LAUNCH_CHECK("wgrad_k3_kernel");
    return CGAN3D_OK;
  }
  if (wgrad_bf16d_ok(g)) {  // other bf16 shapes: partial slabs in ws + their ordered sum into dw, no memset
    int rc = wgrad_bf16_launch(g, gathered, aligned, dw, ws, accumulate, s);
    if (rc) return rc;
    CG_LAUNCH_CHECK("conv_wgrad_bf16_kernel");
    return CGAN3D_OK;
  }
generic:
  if (!ws_clean && ::cg::memset_async(ws, 0, R * g->cout * sizeof(float), s) != hipSuccess) {
    set_error("cgan3d_conv3d_wgrad: memset failed");
    return CGAN3D_EHIP;
  }
  if (g->cout == 1) {
    CG_CHECK_ARG(g->cin % 4 == 0, "cgan3d_conv3d_wgrad: cout==1 needs cin%%4==0");
    const long long R4 = R / 4;
    // one float4 of (tap, channel) accumulators per thread; r4 chunks over blockIdx.y, voxels over x
    const int gy = cg::ceil_div(R4, 256);
    // voxels per block: >= 8 so that a few hundred outputs (the critic's last layer: 12 x 27) still
    // spread over ~160 blocks — each block's voxel loop is a chain of dependent L2 round trips
    // (64 voxels per block: 25.7 us at 64^3 B=4; rocprof, profiles/r02_*)
    long long vpb = (V * gy + 1023) / 1024;
    if (vpb < 8) vpb = 8;
    vpb = (vpb + 7) / 8 * 8;
    dim3 grid(cg::ceil_div(V, vpb), gy);
    ::cg::launch((conv_wgrad_cout1_kernel<1>), grid, dim3(256), 0, s, a, gathered, aligned, ws, vpb);
    CG_LAUNCH_CHECK("conv_wgrad_cout1_kernel");
  } else {
    const int gxb = cg::ceil_div(R, 64);
    const int gz = cg::ceil_div(g->cout, 64);  // 64-channel blocks (cout > 64: 2-D critic)
    long long vpb = wgrad_vpb(V, gxb * gz);
    dim3 grid(gxb, cg::ceil_div(V, vpb), gz);
    const int nb = std::min(4, (g->cout + 15) / 16);
    const bool v4 = (g->cin % 4) == 0;
#define CG_LAUNCH_WG(VV, N) ::cg::launch((conv_wgrad_kernel<VV, N>), grid, dim3(256), 0, s, a, gathered, aligned, ws, vpb)
    if (v4) {
      if (nb == 1) CG_LAUNCH_WG(4, 1); else if (nb == 2) CG_LAUNCH_WG(4, 2); else if (nb == 3) CG_LAUNCH_WG(4, 3); else CG_LAUNCH_WG(4, 4);
    } else {
      if (nb == 1) CG_LAUNCH_WG(1, 1); else if (nb == 2) CG_LAUNCH_WG(1, 2); else if (nb == 3) CG_LAUNCH_WG(1, 3); else CG_LAUNCH_WG(1, 4);
    }
#undef CG_LAUNCH_WG
    CG_LAUNCH_CHECK("conv_wgrad_kernel");
  }
  if (defer) return CGAN3D_OK;  // the caller's cgan3d_wgrad_unpack_multi moves it into dw
  const long long total = R * g->cout;
  CG_CHECK_ARG(total < (1LL << 31), "wgrad unpack: weight too large for 32-bit indexing");
  ::cg::launch(wgrad_unpack_kernel, dim3(cg::ceil_div(total, 256)), dim3(256), 0, s, ws, dw, T, g->cin, g->cout,
                     (long long)g->w_sa, (long long)g->w_sb, accumulate, (int)ws_clean);
  CG_LAUNCH_CHECK("wgrad_unpack_kernel");
  return CGAN3D_OK;
}

// the weight gradient of g runs the generic bf16 kernel into an atomic workspace (the dispatch of
// cgan3d_conv3d_wgrad_ex above reaches wgrad_bf16_launch)
extern "C" int32_t cgan3d_conv3d_wgrad_group_ok(const cgan3d_conv_geom* g) {
  if (!g || validate(g, "cgan3d_conv3d_wgrad_group_ok") || g->planar || g->transposed || g->cout == 1) return 0;
  if (g->k == 7 && g->stride == 1 && (g->cin == 1 || g->cout == 1)) return 0;
  if (c1_wgrad_ok(g) || wgrad_c1_ok(g) || wgrad_s2_ok(g) || wgrad_k3_ok(g)) return 0;
  return wgrad_bf16_ok(g) ? 1 : 0;
}

extern "C" int cgan3d_conv3d_wgrad_group(const cgan3d_conv_geom* geoms, const float* const* gathered,
                                         const float* const* aligned, float* const* ws, int32_t n, void* stream) {
  CG_CHECK_ARG(geoms && gathered && aligned && ws && n > 0 && n <= 4, "cgan3d_conv3d_wgrad_group: 1..4 items");
  for (int i = 0; i < n; ++i) {
    CG_CHECK_ARG(cgan3d_conv3d_wgrad_group_ok(&geoms[i]), "cgan3d_conv3d_wgrad_group: item %d is not a generic bf16 "
                 "weight gradient (cgan3d_conv3d_wgrad_group_ok)", i);
    CG_CHECK_ARG(gathered[i] && aligned[i] && ws[i], "cgan3d_conv3d_wgrad_group: null pointer in item %d", i);
  }
  wgrad_bf16_group_launch(geoms, gathered, aligned, ws, n, (hipStream_t)stream);
  CG_LAUNCH_CHECK("conv_wgrad_bf16_group_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_wgrad_unpack_multi(const cgan3d_unpack_desc* descs, int32_t n, int64_t max_total, void* stream) {
  CG_CHECK_ARG(descs && n > 0 && n <= 65535 && max_total > 0 && max_total < (1LL << 31),
               "cgan3d_wgrad_unpack_multi: need a device descriptor array, 0 < n <= 65535, 0 < max_total < 2^31");
  const unsigned bx = (unsigned)std::min<long long>((max_total + 255) / 256, 1024);
  ::cg::launch(wgrad_unpack_multi_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, descs);
  CG_LAUNCH_CHECK("wgrad_unpack_multi_kernel");
  return CGAN3D_OK;
}
