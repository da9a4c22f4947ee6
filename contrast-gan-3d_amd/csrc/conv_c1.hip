// The critic's single-channel first layer (model/discriminator.py:24-39: Conv3d 1 -> 8, k4 s2 p1,
// bias, LeakyReLU 0.2) in its three roles — forward (also the gradient-penalty forward-mode
// chain, mask epilogue), input-grad (ConvTranspose-shaped, 8 -> 1, only for the interpolated
// samples whose dD/dx the penalty needs) and weight-grad.  One input channel means no channel
// contraction to put on MFMA: these are exact fp32 FMA kernels that read each input voxel once
// through an LDS window and are bound by HBM/L2 traffic (12 x 64^3 inputs per step), not by the
// ~0.4 GFLOP they do.  Tiles: 2 x 8 x 16 output voxels (z, y, x), one per thread.
#include "common.h"

namespace cg {

struct C1Args {
  int n, di, hi, wi, do_, ho, wo;  // gathered (stride-2 input) dims, output dims (fwd roles)
  int tz, ty, tx;                  // tiles per dim
  long long w_sa, w_sb;            // weight strides (input-channel side, output-channel side)
  int tiles_per_block;             // wgrad
};

namespace c1 {
constexpr int TZ = 2, TY = 8, TX = 16;                 // output tile
constexpr int WZ = 2 * TZ + 2, WY = 2 * TY + 2, WX = 2 * TX + 2;  // k4 s2 p1 input window (6 x 18 x 34)
constexpr int RS = 36, PS = 656;                        // LDS row / plane strides (floats): 36 = 4 mod 32,
                                                        // 656 = 16 mod 32 (conflict-free tap-lane reads)
constexpr int WIN = WZ * PS;
}  // namespace c1

// stage the k4 s2 p1 input window of output tile (n, oz0, oy0, ox0) into xs (zero outside); every
// load of the thread is issued before the first LDS store
__device__ __forceinline__ void c1_stage_window(const C1Args& a, const float* __restrict__ x, int nb, int oz0, int oy0,
                                                int ox0, float* xs) {
  using namespace c1;
  constexpr int N = WZ * WY * WX, PER = (N + 255) / 256;
  const int iz0 = 2 * oz0 - 1, iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
  // unconditional loads (clamped index, value masked after: no branch per load), 32-bit offsets
  // within the sample (a sample's volume is far below 2^31 voxels)
  const float* xn = x + (long long)nb * a.di * a.hi * a.wi;
  float v[PER];
  unsigned okm = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int hx = i % WX, r = i / WX, hy = r % WY, hz = r / WY;
    const int iz = iz0 + hz, iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = i < N && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi;
    v[k] = xn[ok ? (iz * a.hi + iy) * a.wi + ix : 0];
    okm |= ok ? 1u << k : 0u;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int hx = i % WX, r = i / WX, hy = r % WY, hz = r / WY;
    if (k + 1 < PER || i < N) xs[hz * PS + hy * RS + hx] = keep_if((okm >> k) & 1u, v[k]);
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __attribute__((aligned(16))) float g_c1_zero[8];  // source of the absent epilogue operands

__device__ __forceinline__ void c1_tile(const C1Args& a, int t, int* nb, int* oz0, int* oy0, int* ox0) {
  const int tx = t % a.tx, r = t / a.tx, ty = r % a.ty, r2 = r / a.ty, tz = r2 % a.tz;
  *nb = r2 / a.tz;
  *oz0 = tz * c1::TZ; *oy0 = ty * c1::TY; *ox0 = tx * c1::TX;
}

// y[o][b] = epi(sum_t x[2o - 1 + t] * w[b][t]), 8 output channels
__global__ __launch_bounds__(256) void c1_fwd_kernel(C1Args a, const float* __restrict__ x, const float* __restrict__ w,
                                                     float* y, Epi ep) {
  using namespace c1;
  __shared__ __attribute__((aligned(16))) float xs[WIN];
  __shared__ __attribute__((aligned(16))) float wsh[64 * 8];  // [tap][b]
  int nb, oz0, oy0, ox0;
  c1_tile(a, blockIdx.x, &nb, &oz0, &oy0, &ox0);
  const int tid = threadIdx.x;
  // both weight loads in flight with the window's (a loop here waited for each in turn)
  const float wv0 = w[(tid & 7) * a.w_sb + (tid >> 3)], wv1 = w[(tid & 7) * a.w_sb + ((tid + 256) >> 3)];
  c1_stage_window(a, x, nb, oz0, oy0, ox0, xs);
  wsh[tid] = wv0;
  wsh[tid + 256] = wv1;
  __syncthreads();
  const int lz = tid >> 7, ly = (tid >> 4) & 7, lx = tid & 15;
  // epilogue operands before the taps (unconditional loads, absent ones from a zero dummy): bias,
  // the LeakyReLU mask of the penalty's forward-mode chain
  const int oz = oz0 + lz, oy = oy0 + ly, ox = ox0 + lx;
  const bool inside = oz < a.do_ && oy < a.ho && ox < a.wo;
  const long long o = inside ? (((long long)nb * a.do_ + oz) * a.ho + oy) * a.wo + ox : 0;
  const bool has_bias = ep.bias != nullptr, has_mask = ep.mask_src != nullptr;
  // integer selects, the pointers made opaque: a select between two load addresses becomes a
  // branch around the load otherwise
  uintptr_t ba = has_bias ? (uintptr_t)ep.bias : (uintptr_t)g_c1_zero;
  uintptr_t ma = has_mask ? (uintptr_t)(ep.mask_src + o * 8) : (uintptr_t)g_c1_zero;
  asm volatile("" : "+s"(ba));
  asm volatile("" : "+v"(ma));
  const f32x4* bp = reinterpret_cast<const f32x4*>(ba);
  const f32x4* mp = reinterpret_cast<const f32x4*>(ma);
  const f32x4 b0 = bp[0], b1 = bp[1], m0 = mp[0], m1 = mp[1];
  f32x2 acc[4];  // channel pairs (2j, 2j + 1): packed fp32 FMA
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x2{0.f, 0.f};
  // (td, th) rolled: unrolled, the compiler hoists all 128 weight reads into registers and spills
#pragma unroll 1
  for (int tdh = 0; tdh < 16; ++tdh)
#pragma unroll
      for (int tw = 0; tw < 4; tw += 2) {
        const int td = tdh >> 2, th = tdh & 3;
        const float2 v = *reinterpret_cast<const float2*>(xs + (2 * lz + td) * PS + (2 * ly + th) * RS + 2 * lx + tw);
        const int t = tdh * 4 + tw;
        const f32x4* wt = reinterpret_cast<const f32x4*>(wsh + t * 8);  // broadcast reads
        const f32x4 w0 = wt[0], w1 = wt[1], w2 = wt[2], w3 = wt[3];
        const f32x2 vx = {v.x, v.x}, vy = {v.y, v.y};
        acc[0] += vx * f32x2{w0[0], w0[1]} + vy * f32x2{w2[0], w2[1]};
        acc[1] += vx * f32x2{w0[2], w0[3]} + vy * f32x2{w2[2], w2[3]};
        acc[2] += vx * f32x2{w1[0], w1[1]} + vy * f32x2{w3[0], w3[1]};
        acc[3] += vx * f32x2{w1[2], w1[3]} + vy * f32x2{w3[2], w3[3]};
      }
  // branch-free epilogue: uniform selects
  const bool relu = ep.act == CGAN3D_ACT_RELU, lrelu = ep.act == CGAN3D_ACT_LRELU;
  const float slope = ep.slope;
  float v[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    float t = acc[b >> 1][b & 1] + (b < 4 ? b0[b & 3] : b1[b & 3]);
    t = relu ? fmaxf(t, 0.f) : t;
    t = (lrelu & (t < 0.f)) ? t * slope : t;
    const float m = b < 4 ? m0[b & 3] : m1[b & 3];
    v[b] = (has_mask & !(m > 0.f)) ? t * slope : t;
  }
  if (!inside) return;
  *reinterpret_cast<f32x4*>(y + o * 8) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(y + o * 8 + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

// input-grad: dx[i] = sum_{t, o : i = 2o - 1 + t} sum_c dz[o][c] * w[c][t]  (i on the fine grid)
// a.di.. = coarse (dz) dims, a.do_.. = fine (dx) dims; tile = 2 x 8 x 16 fine voxels
// res / tnh (CGAN3D_ACT_NEG_DTANH): dx = res - acc * (1 - tnh^2), in place over res allowed.
// sq (optional): sq[block] = sum of dx^2 over the block's outputs (the gradient penalty's per-sample
// norms, cgan3d_gradient_penalty_part: a block never spans two samples)
__global__ __launch_bounds__(256) void c1_dgrad_kernel(C1Args a, const float* __restrict__ dz,
                                                       const float* __restrict__ w, float* dx, const float* res,
                                                       const float* __restrict__ tnh, float* sq) {
  constexpr int GZ = c1::TZ / 2 + 2, GY = c1::TY / 2 + 2, GX = c1::TX / 2 + 2;  // coarse window 3 x 6 x 10
  __shared__ __attribute__((aligned(16))) float gs[GZ * GY * GX * 8];
  __shared__ __attribute__((aligned(16))) float ws[64 * 8];  // [tap][c]
  int nb, oz0, oy0, ox0;
  c1_tile(a, blockIdx.x, &nb, &oz0, &oy0, &ox0);
  const int tid = threadIdx.x;
  const int cz0 = oz0 / 2 - 1, cy0 = oy0 / 2 - 1, cx0 = ox0 / 2 - 1;
  // every global load of the thread (2 weights, <= 3 float4 halves of 8-channel voxels) in flight
  // before the first LDS store
  constexpr int NG = GZ * GY * GX * 2, PER = (NG + 255) / 256;
  const float w0 = w[(tid & 7) * a.w_sa + (tid >> 3)], w1 = w[(tid & 7) * a.w_sa + ((tid + 256) >> 3)];
  // unconditional loads from clamped offsets, masked at the LDS store (no branch per load)
  const float* dzn = dz + (long long)nb * a.di * a.hi * a.wi * 8;
  f32x4 gv[PER];
  unsigned okm = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = tid + 256 * k, h = i & 1, v = i >> 1;
    const int gx = v % GX, r = v / GX, gy = r % GY, gz = r / GY;
    const int cz = cz0 + gz, cy = cy0 + gy, cx = cx0 + gx;
    const bool ok = i < NG && (unsigned)cz < (unsigned)a.di && (unsigned)cy < (unsigned)a.hi && (unsigned)cx < (unsigned)a.wi;
    gv[k] = *reinterpret_cast<const f32x4*>(dzn + (ok ? ((cz * a.hi + cy) * a.wi + cx) * 8 + 4 * h : 0));
    okm |= ok ? 1u << k : 0u;
  }
  // the epilogue's operands (penalty fold: residual, tanh) before the taps as well
  const int lz = tid >> 7, ly = (tid >> 4) & 7, lx = tid & 15;
  const int oz = oz0 + lz, oy = oy0 + ly, ox = ox0 + lx;
  const bool inside = oz < a.do_ && oy < a.ho && ox < a.wo;
  const long long o = inside ? (((long long)nb * a.do_ + oz) * a.ho + oy) * a.wo + ox : 0;
  const bool fold = tnh != nullptr;
  uintptr_t pt = fold ? (uintptr_t)tnh : (uintptr_t)g_c1_zero, pr = fold ? (uintptr_t)res : (uintptr_t)g_c1_zero;
  asm volatile("" : "+s"(pt), "+s"(pr));
  const float tv = reinterpret_cast<const float*>(pt)[fold ? o : 0], rv = reinterpret_cast<const float*>(pr)[fold ? o : 0];
  ws[tid] = w0;
  ws[tid + 256] = w1;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (tid + 256 * k < NG) {
      const bool ok = (okm >> k) & 1u;
      f32x4 m;
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = keep_if(ok, gv[k][e]);
      *reinterpret_cast<f32x4*>(gs + (tid + 256 * k) * 4) = m;
    }
  }
  __syncthreads();
  // per dim: taps t = ((o + 1) & 1) + 2j, coarse o' = (o + 1 - t) / 2, local = o' - c0
  float acc = 0.f;
#pragma unroll
  for (int jz = 0; jz < 2; ++jz)
#pragma unroll
    for (int jy = 0; jy < 2; ++jy)
#pragma unroll
      for (int jx = 0; jx < 2; ++jx) {
        const int tz = ((oz + 1) & 1) + 2 * jz, ty = ((oy + 1) & 1) + 2 * jy, tx = ((ox + 1) & 1) + 2 * jx;
        const int gz = (oz + 1 - tz) / 2 - cz0, gy = (oy + 1 - ty) / 2 - cy0, gx = (ox + 1 - tx) / 2 - cx0;
        const float* gv = gs + ((gz * GY + gy) * GX + gx) * 8;
        const float* wv = ws + ((tz * 4 + ty) * 4 + tx) * 8;
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(gv), g1 = *reinterpret_cast<const f32x4*>(gv + 4);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wv), w1 = *reinterpret_cast<const f32x4*>(wv + 4);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc = fmaf(g0[c], w0[c], acc);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc = fmaf(g1[c], w1[c], acc);
      }
  if (fold) acc = rv - acc * (1.f - tv * tv);
  if (inside) dx[o] = acc;
  if (sq) {  // the block's sum of squares: waves by shuffles, then 4 partials through LDS (ws is free)
    float v = inside ? acc * acc : 0.f;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
    __syncthreads();
    if ((tid & 63) == 0) ws[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) sq[blockIdx.x] = (ws[0] + ws[1]) + (ws[2] + ws[3]);
  }
}

// weight-grad: dw[b][t] += sum_{n,o} x[2o - 1 + t] * dz[o][b]; lane = tap.  G groups of 4 waves per
// block, each reducing its own tiles (tiles t0 + g, t0 + g + G, ...) through its own LDS window, the
// 4 waves of a group splitting a tile's voxels; one atomic add per (b, t) per block at the end (every
// block adds into the same 512 words, so fewer, longer blocks; the groups give each SIMD G waves to
// hide the LDS latency of the voxel loop with).  The next tile's window + dz stay in registers while
// the current one is reduced.
template <int G>
__global__ __launch_bounds__(256 * G) void c1_wgrad_kernel(C1Args a, const float* __restrict__ x,
                                                           const float* __restrict__ dz, float* part, int ntiles) {
  using namespace c1;
  __shared__ __attribute__((aligned(16))) float xs_all[G][WIN];
  __shared__ __attribute__((aligned(16))) float gs_all[G][TZ * TY * TX * 8];
  __shared__ float red[4 * G][8][65];
  constexpr int N = WZ * WY * WX, PER = (N + 255) / 256;
  const int tid = threadIdx.x & 255, grp = threadIdx.x >> 8, t = tid & 63, vg = tid >> 6;
  const int td = t >> 4, th = (t >> 2) & 3, tw = t & 3;
  float* const xs = xs_all[grp];
  float* const gs = gs_all[grp];
  float xv_n[PER];
  f32x4 gv_n[2];
  unsigned okm = 0;  // validity of the staged values (unconditional loads, masked at the LDS store)
  auto load = [&](int tile) {
    int nb, oz0, oy0, ox0;
    c1_tile(a, tile, &nb, &oz0, &oy0, &ox0);
    const int iz0 = 2 * oz0 - 1, iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
    const float* xn = x + (long long)nb * a.di * a.hi * a.wi;
    const float* gn = dz + (long long)nb * a.do_ * a.ho * a.wo * 8;
    okm = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + 256 * k;
      const int hx = i % WX, r = i / WX, hy = r % WY, hz = r / WY;
      const int iz = iz0 + hz, iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = i < N && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi;
      xv_n[k] = xn[ok ? (iz * a.hi + iy) * a.wi + ix : 0];
      okm |= ok ? 1u << k : 0u;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k, h = i & 1, v = i >> 1;
      const int oz = oz0 + (v >> 7), oy = oy0 + ((v >> 4) & 7), ox = ox0 + (v & 15);
      const bool ok = oz < a.do_ && oy < a.ho && ox < a.wo;
      gv_n[k] = *reinterpret_cast<const f32x4*>(gn + (ok ? ((oz * a.ho + oy) * a.wo + ox) * 8 + 4 * h : 0));
      okm |= ok ? 1u << (PER + k) : 0u;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + 256 * k;
      const int hx = i % WX, r = i / WX, hy = r % WY, hz = r / WY;
      if (k + 1 < PER || i < N) xs[hz * PS + hy * RS + hx] = keep_if((okm >> k) & 1u, xv_n[k]);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool ok = (okm >> (PER + k)) & 1u;
      f32x4 g;
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = keep_if(ok, gv_n[k][e]);
      *reinterpret_cast<f32x4*>(gs + (tid + 256 * k) * 4) = g;
    }
  };
  f32x2 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x2{0.f, 0.f};
  const int t0 = blockIdx.x * a.tiles_per_block;
  const int t1 = min(t0 + a.tiles_per_block, ntiles);
  const int iters = (t1 - t0 + G - 1) / G;  // block-uniform: every group meets every barrier
  if (t0 + grp < t1) load(t0 + grp);
  for (int it = 0; it < iters; ++it) {
    const int tile = t0 + it * G + grp;
    lds_barrier();  // previous tile's LDS reads done
    if (tile < t1) store();
    lds_barrier();
    if (tile + G < t1) load(tile + G);
    if (tile < t1) {
#pragma unroll 8
      for (int v = vg * 64; v < vg * 64 + 64; ++v) {
        const int lz = v >> 7, ly = (v >> 4) & 7, lx = v & 15;
        const float xv = xs[(2 * lz + td) * PS + (2 * ly + th) * RS + 2 * lx + tw];
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(gs + v * 8), g1 = *reinterpret_cast<const f32x4*>(gs + v * 8 + 4);
        const f32x2 x2 = {xv, xv};
        acc[0] += x2 * f32x2{g0[0], g0[1]};
        acc[1] += x2 * f32x2{g0[2], g0[3]};
        acc[2] += x2 * f32x2{g1[0], g1[1]};
        acc[3] += x2 * f32x2{g1[2], g1[3]};
      }
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int b = 0; b < 8; ++b) red[w][b][t] = acc[b >> 1][b & 1];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256 * G) {
    const int b = i >> 6, tt = i & 63;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4 * G; ++k) s += red[k][b][tt];
    part[(long long)blockIdx.x * 512 + i] = s;  // i = b * 64 + tt (colsum_kernel adds the rows in order)
  }
}


// roles this file takes (geometries as built by cgan3d_amd/ops.py)
bool c1_fwd_ok(const cgan3d_conv_geom* g) {
  return !g->transposed && !g->reflect && g->cin == 1 && g->cout == 8 && g->k == 4 && g->stride == 2 && g->pad == 1 &&
         g->w_packed == 0;
}
bool c1_dgrad_ok(const cgan3d_conv_geom* g) {
  return g->transposed && !g->reflect && g->cin == 8 && g->cout == 1 && g->k == 4 && g->stride == 2 && g->pad == 1 &&
         g->w_packed == 0 && g->do_ % 2 == 0 && g->ho % 2 == 0 && g->wo % 2 == 0;
}
bool c1_wgrad_ok(const cgan3d_conv_geom* g) { return c1_fwd_ok(g); }

long long c1_dgrad_blocks(const cgan3d_conv_geom* g) {  // per-block sum-of-squares slots (cgan3d_conv3d_sumsq_blocks)
  if (g->planar || !c1_dgrad_ok(g)) return 0;
  return (long long)g->n * ceil_div(g->do_, c1::TZ) * ceil_div(g->ho, c1::TY) * ceil_div(g->wo, c1::TX);
}

static C1Args c1_args(const cgan3d_conv_geom* g) {
  C1Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.tz = ceil_div(g->do_, c1::TZ); a.ty = ceil_div(g->ho, c1::TY); a.tx = ceil_div(g->wo, c1::TX);
  a.w_sa = g->w_sa; a.w_sb = g->w_sb;
  a.tiles_per_block = 1;
  return a;
}

int c1_fwd_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st) {
  CG_CHECK_ARG(!e.residual && !e.minuend && !e.out2 && !e.stats && !e.bn_mode,
               "conv c1: only bias / activation / mask epilogues");
  C1Args a = c1_args(g);
  ::cg::launch(c1_fwd_kernel, dim3(a.n * a.tz * a.ty * a.tx), dim3(256), 0, st, a, x, w, y, e);
  return CGAN3D_OK;
}

int c1_dgrad_launch(const cgan3d_conv_geom* g, const float* dz, const float* w, float* dx, const Epi& e,
                    hipStream_t st) {
  const bool fold = e.act == CGAN3D_ACT_NEG_DTANH;
  CG_CHECK_ARG(!e.bias && !e.minuend && !e.out2 && !e.bn_mode &&
                   (fold ? (e.residual && e.mask_src) : (e.act == CGAN3D_ACT_NONE && !e.residual && !e.mask_src)),
               "conv c1 input-grad: no epilogue but CGAN3D_ACT_NEG_DTANH (residual + mask_src)");
  C1Args a = c1_args(g);
  ::cg::launch(c1_dgrad_kernel, dim3(a.n * a.tz * a.ty * a.tx), dim3(256), 0, st, a, dz, w, dx,
               fold ? e.residual : nullptr, fold ? e.mask_src : nullptr, e.stats);
  return CGAN3D_OK;
}

// per-block partial rows [block][8 x 64] in ws (c1_wgrad_ws_floats), summed into dW in block order by
// colsum_kernel (round 6: the blocks' atomics into dW made the gradient order-dependent)
static int c1_wgrad_grid(const C1Args& a0, int* tpb) {
  const int ntiles = a0.n * a0.tz * a0.ty * a0.tx;
  // at most ~192 blocks (measured: 1024 blocks of one tile each, 36 -> 47 us at 64^3 B=4; 192 blocks of 8
  // tiles at 12 x 64^3 leave CUs to the main stream's kernels: A/B 1.447 / 1.443 / 1.455 vs 1.471 / 1.473 /
  // 1.472 ms/step at 256 blocks).  Small grids keep one tile per block (ntiles / 192 rounds to 0-1).
  *tpb = std::max(1, ntiles / 192);
  return ceil_div(ntiles, *tpb);
}

// a bound for every batch up to g->n (the grid is not monotone in the tile count: 383 tiles take 383
// blocks, 384 take 192), so a workspace sized at the largest batch serves the smaller ones
long long c1_wgrad_ws_floats(const cgan3d_conv_geom* g) {
  if (!c1_wgrad_ok(g)) return 0;
  const C1Args a = c1_args(g);
  return (long long)std::min(a.n * a.tz * a.ty * a.tx, 2 * 192) * 512;
}

int c1_wgrad_launch(const cgan3d_conv_geom* g, const float* x, const float* dz, float* dw, float* ws, hipStream_t st) {
  C1Args a = c1_args(g);
  const int ntiles = a.n * a.tz * a.ty * a.tx;
  const int blocks = c1_wgrad_grid(a, &a.tiles_per_block);
  // two tile groups per block when there are tiles for both
  if (ntiles >= 512)
    ::cg::launch(c1_wgrad_kernel<2>, dim3(blocks), dim3(512), 0, st, a, x, dz, ws, ntiles);
  else
    ::cg::launch(c1_wgrad_kernel<1>, dim3(blocks), dim3(256), 0, st, a, x, dz, ws, ntiles);
  colsum_launch(ws, blocks, 512, 64, dw, (long long)g->w_sb, st);
  return CGAN3D_OK;
}

}  // namespace cg
