// Stride-2 convolution 32 -> 64 channels at the generator's 32 <-> 64 level with every operand of a
// block in LDS (round 5): the second downsampling Conv3d forward (model/generator.py:40-47, k3 s2 p1,
// 32^3 x 32 -> 16^3 x 64 at 64^3 patches) and the input-grad of the first ConvTranspose3d
// (generator.py:61-77; the transpose of a stride-2 transposed conv is this forward mapping).
//
// conv_halo_kernel ran them at 18-20 us per launch (27-64 VALU per MFMA, tap-by-tap weight ring with
// two barriers per tap).  Here the shape of conv_k3m: a block owns a 4 x 4 x 8 output tile x one half
// (32) of the output channels — 256 blocks at 64^3 B=4 — and LDS-DMAs its whole input halo (9 x 9 x
// 17 voxels x 32 channels, 98 KB) and all 27 taps of its channel half (54 KB) once; each wave runs
// its two z-slices (a 32-voxel M tile) x 32 channels over K = 27 taps x 32 on v_mfma_f32_32x32x16_bf16
// (54 MFMAs) with no barrier after the one that publishes the operands.
//
// Conflict-free stride-2 A reads: the 64-byte voxel rows are stored split by x parity — image row
// ((hz * 9 + hy) * 2 + (hx & 1)) * 5 + (hx >> 1) — so a 16-lane group (one z-slice, 4 x 4 (x, y)
// outputs reading input (2x + tx, 2y + ty)) spans four consecutive image rows along x (row mod 4 takes
// all four values) and the 16-byte granule positions are swizzled by (hy >> 1) & 3 (all four along y):
// 16 distinct (row mod 4, position) pairs = all 64 banks, for every tap.  Weight rows (one output
// channel, 64 bytes) swizzle by (c >> 2) & 3 for the same reason.
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_f __attribute__((ext_vector_type(8)));
typedef float f32x16_f __attribute__((ext_vector_type(16)));

constexpr int F64_HX = 9, F64_HY = 9, F64_HZ = 17;             // input halo of a 4 x 4 x 8 output tile
constexpr int F64_IROWS = F64_HZ * F64_HY * 2 * 5;              // 1530 image rows of 64 B
constexpr int F64_HALO = 1536 * 64;                            // 96 DMA instructions of 16 rows
constexpr int F64_TAPB = 32 * 64;                              // one tap's weights, 32 output channels
constexpr int F64_LDS = F64_HALO + 27 * F64_TAPB;              // 153600 B

__device__ __attribute__((aligned(16))) unsigned char g_f64_zero[16];

struct F64Args {
  int n, di, hi, wi, do_, ho, wo;
  int tx, ty, tz;  // output tiles per axis (4, 4, 8)
};

__device__ __forceinline__ int f64_irow(int hz, int hy, int hx) { return ((hz * F64_HY + hy) * 2 + (hx & 1)) * 5 + (hx >> 1); }
__device__ __forceinline__ int f64_fa(int hy) { return (hy >> 1) & 3; }
__device__ __forceinline__ int f64_fw(int c) { return (c >> 2) & 3; }

// A row r (0..31) of an M tile -> (x, y, z-slice zz) (conv_k3m's km_row: a ds_read_b128 lane group
// is one z-slice, 4 x 4 in (x, y))
__device__ __forceinline__ void f64_row(int r, int& x, int& y, int& zz) {
  int idx;
  if (r < 4) { zz = 0; idx = r; }
  else if (r < 12) { zz = 1; idx = r - 4; }
  else if (r < 16) { zz = 0; idx = r - 8; }
  else if (r < 20) { zz = 1; idx = r - 8; }
  else if (r < 28) { zz = 0; idx = r - 12; }
  else { zz = 1; idx = r - 16; }
  x = idx & 3;
  y = idx >> 2;
}

__device__ __forceinline__ void f64_dma16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

// OB: bit 0 — y and bn_z are bf16 (cgan3d_epilogue.out_bf16)
template <int OB>
__global__ __launch_bounds__(256, 1) void conv_f64_kernel(F64Args a, const __bf16* __restrict__ x16,
                                                          const __bf16* __restrict__ wpk, float* __restrict__ y,
                                                          Epi ep) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[F64_LDS];
  __shared__ float red[3][4][32];
  using lds_t = __attribute__((address_space(3))) void*;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = blockIdx.x & 1;
  int t = blockIdx.x >> 1;
  const int txi = t % a.tx;
  t /= a.tx;
  const int tyi = t % a.ty;
  t /= a.ty;
  const int tzi = t % a.tz;
  const int nb = t / a.tz;
  const int ox0 = 4 * txi, oy0 = 4 * tyi, oz0 = 8 * tzi;
  const int co0 = 32 * half;
  const int c = lane & 31, h = lane >> 5;

  // ---- epilogue operands first (conv_k3m): this lane's 16 output offsets and the mode-4 z there
  const bool mode4 = ep.fz.acc_mode == 4;
  int oidx[16];
  float zv[16] = {};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int R = (i & 3) + 8 * (i >> 2) + 4 * h;
    int lx, ly, lzz;
    f64_row(R, lx, ly, lzz);
    const int ox = ox0 + lx, oy = oy0 + ly, oz = oz0 + 2 * wave + lzz;
    const bool ok = ox < a.wo && oy < a.ho && oz < a.do_;
    oidx[i] = ok ? (((nb * a.do_ + oz) * a.ho + oy) * a.wo + ox) * 64 + co0 + c : -1;
  }
  if (mode4) {  // block-uniform
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int zi = oidx[i] >= 0 ? oidx[i] : 0;
      if constexpr ((OB & 1) != 0) zv[i] = (float)reinterpret_cast<const __bf16*>(ep.bn_z)[zi];
      else zv[i] = ep.bn_z[zi];
    }
  }

  // ---- LDS-DMA: the halo image (96 instructions of 16 rows; lane -> row 16 i + lane / 4, 16-byte
  // position lane % 4 holding logical granule position ^ f64_fa(hy)), then the 27 taps' weights of
  // this channel half (54 instructions of 16 output-channel rows)
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_t)smem;
  {
    const int p = lane & 3;
    const int hx0 = 2 * ox0 - 1, hy0 = 2 * oy0 - 1, hz0 = 2 * oz0 - 1;
    // image row ir = ((hz * 9 + hy) * 2 + par) * 5 + xh, decoded once and then stepped by 64 rows per
    // iteration (= 12 x 5 + 4) with carries: the per-iteration divisions by 5 and 9 were most of the
    // kernel's VALU (29 VALU per MFMA, profiles/r05_pmc_sq_step.json)
    int xh, par, hy, hz;
    {
      const int ir0 = 16 * wave + (lane >> 2);
      xh = ir0 % 5;
      const int q = ir0 / 5;
      par = q & 1;
      hy = (q >> 1) % F64_HY;
      hz = (q >> 1) / F64_HY;
    }
    for (int i = wave; i < F64_HALO / 1024; i += 4) {
      const int ir = 16 * i + (lane >> 2);
      const int hx = 2 * xh + par;
      const int ix = hx0 + hx, iy = hy0 + hy, iz = hz0 + hz;
      const bool ok = ir < F64_IROWS && hx < F64_HX && (unsigned)ix < (unsigned)a.wi && (unsigned)iy < (unsigned)a.hi &&
                      (unsigned)iz < (unsigned)a.di;
      const int g = p ^ f64_fa(hy);
      const void* src = ok ? (const void*)(x16 + ((long long)((nb * a.di + iz) * a.hi + iy) * a.wi + ix) * 32 + 8 * g)
                           : (const void*)g_f64_zero;
      f64_dma16(src, __builtin_amdgcn_readfirstlane(lds0 + i * 1024));
      xh += 4;
      const int cx = xh >= 5;
      xh -= cx ? 5 : 0;
      const int t2 = par + cx;  // q = (hz * 9 + hy) * 2 + par advances by 12 + cx
      par = t2 & 1;
      hy += 6 + (t2 >> 1);
      const int cy = hy >= F64_HY;
      hy -= cy ? F64_HY : 0;
      hz += cy;
    }
    for (int j = wave; j < 54; j += 4) {
      const int tp = j >> 1, cw = 16 * (j & 1) + (lane >> 2);
      // packed format 2 keeps logical granule L of (tap, channel) at position L ^ (channel & 3)
      const int L = p ^ f64_fw(cw);
      const __bf16* src = wpk + ((long long)(tp * 64 + co0 + cw) * 32 + 8 * (L ^ (cw & 3)));
      f64_dma16(src, __builtin_amdgcn_readfirstlane(lds0 + F64_HALO + j * 1024));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- 27 taps x 2 K-steps of 16 channels: 54 MFMAs, the next tap's fragments in flight
  int lx, ly, lzz;
  f64_row(c, lx, ly, lzz);
  const int bz = 2 * (2 * wave + lzz), by = 2 * ly, bx = 2 * lx;  // halo coordinates at tap (0, 0, 0)
  int boff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) boff[s] = F64_HALO + c * 64 + 16 * ((2 * s + h) ^ f64_fw(c));
  f32x16_f acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  auto aoff = [&](int tp, int s) {
    const int tz = tp / 9, ty = (tp / 3) % 3, tx = tp % 3;
    const int hy = by + ty;
    return f64_irow(bz + tz, hy, bx + tx) * 64 + 16 * ((2 * s + h) ^ f64_fa(hy));
  };
  bf16x8_f ra[2][2], rb[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    ra[0][s] = *reinterpret_cast<const bf16x8_f*>(smem + aoff(0, s));
    rb[0][s] = *reinterpret_cast<const bf16x8_f*>(smem + boff[s]);
  }
#pragma unroll
  for (int tp = 0; tp < 27; ++tp) {
    const int cur = tp & 1, nxt = cur ^ 1;
    if (tp + 1 < 27) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        ra[nxt][s] = *reinterpret_cast<const bf16x8_f*>(smem + aoff(tp + 1, s));
        rb[nxt][s] = *reinterpret_cast<const bf16x8_f*>(smem + boff[s] + (tp + 1) * F64_TAPB);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[cur][s], rb[cur][s], acc, 0, 0, 0);
  }

  // ---- epilogue: stores, then the statistics of channel co0 + c over this lane's outputs
  const int mode = ep.fz.acc_mode;
  float n1 = 0.f, K = 0.f, s1 = 0.f, s2 = 0.f;
  bool first = true;
  float sc = 0.f, sh = 0.f, mu = 0.f, is = 0.f;
  if (mode4) { sc = ep.bn_ss[co0 + c]; sh = ep.bn_ss[64 + co0 + c]; mu = ep.bn_mi[co0 + c]; is = ep.bn_mi[64 + co0 + c]; }
  const int bact = ep.bn_act;
  const float bslope = ep.bn_slope;
  // round 5b: the statistics mode and the BatchNorm activation as uniform branches around whole loops,
  // and a tile inside the volume (every tile at 64^3) without per-element validity
  const bool full = ox0 + 4 <= a.wo && oy0 + 4 <= a.ho && oz0 + 8 <= a.do_;
  auto store = [&](int o, float v) {
    if constexpr ((OB & 1) != 0) reinterpret_cast<__bf16*>(y)[o] = (__bf16)v;
    else y[o] = v;
  };
  if (mode == 3 && full) {  // shift = the lane's first value
    K = acc[0];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i];
      store(oidx[i], v);
      const float d = v - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
    n1 = 16.f;
  } else if (mode4) {  // (invalid rows: skipped)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (!full && oidx[i] < 0) continue;
      const float v = acc[i];
      store(oidx[i], v);
      const float pre = zv[i] * sc + sh;
      const float gg = bact == CGAN3D_ACT_RELU ? (pre > 0.f ? v : 0.f)
                                               : (bact == CGAN3D_ACT_LRELU ? (pre > 0.f ? v : v * bslope) : v);
      s1 += gg;
      s2 += gg * (zv[i] - mu) * is;
    }
  } else {  // no statistics, or mode 3 on a ragged tile (the shift is the first valid value)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int o = oidx[i];
      if (o < 0) continue;
      const float v = acc[i];
      store(o, v);
      if (mode == 3) {
        if (first) { K = v; first = false; }
        const float d = v - K;
        s1 += d;
        s2 = fmaf(d, d, s2);
        n1 += 1.f;
      }
    }
  }
  if (!mode) return;
  double* const facc = ep.fz.acc_out + (long long)(blockIdx.x % ep.fz.reps) * 2 * 64;
  if (mode == 3) {  // lane (n, mean, M2) -> merged with lane ^ 32 (same channel), then the 4 waves
    float mm = n1 > 0.f ? K + s1 / n1 : 0.f, q = n1 > 0.f ? fmaxf(s2 - s1 * s1 / n1, 0.f) : 0.f, nn = n1;
    {
      const float no = __shfl_xor(nn, 32, 64), mo = __shfl_xor(mm, 32, 64), qo = __shfl_xor(q, 32, 64);
      if (no > 0.f) {
        const float nt = nn + no, dl = mo - mm;
        mm += dl * (no / nt);
        q += qo + dl * dl * (nn * no / nt);
        nn = nt;
      }
    }
    if (h == 0) { red[0][wave][c] = nn; red[1][wave][c] = mm; red[2][wave][c] = q; }
    __syncthreads();
    if (tid < 32) {
      float rn = 0.f, rm = 0.f, rq = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float no = red[0][w][tid], mo = red[1][w][tid], qo = red[2][w][tid];
        if (no > 0.f) {
          const float nt = rn + no, dl = mo - rm;
          rm += dl * (no / nt);
          rq += qo + dl * dl * (rn * no / nt);
          rn = nt;
        }
      }
      if (rn > 0.f) {
        const double S = (double)rm * rn;
        unsafeAtomicAdd(facc + co0 + tid, S);
        unsafeAtomicAdd(facc + 64 + co0 + tid, (double)rq + S * (double)rm);
      }
    }
  } else {  // mode 4: (sum g, sum g * xhat)
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (h == 0) { red[0][wave][c] = s1; red[1][wave][c] = s2; }
    __syncthreads();
    if (tid < 32) {
      unsafeAtomicAdd(facc + co0 + tid, (double)(red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid]));
      unsafeAtomicAdd(facc + 64 + co0 + tid,
                      (double)(red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid]));
    }
  }
}

// Conv3d k3 s2 p1 32 -> 64 with the bf16 input shadow and format-2 packed weights; epilogue: output
// (fp32 / bf16) + fp64-accumulator statistics (mode 3 / 4) or nothing
bool f64_geom_ok(const cgan3d_conv_geom* g) {
#if defined(CGAN3D_NO_T64)
  return false;  // (A/B builds)
#endif
  return k3m_enabled() && g->prec == CGAN3D_PREC_BF16 && g->w_packed == 2 && !g->transposed && !g->reflect && !g->planar && g->k == 3 &&
         g->stride == 2 && g->pad == 1 && g->cin == 32 && g->cout == 64 && g->do_ == (g->di - 1) / 2 + 1 &&
         g->ho == (g->hi - 1) / 2 + 1 && g->wo == (g->wi - 1) / 2 + 1 &&
         (long long)g->n * g->di * g->hi * g->wi * 32 < (1LL << 31) &&
         (long long)g->n * g->do_ * g->ho * g->wo * 64 < (1LL << 31);
}

bool f64_ok(const cgan3d_conv_geom* g, const Epi& e) {
  return f64_geom_ok(g) && e.x16 && !e.bias && !e.residual && !e.mask_src && !e.minuend && !e.out2 && !e.stats &&
         !e.bn_mode && !e.bn_fold && !e.pre.mode && e.act == CGAN3D_ACT_NONE && !e.res16 &&
         (e.fz.acc_mode == 0 || e.fz.acc_mode == 3 || (e.fz.acc_mode == 4 && e.bn_z && e.bn_ss && e.bn_mi));
}

int f64_launch(const cgan3d_conv_geom* g, const __bf16* wp, float* y, const Epi& e, hipStream_t st) {
  F64Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.tx = (a.wo + 3) / 4; a.ty = (a.ho + 3) / 4; a.tz = (a.do_ + 7) / 8;
  const dim3 grid((unsigned)(2 * a.n * a.tx * a.ty * a.tz));
  if (e.out16) ::cg::launch(conv_f64_kernel<1>, grid, dim3(256), 0, st, a, e.x16, wp, y, e);
  else ::cg::launch(conv_f64_kernel<0>, grid, dim3(256), 0, st, a, e.x16, wp, y, e);
  return CGAN3D_OK;
}

}  // namespace cg
