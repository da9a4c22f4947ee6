// Stride-2 convolutions between the generator's 16- and 32-channel levels, bf16 MFMA (gfx950).
//
// Four launches per step share two shapes (model/generator.py:40-47,61-77; blocks.py:23-38):
//  * S2F, Conv3d k3 s2 p1, 16 -> 32 channels (gathered 2S^3 -> aligned S^3): the first
//    downsampling conv forward and the input-grad of the last ConvTranspose3d;
//  * S2T, the transposed mapping, 32 gathered -> 16 channels on the 2x grid: the last
//    ConvTranspose3d forward (output_padding 1) and the first downsampling conv's input-grad.
// conv_halo_kernel does not take them (16-channel K or N side), and the implicit-GEMM kernel
// re-gathers every tap through L1 (110-127 us per launch at 64^3, B=4).  Both kernels here are
// built to be HBM-bound: one block stages its input halo once (fp32 NDHWC -> bf16 LDS), holds
// all of its weight fragments in registers (loaded from L2 before the staging), and writes a
// 128-voxel (S2F) or 1024-voxel (S2T, all 8 parity classes of a tile) output block.
//
// LDS layouts are bank-conflict-free for the MFMA A reads (ds_read_b128 lane groups of
// MI355X_MICROARCH.md §LDS; the swizzles were found by exhaustive search over every tap offset):
//  * S2F: an M tile is 16 consecutive outputs along x; tap (td,th,tw) reads input x = 2x + tw,
//    so the halo keeps each (z, y) input row split by x parity — sub-row [parity][x/2][16 ch],
//    32-byte voxels — and a lane group reads 16 consecutive voxels of one sub-row.  One K step of
//    v_mfma_f32_16x16x32_bf16 covers two taps (16 channels each; g>>1 selects the tap).
//  * S2T: an M tile is 16 consecutive class voxels along x; rows [z][y][17 x][32 ch], 64-byte
//    voxels with granule g stored at g ^ ((x >> 1) & 2).
// Both run the MFMA transposed (A = the weight fragments, B = the staged activations), so a lane
// ends up with 4 consecutive output channels of one voxel: one 16-byte store (and, for the
// input-grad statistics, one 16-byte z load) per voxel and lane instead of four 4-byte ones.
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_s __attribute__((ext_vector_type(4)));

struct S2Args {
  int n, di, hi, wi, do_, ho, wo;
  int cd, ch, cw;  // output grid (S2F) or class grid (S2T)
  int td, th, tw;  // tiles per dim
};

// per-channel sum over the block in the transposed MFMA layout: v[nt][j] is this lane's partial
// for channel nt*16 + 4g + j (over its voxel column r16), summed over the 16 voxel lanes and the
// four waves; every lane receives its channels' block totals
template <int NT>
__device__ __forceinline__ void block_chan_sum(float (&v)[NT][4], float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) v[nt][j] += __shfl_xor(v[nt][j], m, 64);
  lds_barrier();  // red is free (LDS-only: outstanding output stores stay in flight)
  if (r16 == 0) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave * NT * 16 + nt * 16 + 4 * g + j] = v[nt][j];
  }
  lds_barrier();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = nt * 16 + 4 * g + j;
      v[nt][j] = red[c] + red[NT * 16 + c] + red[2 * NT * 16 + c] + red[3 * NT * 16 + c];
    }
}

__device__ __forceinline__ float s2_act(float v, const Epi& ep) {
  if (ep.act == CGAN3D_ACT_RELU) return fmaxf(v, 0.f);
  if (ep.act == CGAN3D_ACT_LRELU) return v > 0.f ? v : v * ep.slope;
  return v;
}

// Block statistics of the fused BatchNorm slab (include/cgan3d.h): mode 1 (sum, M2 about the block
// mean, count), mode 2 (sum g, sum g*xhat).  vals / zv: [U][NT] per lane = channels nt*16 + 4g +
// 0..3 of the lane's voxel in output group u; ok[u]: that voxel is inside the volume.
// fused-statistics mode of an epilogue: 1 / 2 (slab or, cgan3d_bn_fuse acc_mode 3 / 4, fp64 accumulators)
__device__ __forceinline__ int s2_stat_mode(const Epi& ep) {
  return ep.fz.acc_mode == 3 ? 1 : ep.fz.acc_mode == 4 ? 2 : ep.bn_mode;
}
static int s2_host_stat_mode(const Epi& ep) { return ep.fz.acc_mode == 3 ? 1 : ep.fz.acc_mode == 4 ? 2 : ep.bn_mode; }

// write the block's statistic pairs (s, q) of channels nt*16 + 4g + j, summed over the block
// first: mode 1 (sum, M2) or 2 (sum g, sum g*xhat) into slab slot `slot`, or (cgan3d_bn_fuse) into
// replica slot % reps of the fp64 accumulators (mode 1 as (sum, sum of squares = M2 + S * mean))
template <int NT>
__device__ __forceinline__ void s2_stats_write(const Epi& ep, int mode, int C, float (&s)[NT][4], float (&q)[NT][4],
                                               int cnt, int slot) {
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  // after the block sums, lanes 0, 16, 32, 48 of wave 0 hold channels nt*16 + 4g + j
  if (!(tid < 64 && (lane & 15) == 0)) return;
  double* const acc = ep.fz.acc_mode ? ep.fz.acc_out + (long long)(slot % ep.fz.reps) * 2 * C : nullptr;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = nt * 16 + 4 * g + j;
      if (acc) {
        if (mode == 2) {
          unsafeAtomicAdd(acc + c, (double)s[nt][j]);
          unsafeAtomicAdd(acc + C + c, (double)q[nt][j]);
        } else if (cnt) {
          unsafeAtomicAdd(acc + c, (double)s[nt][j]);
          unsafeAtomicAdd(acc + C + c, (double)q[nt][j] + (double)s[nt][j] * (double)s[nt][j] / cnt);
        }
      } else {
        *bn_slot(ep, 0, C, c, slot) = s[nt][j];
        *bn_slot(ep, 1, C, c, slot) = q[nt][j];
      }
    }
  if (mode == 1 && tid == 0 && !acc) *bn_slot(ep, 2, C, 0, slot) = (float)cnt;
}

// mode 1 from the block's outputs: vals[U][NT] per lane = channels nt*16 + 4g + 0..3 of the lane's
// voxel in output group u, ok[u] = that voxel is inside the volume; (sum, M2 about the block mean)
template <int U, int NT>
__device__ __forceinline__ void s2_stats_m1(const Epi& ep, int C, const f32x4 (&vals)[U][NT], const bool (&ok)[U],
                                            int cnt, float* red, int slot) {
  float s[NT][4], q[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[nt][j] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) s[nt][j] += ok[u] ? vals[u][nt][j] : 0.f;
    }
  block_chan_sum<NT>(s, red);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float m = cnt ? s[nt][j] / cnt : 0.f;
      q[nt][j] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float d = ok[u] ? vals[u][nt][j] - m : 0.f;
        q[nt][j] += d * d;
      }
    }
  block_chan_sum<NT>(q, red);
  s2_stats_write<NT>(ep, 1, C, s, q, cnt, slot);
}

// mode 2, streamed: the BatchNorm coefficients of the lane's channels, then s2_m2_add per output
struct S2M2 {
  float sc[4], sh[4], mu[4], inv[4];
};
__device__ __forceinline__ S2M2 s2_m2_coef(const Epi& ep, int C, int c0) {
  S2M2 k;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    k.sc[j] = ep.bn_ss[c0 + j]; k.sh[j] = ep.bn_ss[C + c0 + j];
    k.mu[j] = ep.bn_mi[c0 + j]; k.inv[j] = ep.bn_mi[C + c0 + j];
  }
  return k;
}
__device__ __forceinline__ void s2_m2_add(const Epi& ep, const S2M2& k, f32x4 v, f32x4 z, bool ok, float (&s)[4],
                                          float (&q)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gg = ok ? v[j] * act_grad(z[j] * k.sc[j] + k.sh[j], ep.bn_act, ep.bn_slope) : 0.f;
    s[j] += gg;
    q[j] += gg * (z[j] - k.mu[j]) * k.inv[j];
  }
}

// lo / hi: lane r16 holds the first / second 64-byte half of line r16 (a 128-byte pair of voxels or
// channel halves).  Rotating each by 8 lanes within the 16-lane row (DPP) gives A = lines 0..7 and
// B = lines 8..15 whole: lane r16 of A holds half r16 >> 3 of line r16 & 7, of B of line 8 + (r16 & 7)
__device__ __forceinline__ f32x4 s2_ror8(f32x4 v) {
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    r[j] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[j]), 0x128, 0xf, 0xf, false));
  return r;
}
__device__ __forceinline__ void s2_line_pair(f32x4 lo, f32x4 hi, int r16, f32x4& A, f32x4& B) {
  const f32x4 lo8 = s2_ror8(lo), hi8 = s2_ror8(hi);
  const bool first = r16 < 8;
  A = first ? lo : hi8;
  B = first ? lo8 : hi;
}

__device__ __forceinline__ f32x4 s2_act4(f32x4 v, const Epi& ep) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = s2_act(v[j], ep);
  return v;
}

// ------------------------------------------------------------------------------------------------
// S2F: Conv3d k3 s2 p1, 16 -> 32.  Block = 16 (x) x 4 (y) x 2 (z) outputs; wave w = output row y,
// both z slices (2 M tiles) x 2 N tiles; K = 27 taps x 16 channels in 14 steps of two taps.
constexpr int F_HX = 33, F_HY = 9, F_HZ = 5, F_SX = 17;
constexpr int F_HALO = F_HZ * F_HY * 2 * F_SX * 16;  // bf16 elements (48960 bytes)

template <int MODE>  // statistics mode s2_stat_mode(ep): 0 none, 1 forward, 2 input-grad
__global__ __launch_bounds__(256) void conv_s2f_kernel(S2Args a, const float* __restrict__ x,
                                                       const __bf16* __restrict__ wpk, float* y, Epi ep) {
  constexpr int CI = 16, CO = 32, KSTEPS = 14;
  __shared__ __attribute__((aligned(16))) __bf16 halo[F_HALO];
  __shared__ float red[4 * CO];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tiles = a.td * a.th * a.tw;
  int bid = blockIdx.x;
  const int nb = bid / tiles;
  bid -= nb * tiles;
  const int Z0 = (bid / (a.th * a.tw)) * 2, Y0 = ((bid / a.tw) % a.th) * 4, X0 = (bid % a.tw) * 16;

  // weight fragments of every K step: lane (channel nt*16 + r16, tap 2s + (g>>1), granule g&1)
  bf16x8_s bq[KSTEPS][2];
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) {
    const int t = 2 * s + (g >> 1);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int co = nt * 16 + r16;
      const int tt = t < 27 ? t : 26;
      bq[s][nt] = *reinterpret_cast<const bf16x8_s*>(wpk + ((long long)tt * CO + co) * CI + 8 * ((g & 1) ^ (co & 1)));
      if (t >= 27) bq[s][nt] = bf16x8_s{};
    }
  }

  // halo: input (2*Z0-1 .. +5, 2*Y0-1 .. +9, 2*X0-1 .. +33) -> [hz][hy][x parity][x/2][16] bf16
  if (ep.x16) {  // from the bf16 shadow of the input: 16-byte granules (8 channels) copied as they are
    const int iz0 = 2 * Z0 - 1, iy0 = 2 * Y0 - 1, ix0 = 2 * X0 - 1;
    constexpr int NG = F_HZ * F_HY * F_HX * 2, PG = (NG + 255) / 256;
    const bf16x8_s* xq = reinterpret_cast<const bf16x8_s*>(ep.x16);
    bf16x8_s sb[PG];
#pragma unroll
    for (int k = 0; k < PG; ++k) {
      const int i = tid + 256 * k;
      const int q = i & 1, v = i >> 1;
      const int hx = v % F_HX, r = v / F_HX;
      const int hy = r % F_HY, hz = r / F_HY;
      const int iz = iz0 + hz, iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = i < NG && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi &&
                      (unsigned)ix < (unsigned)a.wi;
      sb[k] = xq[ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * 2 + q : 0];
      if (!ok) sb[k] = bf16x8_s{};
    }
#pragma unroll
    for (int k = 0; k < PG; ++k) {
      const int i = tid + 256 * k;
      if (i >= NG) break;
      const int q = i & 1, v = i >> 1;
      const int hx = v % F_HX, r = v / F_HX;
      const int row = r * 2 + (hx & 1);
      *reinterpret_cast<bf16x8_s*>(halo + (row * F_SX + (hx >> 1)) * CI + 8 * q) = sb[k];
    }
  } else {
    const int iz0 = 2 * Z0 - 1, iy0 = 2 * Y0 - 1, ix0 = 2 * X0 - 1;
    constexpr int NV4 = F_HZ * F_HY * F_HX * 4, PER = (NV4 + 255) / 256, BATCH = 8;
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += BATCH) {
      f32x4 sv[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = tid + 256 * (k0 + k);
        const int c4 = i & 3, v = i >> 2;
        const int hx = v % F_HX, r = v / F_HX;
        const int hy = r % F_HY, hz = r / F_HY;
        const int iz = iz0 + hz, iy = iy0 + hy, ix = ix0 + hx;
        const bool ok = k0 + k < PER && i < NV4 && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi &&
                        (unsigned)ix < (unsigned)a.wi;
        sv[k] = *reinterpret_cast<const f32x4*>(
            x + (ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * CI + 4 * c4 : 0));
        if (!ok) sv[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = tid + 256 * (k0 + k);
        if (k0 + k >= PER || i >= NV4) break;
        const int c4 = i & 3, v = i >> 2;
        const int hx = v % F_HX, r = v / F_HX;
        const int row = r * 2 + (hx & 1);
        bf16x4_s u;
        u[0] = (__bf16)sv[k][0]; u[1] = (__bf16)sv[k][1]; u[2] = (__bf16)sv[k][2]; u[3] = (__bf16)sv[k][3];
        *reinterpret_cast<bf16x4_s*>(halo + (row * F_SX + (hx >> 1)) * CI + 4 * c4) = u;
      }
    }
  }
  __syncthreads();

  // mode-2 statistics: this lane's z values (its voxel, channels nt*16 + 4g .. +3) in flight during
  // the MFMAs
  constexpr int mode = MODE;
  const int oy = Y0 + wave, ox = X0 + r16;
  long long obase[2];
  bool ok[2];
#pragma unroll
  for (int zz = 0; zz < 2; ++zz) {
    const int oz = Z0 + zz;
    ok[zz] = oz < a.cd && oy < a.ch && ox < a.cw;
    obase[zz] = ok[zz] ? ((((long long)nb * a.cd + oz) * a.ch + oy) * a.cw + ox) * CO + 4 * g : 0;
  }
  f32x4 zv[2][2];
#pragma unroll
  for (int zz = 0; zz < 2; ++zz)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      zv[zz][nt] = mode == 2 ? *reinterpret_cast<const f32x4*>(ep.bn_z + obase[zz] + nt * 16) : f32x4{0.f, 0.f, 0.f, 0.f};

  // D[channel][voxel]: A = weights (lane channel r16), B = activations (lane voxel r16)
  f32x4 acc[2][2];
#pragma unroll
  for (int zz = 0; zz < 2; ++zz)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[zz][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) {
    int t = 2 * s + (g >> 1);
    t = t < 27 ? t : 26;  // the padding tap reads valid data against zero weights
    const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
#pragma unroll
    for (int zz = 0; zz < 2; ++zz) {
      const int row = ((2 * zz + td) * F_HY + 2 * wave + th) * 2 + (tw & 1);
      const bf16x8_s av =
          *reinterpret_cast<const bf16x8_s*>(halo + (row * F_SX + r16 + (tw >> 1)) * CI + 8 * (g & 1));
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[zz][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[s][nt], av, acc[zz][nt], 0, 0, 0);
    }
  }

  // ---- epilogue: lane holds output (x = X0 + r16, y = Y0 + wave, z = Z0 + zz), channels nt*16 + 4g .. +3
  f32x4 vals[2][2];
  float s2s[2][4] = {}, s2q[2][4] = {};  // mode 2, streamed
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int c = nt * 16 + 4 * g;
    const f32x4 b4 = ep.bias ? f32x4{ep.bias[c], ep.bias[c + 1], ep.bias[c + 2], ep.bias[c + 3]} : f32x4{0.f, 0.f, 0.f, 0.f};
    S2M2 k2;
    if constexpr (mode == 2) k2 = s2_m2_coef(ep, CO, c);
#pragma unroll
    for (int zz = 0; zz < 2; ++zz) {
      const f32x4 v = s2_act4(acc[zz][nt] + b4, ep);
      if (ok[zz]) *reinterpret_cast<f32x4*>(y + obase[zz] + nt * 16) = v;
      vals[zz][nt] = v;
      if constexpr (mode == 2) s2_m2_add(ep, k2, v, zv[zz][nt], ok[zz], s2s[nt], s2q[nt]);
    }
  }
  const int cnt = max(0, min(2, a.cd - Z0)) * max(0, min(4, a.ch - Y0)) * max(0, min(16, a.cw - X0));
  if constexpr (mode == 1) s2_stats_m1<2, 2>(ep, CO, vals, ok, cnt, red, blockIdx.x);
  if constexpr (mode == 2) {
    block_chan_sum<2>(s2s, red);
    block_chan_sum<2>(s2q, red);
    s2_stats_write<2>(ep, 2, CO, s2s, s2q, cnt, blockIdx.x);
  }
}

// ------------------------------------------------------------------------------------------------
// S2T: transposed k3 s2 p1 (output = 2 x gathered grid), 32 gathered -> 16 channels.  Block = a
// 16 x 4 x 2 tile of class coordinates j, all 8 parity classes r (output 2j + r): wave w = class
// row y, both z slices x 8 classes = 16 M tiles, one N tile; 27 taps, K = 32 channels each.
// Class r, per dim: r = 0 -> tap 1 at gathered j; r = 1 -> tap 0 at j + 1 and tap 2 at j.
constexpr int T_HX = 17, T_HY = 5, T_HZ = 3;
constexpr int T_HALO = T_HZ * T_HY * T_HX * 32;  // bf16 elements (16320 bytes)

template <int R>
struct S2Taps;  // per-dim taps of parity class R: (tap, gathered offset)
template <>
struct S2Taps<0> {
  static constexpr int n = 1;
  static constexpr int t[2] = {1, 1};
  static constexpr int off[2] = {0, 0};
};
template <>
struct S2Taps<1> {
  static constexpr int n = 2;
  static constexpr int t[2] = {0, 2};
  static constexpr int off[2] = {1, 0};
};

// weight granule (tap t, output channel co, K granule q) of the LDS copy: slot q ^ s2t_wsw(co) of
// the (t, co) row — the 16 lanes of every ds_read_b128 lane group hit 16 distinct bank blocks
__device__ __forceinline__ int s2t_wsw(int co) { return (co & 4) >> 1; }

template <int RZ, int RY, int RX>
__device__ __forceinline__ void s2t_class(const __bf16* halo, const __bf16* wts, f32x4 (&acc)[2], int wave, int g,
                                          int r16) {
  using TZ = S2Taps<RZ>;
  using TY = S2Taps<RY>;
  using TX = S2Taps<RX>;
#pragma unroll
  for (int a = 0; a < TZ::n; ++a)
#pragma unroll
    for (int b = 0; b < TY::n; ++b)
#pragma unroll
      for (int c = 0; c < TX::n; ++c) {
        const int t = TZ::t[a] * 9 + TY::t[b] * 3 + TX::t[c];
        const int hx = r16 + TX::off[c];
        const bf16x8_s bw = *reinterpret_cast<const bf16x8_s*>(wts + ((t * 16 + r16) * 4 + (g ^ s2t_wsw(r16))) * 8);
#pragma unroll
        for (int zz = 0; zz < 2; ++zz) {
          const int row = (zz + TZ::off[a]) * T_HY + wave + TY::off[b];
          const bf16x8_s av =
              *reinterpret_cast<const bf16x8_s*>(halo + (row * T_HX + hx) * 32 + 8 * (g ^ ((hx >> 1) & 2)));
          acc[zz] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, av, acc[zz], 0, 0, 0);
        }
      }
}

// Persistent: a block loops over tiles (grid = min(tiles, 2 per CU; 1 for mode 2 without the bf16
// shadow)); the weights are staged into
// LDS once, the next tile's halo is loaded into registers while the current tile's MFMAs and
// epilogue run.
// statistics mode s2_stat_mode(ep): 0 none, 1 forward, 2 input-grad; X16: ep.x16; B16 (ep.out16, round 4):
// the output and the mode-2 z are bf16 (the generator's 64^3 16-channel tensors)
template <int MODE, bool X16, bool B16>
__global__ __launch_bounds__(256, MODE == 2 && !X16 ? 1 : 2) void conv_s2t_kernel(S2Args a, const float* __restrict__ x,
                                                          const __bf16* __restrict__ wpk, float* y, Epi ep, int ntiles) {
  constexpr int CI = 32, CO = 16;
  __shared__ __attribute__((aligned(16))) __bf16 halo[T_HALO];
  __shared__ __attribute__((aligned(16))) __bf16 wts[27 * CO * CI];
  __shared__ float red[4 * CO];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tiles = a.td * a.th * a.tw;
  {  // packed weights (granule (t*CO + co)*4 + (q ^ (co & 3)) holds K granule q) -> LDS, once
    const bf16x8_s* src = reinterpret_cast<const bf16x8_s*>(wpk);
    bf16x8_s* dst = reinterpret_cast<bf16x8_s*>(wts);
    for (int i = tid; i < 27 * CO * 4; i += 256) {
      const int q = i & 3, co = (i >> 2) & 15, t = i >> 6;
      const int kq = q ^ s2t_wsw(co);
      dst[i] = src[(t * CO + co) * 4 + (kq ^ (co & 3))];
    }
  }
  const float4* xf = reinterpret_cast<const float4*>(x);
  const bf16x8_s* xq = reinterpret_cast<const bf16x8_s*>(ep.x16);
  constexpr int NG = T_HZ * T_HY * T_HX * 4, PG = (NG + 255) / 256;    // bf16 shadow granules
  constexpr int NV4 = T_HZ * T_HY * T_HX * 8, PER = (NV4 + 255) / 256;  // fp32 float4s
  bf16x8_s sb[X16 ? PG : 1];
  f32x4 sv[X16 ? 1 : PER];
  auto origin = [&](int tile, int* nb, int* Z0, int* Y0, int* X0) {
    *nb = tile / tiles;
    const int b = tile - *nb * tiles;
    *Z0 = (b / (a.th * a.tw)) * 2; *Y0 = ((b / a.tw) % a.th) * 4; *X0 = (b % a.tw) * 16;
  };
  // halo: gathered (Z0 .. +3, Y0 .. +5, X0 .. +17) -> [hz][hy][hx][32] bf16, granule swizzle
  auto load = [&](int tile) {
    int nb, Z0, Y0, X0;
    origin(tile, &nb, &Z0, &Y0, &X0);
    if constexpr (X16) {
#pragma unroll
      for (int k = 0; k < PG; ++k) {
        const int i = tid + 256 * k;
        const int q = i & 3, v = i >> 2;
        const int hx = v % T_HX, r = v / T_HX;
        const int hy = r % T_HY, hz = r / T_HY;
        const int iz = Z0 + hz, iy = Y0 + hy, ix = X0 + hx;
        const bool ok = i < NG && iz < a.di && iy < a.hi && ix < a.wi;
        sb[k] = xq[ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * 4 + q : 0];
        if (!ok) sb[k] = bf16x8_s{};
      }
    } else {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + 256 * k;
        const int c4 = i & 7, v = i >> 3;
        const int hx = v % T_HX, r = v / T_HX;
        const int hy = r % T_HY, hz = r / T_HY;
        const int iz = Z0 + hz, iy = Y0 + hy, ix = X0 + hx;
        const bool ok = i < NV4 && iz < a.di && iy < a.hi && ix < a.wi;
        const float4 f = xf[ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * (CI / 4) + c4 : 0];
        sv[k] = ok ? f32x4{f.x, f.y, f.z, f.w} : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store = [&]() {
    if constexpr (X16) {
#pragma unroll
      for (int k = 0; k < PG; ++k) {
        const int i = tid + 256 * k;
        if (i >= NG) break;
        const int q = i & 3, v = i >> 2;
        const int hx = v % T_HX;
        *reinterpret_cast<bf16x8_s*>(halo + v * 32 + 8 * (q ^ ((hx >> 1) & 2))) = sb[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + 256 * k;
        if (i >= NV4) break;
        const int c4 = i & 7, v = i >> 3;
        const int hx = v % T_HX;
        bf16x4_s u;
        u[0] = (__bf16)sv[k][0]; u[1] = (__bf16)sv[k][1]; u[2] = (__bf16)sv[k][2]; u[3] = (__bf16)sv[k][3];
        *reinterpret_cast<bf16x4_s*>(halo + v * 32 + 8 * ((c4 >> 1) ^ ((hx >> 1) & 2)) + 4 * (c4 & 1)) = u;
      }
    }
  };
  const f32x4 b4 = ep.bias ? f32x4{ep.bias[4 * g], ep.bias[4 * g + 1], ep.bias[4 * g + 2], ep.bias[4 * g + 3]}
                           : f32x4{0.f, 0.f, 0.f, 0.f};
  S2M2 k2;
  if constexpr (MODE == 2) k2 = s2_m2_coef(ep, CO, 4 * g);
  int tile = blockIdx.x;
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    int nb, Z0, Y0, X0;
    origin(tile, &nb, &Z0, &Y0, &X0);
    // The MFMAs leave lane (g, r16) with channels 4g .. 4g+3 of class voxel jx = X0 + r16; the
    // classes rx = 0 / 1 of one (rz, ry, slice) are the two 64-byte halves of the 128-byte voxel
    // pairs (2jx, 2jx + 1).  The epilogue swaps halves between lanes r16 and r16 ^ 8 (DPP row
    // rotate by 8) so each store writes whole lines: output u = ((rz * 2 + ry) * 2 + zz) * 2 + S
    // holds class voxel jx = X0 + 8S + (r16 & 7), rx = r16 >> 3.  Element offsets of this launch
    // fit 32 bits (s2_launch checks it).
    const int jy = Y0 + wave;
    int obase[16];
    bool ok[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int S = u & 1, zz = (u >> 1) & 1, ry = (u >> 2) & 1, rz = u >> 3;
      const int jz = Z0 + zz, jx = X0 + 8 * S + (r16 & 7), rx = r16 >> 3;
      const bool v_ok = jz < a.cd && jy < a.ch && jx < a.cw;
      ok[u] = v_ok;
      obase[u] = v_ok ? (((nb * a.do_ + 2 * jz + rz) * a.ho + 2 * jy + ry) * a.wo + 2 * jx + rx) * CO + 4 * g : 0;
    }
    __syncthreads();  // every wave done with the previous tile's halo (and the weight staging)
    store();
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load(tile + gridDim.x);  // in flight during this tile's MFMAs

    f32x4 acc[8][2];  // D[channel][voxel]: A = weights (lane channel r16), B = activations (lane voxel r16)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c][0] = acc[c][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    s2t_class<0, 0, 0>(halo, wts, acc[0], wave, g, r16);
    s2t_class<0, 0, 1>(halo, wts, acc[1], wave, g, r16);
    s2t_class<0, 1, 0>(halo, wts, acc[2], wave, g, r16);
    s2t_class<0, 1, 1>(halo, wts, acc[3], wave, g, r16);
    s2t_class<1, 0, 0>(halo, wts, acc[4], wave, g, r16);
    s2t_class<1, 0, 1>(halo, wts, acc[5], wave, g, r16);
    s2t_class<1, 1, 0>(halo, wts, acc[6], wave, g, r16);
    s2t_class<1, 1, 1>(halo, wts, acc[7], wave, g, r16);

    // ---- epilogue: 16-byte stores of whole lines; mode 2 statistics streamed (z loaded here: the
    // second resident block's MFMAs cover the round trip), mode 1 from the held outputs (M2 about
    // the block mean)
    f32x4 vals[MODE == 1 ? 16 : 1][1];
    float s2s[1][4] = {}, s2q[1][4] = {};
#pragma unroll
    for (int p = 0; p < 4; ++p) {  // (rz, ry): classes 2p (rx = 0) and 2p + 1 (rx = 1)
      f32x4 zv[MODE == 2 ? 4 : 1];  // outputs u = 4p .. 4p + 3
      if constexpr (MODE == 2) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if constexpr (B16) {
            const bf16x4_s h = *reinterpret_cast<const bf16x4_s*>(reinterpret_cast<const __bf16*>(ep.bn_z) + obase[4 * p + k]);
            zv[k] = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
          } else {
            zv[k] = *reinterpret_cast<const f32x4*>(ep.bn_z + obase[4 * p + k]);
          }
        }
      }
#pragma unroll
      for (int zz = 0; zz < 2; ++zz) {
        f32x4 out[2];
        s2_line_pair(s2_act4(acc[2 * p][zz] + b4, ep), s2_act4(acc[2 * p + 1][zz] + b4, ep), r16, out[0], out[1]);
#pragma unroll
        for (int S = 0; S < 2; ++S) {
          const int u = (p * 2 + zz) * 2 + S;
          if constexpr (B16) {  // 8 bytes per lane (the two halves of a 64-byte voxel pair from one store)
            bf16x4_s h;
            h[0] = (__bf16)out[S][0]; h[1] = (__bf16)out[S][1]; h[2] = (__bf16)out[S][2]; h[3] = (__bf16)out[S][3];
            if (ok[u]) *reinterpret_cast<bf16x4_s*>(reinterpret_cast<__bf16*>(y) + obase[u]) = h;
          } else {
            if (ok[u]) *reinterpret_cast<f32x4*>(y + obase[u]) = out[S];
          }
          if constexpr (MODE == 1) vals[u][0] = out[S];
          if constexpr (MODE == 2) s2_m2_add(ep, k2, out[S], zv[u - 4 * p], ok[u], s2s[0], s2q[0]);
        }
      }
    }
    const int cnt = 8 * max(0, min(2, a.cd - Z0)) * max(0, min(4, a.ch - Y0)) * max(0, min(16, a.cw - X0));
    if constexpr (MODE == 1) s2_stats_m1<16, 1>(ep, CO, vals, ok, cnt, red, tile);
    if constexpr (MODE == 2) {
      block_chan_sum<1>(s2s, red);
      block_chan_sum<1>(s2q, red);
      s2_stats_write<1>(ep, 2, CO, s2s, s2q, cnt, tile);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// 1: S2F, 2: S2T, 0: neither
int s2_kind(const cgan3d_conv_geom* g) {
  if (g->prec != CGAN3D_PREC_BF16 || g->reflect || g->k != 3 || g->stride != 2 || g->pad != 1) return 0;
  if (!g->transposed && g->cin == 16 && g->cout == 32 && g->do_ == (g->di - 1) / 2 + 1 &&
      g->ho == (g->hi - 1) / 2 + 1 && g->wo == (g->wi - 1) / 2 + 1)
    return 1;
  if (g->transposed && g->cin == 32 && g->cout == 16 && g->do_ == 2 * g->di && g->ho == 2 * g->hi &&
      g->wo == 2 * g->wi)
    return 2;
  return 0;
}

static S2Args s2_args(const cgan3d_conv_geom* g, int kind) {
  S2Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  if (kind == 1) { a.cd = g->do_; a.ch = g->ho; a.cw = g->wo; }
  else { a.cd = g->di; a.ch = g->hi; a.cw = g->wi; }
  a.td = (a.cd + 1) / 2; a.th = (a.ch + 3) / 4; a.tw = (a.cw + 15) / 16;
  return a;
}

long long s2_blocks(const cgan3d_conv_geom* g) {
  const int kind = s2_kind(g);
  if (!kind) return 0;
  S2Args a = s2_args(g, kind);
  return (long long)a.n * a.td * a.th * a.tw;
}

int s2_launch(const cgan3d_conv_geom* g, const float* x, const __bf16* wp, float* y, const Epi& e, hipStream_t st) {
  const int kind = s2_kind(g);
  if (!kind || e.residual || e.mask_src || e.stats || e.minuend || e.out2) {
    set_error("conv_s2: geometry or epilogue not supported (residual/mask/stats/out2)");
    return CGAN3D_EINVAL;
  }
  if (e.out16 && (kind != 2 || !e.x16)) {
    set_error("conv_s2: out_bf16 only on the S2T kernel with the bf16 input shadow");
    return CGAN3D_EINVAL;
  }
  S2Args a = s2_args(g, kind);
  if ((long long)g->n * g->do_ * g->ho * g->wo * g->cout >= (1LL << 31)) {  // 32-bit output offsets
    set_error("conv_s2: output too large for 32-bit element offsets");
    return CGAN3D_EINVAL;
  }
  const long long ntiles = (long long)a.n * a.td * a.th * a.tw;
  const dim3 grid((unsigned)ntiles);
  const int mode = s2_host_stat_mode(e);
#define CG_S2(K, M) ::cg::launch(K<M>, grid, dim3(256), 0, st, a, x, wp, y, e)
  if (kind == 1) { if (mode == 2) CG_S2(conv_s2f_kernel, 2); else if (mode == 1) CG_S2(conv_s2f_kernel, 1); else CG_S2(conv_s2f_kernel, 0); }
#undef CG_S2
  else {  // persistent: two blocks per CU (one for mode 2 from fp32 input: its staging registers)
    const long long per_cu = mode == 2 && !e.x16 ? 1 : 2;
    const dim3 pgrid((unsigned)std::min<long long>(ntiles, per_cu * cu_count()));
#define CG_S2T(M, X, B) ::cg::launch(conv_s2t_kernel<M, X, B>, pgrid, dim3(256), 0, st, a, x, wp, y, e, (int)ntiles)
    if (e.out16) { if (mode == 2) CG_S2T(2, true, true); else if (mode == 1) CG_S2T(1, true, true); else CG_S2T(0, true, true); }
    else if (e.x16) { if (mode == 2) CG_S2T(2, true, false); else if (mode == 1) CG_S2T(1, true, false); else CG_S2T(0, true, false); }
    else { if (mode == 2) CG_S2T(2, false, false); else if (mode == 1) CG_S2T(1, false, false); else CG_S2T(0, false, false); }
#undef CG_S2T
  }
  return CGAN3D_OK;
}

}  // namespace cg
