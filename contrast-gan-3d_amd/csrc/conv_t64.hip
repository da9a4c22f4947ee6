// Stride-2 transposed convolution 64 -> 32 channels at the generator's 32 <-> 64 level, every operand
// of a block resident in LDS (round 5): the first ConvTranspose3d forward (model/generator.py:61-77,
// k3 s2 p1 output_padding 1, 16^3 x 64 -> 32^3 x 32 at 64^3 patches) and the input-grad of the second
// downsampling Conv3d (generator.py:40-47; the same transposed mapping of its dL/dz).
//
// conv_halo_kernel ran these as one block per (parity class, 4^3 class tile): 2048 blocks of 64 output
// voxels x 32 channels with 1-8 taps each, two barriers per tap and the BatchNorm epilogue's three —
// 25-29 us per launch at 64 VALU per MFMA.  Here a block owns a 4^3 class tile
// with ALL EIGHT parity classes (512 output voxels x 32 channels: 1.8 GFLOP over 256 blocks at 64^3 B=4, the shape
// of conv_k3m): the classes share one input halo (tile + 1 per axis, 5^3 voxels) and the 27 taps'
// weights, both put into LDS once by LDS-DMA (the halo and the 27 x 4 KB of packed format-2 weights,
// the image conv_k3m stages for one channel half), then each wave runs its share of the 16 (class,
// 32-voxel M tile) items on v_mfma_f32_32x32x16_bf16 — class r has (1 + r_z)(1 + r_y)(1 + r_x)
// taps, the items are dealt 13 / 13 / 14 / 14 taps to the four waves — with no barrier between
// items.  The halo rows (x padded to 6) and the A-row permutation are conv_k3m's, so every A read is
// conflict-free for every tap shift (km_fa swizzle: a 16-lane group reads one 4 x 4 (x, y) plane).
// Epilogue: fp32 or bf16 output, BatchNorm statistics into the fp64 accumulators (cgan3d_bn_fuse mode
// 3: per-lane sums shifted by the lane's first value, merged once; mode 4 with bn_z / bn_ss / bn_mi).
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int T64_HX = 6, T64_HY = 5, T64_HZ = 5;         // halo (x padded to 6: row parity = hx & 1)
constexpr int T64_ROWS = 152;                              // 150 rows + the last DMA's 2 spare rows
constexpr int T64_HALO = T64_ROWS * 128;                   // 19456 B
constexpr int T64_TAPB = 32 * 128;                         // one tap's weights, 32 output channels
constexpr int T64_LDS = T64_HALO + 27 * T64_TAPB;          // 130048 B
constexpr int T64_ITEMS = 5;                               // most items of a wave

__device__ __attribute__((aligned(16))) unsigned char g_t64_zero[16];

struct T64Args {
  int n, di, hi, wi;  // gathered (class) grid; output 2x
  int tx, ty, tz;     // 4^3 tiles per axis
};

__device__ __forceinline__ int t64_fa(int hx, int hy) { return ((hx >> 1) & 1) | ((hy & 3) << 1); }
__device__ __forceinline__ int t64_fw(int c) { return (c >> 1) & 7; }

// A row r (0..31) of an M tile -> (x, y, z-slice zz): lane group {0-3, 12-15, 20-27} is zz = 0,
// {4-11, 16-19, 28-31} zz = 1, 4 x 4 in (x, y) each (conv_k3m's km_row)
__device__ __forceinline__ void t64_row(int r, int& x, int& y, int& zz) {
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

__device__ __forceinline__ void t64_dma16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

// the taps of class bit b along one axis (ConvTranspose k3 s2 p1: output 2j + b reads input j + d
// through tap t): b = 0 -> t = 1, d = 0; b = 1 -> t = 0, d = 1 and t = 2, d = 0
// one (class R = rz rz ry rx bits, M tile M) item: every tap of the class x 4 K-steps of 16 channels
template <int R, int M>
__device__ __forceinline__ void t64_item(const unsigned char* smem, f32x16_t& acc, int lx, int ly, int lzz, int h,
                                         const int (&boff)[4]) {
  constexpr int RZ = (R >> 2) & 1, RY = (R >> 1) & 1, RX = R & 1;
  constexpr int NZ = 1 + RZ, NY = 1 + RY, NX = 1 + RX;
  const int jx = lx, jy = ly, jz = 2 * M + lzz;
#pragma unroll
  for (int iz = 0; iz < NZ; ++iz)
#pragma unroll
    for (int iy = 0; iy < NY; ++iy)
#pragma unroll
      for (int ix = 0; ix < NX; ++ix) {
        const int tz = RZ == 0 ? 1 : (iz == 0 ? 0 : 2), dz = RZ == 0 ? 0 : (iz == 0 ? 1 : 0);
        const int ty = RY == 0 ? 1 : (iy == 0 ? 0 : 2), dy = RY == 0 ? 0 : (iy == 0 ? 1 : 0);
        const int tx = RX == 0 ? 1 : (ix == 0 ? 0 : 2), dx = RX == 0 ? 0 : (ix == 0 ? 1 : 0);
        const int tap = (tz * 3 + ty) * 3 + tx;
        const int hx = jx + dx, hy = jy + dy, hz = jz + dz;
        const int row = (hz * T64_HY + hy) * T64_HX + hx;
        const int f = t64_fa(hx, hy);
        bf16x8_t av[4], bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = *reinterpret_cast<const bf16x8_t*>(smem + row * 128 + 16 * ((2 * s + h) ^ f));
          bv[s] = *reinterpret_cast<const bf16x8_t*>(smem + boff[s] + tap * T64_TAPB);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[s], bv[s], acc, 0, 0, 0);
      }
}

// OB: bit 0 — y and bn_z are bf16 (cgan3d_epilogue.out_bf16)
template <int OB>
__global__ __launch_bounds__(256, 1) void conv_t64_kernel(T64Args a, const __bf16* __restrict__ x16,
                                                          const __bf16* __restrict__ wpk, float* __restrict__ y,
                                                          Epi ep) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[T64_LDS];
  __shared__ float red[3][4][32];
  using lds_t = __attribute__((address_space(3))) void*;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int t = blockIdx.x;
  const int txi = t % a.tx;
  t /= a.tx;
  const int tyi = t % a.ty;
  t /= a.ty;
  const int tzi = t % a.tz;
  const int nb = t / a.tz;
  const int jx0 = 4 * txi, jy0 = 4 * tyi, jz0 = 4 * tzi;
  const int DO = 2 * a.di, HO = 2 * a.hi, WO = 2 * a.wi;

  // ---- this wave's items (class, M tile): 13 / 13 / 14 / 14 taps
  // w0: (7,0) (3,0) (0,0); w1: (7,1) (3,1) (0,1); w2: (5,0) (5,1) (1,0) (1,1) (4,0); w3: (6,0) (6,1) (2,0) (2,1) (4,1)
  auto item_cls = [&](int k) -> int {
    if (wave == 0) return k == 0 ? 7 : k == 1 ? 3 : k == 2 ? 0 : -1;
    if (wave == 1) return k == 0 ? 7 : k == 1 ? 3 : k == 2 ? 0 : -1;
    if (wave == 2) return k < 2 ? 5 : k < 4 ? 1 : 4;
    return k < 2 ? 6 : k < 4 ? 2 : 4;
  };
  auto item_m = [&](int k) -> int {
    if (wave == 0) return 0;
    if (wave == 1) return 1;
    if (wave == 2) return k == 4 ? 0 : (k & 1);
    return k == 4 ? 1 : (k & 1);
  };
  const int nitems = wave < 2 ? 3 : 5;

  // ---- output offsets (round 5b): lane base + a per-item scalar + a per-row delta, instead of 80
  // offsets of ~12 instructions each held in registers; row i of a lane is R = (i & 3) + 8 (i >> 2) +
  // 4 h (the MFMA's accumulator rows), item (class r, M tile m) outputs voxel 2 j + r with j = tile
  // origin + (lx, ly, 2 m + lzz)
  const int c = lane & 31, h = lane >> 5;
  const bool mode4 = ep.fz.acc_mode == 4;
  const int obase = (((nb * DO + 2 * jz0) * HO + 2 * jy0) * WO + 2 * jx0) * 32 + c;
  auto item_off = [&](int k) -> int {  // wave-uniform
    const int cls = item_cls(k), m = item_m(k);
    return (((4 * m + ((cls >> 2) & 1)) * HO + ((cls >> 1) & 1)) * WO + (cls & 1)) * 32;
  };
  int drow[16];
  unsigned vxy = 0, vz = 0;  // per row: (x, y) inside the volume; its z-slice lzz
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int lx, ly, lzz;
    t64_row((i & 3) + 8 * (i >> 2) + 4 * h, lx, ly, lzz);
    drow[i] = ((2 * lzz * HO + 2 * ly) * WO + 2 * lx) * 32;
    vxy |= (unsigned)(jx0 + lx < a.wi && jy0 + ly < a.hi) << i;
    vz |= (unsigned)lzz << i;
  }
  const bool full = jx0 + 4 <= a.wi && jy0 + 4 <= a.hi && jz0 + 4 <= a.di;  // every row of every item
  auto valid = [&](int k, int i) -> bool {
    return k < nitems && ((vxy >> i) & 1) && jz0 + 2 * item_m(k) + (int)((vz >> i) & 1) < a.di;
  };
  float zv[T64_ITEMS][16];
  if (mode4) {  // block-uniform; the z loads go out before the DMAs so the MFMAs cover their round trip
#pragma unroll
    for (int k = 0; k < T64_ITEMS; ++k) {
      const int ok0 = obase + item_off(k);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int zi = (full ? k < nitems : valid(k, i)) ? ok0 + drow[i] : 0;
        if constexpr ((OB & 1) != 0) zv[k][i] = (float)reinterpret_cast<const __bf16*>(ep.bn_z)[zi];
        else zv[k][i] = ep.bn_z[zi];
      }
    }
  }

  // ---- LDS-DMA: the halo (19 wave-instructions of 8 rows; rows past 150 and voxels outside the
  // volume read zeros), then all 27 taps (one 8-channel quarter per wave each)
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_t)smem;
  {
    const int p = lane & 7;
    for (int i = wave; i < T64_ROWS / 8; i += 4) {
      const int row = 8 * i + (lane >> 3);
      const int hx = row % T64_HX, hy = (row / T64_HX) % T64_HY, hz = row / (T64_HX * T64_HY);
      const int ix = jx0 + hx, iy = jy0 + hy, iz = jz0 + hz;
      const bool ok = row < T64_HX * T64_HY * T64_HZ && hx < 5 && ix < a.wi && iy < a.hi && iz < a.di;
      const int g = p ^ t64_fa(hx, hy);
      const void* src = ok ? (const void*)(x16 + ((long long)((nb * a.di + iz) * a.hi + iy) * a.wi + ix) * 64 + 8 * g)
                           : (const void*)g_t64_zero;
      t64_dma16(src, __builtin_amdgcn_readfirstlane(lds0 + i * 1024));
    }
    const int cw = 8 * wave + (lane >> 3);  // output channel row of the tap image
    // packed format 2 keeps logical granule q of (tap, channel) at position q ^ (channel & 7)
    const __bf16* src = wpk + (long long)cw * 64 + 8 * ((p ^ t64_fw(cw)) ^ (cw & 7));
#pragma unroll
    for (int tp = 0; tp < 27; ++tp)
      t64_dma16(src + (long long)tp * 32 * 64, __builtin_amdgcn_readfirstlane(lds0 + T64_HALO + tp * T64_TAPB + wave * 1024));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- the items
  int lx, ly, lzz;
  t64_row(c, lx, ly, lzz);
  int boff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) boff[s] = T64_HALO + c * 128 + 16 * ((2 * s + h) ^ t64_fw(c));
  f32x16_t acc[T64_ITEMS];
#pragma unroll
  for (int k = 0; k < T64_ITEMS; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[k][i] = 0.f;
  if (wave == 0) {
    t64_item<7, 0>(smem, acc[0], lx, ly, lzz, h, boff);
    t64_item<3, 0>(smem, acc[1], lx, ly, lzz, h, boff);
    t64_item<0, 0>(smem, acc[2], lx, ly, lzz, h, boff);
  } else if (wave == 1) {
    t64_item<7, 1>(smem, acc[0], lx, ly, lzz, h, boff);
    t64_item<3, 1>(smem, acc[1], lx, ly, lzz, h, boff);
    t64_item<0, 1>(smem, acc[2], lx, ly, lzz, h, boff);
  } else if (wave == 2) {
    t64_item<5, 0>(smem, acc[0], lx, ly, lzz, h, boff);
    t64_item<5, 1>(smem, acc[1], lx, ly, lzz, h, boff);
    t64_item<1, 0>(smem, acc[2], lx, ly, lzz, h, boff);
    t64_item<1, 1>(smem, acc[3], lx, ly, lzz, h, boff);
    t64_item<4, 0>(smem, acc[4], lx, ly, lzz, h, boff);
  } else {
    t64_item<6, 0>(smem, acc[0], lx, ly, lzz, h, boff);
    t64_item<6, 1>(smem, acc[1], lx, ly, lzz, h, boff);
    t64_item<2, 0>(smem, acc[2], lx, ly, lzz, h, boff);
    t64_item<2, 1>(smem, acc[3], lx, ly, lzz, h, boff);
    t64_item<4, 1>(smem, acc[4], lx, ly, lzz, h, boff);
  }

  // ---- epilogue: stores, then the statistics of channel c over this lane's outputs.  Round 5b: the
  // statistics mode and the BatchNorm activation are uniform branches around whole loops, and a tile
  // inside the volume (all of them at 64^3) needs no per-element validity (VALU per MFMA 46.7 in
  // profiles/r05_pmc_sq_step.json before)
  const int mode = ep.fz.acc_mode;
  float n1 = 0.f, K = 0.f, s1 = 0.f, s2 = 0.f;
  auto store = [&](int o, float v) {
    if constexpr ((OB & 1) != 0) reinterpret_cast<__bf16*>(y)[o] = (__bf16)v;
    else y[o] = v;
  };
  if (mode == 3 && full) {  // shift = the lane's first value; n = 16 per item
    K = acc[0][0];
#pragma unroll
    for (int k = 0; k < T64_ITEMS; ++k) {
      if (k >= nitems) break;
      const int ok0 = obase + item_off(k);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = acc[k][i];
        store(ok0 + drow[i], v);
        const float d = v - K;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
    }
    n1 = 16.f * nitems;
  } else if (mode4) {
    const float sc = ep.bn_ss[c], sh = ep.bn_ss[32 + c], mu = ep.bn_mi[c], is = ep.bn_mi[32 + c];
    const int bact = ep.bn_act;
    const float bslope = ep.bn_slope;
#pragma unroll
    for (int k = 0; k < T64_ITEMS; ++k) {
      if (k >= nitems) break;
      const int ok0 = obase + item_off(k);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (!full && !valid(k, i)) continue;
        const float v = acc[k][i];
        store(ok0 + drow[i], v);
        const float pre = zv[k][i] * sc + sh;
        const float gg = bact == CGAN3D_ACT_RELU ? (pre > 0.f ? v : 0.f)
                                                 : (bact == CGAN3D_ACT_LRELU ? (pre > 0.f ? v : v * bslope) : v);
        s1 += gg;
        s2 += gg * (zv[k][i] - mu) * is;
      }
    }
  } else {  // no statistics, or mode 3 on a ragged tile (the shift is the first valid value)
    bool first = true;
#pragma unroll
    for (int k = 0; k < T64_ITEMS; ++k) {
      if (k >= nitems) break;
      const int ok0 = obase + item_off(k);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (!full && !valid(k, i)) continue;
        const float v = acc[k][i];
        store(ok0 + drow[i], v);
        if (mode == 3) {
          if (first) { K = v; first = false; }
          const float d = v - K;
          s1 += d;
          s2 = fmaf(d, d, s2);
          n1 += 1.f;
        }
      }
    }
  }
  if (!mode) return;
  double* const facc = ep.fz.acc_out + (long long)(blockIdx.x % ep.fz.reps) * 2 * 32;
  if (mode == 3) {  // lane (n, mean, M2) -> merged with lane ^ 32 (same channel), then the 4 waves
    float mm = n1 > 0.f ? K + s1 / n1 : 0.f, q = n1 > 0.f ? fmaxf(s2 - s1 * s1 / n1, 0.f) : 0.f, nn = n1;
    {
      const float no = __shfl_xor(nn, 32, 64), mo = __shfl_xor(mm, 32, 64), qo = __shfl_xor(q, 32, 64);
      const float nt = nn + no;
      if (no > 0.f) {
        const float dl = mo - mm;
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
        unsafeAtomicAdd(facc + tid, S);
        unsafeAtomicAdd(facc + 32 + tid, (double)rq + S * (double)rm);
      }
    }
  } else {  // mode 4: (sum g, sum g * xhat)
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (h == 0) { red[0][wave][c] = s1; red[1][wave][c] = s2; }
    __syncthreads();
    if (tid < 32) {
      unsafeAtomicAdd(facc + tid, (double)(red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid]));
      unsafeAtomicAdd(facc + 32 + tid, (double)(red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid]));
    }
  }
}

// ConvTranspose3d k3 s2 p1 (output padding 1) 64 -> 32 with the bf16 input shadow and format-2 packed
// weights, epilogue: output (fp32 / bf16) + fp64-accumulator statistics (mode 3 / 4) or nothing
bool t64_geom_ok(const cgan3d_conv_geom* g) {
#if defined(CGAN3D_NO_T64)
  return false;  // (A/B builds)
#endif
  return k3m_enabled() && g->prec == CGAN3D_PREC_BF16 && g->w_packed == 2 && g->transposed && !g->reflect && !g->planar && g->k == 3 &&
         g->stride == 2 && g->pad == 1 && g->cin == 64 && g->cout == 32 && g->do_ == 2 * g->di &&
         g->ho == 2 * g->hi && g->wo == 2 * g->wi && (long long)g->n * g->do_ * g->ho * g->wo * 32 < (1LL << 31);
}

bool t64_ok(const cgan3d_conv_geom* g, const Epi& e) {
  return t64_geom_ok(g) && e.x16 && !e.bias && !e.residual && !e.mask_src && !e.minuend && !e.out2 && !e.stats && !e.bn_mode &&
         !e.bn_fold && !e.pre.mode && e.act == CGAN3D_ACT_NONE && !e.res16 &&
         (e.fz.acc_mode == 0 || e.fz.acc_mode == 3 || (e.fz.acc_mode == 4 && e.bn_z && e.bn_ss && e.bn_mi));
}

int t64_launch(const cgan3d_conv_geom* g, const __bf16* wp, float* y, const Epi& e, hipStream_t st) {
  T64Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi;
  a.tx = (a.wi + 3) / 4; a.ty = (a.hi + 3) / 4; a.tz = (a.di + 3) / 4;
  const dim3 grid((unsigned)(a.n * a.tx * a.ty * a.tz));
  if (e.out16) ::cg::launch(conv_t64_kernel<1>, grid, dim3(256), 0, st, a, e.x16, wp, y, e);
  else ::cg::launch(conv_t64_kernel<0>, grid, dim3(256), 0, st, a, e.x16, wp, y, e);
  return CGAN3D_OK;
}

}  // namespace cg
