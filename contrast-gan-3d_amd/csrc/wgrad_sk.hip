// The critic's middle-layer weight gradients (model/discriminator.py:42-68: Conv3d k4 s2 p1,
// 8 -> 16 -> 32 -> 64 channels) in the gradient-penalty update (trainer/Trainer.py:108-142), round 5.
//
//   dW[t][a][b] = sum_o X(2 o - 1 + t)[a] * dZ(o)[b],  t in 4^3 taps
//
// The generic bf16 weight-gradient kernel (conv_wgrad.hip) owns 64 (tap, channel) rows per block and
// re-gathers X for every 8-tap row block: at 12 samples of 64^3 patches the three layers took 36 us
// in one grouped launch at ~1.5 % MFMA busy (profiles/r05_mfma_busy.json).  Here a block owns an
// output tile of one sample and stages, once, the tile's input window (2T + 2 per dimension, bf16
// rows of the cin channels) and its dZ rows (bf16 rows of cout) in LDS; every tap is then a row
// shift inside the window.  MFMA v_mfma_f32_16x16x32_bf16 with M = (tap, input channel), N = output
// channel, K = the tile's voxels; both operands are read as fragments with ds_read_b64_tr_b16 (a
// 16-lane group reads 4 voxel rows x 16 channels, lane i receiving channel i of the 4 voxels), so
// a tap costs one address per lane and no data movement.  Variants (compile-time tiles):
//   V0  8 -> 16: tile 4 x 8 x 16, all 64 taps per block (wave w: tz = w; an M tile is 2 taps x 8
//       input channels);
//   V1 16 -> 32: tile 4 x 4 x 8, all taps (wave w: tz = w, 16 taps x 2 N tiles);
//   V2 32 -> 64: tile 4 x 4 x 4, one tap plane tz per block (wave w: ty = w; 4 taps x 2 M x 4 N
//       tiles) — the window then holds only the TZ input planes 2 z - 1 + tz.
//   V3 64 -> 1, k4 s1 p1 (the last layer, discriminator.py:70-80; exact fp32 as its other roles): a
//       block per sample, fp32 FMA over the sample's <= 64 output voxels (its own VALU body; in the
//       same launch, so the last layer's weight gradient costs no launch of its own).
// Per-block partial tiles go to a workspace in fragment order (each lane's 4 accumulator values,
// 1 KB contiguous per wave-instruction; no atomics), and the second launch sums them over the
// samples / tiles into dW (+=, torch layout) — the grouped launch's unpack pass, replaced.  The grid
// stays within one round of the 256 CUs (1 block per CU: 4 waves at ~300 registers).
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_s __attribute__((ext_vector_type(4)));
typedef short s16x4_s __attribute__((ext_vector_type(4)));

template <int CIN_, int COUT_, int TZ_, int TY_, int TX_, bool ALLTZ_>
struct SkwV {
  static constexpr int CIN = CIN_, COUT = COUT_, TZ = TZ_, TY = TY_, TX = TX_;
  static constexpr bool ALLTZ = ALLTZ_;                       // all 64 taps per block (else one tz)
  static constexpr int NTG = ALLTZ ? 1 : 4;                   // tap groups (blocks per tile)
  static constexpr int WZ = ALLTZ ? 2 * TZ + 2 : TZ, WY = 2 * TY + 2, WX = 2 * TX + 2;
  static constexpr int XROWS = WZ * WY * WX, ZROWS = TZ * TY * TX;
  static constexpr int XB = 2 * CIN, ZB = 2 * COUT;          // LDS row bytes
  static constexpr int LDS = XROWS * XB + ZROWS * ZB;
  static constexpr int KSTEPS = ZROWS / 32;
  static constexpr int NT = COUT / 16;
  // accumulator tiles per wave
  static constexpr int TPW = CIN == 8 ? 8 : (CIN == 16 ? 16 * NT : 4 * 2 * NT);
};
using SkwV0 = SkwV<8, 16, 4, 8, 16, true>;
using SkwV1 = SkwV<16, 32, 4, 4, 8, true>;
using SkwV2 = SkwV<32, 64, 4, 4, 4, false>;
static_assert(SkwV0::TPW == 8 && SkwV1::TPW == 32 && SkwV2::TPW == 32, "tiles per wave");

// tile i of wave w (tap group tg): its tap (tz, ty, tx) for M rows m < 8 (V0: m >= 8 is tx + 1),
// its first input channel and its N tile
template <class V>
__device__ __forceinline__ void skw_tile(int tg, int w, int i, int& tz, int& ty, int& tx, int& a0, int& nt) {
  if constexpr (V::CIN == 8) {  // wave: tz; tile i = (ty, tx pair)
    tz = w; ty = i >> 1; tx = 2 * (i & 1); a0 = 0; nt = 0;
  } else if constexpr (V::CIN == 16) {  // wave: tz; tile i = (tap (ty, tx), N tile)
    tz = w; ty = (i / V::NT) >> 2; tx = (i / V::NT) & 3; a0 = 0; nt = i % V::NT;
  } else {  // one tz per block; wave: ty; tile i = (tx, M tile, N tile)
    tz = tg; ty = w; tx = i / (2 * V::NT); a0 = 16 * ((i / V::NT) & 1); nt = i % V::NT;
  }
}

struct SkwArgs {
  int n, di, hi, wi, dout, hout, wout;  // volumes (input X, output dZ)
  int tz_n, ty_n, tx_n;                 // tiles per dimension
  const float* x;                       // X  [n][di][hi][wi][cin]
  const float* dz;                      // dZ [n][dout][hout][wout][cout]
  float* ws;                            // partials [block][tile][lane][4]
  float* dw;                            // dW (torch layout, strides w_sa / w_sb), += in the reduce
  long long w_sa, w_sb;
  int variant;                          // 0, 1, 2 (SkwV0..2), 3 (the fp32 64 -> 1 last layer)
  int blocks;                           // tiles * NTG (variant 3: samples)
};

__device__ __forceinline__ bf16x8_s skw_tr(const unsigned char* lds, int off0, int off1) {
  const s16x4_s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_s*)(lds + off0));
  const s16x4_s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_s*)(lds + off1));
  return __builtin_bit_cast(bf16x8_s, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <class V>
__device__ __forceinline__ void skw_block(const SkwArgs& a, int bid, unsigned char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tg = bid % V::NTG, tile = bid / V::NTG;
  int t = tile;
  const int txi = t % a.tx_n;
  t /= a.tx_n;
  const int tyi = t % a.ty_n;
  t /= a.ty_n;
  const int tzi = t % a.tz_n, nb = t / a.tz_n;
  const int oz0 = tzi * V::TZ, oy0 = tyi * V::TY, ox0 = txi * V::TX;
  unsigned char* xs = smem;
  unsigned char* zs = smem + V::XROWS * V::XB;

  // ---- staging: X window rows (input voxel (2 oz0 - 1 + wz or 2 (oz0 + wz) - 1 + tz, 2 oy0 - 1 + wy,
  // 2 ox0 - 1 + wx)) and dZ tile rows, fp32 -> bf16, in 4-channel chunks; rounds of RND chunks per
  // thread, every load of a round before its LDS writes (caps the staging registers)
  constexpr int XC = V::XROWS * (V::CIN / 4), ZC = V::ZROWS * (V::COUT / 4);
  constexpr int RND = 12;
  auto stage = [&](auto is_x, int nch, int c0) {
    constexpr bool X = decltype(is_x)::value;
    f32x4 v[RND];
#pragma unroll
    for (int j = 0; j < RND; ++j) {
      const int c = c0 + tid + 256 * j;
      bool ok = c < nch;
      long long off = 0;
      if constexpr (X) {
        const int row = c / (V::CIN / 4), part = c - row * (V::CIN / 4);
        const int wx = row % V::WX, r2 = row / V::WX, wy = r2 % V::WY, wz = r2 / V::WY;
        const int iz = V::ALLTZ ? 2 * oz0 - 1 + wz : 2 * (oz0 + wz) - 1 + tg;
        const int iy = 2 * oy0 - 1 + wy, ix = 2 * ox0 - 1 + wx;
        ok = ok && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi;
        off = ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * V::CIN + 4 * part : 0;
        v[j] = *reinterpret_cast<const f32x4*>(a.x + off);
      } else {
        const int row = c / (V::COUT / 4), part = c - row * (V::COUT / 4);
        const int lx = row % V::TX, r2 = row / V::TX, ly = r2 % V::TY, lz = r2 / V::TY;
        off = ok ? ((((long long)nb * a.dout + oz0 + lz) * a.hout + oy0 + ly) * a.wout + ox0 + lx) * V::COUT + 4 * part : 0;
        v[j] = *reinterpret_cast<const f32x4*>(a.dz + off);
      }
      if (!ok) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < RND; ++j) {
      const int c = c0 + tid + 256 * j;
      if (c < nch) {
        bf16x4_s b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[j][e];
        *reinterpret_cast<bf16x4_s*>((X ? xs : zs) + c * 8) = b;  // row-major chunks: c * 8 = row * rowbytes + part * 8
      }
    }
  };
  for (int c0 = 0; c0 < ZC; c0 += 256 * RND) stage(std::false_type{}, ZC, c0);
  for (int c0 = 0; c0 < XC; c0 += 256 * RND) stage(std::true_type{}, XC, c0);
  __syncthreads();

  // ---- MFMAs: lane (G = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3) supplies, for read r of a
  // K-step, voxel k = 32 ks + 8 G + 4 r + q of the tile (tile-linear z, y, x) and 4-channel chunk pp
  const int G = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  f32x4 acc[V::TPW];
#pragma unroll
  for (int i = 0; i < V::TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < V::KSTEPS; ++ks) {
    int xb[2], zb[2];  // window row of tap (0, 0, 0) / dZ row of this lane's voxel, per read
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = 32 * ks + 8 * G + 4 * r + q;
      const int lx = k % V::TX, ly = (k / V::TX) % V::TY, lz = k / (V::TX * V::TY);
      xb[r] = ((V::ALLTZ ? 2 * lz : lz) * V::WY + 2 * ly) * V::WX + 2 * lx;
      zb[r] = k;
    }
    bf16x8_s bfr[V::NT];
#pragma unroll
    for (int nt = 0; nt < V::NT; ++nt)
      bfr[nt] = skw_tr(zs, zb[0] * V::ZB + (16 * nt + 4 * pp) * 2, zb[1] * V::ZB + (16 * nt + 4 * pp) * 2);
#pragma unroll
    for (int i = 0; i < V::TPW; ++i) {
      int tz, ty, tx, a0, nt;
      skw_tile<V>(0, wave, i, tz, ty, tx, a0, nt);  // tz of V2 is the block's: not part of the row
      bf16x8_s afr;
      if constexpr (V::CIN == 8) {  // rows 0-7: tap tx, rows 8-15: tap tx + 1
        const int sh = ((V::ALLTZ ? tz : 0) * V::WY + ty) * V::WX + tx + (pp >> 1);
        afr = skw_tr(xs, (xb[0] + sh) * V::XB + (pp & 1) * 8, (xb[1] + sh) * V::XB + (pp & 1) * 8);
      } else {
        const int sh = ((V::ALLTZ ? tz : 0) * V::WY + ty) * V::WX + tx;
        afr = skw_tr(xs, (xb[0] + sh) * V::XB + (a0 + 4 * pp) * 2, (xb[1] + sh) * V::XB + (a0 + 4 * pp) * 2);
      }
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[nt], acc[i], 0, 0, 0);
    }
  }
  // ---- partial tiles, fragment order [block][wave][i][lane][4]
  float* o = a.ws + ((long long)bid * 4 * V::TPW + wave * V::TPW) * 256 + lane * 4;
#pragma unroll
  for (int i = 0; i < V::TPW; ++i) *reinterpret_cast<f32x4*>(o + i * 256) = acc[i];
}

// ---- V3: the last layer (64 -> 1, k4 s1 p1), exact fp32: block = sample; thread = (input channel
// a = tid / 4, tap plane tz = tid % 4) x its 16 taps (ty, tx); partial [sample][a][tap]
constexpr int SKW3_XMAX = 64 * 64;  // <= 64 input voxels x 64 channels (fp32)
__device__ __forceinline__ void skw_last_block(const SkwArgs& a, int nb, unsigned char* smem) {
  float* xs = reinterpret_cast<float*>(smem);
  float* zs = xs + SKW3_XMAX;
  const int tid = threadIdx.x;
  const int vin = a.di * a.hi * a.wi, vout = a.dout * a.hout * a.wout;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(a.x + (long long)nb * vin * 64);
  for (int i = tid; i < vin * 16; i += 256) reinterpret_cast<f32x4*>(xs)[i] = x4[i];
  for (int i = tid; i < vout; i += 256) zs[i] = a.dz[(long long)nb * vout + i];
  __syncthreads();
  const int ch = tid >> 2, tz = tid & 3;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int o = 0; o < vout; ++o) {
    const int ox = o % a.wout, oy = (o / a.wout) % a.hout, oz = o / (a.wout * a.hout);
    const float g = zs[o];
    const int iz = oz - 1 + tz;
    if ((unsigned)iz >= (unsigned)a.di) continue;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int iy = oy - 1 + (j >> 2), ix = ox - 1 + (j & 3);
      if ((unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi)
        acc[j] = fmaf(xs[((iz * a.hi + iy) * a.wi + ix) * 64 + ch], g, acc[j]);
    }
  }
  float* o = a.ws + (long long)nb * 4096 + ch * 64 + tz * 16;
#pragma unroll
  for (int j = 0; j < 16; j += 4) *reinterpret_cast<f32x4*>(o + j) = f32x4{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
}

// A group of up to 4 layers in one launch: item j owns blocks [first[j], first[j + 1])
constexpr int SKW_GROUP = 4;
struct SkwGroup {
  SkwArgs a[SKW_GROUP];
  int first[SKW_GROUP + 1];
  int n;
};

template <int I>
__device__ __forceinline__ void skw_item(const SkwGroup& G, unsigned char* smem) {
  const SkwArgs& a = G.a[I];
  const int bid = blockIdx.x - G.first[I];
  if (a.variant == 0) skw_block<SkwV0>(a, bid, smem);
  else if (a.variant == 1) skw_block<SkwV1>(a, bid, smem);
  else if (a.variant == 2) skw_block<SkwV2>(a, bid, smem);
  else skw_last_block(a, bid, smem);
}

constexpr int skw_max(int x, int y) { return x > y ? x : y; }
constexpr int SKW_LDS = skw_max(skw_max(SkwV0::LDS, SkwV1::LDS), skw_max(SkwV2::LDS, (SKW3_XMAX + 64) * 4));
static_assert(SKW_LDS <= 160 * 1024, "LDS");

__global__ __launch_bounds__(256) void wgrad_sk_kernel(SkwGroup G) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SKW_LDS];
  const int bid = blockIdx.x;
  if (G.n > 3 && bid >= G.first[3]) skw_item<3>(G, smem);
  else if (G.n > 2 && bid >= G.first[2]) skw_item<2>(G, smem);
  else if (G.n > 1 && bid >= G.first[1]) skw_item<1>(G, smem);
  else skw_item<0>(G, smem);
}

// ---- reduce: element e = (tap group tg, tile index, lane, jj) of the partials; a block = EB elements
// x S = 256 / EB slices of the blocks of that tap group (spatial tiles x samples), combined in LDS;
// += into dW[b][a][tap]
template <class V>
__device__ __forceinline__ void skw_reduce_item(const SkwArgs& a, int lb, int EB, float* red) {
  constexpr int PER = 4 * V::TPW * 256;  // floats per block of the main kernel
  const int S = 256 / EB, el = threadIdx.x % EB, sl = threadIdx.x / EB;
  const long long e = (long long)lb * EB + el;
  const int tg = (int)(e / PER), r = (int)(e - (long long)tg * PER);
  const int nsp = a.blocks / V::NTG;
  const float* p = a.ws + (long long)tg * PER + r;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int sp = sl;
  for (; sp + 3 * S < nsp; sp += 4 * S) {
    s0 += p[(long long)(sp + 0 * S) * V::NTG * PER];
    s1 += p[(long long)(sp + 1 * S) * V::NTG * PER];
    s2 += p[(long long)(sp + 2 * S) * V::NTG * PER];
    s3 += p[(long long)(sp + 3 * S) * V::NTG * PER];
  }
  for (; sp < nsp; sp += S) s0 += p[(long long)sp * V::NTG * PER];
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sl != 0) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += red[k * EB + el];
  const int jj = r & 3, lane = (r >> 2) & 63, ti = r >> 8, w = ti / V::TPW, i = ti - w * V::TPW;
  int tz, ty, tx, a0, nt;
  skw_tile<V>(tg, w, i, tz, ty, tx, a0, nt);
  const int m = 4 * (lane >> 4) + jj, n = lane & 15;
  int ch = a0 + m;
  if (V::CIN == 8 && m >= 8) {
    ch = m - 8;
    tx += 1;
  }
  const int tap = (tz * 4 + ty) * 4 + tx, b = 16 * nt + n;
  float* d = a.dw + (long long)b * a.w_sb + (long long)ch * a.w_sa + tap;
  *d += s;
}

struct SkwReduce {
  SkwArgs a[SKW_GROUP];
  int first[SKW_GROUP + 1];  // block ranges
  int eb[SKW_GROUP];         // elements per block (256 / slices)
  int n;
};

// the last layer's partials [sample][a][tap]: thread = element, summed over the samples
__device__ __forceinline__ void skw_reduce_last(const SkwArgs& a, int lb) {
  const int e = lb * 256 + threadIdx.x;
  if (e >= 4096) return;
  float s = 0.f;
  for (int sp = 0; sp < a.blocks; ++sp) s += a.ws[(long long)sp * 4096 + e];
  a.dw[(long long)(e >> 6) * a.w_sa + (e & 63)] += s;
}

__global__ __launch_bounds__(256) void wgrad_sk_reduce_kernel(SkwReduce R) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < R.n && b >= R.first[j + 1]) ++j;
  const SkwArgs& a = R.a[j];
  if (a.variant == 0) skw_reduce_item<SkwV0>(a, b - R.first[j], R.eb[j], red);
  else if (a.variant == 1) skw_reduce_item<SkwV1>(a, b - R.first[j], R.eb[j], red);
  else if (a.variant == 2) skw_reduce_item<SkwV2>(a, b - R.first[j], R.eb[j], red);
  else skw_reduce_last(a, b - R.first[j]);
}

// ---- host side
int wgrad_sk_variant(const cgan3d_conv_geom* g) {
  if (g->transposed || g->reflect || g->planar || g->k != 4 || g->pad != 1) return -1;
  // the last layer (k4 s1, 64 -> 1, exact fp32 in every precision): 4^3 -> 3^3 at 64^3 patches
  if (g->stride == 1 && g->cout == 1 && g->cin == 64 && (long long)g->di * g->hi * g->wi <= 64 &&
      (long long)g->do_ * g->ho * g->wo <= 64 && g->do_ == g->di - 1 && g->ho == g->hi - 1 && g->wo == g->wi - 1)
    return 3;
  if (g->prec != CGAN3D_PREC_BF16 || g->stride != 2) return -1;
  if (g->di != 2 * g->do_ || g->hi != 2 * g->ho || g->wi != 2 * g->wo) return -1;
  if ((long long)g->n * g->di * g->hi * g->wi * g->cin >= (1LL << 40)) return -1;
  auto fits = [&](int tz, int ty, int tx) { return g->do_ % tz == 0 && g->ho % ty == 0 && g->wo % tx == 0; };
  if (g->cin == 8 && g->cout == 16 && fits(SkwV0::TZ, SkwV0::TY, SkwV0::TX)) return 0;
  if (g->cin == 16 && g->cout == 32 && fits(SkwV1::TZ, SkwV1::TY, SkwV1::TX)) return 1;
  if (g->cin == 32 && g->cout == 64 && fits(SkwV2::TZ, SkwV2::TY, SkwV2::TX)) return 2;
  return -1;
}

static SkwArgs skw_args(const cgan3d_conv_geom* g, int v) {
  SkwArgs a{};
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.dout = g->do_; a.hout = g->ho; a.wout = g->wo;
  a.variant = v;
  a.w_sa = g->w_sa; a.w_sb = g->w_sb;
  if (v == 3) {
    a.blocks = g->n;
    return a;
  }
  int tz, ty, tx, ntg;
  if (v == 0) { tz = SkwV0::TZ; ty = SkwV0::TY; tx = SkwV0::TX; ntg = SkwV0::NTG; }
  else if (v == 1) { tz = SkwV1::TZ; ty = SkwV1::TY; tx = SkwV1::TX; ntg = SkwV1::NTG; }
  else { tz = SkwV2::TZ; ty = SkwV2::TY; tx = SkwV2::TX; ntg = SkwV2::NTG; }
  a.tz_n = g->do_ / tz; a.ty_n = g->ho / ty; a.tx_n = g->wo / tx;
  a.blocks = g->n * a.tz_n * a.ty_n * a.tx_n * ntg;
  a.w_sa = g->w_sa; a.w_sb = g->w_sb;
  return a;
}

static long long skw_tpw(int v) { return v == 0 ? SkwV0::TPW : (v == 1 ? SkwV1::TPW : SkwV2::TPW); }

long long wgrad_sk_ws_floats(const cgan3d_conv_geom* g) {
  const int v = wgrad_sk_variant(g);
  if (v < 0) return 0;
  const SkwArgs a = skw_args(g, v);
  return v == 3 ? (long long)a.blocks * 4096 : (long long)a.blocks * 4 * skw_tpw(v) * 256;
}

int wgrad_sk_launch(const cgan3d_conv_geom* geoms, const float* const* gathered, const float* const* aligned,
                    float* const* ws, float* const* dw, int n, hipStream_t st) {
  SkwGroup G{};
  SkwReduce R{};
  G.n = R.n = n;
  for (int i = 0; i < n; ++i) {
    const int v = wgrad_sk_variant(&geoms[i]);
    SkwArgs a = skw_args(&geoms[i], v);
    a.x = gathered[i]; a.dz = aligned[i]; a.ws = ws[i]; a.dw = dw[i];
    G.a[i] = R.a[i] = a;
    G.first[i + 1] = G.first[i] + a.blocks;
    if (v == 3) {  // 4096 elements, one per thread
      R.eb[i] = 256;
      R.first[i + 1] = R.first[i] + 16;
      continue;
    }
    const int ntg = v == 2 ? SkwV2::NTG : 1;
    const long long elems = (long long)ntg * 4 * skw_tpw(v) * 256;
    // slices per element: ~12 partials per thread (the sums over up to a few hundred blocks stay short)
    const int nsp = a.blocks / ntg;
    int S = 1;
    while (S < 16 && nsp > 12 * S) S *= 2;
    R.eb[i] = 256 / S;
    R.first[i + 1] = R.first[i] + (int)(elems / R.eb[i]);
  }
  ::cg::launch(wgrad_sk_kernel, dim3(G.first[n]), dim3(256), 0, st, G);
  ::cg::launch(wgrad_sk_reduce_kernel, dim3((unsigned)R.first[n]), dim3(256), 0, st, R);
  return CGAN3D_OK;
}

}  // namespace cg

using namespace cg;

extern "C" int32_t cgan3d_conv3d_wgrad_sk_ok(const cgan3d_conv_geom* g) {
  return g && wgrad_sk_variant(g) >= 0 ? 1 : 0;
}

extern "C" int64_t cgan3d_conv3d_wgrad_sk_ws_floats(const cgan3d_conv_geom* g) {
  return g ? wgrad_sk_ws_floats(g) : 0;
}

extern "C" int cgan3d_conv3d_wgrad_sk(const cgan3d_conv_geom* geoms, const float* const* gathered,
                                      const float* const* aligned, float* const* ws, float* const* dw, int32_t n,
                                      void* stream) {
  CG_CHECK_ARG(geoms && gathered && aligned && ws && dw && n >= 1 && n <= SKW_GROUP,
               "cgan3d_conv3d_wgrad_sk: bad arguments (1..4 items)");
  for (int i = 0; i < n; ++i) {
    CG_CHECK_ARG(wgrad_sk_variant(&geoms[i]) >= 0, "cgan3d_conv3d_wgrad_sk: item %d not eligible", i);
    CG_CHECK_ARG(gathered[i] && aligned[i] && ws[i] && dw[i], "cgan3d_conv3d_wgrad_sk: null pointer in item %d", i);
    CG_CHECK_ARG(!(((uintptr_t)gathered[i] | (uintptr_t)aligned[i] | (uintptr_t)ws[i]) & 15),
                 "cgan3d_conv3d_wgrad_sk: operands must be 16-byte aligned");
  }
  const int rc = wgrad_sk_launch(geoms, gathered, aligned, ws, dw, n, (hipStream_t)stream);
  if (rc) return rc;
  CG_LAUNCH_CHECK("wgrad_sk_kernel");
  return CGAN3D_OK;
}
