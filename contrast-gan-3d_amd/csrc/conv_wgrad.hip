// Weight gradients of the 3x3 / 4x4 convolutions on bf16 MFMA (CGAN3D_PREC_BF16 geometries).
//
// dW[t, a, b] = sum_o G(o*s - p + t, a) * O(o, b) — the autograd weight gradient of Conv3d
// (model/blocks.py:29-38, discriminator.py:24-80) and, with the roles of the operands swapped by
// the caller, of ConvTranspose3d (blocks.py:23-25).  GEMM: M = (t, a) rows, N = b, K = output
// voxels.  A block owns 64 rows (one tap x 64 channels, or 2-4 taps of 32/16 channels) x all
// output channels (<= 64) and walks a chunk of output voxels 64 at a time:
//
//  * staging: half the threads gather G (f32x4 = 4 channels of one voxel, 8 voxels each), half
//    load O; both are written TRANSPOSED as bf16 —
//    [row][voxel] and [b][voxel] with voxels contiguous — 16 bytes per store, so each MFMA
//    fragment (8 consecutive voxels of one row or column) is one ds_read_b128;
//  * the next chunk's global loads are issued before the MFMAs of the current one;
//  * v_mfma_f32_16x16x32_bf16, fp32 accumulation; per-block results are added into the packed
//    [t][a][b] workspace (then unpacked, conv.hip).
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_w __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_w __attribute__((ext_vector_type(4)));
typedef float f32x16_w __attribute__((ext_vector_type(16)));

struct WgArgs {
  int n, di, hi, wi, do_, ho, wo, cin, cout, k, s, p, reflect;
  int R;            // k^3 * cin
  long long V;      // output voxels
  long long vpb;    // voxels per block (multiple of 64)
};

constexpr int WG_KV = 64, WG_LD = WG_KV + 8;  // voxels per stage; LDS row (bf16) incl. 16 B pad

__device__ __forceinline__ int wg_coord(int i, int n, int reflect) {
  if (reflect) return reflect_idx(i, n);
  return (i >= 0 && i < n) ? i : -1;
}

// PART (round 6): block (bx, by) stores its sums into partial slab `by` of dwp ([slab][t][a][b], summed in
// slab order by wgrad_reduce_ta_kernel) instead of adding them atomically (the grouped launch)
template <int NB, bool ROW8, bool PART = false>
__device__ __forceinline__ void wgrad_bf16_block(const WgArgs& a, const float* __restrict__ gx,
                                                 const float* __restrict__ go, float* dwp, int bx, int by,
                                                 __bf16* As, __bf16* Gs) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = bx * 64;
  const long long vbeg = (long long)by * a.vpb;
  const long long vend = vbeg + a.vpb < a.V ? vbeg + a.vpb : a.V;

  // staging role (wave-uniform): waves 0-1 gather G rows (4rq..4rq+3 = one tap, 4 channels),
  // waves 2-3 load O columns (4rq..4rq+3); lanes with consecutive vo write consecutive 16-byte
  // chunks of one LDS row (conflict-free), 8 lanes with consecutive rq read 128 contiguous bytes
  const bool isA = wave < 2;
  const int vo = tid & 7, rq = (tid >> 3) & 15;
  int td = 0, th = 0, tw = 0, ca = 0;
  bool rowok;
  if (isA) {
    const int r = r0 + 4 * rq;
    rowok = r < a.R;
    const int t = rowok ? r / a.cin : 0;
    ca = rowok ? r - t * a.cin : 0;  // cin % 4 == 0: the 4 rows share the tap
    td = t / (a.k * a.k); th = (t / a.k) % a.k; tw = t % a.k;
  } else {
    rowok = 4 * rq < a.cout;
  }

  auto load = [&](f32x4 (&st)[8], long long vb) {
    // 8 consecutive output voxels 8vo..8vo+7 of the chunk; ROW8 (W % 8 == 0, chunk starts at a
    // multiple of 8): one output row, decoded once
    const int lin0 = (int)(vb + 8 * vo);
    int ow = lin0 % a.wo, q = lin0 / a.wo;
    int oh = q % a.ho;
    q /= a.ho;
    int od = q % a.do_, nb = q / a.do_;
    const int id = wg_coord(od * a.s - a.p + td, a.di, a.reflect);
    const int ih = wg_coord(oh * a.s - a.p + th, a.hi, a.reflect);
    const long long rowA = (((long long)nb * a.di + id) * a.hi + ih) * a.wi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int lin = lin0 + j;
      long long off = -1;
      if (rowok && lin < vend) {
        if (isA) {
          if (ROW8) {
            const int iw = wg_coord((ow + j) * a.s - a.p + tw, a.wi, a.reflect);
            if ((id | ih | iw) >= 0) off = (rowA + iw) * a.cin + ca;
          } else {
            const int id2 = wg_coord(od * a.s - a.p + td, a.di, a.reflect);
            const int ih2 = wg_coord(oh * a.s - a.p + th, a.hi, a.reflect);
            const int iw2 = wg_coord(ow * a.s - a.p + tw, a.wi, a.reflect);
            if ((id2 | ih2 | iw2) >= 0) off = ((((long long)nb * a.di + id2) * a.hi + ih2) * a.wi + iw2) * a.cin + ca;
          }
        } else {
          off = (long long)lin * a.cout + 4 * rq;
        }
      }
      const float* src = isA ? gx : go;
      st[j] = *reinterpret_cast<const f32x4*>(src + (off >= 0 ? off : 0));
      if (off < 0) st[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!ROW8 && ++ow == a.wo) {
        ow = 0;
        if (++oh == a.ho) {
          oh = 0;
          if (++od == a.do_) { od = 0; ++nb; }
        }
      }
    }
  };
  auto store = [&](const f32x4 (&st)[8]) {
    __bf16* base = (isA ? As : Gs) + (4 * rq) * WG_LD + 8 * vo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bf16x8_w v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)st[j][e];
      *reinterpret_cast<bf16x8_w*>(base + e * WG_LD) = v;
    }
  };

  f32x4 acc[NB];
#pragma unroll
  for (int nt = 0; nt < NB; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;
  // the next chunk's global loads are in flight during this chunk's MFMAs; lds_barrier() keeps
  // them in flight across the barriers
  f32x4 st[8];
  load(st, vbeg);
  for (long long vb = vbeg; vb < vend; vb += WG_KV) {
    lds_barrier();  // the previous stage's fragments have been read
    store(st);
    lds_barrier();
    if (vb + WG_KV < vend) load(st, vb + WG_KV);
#pragma unroll
    for (int ks = 0; ks < WG_KV / 32; ++ks) {
      const bf16x8_w av = *reinterpret_cast<const bf16x8_w*>(As + (wave * 16 + r16) * WG_LD + ks * 32 + 8 * g);
#pragma unroll
      for (int nt = 0; nt < NB; ++nt) {
        const bf16x8_w bv = *reinterpret_cast<const bf16x8_w*>(Gs + (nt * 16 + r16) * WG_LD + ks * 32 + 8 * g);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[nt], 0, 0, 0);
      }
    }
  }
  // lane holds dW rows r0 + wave*16 + 4g + jj, column nt*16 + r16
#pragma unroll
  for (int nt = 0; nt < NB; ++nt) {
    const int b = nt * 16 + r16;
    if (b >= a.cout) continue;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int r = r0 + wave * 16 + 4 * g + jj;
      if (r < a.R) {
        if constexpr (PART) dwp[((long long)by * a.R + r) * a.cout + b] = acc[nt][jj];
        else atomicAdd(dwp + (long long)r * a.cout + b, acc[nt][jj]);
      }
    }
  }
}

template <int NB, bool ROW8>
__global__ __launch_bounds__(256) void conv_wgrad_bf16_kernel(WgArgs a, const float* __restrict__ gx,
                                                              const float* __restrict__ go, float* dwp) {
  __shared__ __attribute__((aligned(16))) __bf16 As[64 * WG_LD];  // [row][voxel]
  __shared__ __attribute__((aligned(16))) __bf16 Gs[64 * WG_LD];  // [b][voxel]
  wgrad_bf16_block<NB, ROW8, true>(a, gx, go, dwp, blockIdx.x, blockIdx.y, As, Gs);
}

// dW[b * w_sb + a * w_sa + t] (+)= sum_p ws[p][t][a][b] (T taps, A gathered x B aligned channels): the
// partial slabs of conv_wgrad_bf16_kernel, read along their layout (64 consecutive elements per block x NC
// chunks of the P slabs, one wave per chunk, 8 loads in flight per lane), chunks combined in a fixed order
__global__ __launch_bounds__(1024) void wgrad_reduce_ta_kernel(const float* __restrict__ ws, int P, int NC, int T,
                                                               int A, int B, float* dw, long long w_sa, long long w_sb,
                                                               int accumulate) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6;
  const long long E = (long long)T * A * B, e = (long long)blockIdx.x * 64 + lane;
  const bool ok = e < E;
  const int pc = (P + NC - 1) / NC, p0 = c * pc, p1 = min(P, p0 + pc);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  for (int p = p0; p < p1; p += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = ws[(long long)(p + j < p1 ? p + j : p0) * E + (ok ? e : 0)];
      s[j] += p + j < p1 ? v : 0.f;
    }
  part[c][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (c == 0 && ok) {
    float v = 0.f;
    for (int k = 0; k < NC; ++k) v += part[k][lane];
    const int b = (int)(e % B), r = (int)(e / B), a = r % A, t = r / A;
    float* o = dw + (long long)b * w_sb + (long long)a * w_sa + t;
    *o = accumulate ? *o + v : v;
  }
}

// ---- several of those weight gradients in one launch (cgan3d_conv3d_wgrad_group): item i owns the
// blocks [first[i], first[i + 1]) of a 1-D grid; each block runs the single kernel's body with its
// item's operands (the critic's middle layers after the penalty's forward-mode chain: independent
// grids of 100-300 blocks that each leave most of the chip idle and pay a launch apiece)
constexpr int WG_GROUP = 4;
struct WgGroup {
  WgArgs a[WG_GROUP];
  const float* gx[WG_GROUP];
  const float* go[WG_GROUP];
  float* dwp[WG_GROUP];
  int gxb[WG_GROUP];          // row blocks of the item (its grid's x extent)
  int nb[WG_GROUP];           // 16-column tiles (cout / 16, rounded up)
  int row8[WG_GROUP];         // W % 8 == 0
  int first[WG_GROUP + 1];
  int n;
};

// item I's operands indexed at compile time (a runtime index into the kernel-argument arrays makes
// hipcc copy the whole struct to scratch)
template <int I>
__device__ __forceinline__ void wgrad_group_item(const WgGroup& G, __bf16* As, __bf16* Gs) {
  const int b = blockIdx.x - G.first[I], bx = b % G.gxb[I], by = b / G.gxb[I];
#define CG_WGG(N) (G.row8[I] ? wgrad_bf16_block<N, true>(G.a[I], G.gx[I], G.go[I], G.dwp[I], bx, by, As, Gs) \
                             : wgrad_bf16_block<N, false>(G.a[I], G.gx[I], G.go[I], G.dwp[I], bx, by, As, Gs))
  if (G.nb[I] == 1) CG_WGG(1); else if (G.nb[I] == 2) CG_WGG(2); else if (G.nb[I] == 3) CG_WGG(3); else CG_WGG(4);
#undef CG_WGG
}

__global__ __launch_bounds__(256) void conv_wgrad_bf16_group_kernel(WgGroup G) {
  __shared__ __attribute__((aligned(16))) __bf16 As[64 * WG_LD];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[64 * WG_LD];
  const int bid = blockIdx.x;
  if (G.n > 3 && bid >= G.first[3]) wgrad_group_item<3>(G, As, Gs);
  else if (G.n > 2 && bid >= G.first[2]) wgrad_group_item<2>(G, As, Gs);
  else if (G.n > 1 && bid >= G.first[1]) wgrad_group_item<1>(G, As, Gs);
  else wgrad_group_item<0>(G, As, Gs);
}

// ---- single-channel input, few output channels (the critic's first layer, 1 -> 8, k4 s2):
// M x N = 64 taps x 8 is too small for MFMA tiles, K = every output voxel.  A thread owns one tap
// and all output channels; the 64 lanes of a wave are the 64 taps of ONE output voxel, so the
// aligned-operand loads are wave-wide broadcasts and the gathered loads hit one 4x4x4 window.
// Per block: fp32 partial sums over its voxel chunk, combined across the waves in LDS, then one
// atomic add per (tap, channel) into dW (zeroed by the caller unless accumulating).  fp32 FMA.
template <int COUT>
__global__ __launch_bounds__(256) void conv_wgrad_c1_kernel(WgArgs a, const float* __restrict__ gx,
                                                            const float* __restrict__ go, float* dw, long long w_sb) {
  constexpr int VL = 4;  // voxel lanes (waves) per block; T = 64 taps per wave
  __shared__ float red[VL][64][COUT + 1];
  const int tid = threadIdx.x, t = tid & 63, vl = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool tok = t < a.R;
  const int td = t / (a.k * a.k), th = (t / a.k) % a.k, tw = t % a.k;
  const long long vbeg = (long long)blockIdx.x * a.vpb;
  const long long vend = vbeg + a.vpb < a.V ? vbeg + a.vpb : a.V;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
  long long v = vbeg + vl;
  int ow = (int)(v % a.wo), q = (int)(v / a.wo);
  int oh = q % a.ho;
  q /= a.ho;
  int od = q % a.do_, nb = q / a.do_;
  for (; v < vend; v += VL) {
    const int id = wg_coord(od * a.s - a.p + td, a.di, a.reflect);
    const int ih = wg_coord(oh * a.s - a.p + th, a.hi, a.reflect);
    const int iw = wg_coord(ow * a.s - a.p + tw, a.wi, a.reflect);
    const bool ok = tok && (id | ih | iw) >= 0;
    float xv = gx[ok ? (((long long)nb * a.di + id) * a.hi + ih) * a.wi + iw : 0];
    xv = ok ? xv : 0.f;
    const f32x4* g4 = reinterpret_cast<const f32x4*>(go + v * COUT);
#pragma unroll
    for (int c4 = 0; c4 < COUT / 4; ++c4) {
      const f32x4 gv = g4[c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * c4 + e] = fmaf(xv, gv[e], acc[4 * c4 + e]);
    }
    ow += VL;
    while (ow >= a.wo) {
      ow -= a.wo;
      if (++oh == a.ho) {
        oh = 0;
        if (++od == a.do_) { od = 0; ++nb; }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < COUT; ++c) red[vl][t][c] = acc[c];
  __syncthreads();
  for (int i = tid; i < 64 * COUT; i += 256) {
    const int tt = i / COUT, c = i - tt * COUT;
    if (tt < a.R) {
      float sum = 0.f;
#pragma unroll
      for (int l = 0; l < VL; ++l) sum += red[l][tt][c];
      atomicAdd(dw + c * w_sb + tt, sum);
    }
  }
}

bool wgrad_c1_ok(const cgan3d_conv_geom* g) {
  return !g->transposed && g->cin == 1 && g->k * g->k * g->k <= 64 && (g->cout == 4 || g->cout == 8 || g->cout == 16);
}

// atomically adds into dw (torch layout, zeroed by the caller unless accumulating)
int wgrad_c1_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw, hipStream_t st) {
  WgArgs a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.cin = 1; a.cout = g->cout; a.k = g->k; a.s = g->stride; a.p = g->pad; a.reflect = g->reflect;
  a.R = g->k * g->k * g->k;
  a.V = (long long)g->n * g->do_ * g->ho * g->wo;
  long long blocks = (a.V + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  a.vpb = (a.V + blocks - 1) / blocks;
  a.vpb = (a.vpb + 3) / 4 * 4;
  dim3 grid((unsigned)((a.V + a.vpb - 1) / a.vpb));
#define CG_WC1(C) ::cg::launch((conv_wgrad_c1_kernel<C>), grid, dim3(256), 0, st, a, gathered, aligned, dw, (long long)g->w_sb)
  if (g->cout == 4) CG_WC1(4); else if (g->cout == 8) CG_WC1(8); else CG_WC1(16);
#undef CG_WC1
  return CGAN3D_OK;
}

constexpr int g_wgrad_blocks = 1024;  // target grid size

bool wgrad_bf16_ok(const cgan3d_conv_geom* g) {
  return g->prec == CGAN3D_PREC_BF16 && !g->transposed && g->cin % 4 == 0 && g->cout % 4 == 0 && g->cout <= 64 &&
         g->cout >= 4;
}

static WgArgs wgrad_bf16_args(const cgan3d_conv_geom* g, int* gxb, int* gyb) {
  WgArgs a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.cin = g->cin; a.cout = g->cout; a.k = g->k; a.s = g->stride; a.p = g->pad; a.reflect = g->reflect;
  a.R = g->k * g->k * g->k * g->cin;
  a.V = (long long)g->n * g->do_ * g->ho * g->wo;
  const int gx = (a.R + 63) / 64;
  // ~1024 blocks over the chip (fewer partial sums to add), >= 4 stages (256 voxels) per block
  long long gy = g_wgrad_blocks / gx;
  if (gy < 1) gy = 1;
  long long vpb = (a.V + gy - 1) / gy;
  if (vpb < 4 * WG_KV) vpb = 4 * WG_KV;
  a.vpb = (vpb + WG_KV - 1) / WG_KV * WG_KV;
  *gxb = gx;
  *gyb = (int)((a.V + a.vpb - 1) / a.vpb);
  return a;
}

// adds into the packed [t][a][b] workspace dwp (zeroed by the caller)
long long wgrad_bf16_ws_floats(const cgan3d_conv_geom* g) {
  if (!wgrad_bf16_ok(g)) return 0;
  int gxb, gyb;
  const WgArgs a = wgrad_bf16_args(g, &gxb, &gyb);
  return (long long)gyb * a.R * g->cout;
}

// partial slabs into ws (wgrad_bf16_ws_floats), then their ordered sum into dw (round 6: deterministic;
// the blocks of one row chunk added into one workspace by atomics before)
int wgrad_bf16_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw, float* dwp,
                      int accumulate, hipStream_t st) {
  int gxb, gyb;
  const WgArgs a = wgrad_bf16_args(g, &gxb, &gyb);
  dim3 grid(gxb, gyb);
  const int nb = (g->cout + 15) / 16;
#define CG_WGB(N, R8) ::cg::launch((conv_wgrad_bf16_kernel<N, R8>), grid, dim3(256), 0, st, a, gathered, aligned, dwp)
  if (g->wo % 8 == 0) {  // chunks are 64-voxel aligned: 8 | W keeps each thread's 8 voxels in one row
    if (nb == 1) CG_WGB(1, true); else if (nb == 2) CG_WGB(2, true); else if (nb == 3) CG_WGB(3, true); else CG_WGB(4, true);
  } else {
    if (nb == 1) CG_WGB(1, false); else if (nb == 2) CG_WGB(2, false); else if (nb == 3) CG_WGB(3, false);
    else CG_WGB(4, false);
  }
#undef CG_WGB
  const long long E = (long long)a.R * g->cout;
  const int nc = std::max(1, std::min(16, (gyb + 7) / 8));  // ~8 slabs per lane
  ::cg::launch(wgrad_reduce_ta_kernel, dim3((unsigned)((E + 63) / 64)), dim3(64 * nc), 0, st, dwp, gyb, nc,
               g->k * g->k * g->k, g->cin, g->cout, dw, (long long)g->w_sa, (long long)g->w_sb, accumulate);
  return CGAN3D_OK;
}

int wgrad_bf16_group_launch(const cgan3d_conv_geom* geoms, const float* const* gathered, const float* const* aligned,
                            float* const* ws, int n, hipStream_t st) {
  WgGroup G{};
  G.n = n;
  G.first[0] = 0;
  for (int i = 0; i < n; ++i) {
    int gxb, gyb;
    G.a[i] = wgrad_bf16_args(&geoms[i], &gxb, &gyb);
    G.gx[i] = gathered[i]; G.go[i] = aligned[i]; G.dwp[i] = ws[i];
    G.gxb[i] = gxb;
    G.nb[i] = (geoms[i].cout + 15) / 16;
    G.row8[i] = geoms[i].wo % 8 == 0;
    G.first[i + 1] = G.first[i] + gxb * gyb;
  }
  ::cg::launch(conv_wgrad_bf16_group_kernel, dim3(G.first[n]), dim3(256), 0, st, G);
  return CGAN3D_OK;
}

// ---- ResNet-block weight gradient (k3 s1 p1, 64 -> 64, bf16 MFMA), SURVEY.md §8 a2/a5:
// dW[t][a][b] = sum_o X(o + t - 1)[a] * dZ(o)[b].  Block = (tap plane td, chunk p of the output
// voxels); wave w owns input channels 16w..16w+15 x all 64 output channels x the 9 taps of the
// plane (36 accumulator tiles).  K = output voxels in units of 4 (y) x 8 (x) = 32, two units per
// LDS stage.  Both operands stay NDHWC ([voxel][channel] bf16 rows of 128 B) in LDS and are read
// as MFMA fragments with ds_read_b64_tr_b16 (lane i of a 16-lane group receives channel i of 4
// voxel rows, whatever those rows' addresses): the tap shift is just another row address, so the
// X halo is staged once per unit and serves all 9 taps.  16-channel chunks of a row are XOR-
// swizzled by ((x >> 1) + 2y) & 3: the 8 rows a 32-lane half reads (4 consecutive x, 2 y) land
// on 8 distinct 8-bank groups, for every tap.  Per-block partials go to ws[p][t][b][a] (plain
// stores), wgrad_reduce_lin_kernel sums them into dW's layout.  B16: both operands come from their
// bf16 shadows (8-byte loads of the same 4 channels, stored as they are: half the bytes, no
// conversion, bit-identical partials).
namespace wk3 {
constexpr int UPS = 4;                          // units per LDS stage
constexpr int EX = 10, EY = 4;                  // X rows of one unit for one th: 4 (y) x 10 (x) voxels
constexpr int XROWS = UPS * EX * EY, ZROWS = UPS * 32;  // rows per stage
constexpr int STAGE_BYTES = (XROWS + ZROWS) * 128;
__device__ __forceinline__ int swz(int x, int y) { return ((x >> 1) + 2 * y) & 3; }
}  // namespace wk3

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_w tr_pair(const unsigned char* lds, int off0, int off1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + off0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + off1));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_w, v);
}

struct Wk3Args {
  int n, d, h, w;
  int units;      // n * d * (h/4) * (w/8)
  int upb;        // units per block (even)
  int probe;      // phase probes (common.h CG_PROBE)
};

template <bool B16>
__global__ __launch_bounds__(512, 2) void wgrad_k3_kernel(Wk3Args a, const float* __restrict__ x,
                                                          const float* __restrict__ dz, const __bf16* __restrict__ x16,
                                                          const __bf16* __restrict__ dz16, float* __restrict__ ws) {
  // block = (voxel chunk p, tap row tdh = (td, th)): the 3 taps tw of that row x 64 x 64; 8 waves:
  // wave w owns input channels 16*(w & 3) .. +15 and output-channel tiles 2*(w >> 2), +1.  Nine
  // tap rows instead of one chunk per block keeps the split-K partials (P x |dW|) small.
  using namespace wk3;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int at = wave & 3, bh = wave >> 2;
  const int tdh = blockIdx.y, td = tdh / 3, th = tdh % 3, p = blockIdx.x;
  const int u0 = p * a.upb;
  const int yb_n = a.h >> 2, xb_n = a.w >> 3;
  const long long plane = (long long)a.h * a.w;
  const int q4 = tid & 15, rbase = tid >> 4;
  struct Unit { long long corner; int z, yb, xb; bool ok; };
  auto unit = [&](int uu) {
    Unit r;
    r.ok = uu < u0 + a.upb && uu < a.units;
    const int xb = uu % xb_n, q = uu / xb_n, yb = q % yb_n, zq = q / yb_n;
    r.z = zq % a.d;
    r.yb = yb; r.xb = xb;
    r.corner = (long long)zq * plane + (long long)(yb * 4) * a.w + xb * 8;  // zq = nb * d + z
    return r;
  };
  constexpr int NXK = XROWS * 16 / 512, NZK = ZROWS * 16 / 512;  // 5, 4 float4 per thread
  using SV = std::conditional_t<B16, bf16x4_w, f32x4>;
  SV sx[2][NXK], sz[2][NZK];  // two stages of loads in flight (register slots)
  auto load = [&](int s, int sl) {
    const Unit U0 = unit(u0 + UPS * s), U1 = unit(u0 + UPS * s + 1), U2 = unit(u0 + UPS * s + 2),
               U3 = unit(u0 + UPS * s + 3);
#pragma unroll
    for (int k = 0; k < NXK; ++k) {
      const int row = rbase + 32 * k;
      const int u = row / (EX * EY), r = row - u * EX * EY;
      const int hy = r / EX, hx = r - hy * EX;
      const Unit V = u == 0 ? U0 : (u == 1 ? U1 : (u == 2 ? U2 : U3));
      const int iz = V.z + td - 1, iy = V.yb * 4 + hy + th - 1, ix = V.xb * 8 + hx - 1;
      const bool ok = V.ok && (unsigned)iz < (unsigned)a.d && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      const long long off = V.corner + (long long)(td - 1) * plane + (long long)(hy + th - 1) * a.w + (hx - 1);
      if constexpr (B16) sx[sl][k] = ok ? *reinterpret_cast<const bf16x4_w*>(x16 + off * 64 + 4 * q4) : bf16x4_w{};
      else sx[sl][k] = ok ? *reinterpret_cast<const f32x4*>(x + off * 64 + 4 * q4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < NZK; ++k) {
      const int row = rbase + 32 * k;
      const int u = row >> 5, r = row & 31;
      const Unit V = u == 0 ? U0 : (u == 1 ? U1 : (u == 2 ? U2 : U3));
      const long long off = V.corner + (long long)(r >> 3) * a.w + (r & 7);
      if constexpr (B16) sz[sl][k] = V.ok ? *reinterpret_cast<const bf16x4_w*>(dz16 + off * 64 + 4 * q4) : bf16x4_w{};
      else sz[sl][k] = V.ok ? *reinterpret_cast<const f32x4*>(dz + off * 64 + 4 * q4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store = [&](int buf, int sl) {
    unsigned char* base = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int k = 0; k < NXK; ++k) {
      const int row = rbase + 32 * k;
      const int r = row % (EX * EY);
      const int hy = r / EX, hx = r - hy * EX;
      bf16x4_w v;
      if constexpr (B16) v = sx[sl][k];
      else { v[0] = (__bf16)sx[sl][k][0]; v[1] = (__bf16)sx[sl][k][1]; v[2] = (__bf16)sx[sl][k][2]; v[3] = (__bf16)sx[sl][k][3]; }
      *reinterpret_cast<bf16x4_w*>(base + row * 128 + (((q4 >> 2) ^ swz(hx, hy)) * 32) + (q4 & 3) * 8) = v;
    }
#pragma unroll
    for (int k = 0; k < NZK; ++k) {
      const int row = rbase + 32 * k;
      const int r = row & 31;
      bf16x4_w v;
      if constexpr (B16) v = sz[sl][k];
      else { v[0] = (__bf16)sz[sl][k][0]; v[1] = (__bf16)sz[sl][k][1]; v[2] = (__bf16)sz[sl][k][2]; v[3] = (__bf16)sz[sl][k][3]; }
      *reinterpret_cast<bf16x4_w*>(base + (XROWS + row) * 128 + (((q4 >> 2) ^ swz(r & 7, r >> 3)) * 32) + (q4 & 3) * 8) = v;
    }
  };

  f32x4 acc[3][2];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int bt = 0; bt < 2; ++bt) acc[t][bt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  int boff[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int bt = 2 * bh + j;
    boff[j][0] = (XROWS + g * 8 + q) * 128 + ((bt ^ swz(q, g)) * 32) + pp * 8;
    boff[j][1] = (XROWS + g * 8 + q + 4) * 128 + ((bt ^ swz(q + 4, g)) * 32) + pp * 8;
  }
  const int nstages = a.upb / UPS;
  auto stage = [&](int s, int sl) {  // sl == s & 1 (compile-time after the unroll below)
    store(sl, sl);
    lds_barrier();
    if (s + 2 < nstages) load(s + 2, sl);
    const unsigned char* base = smem + sl * STAGE_BYTES;
#pragma unroll
    for (int u = 0; u < UPS; ++u) {
      bf16x8_w bfr[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tr_pair(base + u * 32 * 128, boff[j][0], boff[j][1]);
#pragma unroll
      for (int tw = 0; tw < 3; ++tw) {
        const int hy = g, hx0 = q + tw, hx1 = q + 4 + tw;
        const int r0 = u * (EX * EY) + hy * EX + hx0, r1 = r0 + 4;
        const bf16x8_w afr = tr_pair(base, r0 * 128 + ((at ^ swz(hx0, hy)) * 32) + pp * 8,
                                     r1 * 128 + ((at ^ swz(hx1, hy)) * 32) + pp * 8);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[tw][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[j], acc[tw][j], 0, 0, 0);
      }
    }
    // no trailing barrier: the next stage stores into the other LDS buffer, last read one stage
    // earlier, before every wave passed this stage's barrier
  };
  if (nstages > 0) load(0, 0);
  if (nstages > 1) load(1, 1);
  for (int s = 0; s < nstages; s += 2) {
    stage(s, 0);
    if (s + 1 < nstages) stage(s + 1, 1);
  }
  // partials: lane holds a = 16*at + 4g + jj (jj = 0..3), b = 16*bt + (lane & 15)
  const int bl = lane & 15;
#pragma unroll
  for (int tw = 0; tw < 3; ++tw)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tap = tdh * 3 + tw, bt = 2 * bh + j;
      *reinterpret_cast<f32x4*>(ws + ((((long long)p * 27 + tap) * 64 + bt * 16 + bl) * 64 + 16 * at + 4 * g)) =
          acc[tw][j];
    }
}

// ---- the same weight gradient, round 4 (wgrad_k3m_kernel): the block's operand stream through
// LDS by LDS-DMA and v_mfma_f32_32x32x16_bf16.  Same decomposition (block = voxel chunk p x tap row
// (td, th), the 3 taps tw; per-block partials -> wgrad_reduce_lin_kernel), 4 waves: wave w owns the
// 32 x 32 tile (input channels 32 (w & 1) .., output channels 32 (w >> 1) ..) of the 3 taps.  A
// stage = 4 units (4 y x 8 x output voxels at one z): X rows of the tap row's window (4 y x 10 x
// per unit: one staged window serves tw = 0, 1, 2) and dZ rows, 128 B each, DMA'd lane-linearly
// into one of 4 ring slots three stages ahead of the MFMAs (no staging registers, no conversion,
// no per-element index math).  MFMA operands by ds_read_b64_tr_b16 (one 16-lane group reads 4
// voxel rows x 16 channels, lane i receiving channel i): K-step = 16 voxels = 2 y-rows x 8 x, a
// lane's 8 K-values one y-row's x = 0..7.  Rows keep 16-byte chunk c at c ^ (4 ((r >> 1) & 1)):
// the 4 consecutive voxel rows of a transposed read then cover all 64 banks once (conflict-free
// for every tw shift).  Both operands from their bf16 shadows; fp32 operands stay on wgrad_k3_kernel.
namespace wkm {
constexpr int UPS = 4;                  // units per stage
constexpr int XR = 40, ZR = 32;         // X / dZ rows per unit
constexpr int XROWS = UPS * XR;         // 160
constexpr int ZROWS = UPS * ZR;         // 128
constexpr int SROWS = XROWS + ZROWS;    // 288 rows = 36 DMA wave-instructions per stage
constexpr int SBYTES = SROWS * 128;     // 36864
constexpr int NSLOT = 4;                // ring slots (3 stages in flight ahead)
constexpr int DPW = SROWS / 8 / 4;      // DMA instructions per wave per stage (9)
__device__ __forceinline__ int swz(int r) { return ((r >> 1) & 1) << 2; }
}  // namespace wkm

__device__ __attribute__((aligned(16))) unsigned char g_wkm_zero[16];

__device__ __forceinline__ void wkm_dma16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

__device__ __forceinline__ bf16x8_w wkm_tr(const unsigned char* lds, int off0, int off1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + off0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + off1));
  return __builtin_bit_cast(bf16x8_w, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__global__ __launch_bounds__(256, 1) void wgrad_k3m_kernel(Wk3Args a, const __bf16* __restrict__ x16,
                                                           const __bf16* __restrict__ dz16, float* __restrict__ ws) {
  using namespace wkm;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NSLOT * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ah = wave & 1, bh = wave >> 1;
  const int tdh = blockIdx.y, td = tdh / 3, th = tdh % 3, p = blockIdx.x;
  const int u0 = p * a.upb, un = min(a.upb, a.units - u0);
  const int nst = (un + UPS - 1) / UPS;
  const int yb_n = a.h >> 2, xb_n = a.w >> 3;
  const long long plane = (long long)a.h * a.w;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;

  // ---- DMA of stage s into slot s % NSLOT: wave w issues instructions j = w + 4i (i < DPW); an
  // instruction covers 8 rows, lane -> row 8j + lane / 8, 16-byte position lane % 8 (holding chunk
  // position ^ swz(row))
  auto issue = [&](int s) {
    if (CG_PROBE(a.probe, 2)) return;
    // the stage's 4 units (wave-uniform: scalar arithmetic): first voxel of the X window / dZ rows
    long long xo[UPS], zo[UPS];
    int zz[UPS], yy[UPS], xx[UPS];
    bool uo[UPS];
#pragma unroll
    for (int u = 0; u < UPS; ++u) {
      const int uu = u0 + UPS * s + u;
      uo[u] = uu < u0 + un;
      const int xb = uu % xb_n, q = uu / xb_n, yb = q % yb_n, zq = q / yb_n;
      zz[u] = zq % a.d + td - 1;
      yy[u] = yb * 4 + th - 1;
      xx[u] = xb * 8 - 1;
      xo[u] = (long long)(zq + td - 1) * plane + (long long)yy[u] * a.w + xx[u];
      zo[u] = (long long)zq * plane + (long long)(yb * 4) * a.w + xb * 8;
    }
    const int pos = lane & 7, lr = lane >> 3;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int j = wave + 4 * i;  // instruction: 8 rows of one unit (40 and 32 are multiples of 8)
      const void* src = g_wkm_zero;
      if (j < XROWS / 8) {
        const int u = j / 5, rr = (j - 5 * u) * 8 + lr, hy = rr / 10, hx = rr - 10 * hy;
        const int chunk = pos ^ swz(8 * j + lr);
        if (uo[u] && (unsigned)zz[u] < (unsigned)a.d && (unsigned)(yy[u] + hy) < (unsigned)a.h &&
            (unsigned)(xx[u] + hx) < (unsigned)a.w)
          src = x16 + ((xo[u] + (long long)hy * a.w + hx) * 64 + 8 * chunk);
      } else {
        const int jz = j - XROWS / 8, u = jz >> 2, rr = (jz & 3) * 8 + lr;
        const int chunk = pos ^ swz(8 * jz + lr);
        if (uo[u]) src = dz16 + ((zo[u] + (long long)(rr >> 3) * a.w + (rr & 7)) * 64 + 8 * chunk);
      }
      wkm_dma16(src, __builtin_amdgcn_readfirstlane(lds0 + (s % NSLOT) * SBYTES + j * 1024));
    }
  };

  // ---- per-lane transposed-read offsets inside a stage (bytes): 16-lane group G = lane >> 4 reads
  // channels 16 (G & 1) .. of its operand half; lane 4q + pp supplies row q's channels 4pp .. 4pp+3;
  // K-step ks, lane half h (= G >> 1): y-row 2 ks + h, x = q (first read) and q + 4 (second)
  const int G = lane >> 4, h = G >> 1, q = (lane & 15) >> 2, pp = lane & 3;
  const int cha = 32 * ah + 16 * (G & 1) + 4 * pp;  // input channel of this lane's A read
  const int chb = 32 * bh + 16 * (G & 1) + 4 * pp;  // output channel of its B read
  auto roff = [&](int r, int ch) { return r * 128 + (((ch >> 3) ^ swz(r)) << 4) + (ch & 7) * 2; };
  f32x16_w acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int npre = nst < NSLOT - 1 ? nst : NSLOT - 1;
  for (int s = 0; s < npre; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    // this wave's DMAs of stage s have landed (the younger stages' DPW each still in flight) ...
    const int ahead = min(nst - 1 - s, NSLOT - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ... every wave's, and every wave is done reading slot (s - 1) % NSLOT
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NSLOT - 1 < nst) issue(s + NSLOT - 1);
    const unsigned char* base = smem + (s % NSLOT) * SBYTES;
    // 24 steps k = (unit u, K-step ks, tap tw) = (k / 6, (k / 3) % 2, k % 3); the A fragment of step
    // k + PD (and the B fragment it starts) in flight while MFMA k runs (source order pinned)
    constexpr int PD = 4, NB = 4;
    bf16x8_w ra[PD], rb[NB];
    auto lda = [&](int k) {
      const int u = k / 6, ks = (k / 3) & 1, tw = k % 3, y = 2 * ks + h;
      const int xr = u * XR + y * 10 + tw;  // X window rows of x + tw - 1
      ra[k % PD] = wkm_tr(base, roff(xr + q, cha), roff(xr + q + 4, cha));
    };
    auto ldb = [&](int k) {  // the dZ fragment of steps 3 (k / 3) .. + 2
      const int u = k / 6, ks = (k / 3) & 1, y = 2 * ks + h;
      const int zr = XROWS + u * ZR + y * 8;  // dZ rows of y-row y, x = 0..7
      rb[(k / 3) % NB] = wkm_tr(base, roff(zr + q, chb), roff(zr + q + 4, chb));
    };
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      if (k % 3 == 0) ldb(k);
      lda(k);
    }
#pragma unroll
    for (int k = 0; k < (CG_PROBE(a.probe, 1) ? 0 : 6 * UPS); ++k) {
      const bf16x8_w av = ra[k % PD], bv = rb[(k / 3) % NB];
      if (k + PD < 6 * UPS) {
        if ((k + PD) % 3 == 0) ldb(k + PD);
        lda(k + PD);
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[k % 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[k % 3], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partials ws[p][tap][b][a]: lane holds a = 32 ah + (i & 3) + 8 (i >> 2) + 4 (lane >> 5), b = 32 bh + (lane & 31)
  const int b = 32 * bh + (lane & 31), a0 = 32 * ah + 4 * (lane >> 5);
  if (CG_PROBE(a.probe, 4)) return;
#pragma unroll
  for (int tw = 0; tw < 3; ++tw) {
    float* o = ws + (((long long)p * 27 + tdh * 3 + tw) * 64 + b) * 64 + a0;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *reinterpret_cast<f32x4*>(o + 8 * g4) =
          f32x4{acc[tw][4 * g4], acc[tw][4 * g4 + 1], acc[tw][4 * g4 + 2], acc[tw][4 * g4 + 3]};
  }
}

// dW[b * w_sb + a * w_sa + t] (+)= sum_p ws[p][t][b][a] (27 taps, A gathered x B aligned channels),
// read along the partials' own layout: block = 64 consecutive elements e = (t, b, a) x NC chunks of
// the P partials (wave = chunk), so every wave load is 256 contiguous bytes; each lane sums its
// chunk with 8 loads in flight and the chunks are combined in a fixed order (deterministic).
// Against a block per (b, 16 a, 9 taps) reading 64-byte pieces: 10.8 -> 6.7 us per launch.
__global__ __launch_bounds__(1024) void wgrad_reduce_lin_kernel(const float* __restrict__ ws, int P, int NC, int A,
                                                                int B, float* dw, long long w_sa, long long w_sb,
                                                                int accumulate) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6;
  const long long E = 27LL * A * B, e = (long long)blockIdx.x * 64 + lane;
  const bool ok = e < E;
  const int pc = (P + NC - 1) / NC, p0 = c * pc, p1 = min(P, p0 + pc);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  for (int p = p0; p < p1; p += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = ws[(long long)(p + j < p1 ? p + j : p0) * E + (ok ? e : 0)];
      s[j] += p + j < p1 ? v : 0.f;
    }
  part[c][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (c == 0 && ok) {
    float v = 0.f;
    for (int k = 0; k < NC; ++k) v += part[k][lane];
    const int a = (int)(e % A), r = (int)(e / A), b = r % B, t = r / B;
    float* o = dw + (long long)b * w_sb + (long long)a * w_sa + t;
    *o = accumulate ? *o + v : v;
  }
}

// dW (+)= sum over the P partials ws[p][27][B][A]
static void wgrad_reduce_launch(const float* ws, int P, int A, int B, float* dw, long long w_sa, long long w_sb,
                                int accumulate, hipStream_t st) {
  const int nc = std::max(1, std::min(16, (P + 7) / 8));  // ~8 partials per lane
  const long long E = 27LL * A * B;
  ::cg::launch(wgrad_reduce_lin_kernel, dim3((unsigned)((E + 63) / 64)), dim3(64 * nc), 0, st, ws, P, nc, A, B, dw,
               w_sa, w_sb, accumulate);
}

// ---- stride-2 weight gradients of both generator levels (bf16 MFMA), from bf16 shadows or fp32
// operands: dW[t][a][b] = sum_o X(2o - 1 + t)[a] * dZ(o)[b] with X the CI-channel operand on the 2x grid.
//   <CI, CO> = <16, 32>: the first down-sampling Conv3d 16 -> 32 (generator.py:40-47) and, operands
//   swapped, the last ConvTranspose3d 32 -> 16 (generator.py:61-77; its output-grad is the gathered
//   operand);  <32, 64> (round 6): the second down-sampling conv and the first up-sampling
//   ConvTranspose — the 32 <-> 64 level, on the generic kernel before (26-41 us per launch beside the
//   backward at ~2.5 % MFMA busy).
// A block stages a slab (one output plane, 4 rows, OC = 512 / CI columns) of both operands once — X's
// 3 x 9 x (2 OC + 1) window (~60 KB either way) serves all 27 taps — and reads MFMA fragments with
// ds_read_b64_tr_b16 (any tap shift is a row address).  Layouts, each chosen so the 32 lanes of a
// transposed read hit distinct banks: X rows of 2 CI bytes with one pad voxel per 16 along x (lanes 8
// output columns apart land 64 B apart) and, at CI = 32, the two 16-channel halves swapped on bit 2 of
// the window column; dZ rows of 2 CO bytes with their 16-channel quarters permuted by bits 1 and 3 (CO
// 64) / bit 3 (CO 32) of the column.  K-step = 32 output voxels (one row of 32, or two rows of 16).
// Waves: tap group (w & 3: taps w & 3 + 4i) x 16-channel output tile (w >> 2; CO = 64: two blocks per slab
// range, blockIdx.y the 32-channel half), every input channel.  The
// next slab's 16-byte loads are in registers during the current slab's MFMAs.  Per-block partials
// ws[p][t][b][a] -> wgrad_reduce_lin_kernel (fixed order).
namespace ws2 {
template <int CI>
struct Geo {
  static constexpr int OC = 512 / CI, XW = 2 * OC + 1, XRS = XW + XW / 16 + 1;  // window columns, padded row
  static constexpr int XB = 2 * CI, XI = XB / 16, XPS = 9 * XRS;                // row bytes / items, plane stride
  static constexpr int XBYTES = 3 * XPS * XB;
  static constexpr int NX = 3 * 9 * XW * XI, NXT = (NX + 511) / 512;
};
__device__ __forceinline__ int xcol(int c) { return c + (c >> 4); }
}  // namespace ws2

struct Ws2Args {
  int n, di, hi, wi, do_, ho, wo;
  int slabs, spb;  // slabs in all, per block
};

// B16: both operands from bf16 shadows (bit-identical: fp32 ones are rounded); SPB > 0: every block takes
// exactly SPB slabs (the launcher checks), so the slab loop unrolls into straight-line code and the compiler's
// vmcnt waits before each LDS store count only the slab being stored (a loop-carried prefetch made it wait
// for every load in flight)
template <int CI, int CO, bool B16, int SPB = 0>
__global__ __launch_bounds__(512) void wgrad_s2_kernel(Ws2Args a, const float* __restrict__ x,
                                                       const float* __restrict__ dz, const __bf16* __restrict__ x16,
                                                       const __bf16* __restrict__ dz16, float* __restrict__ ws) {
  using Gm = ws2::Geo<CI>;
  using ws2::xcol;
  constexpr int OC = Gm::OC, XW = Gm::XW, XRS = Gm::XRS, XPS = Gm::XPS, XB = Gm::XB, XI = Gm::XI;
  constexpr int NX = Gm::NX, NXT = Gm::NXT;
  constexpr int ZB = 2 * CO, ZI = ZB / 16, NZ = 4 * OC * ZI, NZT = (NZ + 511) / 512;
  constexpr int AT = CI / 16, BTW = 1, KS = 4 * OC / 32, NTAP = 7;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Gm::XBYTES + 4 * OC * ZB];
  unsigned char* const zs = smem + Gm::XBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // blockIdx.y: which 32 output channels (CO = 64: the two halves in two blocks, each wave one 16-channel
  // tile — 56 accumulator registers instead of 112, which spilled)
  const int tg = wave & 3, bh = 2 * (int)blockIdx.y + (wave >> 2);
  const int p = blockIdx.x;
  const int s0 = p * a.spb, s1 = min(s0 + a.spb, a.slabs);
  const int yg_n = a.ho >> 2, xc_n = a.wo / OC;
  // two slabs in flight in registers from the bf16 shadows (round 6b; one with fp32 operands, which
  // take twice the registers): the next-but-one slab's loads overlap the current slab's MFMAs
  constexpr int DEPTH = B16 && CI == 16 ? 2 : 1;  // (<32, 64>: two slabs spilled)
  bf16x8_w hx[B16 ? DEPTH : 1][B16 ? NXT : 1], hz[B16 ? DEPTH : 1][B16 ? NZT : 1];
  f32x4 fx[B16 ? 1 : 2 * NXT], fz[B16 ? 1 : 2 * NZT];
  // the window's out-of-volume items load a valid address (element 0) and are zeroed at the LDS store:
  // a select on the loaded value right after the load would make the compiler wait for it there,
  // which turned the prefetch into a serial load
  static_assert(NXT <= 32, "one validity bit per staged X item");
  unsigned okm[DEPTH];
  auto load = [&](int sl, int rb) {
    okm[rb] = 0u;
    const int xc = sl % xc_n, q1 = sl / xc_n, yg = q1 % yg_n, zq = q1 / yg_n;  // zq = nb * do + oz
    const int oz = zq % a.do_, nb = zq / a.do_;
    const int iz0 = 2 * oz - 1, iy0 = 8 * yg - 1, ix0 = 2 * OC * xc - 1;
#pragma unroll
    for (int k = 0; k < NXT; ++k) {
      const int i = tid + 512 * k, qi = i % XI, v = i / XI;
      const int c = v % XW, r = (v / XW) % 9, pl = v / (9 * XW);
      const int iz = iz0 + pl, iy = iy0 + r, ix = ix0 + c;
      const bool ok = i < NX && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi;
      const long long o = ok ? ((((long long)nb * a.di + iz) * a.hi + iy) * a.wi + ix) * CI + 8 * qi : 0;
      okm[rb] |= (ok ? 1u : 0u) << k;
      if constexpr (B16) {
        hx[rb][k] = *reinterpret_cast<const bf16x8_w*>(x16 + o);
      } else {
        fx[2 * k] = *reinterpret_cast<const f32x4*>(x + o);
        fx[2 * k + 1] = *reinterpret_cast<const f32x4*>(x + o + 4);
      }
    }
#pragma unroll
    for (int k = 0; k < NZT; ++k) {
      const int i = tid + 512 * k, qi = i % ZI, v = i / ZI;  // v = u * OC + column
      const int oy = 4 * yg + v / OC, ox = OC * xc + v % OC;
      const long long o = ((((long long)nb * a.do_ + oz) * a.ho + oy) * a.wo + ox) * CO + 8 * qi;
      if constexpr (B16) {
        hz[rb][k] = *reinterpret_cast<const bf16x8_w*>(dz16 + o);
      } else {
        fz[2 * k] = *reinterpret_cast<const f32x4*>(dz + o);
        fz[2 * k + 1] = *reinterpret_cast<const f32x4*>(dz + o + 4);
      }
    }
  };
  auto cvt = [](const f32x4& lo, const f32x4& hi) {
    bf16x8_w h;
#pragma unroll
    for (int e = 0; e < 4; ++e) { h[e] = (__bf16)lo[e]; h[4 + e] = (__bf16)hi[e]; }
    return h;
  };
  // byte offset of 16-channel group `at` of window column cc inside its X row / of quarter `bt` of dZ
  // column c inside its row (the bank swizzles above)
  auto xhalf = [](int at, int cc) { return CI == 16 ? 0 : ((at ^ ((cc >> 2) & 1)) * 32); };
  auto zq = [](int bt, int c) {
    return (CO == 32 ? (bt ^ ((c >> 3) & 1)) : (bt ^ (((c >> 1) & 1) | (((c >> 3) & 1) << 1)))) * 32;
  };
  auto store = [&](int rb) {
#pragma unroll
    for (int k = 0; k < NXT; ++k) {
      const int i = tid + 512 * k, qi = i % XI, v = i / XI;
      if (i >= NX) break;
      const int c = v % XW, r = (v / XW) % 9, pl = v / (9 * XW);
      bf16x8_w h;
      if constexpr (B16) h = hx[rb][k];
      else h = cvt(fx[2 * k], fx[2 * k + 1]);
      if (!((okm[rb] >> k) & 1u)) h = bf16x8_w{};
      *reinterpret_cast<bf16x8_w*>(smem + (pl * XPS + r * XRS + xcol(c)) * XB + xhalf(qi >> 1, c) + (qi & 1) * 16) = h;
    }
#pragma unroll
    for (int k = 0; k < NZT; ++k) {
      const int i = tid + 512 * k, qi = i % ZI, v = i / ZI, c = v % OC;
      bf16x8_w h;
      if constexpr (B16) h = hz[rb][k];
      else h = cvt(fz[2 * k], fz[2 * k + 1]);
      *reinterpret_cast<bf16x8_w*>(zs + v * ZB + zq(qi >> 1, c) + (qi & 1) * 16) = h;
    }
  };
  f32x4 acc[NTAP][AT][BTW];
#pragma unroll
  for (int i = 0; i < NTAP; ++i)
#pragma unroll
    for (int at = 0; at < AT; ++at)
#pragma unroll
      for (int j = 0; j < BTW; ++j) acc[i][at][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  auto mfmas = [&]() {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      // this lane's two voxels of the K-step: kv0 = 8g + q and kv0 + 4 (same output row)
      const int kv0 = 8 * g + q;
      const int u = OC == 32 ? s : 2 * s + (kv0 >> 4);
      const int c0 = OC == 32 ? kv0 : (kv0 & 15), c1 = c0 + 4;
      bf16x8_w bfr[BTW];
#pragma unroll
      for (int j = 0; j < BTW; ++j) {
        const int bt = bh * BTW + j;
        bfr[j] = tr_pair(zs, (u * OC + c0) * ZB + zq(bt, c0) + pp * 8, (u * OC + c1) * ZB + zq(bt, c1) + pp * 8);
      }
#pragma unroll
      for (int i = 0; i < NTAP; ++i) {
        const int t = tg + 4 * i;
        if (t < 27) {  // wave-uniform
          const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
          const int rb = td * XPS + (2 * u + th) * XRS;
          const int cc0 = 2 * c0 + tw, cc1 = 2 * c1 + tw;
#pragma unroll
          for (int at = 0; at < AT; ++at) {
            const bf16x8_w afr = tr_pair(smem, (rb + xcol(cc0)) * XB + xhalf(at, cc0) + pp * 8,
                                         (rb + xcol(cc1)) * XB + xhalf(at, cc1) + pp * 8);
#pragma unroll
            for (int j = 0; j < BTW; ++j) acc[i][at][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[j], acc[i][at][j], 0, 0, 0);
          }
        }
      }
    }
  };
  if constexpr (SPB > 0) {
    load(s0, 0);
    if (DEPTH == 2 && SPB > 1) load(s0 + 1, DEPTH - 1);
#pragma unroll
    for (int k = 0; k < SPB; k += DEPTH) {
      lds_barrier();
      store(0);
      lds_barrier();
      if (k + DEPTH < SPB) load(s0 + k + DEPTH, 0);
      mfmas();
      if (DEPTH == 2 && k + 1 < SPB) {
        lds_barrier();
        store(DEPTH - 1);
        lds_barrier();
        if (k + 1 + DEPTH < SPB) load(s0 + k + 1 + DEPTH, DEPTH - 1);
        mfmas();
      }
    }
  } else {
  if (s0 < s1) load(s0, 0);
  if (DEPTH == 2 && s0 + 1 < s1) load(s0 + 1, DEPTH - 1);
  for (int sl = s0; sl < s1; sl += DEPTH) {
    lds_barrier();  // the previous slab's fragment reads are done
    store(0);
    lds_barrier();
    if (sl + DEPTH < s1) load(sl + DEPTH, 0);
    mfmas();
    if (DEPTH == 2 && sl + 1 < s1) {  // block-uniform
      lds_barrier();
      store(DEPTH - 1);
      lds_barrier();
      if (sl + 1 + DEPTH < s1) load(sl + 1 + DEPTH, DEPTH - 1);
      mfmas();
    }
  }
  }
  // partials ws[p][t][b][a]: lane holds a = 16 at + 4g + jj, b = 16 bt + (lane & 15)
  const int bl = lane & 15;
#pragma unroll
  for (int i = 0; i < NTAP; ++i) {
    const int t = tg + 4 * i;
    if (t < 27)
#pragma unroll
      for (int at = 0; at < AT; ++at)
#pragma unroll
        for (int j = 0; j < BTW; ++j)
          *reinterpret_cast<f32x4*>(ws + ((((long long)p * 27 + t) * CO + (bh * BTW + j) * 16 + bl) * CI + at * 16 + 4 * g)) =
              acc[i][at][j];
  }
}

static int g_wk3_P = 28;  // cgan3d_set_tuning key 9: voxel chunks (blocks per tap plane); 0 = off
static int g_wk3m = 1;    // cgan3d_set_tuning key 16: 0 keeps the bf16 ResNet weight grads on wgrad_k3_kernel (A/B)

void wgrad_k3m_set(int v) { g_wk3m = v; }

void wgrad_k3_set_chunks(int v) { g_wk3_P = v; }

bool wgrad_k3_ok(const cgan3d_conv_geom* g) {
  return g_wk3_P > 0 && g->prec == CGAN3D_PREC_BF16 && !g->transposed && !g->reflect && g->k == 3 && g->stride == 1 && g->pad == 1 &&
         g->cin == 64 && g->cout == 64 && g->di == g->do_ && g->hi == g->ho && g->wi == g->wo && g->ho % 4 == 0 &&
         g->wo % 8 == 0;
}

static void wgrad_k3_geometry(const cgan3d_conv_geom* g, Wk3Args* a, int* P) {
  a->n = g->n; a->d = g->do_; a->h = g->ho; a->w = g->wo;
  a->units = g->n * g->do_ * (g->ho / 4) * (g->wo / 8);
  int p = std::max(1, std::min(g_wk3_P, (a->units + wk3::UPS - 1) / wk3::UPS));
  int upb = (a->units + p - 1) / p;
  upb = (upb + wk3::UPS - 1) / wk3::UPS * wk3::UPS;
  *P = (a->units + upb - 1) / upb;
  a->upb = upb;
  a->probe = g_probe;
}

long long wgrad_k3_ws_floats(const cgan3d_conv_geom* g) {
  if (!wgrad_k3_ok(g)) return 0;
  Wk3Args a;
  int P;
  wgrad_k3_geometry(g, &a, &P);
  return (long long)P * 27 * 64 * 64;
}

int wgrad_k3_partials(const cgan3d_conv_geom* g) {
  if (!wgrad_k3_ok(g)) return 0;
  Wk3Args a;
  int P;
  wgrad_k3_geometry(g, &a, &P);
  return P;
}

// every deferred ResNet weight gradient of a backward in one launch (blockIdx.y = descriptor)
struct ReduceMulti {
  cgan3d_reduce_desc d[16];
  int n;
};

__global__ __launch_bounds__(1024) void wgrad_reduce_multi_kernel(ReduceMulti R) {
  const cgan3d_reduce_desc& d = R.d[blockIdx.y];
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6, NC = blockDim.x >> 6;
  const int A = d.cin, B = d.cout, P = d.P;
  const long long E = 27LL * A * B, e = (long long)blockIdx.x * 64 + lane;
  const bool ok = e < E;
  const int pc = (P + NC - 1) / NC, p0 = c * pc, p1 = min(P, p0 + pc);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  for (int p = p0; p < p1; p += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = d.ws[(long long)(p + j < p1 ? p + j : p0) * E + (ok ? e : 0)];
      s[j] += p + j < p1 ? v : 0.f;
    }
  part[c][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (c == 0 && ok) {
    float v = 0.f;
    for (int k = 0; k < NC; ++k) v += part[k][lane];
    const int a = (int)(e % A), r = (int)(e / A), b = r % B, t = r / B;
    float* o = d.dw + (long long)b * d.sb + (long long)a * d.sa + t;
    *o = d.accumulate ? *o + v : v;
  }
}

int wgrad_k3_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, const __bf16* g16,
                    const __bf16* a16, float* dw, int accumulate, float* ws, hipStream_t st, bool defer_reduce) {
  Wk3Args a;
  int P;
  wgrad_k3_geometry(g, &a, &P);
  if (g16 && a16 && g_wk3m)
    ::cg::launch(wgrad_k3m_kernel, dim3(P, 9), dim3(256), 0, st, a, g16, a16, ws);
  else if (g16 && a16)
    ::cg::launch(wgrad_k3_kernel<true>, dim3(P, 9), dim3(512), 0, st, a, gathered, aligned, g16, a16, ws);
  else
    ::cg::launch(wgrad_k3_kernel<false>, dim3(P, 9), dim3(512), 0, st, a, gathered, aligned, g16, a16, ws);
  if (!defer_reduce) wgrad_reduce_launch(ws, P, 64, 64, dw, (long long)g->w_sa, (long long)g->w_sb, accumulate, st);
  return CGAN3D_OK;
}

}  // namespace cg

extern "C" int32_t cgan3d_conv3d_wgrad_partials(const cgan3d_conv_geom* g) { return g ? cg::wgrad_k3_partials(g) : 0; }

extern "C" int cgan3d_wgrad_reduce_multi(const cgan3d_reduce_desc* descs, int32_t n, void* stream) {
  CG_CHECK_ARG(descs && n >= 1 && n <= 16, "cgan3d_wgrad_reduce_multi: 1..16 descriptors");
  cg::ReduceMulti R{};
  R.n = n;
  int pmax = 1, emax = 1;
  for (int i = 0; i < n; ++i) {
    const cgan3d_reduce_desc& d = descs[i];
    CG_CHECK_ARG(d.ws && d.dw && d.P > 0 && d.cin > 0 && d.cout > 0, "cgan3d_wgrad_reduce_multi: bad descriptor %d", i);
    R.d[i] = d;
    pmax = std::max(pmax, (int)d.P);
    emax = std::max(emax, 27 * d.cin * d.cout);
  }
  const int nc = std::max(1, std::min(16, (pmax + 7) / 8));
  ::cg::launch(cg::wgrad_reduce_multi_kernel, dim3((unsigned)((emax + 63) / 64), (unsigned)n), dim3(64 * nc), 0,
               (hipStream_t)stream, R);
  CG_LAUNCH_CHECK("wgrad_reduce_multi_kernel");
  return CGAN3D_OK;
}

namespace cg {

static int g_ws2_P = 128;  // cgan3d_set_tuning key 10: blocks of wgrad_s2_kernel; 0 = off

void wgrad_s2_set_blocks(int v) { g_ws2_P = v; }

bool wgrad_s2_ok(const cgan3d_conv_geom* g) {
  const bool c16 = g->cin == 16 && g->cout == 32, c32 = g->cin == 32 && g->cout == 64;
  const int oc = c32 ? 16 : 32;
  return g_ws2_P > 0 && g->prec == CGAN3D_PREC_BF16 && !g->transposed && !g->reflect && g->k == 3 && g->stride == 2 &&
         g->pad == 1 && (c16 || c32) && g->ho % 4 == 0 && g->wo % oc == 0 &&
         (long long)2 * g->do_ - 1 <= g->di && (long long)2 * g->ho - 1 <= g->hi && (long long)2 * g->wo - 1 <= g->wi;
}

static void wgrad_s2_geometry(const cgan3d_conv_geom* g, Ws2Args* a, int* P) {
  a->n = g->n; a->di = g->di; a->hi = g->hi; a->wi = g->wi; a->do_ = g->do_; a->ho = g->ho; a->wo = g->wo;
  const int oc = g->cin == 32 ? 16 : 32;
  a->slabs = g->n * g->do_ * (g->ho / 4) * (g->wo / oc);
  // the 32 <-> 64 level: half the blocks (its partial rows are four times as long)
  const int pmax = g->cin == 32 ? std::max(1, g_ws2_P / 2) : g_ws2_P;
  const int p = std::max(1, std::min(pmax, a->slabs));
  a->spb = (a->slabs + p - 1) / p;
  *P = (a->slabs + a->spb - 1) / a->spb;
}

long long wgrad_s2_ws_floats(const cgan3d_conv_geom* g) {
  if (!wgrad_s2_ok(g)) return 0;
  Ws2Args a;
  int P;
  wgrad_s2_geometry(g, &a, &P);
  return (long long)P * 27 * g->cin * g->cout;
}

int wgrad_s2_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, const __bf16* g16,
                    const __bf16* a16, float* dw, int accumulate, float* ws, hipStream_t st) {
  Ws2Args a;
  int P;
  wgrad_s2_geometry(g, &a, &P);
  const bool b16 = g16 && a16;
  const int spb = a.slabs % a.spb == 0 ? a.spb : 0;  // every block full: the unrolled variants
#define CG_WS2(CI, CO, B, S) ::cg::launch(wgrad_s2_kernel<CI, CO, B, S>, dim3(P, CO / 32), dim3(512), 0, st, a, \
                                          gathered, aligned, g16, a16, ws)
#define CG_WS2_ALL(CI, CO)                                                                  \
  do {                                                                                      \
    if (!b16) CG_WS2(CI, CO, false, 0);                                                     \
    else if (spb == 8) CG_WS2(CI, CO, true, 8);                                             \
    else if (spb == 4) CG_WS2(CI, CO, true, 4);                                             \
    else if (spb == 2) CG_WS2(CI, CO, true, 2);                                             \
    else CG_WS2(CI, CO, true, 0);                                                           \
  } while (0)
  if (g->cin == 32) CG_WS2_ALL(32, 64);
  else CG_WS2_ALL(16, 32);
#undef CG_WS2_ALL
#undef CG_WS2
  wgrad_reduce_launch(ws, P, g->cin, g->cout, dw, (long long)g->w_sa, (long long)g->w_sb, accumulate, st);
  return CGAN3D_OK;
}

}  // namespace cg
