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

template <int NB, bool ROW8>
__global__ __launch_bounds__(256) void conv_wgrad_bf16_kernel(WgArgs a, const float* __restrict__ gx,
                                                              const float* __restrict__ go, float* dwp) {
  __shared__ __attribute__((aligned(16))) __bf16 As[64 * WG_LD];  // [row][voxel]
  __shared__ __attribute__((aligned(16))) __bf16 Gs[64 * WG_LD];  // [b][voxel]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.x * 64;
  const long long vbeg = (long long)blockIdx.y * a.vpb;
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
      if (r < a.R) atomicAdd(dwp + (long long)r * a.cout + b, acc[nt][jj]);
    }
  }
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

static int g_wgrad_blocks = 1024;  // target grid size (cgan3d_set_tuning key 1)

void wgrad_bf16_set_blocks(int v) { g_wgrad_blocks = v > 0 ? v : 1024; }

bool wgrad_bf16_ok(const cgan3d_conv_geom* g) {
  return g->prec == CGAN3D_PREC_BF16 && !g->transposed && g->cin % 4 == 0 && g->cout % 4 == 0 && g->cout <= 64 &&
         g->cout >= 4;
}

// adds into the packed [t][a][b] workspace dwp (zeroed by the caller)
int wgrad_bf16_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dwp,
                      hipStream_t st) {
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
  dim3 grid(gx, (unsigned)((a.V + a.vpb - 1) / a.vpb));
  const int nb = (g->cout + 15) / 16;
#define CG_WGB(N, R8) ::cg::launch((conv_wgrad_bf16_kernel<N, R8>), grid, dim3(256), 0, st, a, gathered, aligned, dwp)
  if (g->wo % 8 == 0) {  // chunks are 64-voxel aligned: 8 | W keeps each thread's 8 voxels in one row
    if (nb == 1) CG_WGB(1, true); else if (nb == 2) CG_WGB(2, true); else if (nb == 3) CG_WGB(3, true); else CG_WGB(4, true);
  } else {
    if (nb == 1) CG_WGB(1, false); else if (nb == 2) CG_WGB(2, false); else if (nb == 3) CG_WGB(3, false);
    else CG_WGB(4, false);
  }
#undef CG_WGB
  return CGAN3D_OK;
}

}  // namespace cg
