// Implicit-GEMM convolution, forward / input-grad roles, fp32 or bf16 MFMA (gfx950).
//
// Same gather formulation as conv.hip (include/cgan3d.h geometry; stride-s transposed launches
// split into s^3 parity classes), restructured for throughput:
//  * weights pre-packed once per optimiser step into [tap][cin][cout] rows (cgan3d_pack_weights),
//    so each K-chunk's B tile is a few contiguous float4 rows;
//  * the next K-chunk's A gather and B rows are prefetched into registers while the MFMAs of the
//    current chunk run (one LDS buffer + register double-buffering, one barrier pair per chunk);
//  * the class's valid-tap table lives in LDS (built once per block), so a chunk's gather needs no
//    integer division beyond a shift when cin is a power of two;
//  * two tile shapes: 64 voxels x all output channels (4 waves along M) for large grids, 32 voxels
//    x 32 channels (2 x 2 waves, N split over blockIdx.y) when the grid would not fill 256 CUs;
//  * PREC = 0: v_mfma_f32_16x16x4_f32 (exact f32, the parity path); PREC = 1: operands rounded to
//    bf16 when staged into LDS, v_mfma_f32_16x16x32_bf16 with f32 accumulation.
// Epilogue (bias, activation, LeakyReLU mask, residual, tanh, BatchNorm partial statistics) as in
// conv.hip.
#include "common.h"

namespace cg {
int g_probe = 0;


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct GemmArgs {
  int n, di, hi, wi, do_, ho, wo, cin, cout, k, s, p, transposed, reflect;
  int kd, sd, pd;  // depth-axis kernel / stride / pad: (k, s, p), or (1, 1, 0) for planar (2-D)
  long long sa, sb;
  int packed, ldb;
  int cd, ch, cw;
  long long class_vox;
  int tiles_per_class, nclass;
  int cin_shift;
};

static int ilog2_exact(int v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

struct GemmCfg {
  int wm, nbw, bm, bn, gy;
};

// grids with fewer 64-voxel tiles than this use the 32 x 32 tile (more, smaller blocks: latency
// hiding for the 16^3-voxel ResNet layers)
constexpr int g_small_tile_below = 1024;

// deterministic tile-shape choice (also sizes the BatchNorm statistics buffer)
static GemmCfg gemm_cfg(const cgan3d_conv_geom* g) {
  GemmCfg c;
  const int nbt = g->cout <= 16 ? 1 : (g->cout <= 32 ? 2 : 4);
  long long cls = 1, cv;
  if (g->transposed && g->stride > 1) {
    const int sd = geom_sd(g), s = g->stride;
    cls = (long long)sd * s * s;
    cv = (long long)g->n * ((g->do_ + sd - 1) / sd) * ((g->ho + s - 1) / s) * ((g->wo + s - 1) / s);
  } else {
    cv = (long long)g->n * g->do_ * g->ho * g->wo;
  }
  const long long blocks64 = cls * ((cv + 63) / 64);
  if (blocks64 < g_small_tile_below && g->cout > 16) {
    c.wm = 2; c.nbw = 1; c.bm = 32; c.bn = 32; c.gy = (g->cout + 31) / 32;
  } else {
    c.wm = 4; c.nbw = nbt; c.bm = 64; c.bn = 16 * nbt; c.gy = (g->cout + c.bn - 1) / c.bn;  // > 1: cout > 64
  }
  return c;
}

static bool gemm_args(const cgan3d_conv_geom* g, const GemmCfg& c, GemmArgs* a) {
  a->n = g->n; a->di = g->di; a->hi = g->hi; a->wi = g->wi;
  a->do_ = g->do_; a->ho = g->ho; a->wo = g->wo; a->cin = g->cin; a->cout = g->cout;
  a->k = g->k; a->s = g->stride; a->p = g->pad; a->transposed = g->transposed; a->reflect = g->reflect;
  a->sa = g->w_sa; a->sb = g->w_sb; a->packed = g->w_packed; a->ldb = (g->cout + 3) / 4 * 4;
  a->kd = geom_kd(g); a->sd = geom_sd(g); a->pd = geom_pd(g);
  if (g->transposed && g->stride > 1) {
    // parity classes of an output grid not divisible by the stride: ceil-sized class grids, the
    // voxels past the grid's end masked per row (a stride-2 conv's input-grad on odd dims)
    const int s = g->stride;
    a->cd = (g->do_ + a->sd - 1) / a->sd; a->ch = (g->ho + s - 1) / s; a->cw = (g->wo + s - 1) / s;
    a->nclass = a->sd * s * s;
  } else {
    a->cd = g->do_; a->ch = g->ho; a->cw = g->wo; a->nclass = 1;
  }
  a->class_vox = (long long)g->n * a->cd * a->ch * a->cw;
  a->tiles_per_class = (int)((a->class_vox + c.bm - 1) / c.bm);
  a->cin_shift = ilog2_exact(g->cin);
  return true;
}

__device__ __forceinline__ int gg_coord(int base, int off, int n, int reflect) {
  int i = base + off;
  if (reflect) return reflect_idx(i, n);
  return (i >= 0 && i < n) ? i : -1;
}

template <int PREC>
struct Lds {
  static constexpr int KC = 32;
  static constexpr int LD = PREC ? KC + 8 : KC + 4;  // elements per row (80 B bf16 / 144 B f32)
  using T = typename std::conditional<PREC, __bf16, float>::type;
};

template <int PREC, int VEC, int WM, int NBW>
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmArgs a, const float* __restrict__ x,
                                                        const float* __restrict__ w, float* y, Epi ep) {
  constexpr int WN = 4 / WM, BM = 16 * WM, BN = 16 * NBW * WN, KC = 32;
  constexpr int LD = Lds<PREC>::LD;
  using T = typename Lds<PREC>::T;
  constexpr int A_SLOTS = VEC == 4 ? BM * KC / 4 / 256 : BM * KC / 256;  // per thread
  constexpr int B_SLOTS = (BN * KC / 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) T As[BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LD];
  __shared__ int row_n[BM], row_b[3][BM], row_out[BM];
  __shared__ int tap_off[3][352], tap_lin[352];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int cls = blockIdx.x / a.tiles_per_class;
  const int tile = blockIdx.x - cls * a.tiles_per_class;
  const int co0 = blockIdx.y * BN;
  const int s = a.s, k = a.k, p = a.p;
  int rd = 0, rh = 0, rw = 0;
  if (a.transposed) { rd = cls / (s * s); rh = (cls / s) % s; rw = cls % s; }
  int f[3], st[3], cnt[3];
  const int sq[3] = {a.sd, s, s}, pq[3] = {a.pd, p, p}, kq[3] = {a.kd, k, k};
  {
    const int r3[3] = {rd, rh, rw};
    for (int q = 0; q < 3; ++q) {
      if (a.transposed) {
        f[q] = (r3[q] + pq[q]) % sq[q]; st[q] = sq[q];
        cnt[q] = f[q] < kq[q] ? (kq[q] - f[q] + sq[q] - 1) / sq[q] : 0;
      } else {
        f[q] = 0; st[q] = 1; cnt[q] = kq[q];
      }
    }
  }
  const int ntap = cnt[0] * cnt[1] * cnt[2];
  const int KT = ntap * a.cin;
  for (int j = tid; j < ntap; j += 256) {
    const int mw = j % cnt[2], mh = (j / cnt[2]) % cnt[1], md = j / (cnt[1] * cnt[2]);
    const int td = f[0] + st[0] * md, th = f[1] + st[1] * mh, tw = f[2] + st[2] * mw;
    if (a.transposed) {
      tap_off[0][j] = (rd + a.pd - td) / a.sd; tap_off[1][j] = (rh + p - th) / s; tap_off[2][j] = (rw + p - tw) / s;
    } else {
      tap_off[0][j] = td; tap_off[1][j] = th; tap_off[2][j] = tw;
    }
    tap_lin[j] = (td * k + th) * k + tw;
  }
  const long long v0 = (long long)tile * BM;
  if (tid < BM) {
    const long long lin = v0 + tid;
    if (lin < a.class_vox) {
      int jw, jh, jd, nb;
      unflatten4(lin, a.cw, a.ch, a.cd, jw, jh, jd, nb);
      int od, oh, ow;
      if (a.transposed) {
        od = jd * a.sd + rd; oh = jh * s + rh; ow = jw * s + rw;
        row_b[0][tid] = jd; row_b[1][tid] = jh; row_b[2][tid] = jw;
      } else {
        od = jd; oh = jh; ow = jw;
        row_b[0][tid] = jd * a.sd - a.pd; row_b[1][tid] = jh * s - p; row_b[2][tid] = jw * s - p;
      }
      const bool inside = od < a.do_ && oh < a.ho && ow < a.wo;  // ceil-sized class grids
      row_n[tid] = inside ? nb * a.di : -1;
      row_out[tid] = inside ? ((nb * a.do_ + od) * a.ho + oh) * a.wo + ow : -1;
    } else {
      row_n[tid] = -1; row_out[tid] = -1;
      row_b[0][tid] = row_b[1][tid] = row_b[2][tid] = 0;
    }
  }
  __syncthreads();

  // ---- register prefetch buffers
  f32x4 ra4[VEC == 4 ? A_SLOTS : 1];
  float ra1[VEC == 4 ? 1 : A_SLOTS];
  f32x4 rb[B_SLOTS];
  // which loaded operands are live: applied in store_chunk, after the MFMAs the loads overlap (a mask
  // applied right after the load would wait for it there)
  bool oka[A_SLOTS], okb[B_SLOTS][4];

  auto decode = [&](int kk, int* j, int* ci) {
    if (a.cin_shift >= 0) { *j = kk >> a.cin_shift; *ci = kk & (a.cin - 1); }
    else { *j = kk / a.cin; *ci = kk - *j * a.cin; }
  };
  auto gather = [&](int r, int j, int ci) -> long long {  // element offset or -1
    const int nb = row_n[r];
    if (nb < 0) return -1;
    const int id = gg_coord(row_b[0][r], tap_off[0][j], a.di, a.reflect);
    const int ih = gg_coord(row_b[1][r], tap_off[1][j], a.hi, a.reflect);
    const int iw = gg_coord(row_b[2][r], tap_off[2][j], a.wi, a.reflect);
    if ((id | ih | iw) < 0) return -1;
    return ((long long)((nb + id) * a.hi + ih) * a.wi + iw) * a.cin + ci;
  };
  // Every load is issued unconditionally from a clamped, valid address and a dead operand is selected
  // to zero afterwards: loads under branches (kk < KT, the gathered voxel inside the volume, co < cout)
  // each waited for their own round trip (round 4: 18-59 vmcnt(0) per kernel before).
  auto load_chunk = [&](int kc0) {
    if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int sl = tid + 256 * i, r = sl >> 3, kk = kc0 + (sl & 7) * 4;
        int j, ci;
        decode(min(kk, KT - 1), &j, &ci);
        const long long o = gather(r, j, ci);
        oka[i] = kk < KT && o >= 0;
        ra4[i] = *reinterpret_cast<const f32x4*>(x + (oka[i] ? o : 0));
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int sl = tid + 256 * i, r = sl >> 5, kk = kc0 + (sl & 31);
        int j, ci;
        decode(min(kk, KT - 1), &j, &ci);
        const long long o = gather(r, j, ci);
        oka[i] = kk < KT && o >= 0;
        ra1[i] = x[oka[i] ? o : 0];
      }
    }
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      const int sl = min(tid + 256 * i, BN * KC / 4 - 1);
      const int kr = sl / (BN / 4), c4 = sl - kr * (BN / 4), kk = kc0 + kr;
      const int co = co0 + 4 * c4;
      const bool live = tid + 256 * i < BN * KC / 4 && kk < KT && co < a.cout;
      int j, ci;
      decode(min(kk, KT - 1), &j, &ci);
      // one code path for both weight layouts (addresses selected, not loaded values: a value merged
      // from two branches made the compiler wait for it at the merge, before the MFMAs it should
      // overlap): packed rows [tap][cin][ldb >= cout rounded up to 4], or torch's strided layout
      // element (co + e) of the row at b0 + idx * bs, idx clamped into the row
      const long long b0 = a.packed ? ((long long)tap_lin[j] * a.cin + ci) * a.ldb : (long long)ci * a.sa + tap_lin[j];
      const long long bs = a.packed ? 1 : a.sb;
      const int cl = a.packed ? a.ldb - 1 : a.cout - 1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rb[i][e] = w[b0 + (long long)min(co + e, cl) * bs];
        okb[i][e] = live && co + e < a.cout;
      }
    }
  };
  auto store_chunk = [&]() {
    if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int sl = tid + 256 * i, r = sl >> 3, e0 = (sl & 7) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) As[r * LD + e0 + e] = (T)keep_if(oka[i], ra4[i][e]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int sl = tid + 256 * i;
        As[(sl >> 5) * LD + (sl & 31)] = (T)keep_if(oka[i], ra1[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      const int sl = tid + 256 * i;
      if (sl < BN * KC / 4) {
        const int kr = sl / (BN / 4), c4 = sl - kr * (BN / 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) Bs[(4 * c4 + e) * LD + kr] = (T)keep_if(okb[i][e], rb[i][e]);
      }
    }
  };

  f32x4 acc[NBW];
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;
  const int arow = (wm * 16 + r16) * LD;

  if (KT > 0) load_chunk(0);
  for (int kc0 = 0; kc0 < KT; kc0 += KC) {
    store_chunk();
    lds_barrier();
    if (kc0 + KC < KT) load_chunk(kc0 + KC);  // prefetch: in flight during the MFMAs below
    if constexpr (PREC == 0) {
#pragma unroll
      for (int q = 0; q < KC / 16; ++q) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(&As[arow + 16 * q + 4 * g]);
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) {
          const f32x4 bv =
              *reinterpret_cast<const f32x4*>(&Bs[((wn * NBW + nb) * 16 + r16) * LD + 16 * q + 4 * g]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], acc[nb], 0, 0, 0);
        }
      }
    } else {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(&As[arow + 8 * g]);
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&Bs[((wn * NBW + nb) * 16 + r16) * LD + 8 * g]);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[nb], 0, 0, 0);
      }
    }
    lds_barrier();
  }

  // ---- epilogue: lane holds rows wm*16 + 4g + j, column co0 + (wn*NBW + nb)*16 + r16
  float vals[NBW][4];
  bool rowv[4];
  int rowo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rowo[j] = row_out[wm * 16 + 4 * g + j];
    rowv[j] = rowo[j] >= 0;
  }
  // residual / BatchNorm-input operands: every load issued before the first use
  float resv[NBW][4], zv[NBW][4];
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int c = co0 + (wn * NBW + nb) * 16 + r16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long o = (rowv[j] && c < a.cout) ? (long long)rowo[j] * a.cout + c : 0;
      resv[nb][j] = ep.residual ? ep.residual[o] : 0.f;
      zv[nb][j] = ep.bn_mode == 2 ? ep.bn_z[o] : 0.f;
    }
  }
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int c = co0 + (wn * NBW + nb) * 16 + r16;
    const bool cv = c < a.cout;
    const float b = (ep.bias && cv) ? ep.bias[c] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[nb][j] + b;
      if (ep.act == CGAN3D_ACT_RELU) v = fmaxf(v, 0.f);
      else if (ep.act == CGAN3D_ACT_LRELU) v = v > 0.f ? v : v * ep.slope;
      else if (ep.act == CGAN3D_ACT_TANH) v = tanhf(v);
      if (rowv[j] && cv) {
        const long long o = (long long)rowo[j] * a.cout + c;
        if (ep.mask_src) v = ep.mask_src[o] > 0.f ? v : v * ep.slope;
        v += resv[nb][j];
        y[o] = v;
      }
      vals[nb][j] = (rowv[j] && cv) ? v : 0.f;
    }
  }
  if (ep.stats || ep.bn_mode == 1) {  // (sum, M2 about the block mean, count): block-major or slab
    lds_barrier();
    float* red = reinterpret_cast<float*>(As);  // [WM][BN]  (<= 4*64 floats)
    __shared__ float bmean[64];
    int cntv = 0;
    for (int r = 0; r < BM; ++r) cntv += row_out[r] >= 0;
    const long long sbase = (long long)blockIdx.x * (2 * a.cout + 1);
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      float sum = vals[nb][0] + vals[nb][1] + vals[nb][2] + vals[nb][3];
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      if (g == 0) red[wm * BN + (wn * NBW + nb) * 16 + r16] = sum;
    }
    lds_barrier();
    if (tid < BN) {
      float S = 0.f;
      for (int q = 0; q < WM; ++q) S += red[q * BN + tid];
      bmean[tid] = cntv ? S / cntv : 0.f;
      if (co0 + tid < a.cout) {
        if (ep.stats) ep.stats[sbase + co0 + tid] = S;
        else *bn_slot(ep, 0, a.cout, co0 + tid, blockIdx.x) = S;
      }
    }
    lds_barrier();
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int cl = (wn * NBW + nb) * 16 + r16;
      const float m = bmean[cl];
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = (rowv[j] && co0 + cl < a.cout) ? vals[nb][j] - m : 0.f;
        q += d * d;
      }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) red[wm * BN + cl] = q;
    }
    lds_barrier();
    if (tid < BN) {
      float M2 = 0.f;
      for (int q = 0; q < WM; ++q) M2 += red[q * BN + tid];
      if (co0 + tid < a.cout) {
        if (ep.stats) ep.stats[sbase + a.cout + co0 + tid] = M2;
        else *bn_slot(ep, 1, a.cout, co0 + tid, blockIdx.x) = M2;
      }
    }
    if (tid == 0 && blockIdx.y == 0) {
      if (ep.stats) ep.stats[sbase + 2 * a.cout] = (float)cntv;
      else *bn_slot(ep, 2, a.cout, 0, blockIdx.x) = (float)cntv;
    }
  }
  if (ep.bn_mode == 2) {  // fused BatchNorm backward statistics: this block's slot of the slab
    float p1[NBW], p2[NBW];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int c = co0 + (wn * NBW + nb) * 16 + r16;
      p1[nb] = 0.f;
      p2[nb] = 0.f;
      if (c < a.cout) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (rowv[j]) bn_pair_z(ep, vals[nb][j], zv[nb][j], c, a.cout, &p1[nb], &p2[nb]);
      }
      p1[nb] += __shfl_xor(p1[nb], 16, 64);
      p1[nb] += __shfl_xor(p1[nb], 32, 64);
      p2[nb] += __shfl_xor(p2[nb], 16, 64);
      p2[nb] += __shfl_xor(p2[nb], 32, 64);
    }
    lds_barrier();
    float* red = reinterpret_cast<float*>(As);  // [2][WM][BN]
    if (g == 0) {
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        red[wm * BN + (wn * NBW + nb) * 16 + r16] = p1[nb];
        red[(WM + wm) * BN + (wn * NBW + nb) * 16 + r16] = p2[nb];
      }
    }
    lds_barrier();
    if (tid < BN && co0 + tid < a.cout) {
      float S1 = 0.f, S2 = 0.f;
      for (int q = 0; q < WM; ++q) { S1 += red[q * BN + tid]; S2 += red[(WM + q) * BN + tid]; }
      *bn_slot(ep, 0, a.cout, co0 + tid, blockIdx.x) = S1;
      *bn_slot(ep, 1, a.cout, co0 + tid, blockIdx.x) = S2;
    }
  }
}

// packed [t][a][b] (b contiguous, row length round_up(cout, 4)) from the strided torch layout
__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wp, int T,
                                                           int cin, int cout, int ldb, long long sa, long long sb,
                                                           long long total) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i % ldb);
    const long long r = i / ldb;
    const int ai = (int)(r % cin), t = (int)(r / cin);
    wp[i] = b < cout ? w[ai * sa + b * sb + t] : 0.f;
  }
}

// one packed copy (descriptor d), this block being block bx of nbx working on it
__device__ __forceinline__ void pack_one(const cgan3d_pack_desc& d, long long bx, long long nbx) {
  const long long s0 = bx * blockDim.x + threadIdx.x, st = nbx * blockDim.x;
  if (d.format == 3) {  // conv_sk bf16 [b][tap][a]
    __bf16* wp = reinterpret_cast<__bf16*>(d.wp);
    const long long total = (long long)d.taps * d.cout * d.cin;
    for (long long i = s0; i < total; i += st) {
      const int ai = (int)(i % d.cin);
      const long long r = i / d.cin;
      const int t = (int)(r % d.taps), b = (int)(r / d.taps);
      wp[i] = (__bf16)d.w[ai * d.sa + b * d.sb + t];
    }
    return;
  }
  if (d.format == 2) {  // halo bf16 [tap][b][a], granules of a swizzled by b
    __bf16* wp = reinterpret_cast<__bf16*>(d.wp);
    const long long total = (long long)d.taps * d.cout * d.cin;
    const int ng = d.cin / 8;
    for (long long i = s0; i < total; i += st) {
      const int ai = (int)(i % d.cin);
      const long long r = i / d.cin;
      const int b = (int)(r % d.cout), t = (int)(r / d.cout);
      wp[r * d.cin + ((ai / 8) ^ (b & (ng - 1))) * 8 + (ai & 7)] = (__bf16)d.w[ai * d.sa + b * d.sb + t];
    }
    return;
  }
  const long long total = (long long)d.taps * d.cin * d.ldb;
  for (long long i = s0; i < total; i += st) {
    const int b = (int)(i % d.ldb);
    const long long r = i / d.ldb;
    const int ai = (int)(r % d.cin), t = (int)(r / d.cin);
    d.wp[i] = b < d.cout ? d.w[ai * d.sa + b * d.sb + t] : 0.f;
  }
}

__global__ __launch_bounds__(256) void pack_multi_kernel(const cgan3d_pack_desc* __restrict__ descs) {
  pack_one(descs[blockIdx.y], blockIdx.x, gridDim.x);
}

// element `off` of a contiguous weight (taps innermost; the smaller of the sa / sb strides is the
// inner channel index) written into descriptor d's packed copy: the inverse of pack_one's gather
__device__ __forceinline__ void pack_elem(const cgan3d_pack_desc& d, int off, float val) {
  const int taps = d.taps, t = off % taps, r = off / taps;
  int ai, b;
  if (d.sa <= d.sb) {
    ai = r % d.cin;
    b = r / d.cin;
  } else {
    b = r % d.cout;
    ai = r / d.cout;
  }
  if (d.format == 3) {
    reinterpret_cast<__bf16*>(d.wp)[(b * taps + t) * d.cin + ai] = (__bf16)val;
  } else if (d.format == 2) {
    const int ng = d.cin / 8;
    reinterpret_cast<__bf16*>(d.wp)[(t * d.cout + b) * d.cin + ((ai / 8) ^ (b & (ng - 1))) * 8 + (ai & 7)] =
        (__bf16)val;
  } else {
    d.wp[(t * d.cin + ai) * d.ldb + b] = val;
  }
}

// Adam over the arena at step hyper[4] (+ 1 with `tick`), each updated parameter also written
// into every packed copy of its weight (ndesc > 0), and with `tick` the last block out advances
// hyper[4] (every block read the old step before taking its ticket).  One optimiser step of a
// network is then one launch instead of adam_tick_kernel -> Adam -> pack_multi_kernel, same bits.
// A block works on 256 consecutive parameters at a time and scans the descriptors once per chunk
// (uniform, scalar), so a thread only decodes the one or two packed positions of its own element.
__global__ __launch_bounds__(256) void adam_pack_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, long long n,
                                                        float* hyper, const cgan3d_pack_desc* __restrict__ descs,
                                                        int ndesc, int tick, unsigned* ticket) {
  // tick 0: the step was advanced before (cgan3d_adam_tick); 1: use step + 1 and advance it here
  // (last block out); 2: use step + 1, leave it (cgan3d_adam_range, a part updated ahead of the rest)
  const AdamK k = adam_k(hyper, tick ? hyper[4] + 1.f : hyper[4]);
  if (ndesc == 0 && !((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                       reinterpret_cast<uintptr_t>(v)) & 15)) {
    // no packed copies to refresh: four elements per lane (16-byte loads and stores), same arithmetic
    const long long n4 = n >> 2;
    f32x4* p4 = reinterpret_cast<f32x4*>(p);
    f32x4* m4 = reinterpret_cast<f32x4*>(m);
    f32x4* v4 = reinterpret_cast<f32x4*>(v);
    const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
    // ADAM_U float4 groups of a thread loaded before the first is updated (adam_launch sizes the grid
    // at ~4 per thread: a single group in flight per lane left each of them a full HBM latency apart)
    constexpr int ADAM_U = 4;
    const long long st = (long long)gridDim.x * 256;
    for (long long i0 = (long long)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += ADAM_U * st) {
      f32x4 gi[ADAM_U], mi[ADAM_U], vi[ADAM_U], pi[ADAM_U];
#pragma unroll
      for (int u = 0; u < ADAM_U; ++u) {
        const long long i = min(i0 + u * st, n4 - 1);  // clamped duplicates are loaded, never stored
        gi[u] = g4[i]; mi[u] = m4[i]; vi[u] = v4[i]; pi[u] = p4[i];
      }
#pragma unroll
      for (int u = 0; u < ADAM_U; ++u) {
        const long long i = i0 + u * st;
        if (i >= n4) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = mi[u][e], b = vi[u][e], c = pi[u][e];
          adam_vals(k, gi[u][e], a, b, c);
          mi[u][e] = a; vi[u][e] = b; pi[u][e] = c;
        }
        m4[i] = mi[u];
        v4[i] = vi[u];
        p4[i] = pi[u];
      }
    }
    for (long long i = 4 * n4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
      adam_elem(k, p, g, m, v, i);
    if (tick == 1 && last_block_out(ticket)) hyper[4] += 1.f;
    return;
  }
  for (long long base = (long long)blockIdx.x * 256; base < n; base += (long long)gridDim.x * 256) {
    const long long i = base + threadIdx.x;
    const bool live = i < n;
    const float pi = live ? adam_elem(k, p, g, m, v, i) : 0.f;
    for (int j = 0; j < ndesc; ++j) {
      const cgan3d_pack_desc d = descs[j];
      const long long lo = d.w - p, hi = lo + (long long)d.taps * d.cin * d.cout;
      if (hi <= base || lo >= base + 256) continue;  // uniform: this chunk holds none of it
      if (live && i >= lo && i < hi) pack_elem(d, (int)(i - lo), pi);
    }
  }
  if (tick == 1 && last_block_out(ticket)) hyper[4] += 1.f;
}

void adam_launch(float* p, const float* g, float* m, float* v, long long n, float* hyper,
                 const cgan3d_pack_desc* descs, int ndesc, int tick, unsigned* ticket, hipStream_t st) {
  // vector path: ~4 float4 per thread, at most 256 blocks — the step tick's "last block out" ticket is
  // one global atomic per block, and a thousand of them on one address took ~12 us
  const int blocks = ndesc ? (int)std::min<long long>((n + 255) / 256, 1024)
                           : (int)std::max<long long>(1, std::min<long long>((n / 4 + 1023) / 1024, 256));
  ::cg::launch(adam_pack_kernel, dim3(blocks), dim3(256), 0, st, p, g, m, v, n, hyper, descs, ndesc, tick, ticket);
}

int gemm_blocks(const cgan3d_conv_geom* g, long long* mblocks) {
  GemmCfg c = gemm_cfg(g);
  GemmArgs a;
  if (!gemm_args(g, c, &a)) return -1;
  *mblocks = (long long)a.nclass * a.tiles_per_class;
  return 0;
}

int gemm_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st) {
  GemmCfg c = gemm_cfg(g);
  GemmArgs a;
  if (!gemm_args(g, c, &a)) {
    set_error("cgan3d_conv3d_fwd: transposed output dims must be divisible by the stride");
    return CGAN3D_EINVAL;
  }
  dim3 grid(a.nclass * a.tiles_per_class, c.gy);
  const bool v4 = g->cin % 4 == 0;
  const int prec = g->prec;
#define CG_GL(P, V, W, N) ::cg::launch((conv_gemm_kernel<P, V, W, N>), grid, dim3(256), 0, st, a, x, w, y, e)
#define CG_GL_NB(P, V)                                    \
  do {                                                    \
    if (c.wm == 2) CG_GL(P, V, 2, 1);                     \
    else if (c.nbw == 1) CG_GL(P, V, 4, 1);               \
    else if (c.nbw == 2) CG_GL(P, V, 4, 2);               \
    else CG_GL(P, V, 4, 4);                               \
  } while (0)
  if (prec == CGAN3D_PREC_BF16) {
    if (v4) CG_GL_NB(1, 4); else CG_GL_NB(1, 1);
  } else {
    if (v4) CG_GL_NB(0, 4); else CG_GL_NB(0, 1);
  }
#undef CG_GL_NB
#undef CG_GL
  return CGAN3D_OK;
}

}  // namespace cg

using namespace cg;

extern "C" int64_t cgan3d_packed_weight_floats(const cgan3d_conv_geom* g) {
  if (!g) return -1;
  if (g->w_packed == 2 || g->w_packed == 3) return ((int64_t)geom_taps(g) * g->cin * g->cout + 1) / 2;  // bf16
  return (int64_t)geom_taps(g) * g->cin * ((g->cout + 3) / 4 * 4);
}

extern "C" int cgan3d_pack_weights(const cgan3d_conv_geom* g, const float* w, float* wp, void* stream) {
  CG_CHECK_ARG(g && w && wp, "cgan3d_pack_weights: null pointer");
  CG_CHECK_ARG(g->w_packed != 3, "cgan3d_pack_weights: format 3 is packed by cgan3d_pack_weights_multi");
  CG_CHECK_ARG(!g->planar || g->w_packed == 1, "cgan3d_pack_weights: planar geometries use format 1");
  if (g->w_packed == 2) {
    CG_CHECK_ARG(halo_format_ok(g), "cgan3d_pack_weights: geometry not halo-eligible");
    halo_pack(g, w, wp, (hipStream_t)stream);
    CG_LAUNCH_CHECK("pack_halo_kernel");
    return CGAN3D_OK;
  }
  const int T = geom_taps(g), ldb = (g->cout + 3) / 4 * 4;
  const long long total = (long long)T * g->cin * ldb;
  int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
  ::cg::launch(pack_weights_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wp, T, g->cin, g->cout,
                     ldb, (long long)g->w_sa, (long long)g->w_sb, total);
  CG_LAUNCH_CHECK("pack_weights_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_pack_weights_multi(const cgan3d_pack_desc* descs, int32_t n, int64_t max_total, void* stream) {
  CG_CHECK_ARG(descs && n > 0 && n <= 65535 && max_total > 0, "cgan3d_pack_weights_multi: bad args");
  int bx = (int)std::min<long long>((max_total + 255) / 256, 256);
  ::cg::launch(pack_multi_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, descs);
  CG_LAUNCH_CHECK("pack_multi_kernel");
  return CGAN3D_OK;
}

extern "C" int32_t cgan3d_halo_eligible(const cgan3d_conv_geom* g) {
  return g && !g->planar && halo_format_ok(g) ? 1 : 0;
}

extern "C" int32_t cgan3d_packed_format(const cgan3d_conv_geom* g) {
  if (!g) return 0;
  if (g->planar) return 1;
  if (sk_format_ok(g)) return 3;
  if (g->prec == CGAN3D_PREC_BF16 && halo_format_ok(g)) return 2;
  return 1;
}

extern "C" int cgan3d_set_tuning(int32_t key, int32_t value) {
  // six keys, each choosing between correct launch shapes or kernels (tests compare kernels through
  // 13 / 15 / 16); anything else is rejected
  switch (key) {
    case 9: CG_CHECK_ARG(value >= 0, "cgan3d_set_tuning 9: chunks >= 0"); wgrad_k3_set_chunks(value); return CGAN3D_OK;
    case 10: CG_CHECK_ARG(value >= 0, "cgan3d_set_tuning 10: blocks >= 0"); wgrad_s2_set_blocks(value); return CGAN3D_OK;
    case 13:
      CG_CHECK_ARG(value == -1 || value == 0 || value == 8 || value == 16, "cgan3d_set_tuning 13: -1, 0, 8 or 16");
      k7s_set(value);
      return CGAN3D_OK;
    case 15: CG_CHECK_ARG(value == 0 || value == 1, "cgan3d_set_tuning 15: 0 or 1"); k3m_set(value); return CGAN3D_OK;
    case 16: CG_CHECK_ARG(value == 0 || value == 1, "cgan3d_set_tuning 16: 0 or 1"); wgrad_k3m_set(value); return CGAN3D_OK;
    case 20: CG_CHECK_ARG(value > 0, "cgan3d_set_tuning 20: blocks > 0"); k7wg_blocks_set(value); return CGAN3D_OK;
    case 21:  // round 6: output planes per streamed-plane 1 -> 16 k7 block (0 auto; -1: the k7m_n2w kernel)
      CG_CHECK_ARG(value >= -1 && value <= 64, "cgan3d_set_tuning 21: -1 .. 64"); k7p_set(value); return CGAN3D_OK;
#ifdef CGAN3D_PROBES
    case 90: g_probe = value; return CGAN3D_OK;  // phase probes (common.h CG_PROBE), timing only
#endif
    default: break;
  }
  set_error("cgan3d_set_tuning: unknown key %d", key);
  return CGAN3D_EINVAL;
}

extern "C" int cgan3d_adam_range(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                 const float* hyper, void* stream) {
  CG_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && hyper, "cgan3d_adam_range: null pointer");
  CG_CHECK_ARG(n > 0, "cgan3d_adam_range: bad size");
  adam_launch(param, grad, exp_avg, exp_avg_sq, (long long)n, const_cast<float*>(hyper), nullptr, 0, 2, nullptr,
              (hipStream_t)stream);
  CG_LAUNCH_CHECK("adam_pack_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_adam_pack(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                float* hyper, const cgan3d_pack_desc* descs, int32_t ndesc, uint32_t* ticket,
                                void* stream) {
  CG_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && hyper && ticket, "cgan3d_adam_pack: null pointer");
  CG_CHECK_ARG(n > 0 && ndesc >= 0 && ndesc <= 256 && (ndesc == 0 || descs), "cgan3d_adam_pack: bad sizes");
  adam_launch(param, grad, exp_avg, exp_avg_sq, (long long)n, hyper, descs, (int)ndesc, 1, (unsigned*)ticket,
              (hipStream_t)stream);
  CG_LAUNCH_CHECK("adam_pack_kernel");
  return CGAN3D_OK;
}
