// Small-grid convolutions on bf16 MFMA with the K dimension split over the waves: the critic's
// middle layers (model/discriminator.py:42-68, Conv3d k4 s2 p1, 8 -> 16 -> 32 -> 64 channels) in
// their forward, input-grad (ConvTranspose-shaped, stride-2 parity classes) and gradient-penalty
// forward-mode roles.  At 64^3 patches these layers have 768 - 49k output voxels but 512 - 2048
// reduction terms each, so a block per 64-voxel tile walking all taps in series (conv_halo,
// conv_gemm) leaves most CUs idle and every block latency-bound.  Here:
//
//  * M tile = 16 output voxels of one parity class; K = class taps x cin, ordered (tap, channel);
//  * MT = 1: the four waves take K-steps w, w + 4, ... of the same 16 x (16 NT) tile and are summed
//    once through LDS (4x the blocks of a 64-row tiling); MT = 4: each wave its own 16 rows, all K
//    (short K, many rows);
//  * operands straight from L2, no LDS staging: activations = 8 consecutive K = 8 channels of one
//    gathered voxel (two float4, converted to bf16), weights = packed format 3, bf16 [b][tap][a],
//    one 16-byte load per fragment; the next K-step's loads are in flight during the current MFMAs;
//  * MFMA transposed (A = weights, B = activations): a lane ends with 4 channels of one output
//    voxel, so the epilogue (bias / activation / LeakyReLU-mask / residual) moves 16 bytes per
//    lane access; per-block BatchNorm statistics (sum, M2, count) for the BatchNorm critic of the
//    weight-clip configuration;
//  * N split (round 5): few row tiles with a long K (the 32 -> 64 layer: 48 tiles at 12 samples, 16 at
//    4, K = 2048) left each block pulling all 256 KB of weights through one CU; there every block takes
//    one 16-channel slice of the tile (64 KB of weights), nt blocks per tile.  A split of K over blocks
//    (no-return atomics into a zeroed workspace + a ticket, the last block running the epilogue) was
//    built and measured slower (1.420-1.435 vs 1.402-1.405 ms/step) and removed.
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_k __attribute__((ext_vector_type(8)));

// n / d for n < 2^31 by multiply-high (Granlund-Montgomery; mul and sh computed on the host): the row
// setup's three runtime divisions were ~30 VALU each, in series before every block's first load
struct SkDiv {
  unsigned mul;
  int sh;
};
__device__ __forceinline__ unsigned sk_div(unsigned n, SkDiv d) { return (__umulhi(n, d.mul) + n) >> d.sh; }
static SkDiv sk_divisor(unsigned d) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  return SkDiv{(unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
}

__device__ __attribute__((aligned(16))) float g_sk_zero[8];  // the dead operands' source

struct SkArgs {
  int n, di, hi, wi, do_, ho, wo, cin, cout, k, s, p, transposed;
  int nclass, cd, ch, cw;  // parity-class grid (transposed stride 2) or the output grid
  SkDiv dcw, dch, dcd;     // their divisors
  int mblocks;             // blocks per class
  int ktot;                // k^3 * cin: packed weight row length
  int cin_log2;            // cin is a power of two (sk_format_ok)
  int nsplit;              // blocks per row tile, each 16 NT of the output channels (MT == 1)
};

__device__ __forceinline__ void sk_class(int r, int k, int s, int p, int transposed, int* f, int* st, int* cnt) {
  if (transposed) {
    *f = (r + p) % s; *st = s; *cnt = *f < k ? (k - *f + s - 1) / s : 0;
  } else {
    *f = 0; *st = 1; *cnt = k;
  }
}

// W: waves per block (MT == 1 splits K over them); NKC: compile-time K-steps per wave (0: runtime);
// MODE (round 5b): 1 a forward conv (4 taps per axis), 2 a stride-2 transposed one (2 taps per axis
// and parity class), 0 anything else (runtime tap geometry) — the tap decode and the class geometry
// then fold to shifts and constants (VALU per MFMA 43-85 in profiles/r05_pmc_sq_step.json before)
// CL: log2 of cin as a compile-time constant (the critic's 8 - 64 channels; 0: runtime) — with the
// tap geometry and NKC fixed, a lane's K-step offsets fold to constants plus its lane-group term
template <int MT, int NT, int W, int NKC, int MODE, int CL>
__global__ __launch_bounds__(64 * W) void conv_sk_kernel(SkArgs a, const float* __restrict__ x,
                                                         const __bf16* __restrict__ wp, float* y, Epi ep) {
  __shared__ int rowo[16 * MT];
  __shared__ int rowb[3][16 * MT];  // gathered-grid base coordinate per row (gathered = base + tq)
  __shared__ int rown[16 * MT];
  __shared__ __attribute__((aligned(16))) f32x4 red[W - 1][NT][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // N split (MT == 1): the a.nsplit blocks of a row tile take consecutive 16 NT-channel slices
  const int nsp = MT == 1 ? a.nsplit : 1;
  const int tile = (int)blockIdx.x / nsp, cb = ((int)blockIdx.x - tile * nsp) * 16 * NT;
  const int cls = tile / a.mblocks, mb = tile - cls * a.mblocks;
  const int s = MODE == 2 ? 2 : a.s;  // the conv's stride (a forward conv keeps its own)
  const bool trans = MODE == 1 ? false : MODE == 2 ? true : (a.transposed != 0);
  int r3[3] = {0, 0, 0};
  if (MODE == 2) { r3[0] = cls >> 2; r3[1] = (cls >> 1) & 1; r3[2] = cls & 1; }
  else if (trans) { r3[0] = cls / (s * s); r3[1] = (cls / s) % s; r3[2] = cls % s; }
  int fz, sz, nz, fy, sy, ny, fx, sx, nx;
  if (MODE == 1) {
    fz = fy = fx = 0; sz = sy = sx = 1; nz = ny = nx = 4;
  } else if (MODE == 2) {  // k4 s2: class bit r reads taps f, f + 2 with f = (r + p) & 1
    fz = (r3[0] + a.p) & 1; fy = (r3[1] + a.p) & 1; fx = (r3[2] + a.p) & 1;
    sz = sy = sx = 2; nz = ny = nx = 2;
  } else {
    sk_class(r3[0], a.k, s, a.p, trans, &fz, &sz, &nz);
    sk_class(r3[1], a.k, s, a.p, trans, &fy, &sy, &ny);
    sk_class(r3[2], a.k, s, a.p, trans, &fx, &sx, &nx);
  }
  const int ntap = nz * ny * nx;
  (void)sz;
  (void)sy;
  (void)sx;
  if (tid < 16 * MT) {
    // 32-bit index math (sk_format_ok bounds every volume below 2^31 elements)
    const unsigned m = (unsigned)mb * 16 * MT + tid;
    const unsigned cvox = (unsigned)a.n * a.cd * a.ch * a.cw;
    unsigned q = sk_div(m, a.dcw);
    const int jx = (int)(m - q * a.cw);
    unsigned q2 = sk_div(q, a.dch);
    const int jy = (int)(q - q2 * a.ch);
    q = sk_div(q2, a.dcd);
    const int jz = (int)(q2 - q * a.cd), nb = (int)q;
    const bool ok = m < cvox;
    int od = jz, oh = jy, ow = jx;
    if (trans) {
      od = jz * s + r3[0]; oh = jy * s + r3[1]; ow = jx * s + r3[2];
      rowb[0][tid] = jz; rowb[1][tid] = jy; rowb[2][tid] = jx;
    } else {
      rowb[0][tid] = jz * s - a.p; rowb[1][tid] = jy * s - a.p; rowb[2][tid] = jx * s - a.p;
    }
    rowo[tid] = ok ? ((nb * a.do_ + od) * a.ho + oh) * a.wo + ow : -1;
    rown[tid] = nb;
  }
  __syncthreads();

  const int g = lane >> 4, r16 = lane & 15;
  const int mt = MT == 1 ? 0 : wave;
  const int row = mt * 16 + r16;
  const bool rok = rowo[row] >= 0;
  const int bz = rowb[0][row], by = rowb[1][row], bx = rowb[2][row], nb = rown[row];
  // tap j of the class = digits (md, mh, mw) in base 4 (forward: t = m) or 2 (transposed: t = f + s m,
  // gathered coordinate j + (r + p - t) / s = C - m), decoded in registers (round 5: the round-4 tap
  // tables in LDS put dependent LDS reads in front of every K-step's global loads)
  const int lg = MODE == 1 ? 2 : MODE == 2 ? 1 : (nz == 2 ? 1 : 2), lm = (1 << lg) - 1, sg = trans ? -1 : 1;
  const int st = trans ? s : 1;
  const int Cz = bz + (MODE == 2 ? (r3[0] + a.p - fz) >> 1 : trans ? (r3[0] + a.p - fz) / s : 0);
  const int Cy = by + (MODE == 2 ? (r3[1] + a.p - fy) >> 1 : trans ? (r3[1] + a.p - fy) / s : 0);
  const int Cx = bx + (MODE == 2 ? (r3[2] + a.p - fx) >> 1 : trans ? (r3[2] + a.p - fx) / s : 0);
  const int HW = a.hi * a.wi;
  const int gbase = ((nb * a.di + Cz) * a.hi + Cy) * a.wi + Cx;
  const int cl = CL > 0 ? CL : a.cin_log2, cin = 1 << cl;
  const int KS = ntap * cin / 32;
  const int kend = KS;
  const int ks0 = MT == 1 ? wave : 0, kstep = MT == 1 ? W : 1;

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // K loop (round 4).  Every slot is reloaded unconditionally from a clamped, always-valid address
  // and dead operands are zeroed by a select, so nothing in the loop branches.  NKC > 0 (the wave's
  // K-steps fit in NKC, the launcher's choice): the loop is straight-line code with a ring of
  // PF = min(NKC, 8) register slots, so the compiler counts the loads in flight and each MFMA waits
  // only for its own slot (vmcnt(N)).  The round-3 loop (a runtime trip count, a branch per slot)
  // waited for vmcnt(0) before every MFMA and again for the loop-carried register copies: one L2
  // round trip per K-step, 17 us for the 16-block 32 -> 64 layer's 8 K-steps per wave.  NKC == 0:
  // the runtime loop, for long K (many rows, MT == 4).
  constexpr int PF = NKC > 0 ? (NKC < 8 ? NKC : 8) : 4;
  f32x4 xa0[PF], xa1[PF];  // A: 8 fp32 channels of one gathered voxel
  bf16x8_k bb[PF][NT];     // B fragments
  const int nk = ks0 < kend ? (kend - ks0 + kstep - 1) / kstep : 0;  // this wave's K-steps (wave-uniform)
  auto load = [&](int q, int sl) {
    const bool live = q < nk;
    const int ks = ks0 + min(q, max(nk - 1, 0)) * kstep;
    const int k0 = ks * 32 + 8 * g;
    const int j = k0 >> cl, a0 = k0 & (cin - 1);
    const int md = j >> (2 * lg), mh = (j >> lg) & lm, mw = j & lm;
    const int iz = Cz + sg * md, iy = Cy + sg * mh, ix = Cx + sg * mw;
    const bool ok = live && rok && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi &&
                    (unsigned)ix < (unsigned)a.wi;
    // 32-bit element offsets (sk_launch checks the sizes); a dead operand reads 8 zeros (round 5b: one
    // 64-bit select per K-step instead of 8 selects on the loaded values)
    const float* src = ok ? x + ((gbase + sg * (md * HW + mh * a.wi + mw)) << cl) + a0 : g_sk_zero;
    xa0[sl] = *reinterpret_cast<const f32x4*>(src);
    xa1[sl] = *reinterpret_cast<const f32x4*>(src + 4);
    const int wk = ((((fz + st * md) * 4 + fy + st * mh) * 4 + fx + st * mw) << cl) + a0;  // k == 4
#pragma unroll
    for (int t = 0; t < NT; ++t)  // columns past cout (cout = 8) read a valid row; their outputs are never stored
      bb[sl][t] = *reinterpret_cast<const bf16x8_k*>(wp + min(cb + t * 16 + r16, a.cout - 1) * a.ktot + wk);
  };
  auto step = [&](int sl) {
    bf16x8_k av;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      av[e] = (__bf16)xa0[sl][e];
      av[4 + e] = (__bf16)xa1[sl][e];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[sl][t], av, acc[t], 0, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < PF; ++i) load(i, i);
  if constexpr (NKC > 0) {
#pragma unroll
    for (int q = 0; q < NKC; ++q) {
      step(q % PF);
      if (q + PF < NKC) load(q + PF, q % PF);  // compile-time condition
    }
  } else {
    for (int q0 = 0; q0 < nk; q0 += PF) {
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        step(i);
        load(q0 + i + PF, i);
      }
    }
  }
  if (MT == 1) {  // combine the waves' K partials in wave 0
    if (wave > 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t) red[wave - 1][t][lane] = acc[t];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 r = red[0][t][lane];
#pragma unroll
      for (int q = 1; q < W - 1; ++q) r += red[q][t][lane];
      acc[t] += r;
    }
  }
  // epilogue: the MFMA ran transposed (A = weights, B = activations), so lane (g, r16) holds
  // channels t*16 + 4g .. +3 of row mt*16 + r16: one 16-byte store (and mask / residual load) per
  // lane and N tile (cout % 8 == 0: a lane's four channels are all in range or all out)
  const int ro = rowo[mt * 16 + r16];
  float vals[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c0 = cb + t * 16 + 4 * g;
    const bool ok = c0 < a.cout && ro >= 0;
    f32x4 v = acc[t];
    if (ep.bias && c0 < a.cout) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[jj] += ep.bias[c0 + jj];
    }
    if (ep.act == CGAN3D_ACT_RELU) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[jj] = fmaxf(v[jj], 0.f);
    } else if (ep.act == CGAN3D_ACT_LRELU) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[jj] = v[jj] > 0.f ? v[jj] : v[jj] * ep.slope;
    }
    if (ok) {
      const int o = ro * a.cout + c0;
      if (ep.mask_src) {
        const f32x4 m = *reinterpret_cast<const f32x4*>(ep.mask_src + o);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[jj] = m[jj] > 0.f ? v[jj] : v[jj] * ep.slope;
      }
      if (ep.residual) v += *reinterpret_cast<const f32x4*>(ep.residual + o);
      *reinterpret_cast<f32x4*>(y + o) = v;
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) vals[t][jj] = ok ? v[jj] : 0.f;
  }
  if (ep.stats) {  // (sum, M2 about the row mean, count) of this wave's 16 rows: one stats row per
                   // block (MT == 1) or per wave (MT == 4); rows are the 16 lanes of a lane group
    int cnt = 0;
    for (int r = 0; r < 16; ++r) cnt += rowo[mt * 16 + r] >= 0;
    const long long sb = ((long long)tile * MT + mt) * (2 * a.cout + 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c0 = cb + t * 16 + 4 * g;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        float S = vals[t][jj];
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) S += __shfl_xor(S, off, 64);
        const float mean = cnt ? S / cnt : 0.f;
        const float d = ro >= 0 ? vals[t][jj] - mean : 0.f;
        float q = d * d;
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
        if (r16 == 0 && c0 < a.cout) {
          ep.stats[sb + c0 + jj] = S;
          ep.stats[sb + a.cout + c0 + jj] = q;
        }
      }
    }
    if (lane == 0) ep.stats[sb + 2 * a.cout] = (float)cnt;
  }
}

// geometry (ignoring the weight format): the critic's k4 convs, bf16
bool sk_format_ok(const cgan3d_conv_geom* g) {
  if (g->prec != CGAN3D_PREC_BF16 || g->reflect || g->k != 4 || g->cin % 8 || g->cout % 8 || g->cout > 64) return false;
  if (g->stride != 1 && g->stride != 2) return false;  // taps per dim 4 or 2 (the kernel's digit decode)
  if (g->cin & (g->cin - 1)) return false;  // power of two: shift / mask index math
  if ((long long)g->n * g->di * g->hi * g->wi * g->cin >= (1LL << 31) ||
      (long long)g->n * g->do_ * g->ho * g->wo * g->cout >= (1LL << 31))
    return false;  // 32-bit element offsets
  if (g->transposed && g->stride > 1 && (g->do_ % g->stride || g->ho % g->stride || g->wo % g->stride)) return false;
  // every parity class's K (taps x cin) a multiple of 32
  const int kd = g->transposed ? (g->k + g->stride - 1) / g->stride : g->k;  // taps per dim (k % s == 0 here)
  if (g->transposed && g->k % g->stride) return false;
  return (kd * kd * kd * g->cin) % 32 == 0;
}

bool sk_ok(const cgan3d_conv_geom* g) { return g->w_packed == 3 && sk_format_ok(g); }

static SkArgs sk_args(const cgan3d_conv_geom* g, int* mt) {
  SkArgs a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.cin = g->cin; a.cout = g->cout; a.k = g->k; a.s = g->stride; a.p = g->pad; a.transposed = g->transposed;
  if (g->transposed && g->stride > 1) {
    a.nclass = g->stride * g->stride * g->stride;
    a.cd = g->do_ / g->stride; a.ch = g->ho / g->stride; a.cw = g->wo / g->stride;
  } else {
    a.nclass = 1; a.cd = g->do_; a.ch = g->ho; a.cw = g->wo;
  }
  const int kd = g->transposed ? g->k / g->stride : g->k;
  const int ks = kd * kd * kd * g->cin / 32;
  const long long cvox = (long long)a.n * a.cd * a.ch * a.cw;
  // long K on a small grid: split K over the waves; short K or many rows: one 16-row tile per wave
  *mt = (ks >= 8 && (long long)a.nclass * ((cvox + 15) / 16) < 1024) ? 1 : 4;
  a.mblocks = (int)((cvox + 16 * *mt - 1) / (16 * *mt));
  a.ktot = g->k * g->k * g->k * g->cin;
  a.cin_log2 = 0;
  while ((1 << a.cin_log2) < g->cin) ++a.cin_log2;
  a.nsplit = 1;
  a.dcw = sk_divisor((unsigned)a.cw);
  a.dch = sk_divisor((unsigned)a.ch);
  a.dcd = sk_divisor((unsigned)a.cd);
  return a;
}

long long sk_blocks(const cgan3d_conv_geom* g) {  // rows of the statistics epilogue (per row tile)
  int mt;
  SkArgs a = sk_args(g, &mt);
  return (long long)a.nclass * a.mblocks * mt;
}

int sk_launch(const cgan3d_conv_geom* g, const float* x, const __bf16* wp, float* y, const Epi& e, hipStream_t st) {
  CG_CHECK_ARG(!e.out2 && !e.minuend && !e.bn_mode, "conv_sk: no out2 / BatchNorm-slab epilogue");
  CG_CHECK_ARG(!(((uintptr_t)y | (uintptr_t)e.mask_src | (uintptr_t)e.residual) & 15),
               "conv_sk: output / mask / residual must be 16-byte aligned (float4 epilogue)");
  int mt;
  SkArgs a = sk_args(g, &mt);
  const int nt = (g->cout + 15) / 16;
  // K-steps per wave, as a compile-time trip count where it is short (every parity class has the
  // same tap count here: k % s == 0)
  const int kd = g->transposed ? g->k / g->stride : g->k;
  const int KS = kd * kd * kd * g->cin / 32;
  // N split (round 5): few row tiles with a long K (the 32 -> 64 layer, K = 2048) — each block reads
  // only its 16 output channels' weights (64 KB instead of 256 KB through one CU), nt blocks per tile
  const long long tiles = (long long)a.nclass * a.mblocks;
  const int ns = (mt == 1 && !e.stats && KS >= 64 && tiles < 192) ? nt : 1;
  a.nsplit = ns;
  const int ntb = nt / ns;
  const dim3 grid((unsigned)(tiles * ns));
  const bool wide = mt == 1 && tiles < 128 && !e.stats;
  const int w = wide ? 8 : 4;
  const int nk = mt == 1 ? (KS + w - 1) / w : KS;
  const int nkc = nk <= 4 ? 4 : nk <= 8 ? 8 : nk <= 16 ? 16 : 0;
  const int mode = !g->transposed ? 1 : g->stride == 2 ? 2 : 0;
  auto go = [&](auto mt_c, auto w_c) {
    constexpr int M = decltype(mt_c)::value, W = decltype(w_c)::value;
    auto by_nt = [&](auto nkc_c) {
      constexpr int K = decltype(nkc_c)::value;
      const dim3 block(64 * W);
      auto by_mode = [&](auto nt_c) {
        constexpr int N = decltype(nt_c)::value;
        auto by_cl = [&](auto mode_c) {
          constexpr int MO = decltype(mode_c)::value;
          if (a.cin_log2 == 3) ::cg::launch((conv_sk_kernel<M, N, W, K, MO, 3>), grid, block, 0, st, a, x, wp, y, e);
          else if (a.cin_log2 == 4) ::cg::launch((conv_sk_kernel<M, N, W, K, MO, 4>), grid, block, 0, st, a, x, wp, y, e);
          else if (a.cin_log2 == 5) ::cg::launch((conv_sk_kernel<M, N, W, K, MO, 5>), grid, block, 0, st, a, x, wp, y, e);
          else if (a.cin_log2 == 6) ::cg::launch((conv_sk_kernel<M, N, W, K, MO, 6>), grid, block, 0, st, a, x, wp, y, e);
          else ::cg::launch((conv_sk_kernel<M, N, W, K, MO, 0>), grid, block, 0, st, a, x, wp, y, e);
        };
        if (mode == 1) by_cl(std::integral_constant<int, 1>{});
        else if (mode == 2) by_cl(std::integral_constant<int, 2>{});
        else ::cg::launch((conv_sk_kernel<M, N, W, K, 0, 0>), grid, block, 0, st, a, x, wp, y, e);
      };
      if (ntb == 1) by_mode(std::integral_constant<int, 1>{});
      else if (ntb == 2) by_mode(std::integral_constant<int, 2>{});
      else if (ntb == 3) by_mode(std::integral_constant<int, 3>{});
      else by_mode(std::integral_constant<int, 4>{});
    };
    if (nkc == 4) by_nt(std::integral_constant<int, 4>{});
    else if (nkc == 8) by_nt(std::integral_constant<int, 8>{});
    else if (nkc == 16) by_nt(std::integral_constant<int, 16>{});
    else by_nt(std::integral_constant<int, 0>{});
  };
  // very few row tiles with a long K (the 32 -> 64 layer at 4 samples: 16 blocks x 64 K-steps):
  // 8 waves per block split K, half the serial K-steps per wave
  // (A/B at 64^3 B=4: 1.602 vs 1.609 ms/step with 4 waves)
  if (wide) go(std::integral_constant<int, 1>{}, std::integral_constant<int, 8>{});
  else if (mt == 1) go(std::integral_constant<int, 1>{}, std::integral_constant<int, 4>{});
  else go(std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{});
  return CGAN3D_OK;
}

}  // namespace cg
