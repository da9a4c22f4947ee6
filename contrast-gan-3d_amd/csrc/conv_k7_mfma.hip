// Generator first / last convolutions (k = 7, stride 1, 16 <-> 1 channels) on bf16 MFMA.
//
// Same four roles as conv_k7.hip (model/generator.py:31-38 first conv, generator.py:78-85 last conv
// and their weight/input gradients), taken when the geometry asks for CGAN3D_PREC_BF16.  With one
// side single-channel there is no channel pair to make a GEMM of, so each kernel builds one out of
// the taps:
//
//  * n2w (1 -> 16):  M = 16 outputs along W, N = the 16 channels, K = (td, th, tw padded to 8).
//    A[ow][(td,th,tw)] = x[d+td][h+th][ow+tw] is an "unfolded" single-channel halo: every (row, ow)
//    keeps its 8-voxel window as one 16-byte bf16 vector, so the A fragment is one ds_read_b128.
//  * w2n (16 -> 1):  M = 16 outputs along W, N = a 4 x 4 block of (od, oh) output rows (a Toeplitz
//    weight operand: B[(id,ih,tw,c)][(od,oh)] = W[c][id-od][ih-oh][tw], zero off the band), K runs
//    over the 10 x 10 input rows x 8 tw x 16 channels.  Half of that B is zero; the alternative
//    (N = 1) would waste 15/16.
//
// fp32 accumulation; inputs are rounded to bf16 while staging, like the implicit-GEMM bf16 path.
#include "k7.h"

namespace cg {

typedef __bf16 bf16x8_k __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_k __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_k __attribute__((ext_vector_type(2)));

// Staging from global memory with every load of the thread in flight at once: element i < total
// of the tile comes from src[off(i)] (off < 0: zero).  Loads use clamped addresses and no
// branches (a branch per load makes hipcc wait for each one in turn), then `put(i, value)`.
template <int PER, class T, class Off, class Put>
__device__ __forceinline__ void k7m_stage(const T* __restrict__ src, int total, Off off, Put put) {
  T v[PER];
  bool ok[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + 256 * k;
    const long long o = i < total ? off(i) : -1;
    ok[k] = o >= 0;
    v[k] = src[ok[k] ? o : 0];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i < total) put(i, ok[k] ? v[k] : T{});
  }
}

// ---- n2w: 4 (d) x 8 (h) x 16 (w) output tiles, wave = one d-slice (8 rows of 16 voxels = 8 M tiles).
// Persistent blocks loop over tiles: the 13 B fragments (weights) stay in registers for the whole
// launch, the next tile's x halo is loaded into registers during the current tile's MFMAs, and the
// "unfolded" A image us[row][ow][8 taps] = x[row][ow .. ow + 7] is built from the bf16 halo rows by
// byte-aligning register pairs (no per-element LDS reads).  Bank-conflict-free: a b128 lane group
// of the A read covers ow 0..15 = the 16 bank blocks.
constexpr int N_TD = 4, N_TH = 8, N_TW = 16;
constexpr int N_HD = N_TD + 6, N_HH = N_TH + 6, N_HW = N_TW + 6, N_HWP = 24;  // x halo rows (22 used)
constexpr int N_ROWS = N_HD * N_HH;
constexpr int N_PAIRS = 52;                                 // 49 (td, th) pairs padded to 13 K-steps
#ifndef N_US_PAD
#define N_US_PAD 8
#endif
// unfolded-image row stride (bf16): 256 bytes + N_US_PAD elements — the unfold's 16-byte stores of
// rows r .. r+3 (one ds_write lane group) land on distinct banks instead of 4-way conflicts
constexpr int N_US = N_TW * 8 + N_US_PAD;
constexpr int N_X = N_ROWS * N_HW / 2, N_X_PER = (N_X + 255) / 256;  // halo value pairs (w, w + 1)

// sum over the 16 lanes of a row (the voxel lanes r16 of a transposed MFMA tile)
__device__ __forceinline__ float k7m_rowsum16(float v) {
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// B16 (round 4, cgan3d_epilogue.out_bf16): y and the fold's z are bf16 (the 64^3 16-channel tensors of
// the generator); the statistics come from the fp32 accumulators either way
template <bool B16>
__global__ __launch_bounds__(256, 2) void k7m_n2w_kernel(K7Args a, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* __restrict__ y,
                                                         float* stats, float* bn_part, int tiles_per_block, int ntiles,
                                                         K7Fold fb, double* acc1, int reps1) {
  constexpr int C = 16;
  __shared__ __attribute__((aligned(16))) __bf16 us[N_ROWS * N_US];  // [row][ow][8 taps], rows N_US apart
  __shared__ __attribute__((aligned(16))) __bf16 xs[N_ROWS * N_HWP];     // [row][24]
  __shared__ __attribute__((aligned(16))) __bf16 wt[N_PAIRS * C * 8];    // [pair][c][tw8]
  __shared__ float red[4][C];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  k7m_stage<(N_PAIRS * C * 8 + 255) / 256>(
      w, N_PAIRS * C * 8,
      [&](int i) -> long long {
        const int tw = i & 7, c = (i >> 3) & 15, p = i >> 7;
        if (p >= 49 || tw >= K7) return -1;
        const int t = p * K7 + tw;
        return (long long)c * a.wc + (a.flip ? KT7 - 1 - t : t);
      },
      [&](int i, float v) { wt[i] = (__bf16)v; });
  for (int r = tid; r < N_ROWS; r += 256) {  // row tails (read by the unfold, never stored)
    xs[r * N_HWP + N_HW] = (__bf16)0.f;
    xs[r * N_HWP + N_HW + 1] = (__bf16)0.f;
  }
  lds_barrier();
  bf16x8_k bv[N_PAIRS / 4];  // K-step ks: pair 4ks + g, tw 0..7, channel r16
#pragma unroll
  for (int ks = 0; ks < N_PAIRS / 4; ++ks) bv[ks] = *reinterpret_cast<const bf16x8_k*>(wt + ((4 * ks + g) * C + r16) * 8);
  int aoff[N_PAIRS / 4];  // A image offset of this lane's pair (rows past pair 48: any finite row)
#pragma unroll
  for (int ks = 0; ks < N_PAIRS / 4; ++ks) {
    const int pa = min(4 * ks + g, 48), td = pa / K7, th = pa - td * K7;
    aoff[ks] = (td * N_HH + th) * N_US + r16 * 8;
  }
  int xc[N_X_PER];  // this thread's halo pairs: packed (hd, hh, hw even), -1 past the halo
#pragma unroll
  for (int k = 0; k < N_X_PER; ++k) {
    const int i = tid + 256 * k, hw = 2 * (i % (N_HW / 2)), row = i / (N_HW / 2);
    xc[k] = i < N_X ? ((row / N_HH) | ((row % N_HH) << 8) | (hw << 16)) : -1;
  }
  float xb[N_X_PER][2];
  // element offset of each of this thread's halo pairs relative to the tile's halo origin: a tile whose
  // halo lies inside the volume (no reflect, no zero) loads from tile base + coff (round 5: the
  // per-element reflect / range math was ~40 VALU per pair and most of a tile's VALU)
  int coff[N_X_PER];
#pragma unroll
  for (int k = 0; k < N_X_PER; ++k) {
    const int c = xc[k];
    coff[k] = c >= 0 ? ((c & 255) * a.hi + ((c >> 8) & 255)) * a.wi + (c >> 16) : 0;
  }
  auto tile_origin = [&](int tile, int* n, int* d0, int* h0, int* w0) {
    int r = tile;
    const int tw_ = r % a.tiles_w; r /= a.tiles_w;
    const int th_ = r % a.tiles_h; r /= a.tiles_h;
    const int td_ = r % a.tiles_d; *n = r / a.tiles_d;
    *d0 = td_ * N_TD; *h0 = th_ * N_TH; *w0 = tw_ * N_TW;
  };
  auto load = [&](int tile) {
    int n, d0, h0, w0;
    tile_origin(tile, &n, &d0, &h0, &w0);
    const int hd0 = d0 - a.P, hh0 = h0 - a.P, hw0 = w0 - a.P;  // block-uniform
    if (hd0 >= 0 && hd0 + N_HD <= a.di && hh0 >= 0 && hh0 + N_HH <= a.hi && hw0 >= 0 && hw0 + N_HW <= a.wi &&
        !CG_PROBE(a.probe, 2)) {
      const float* xt = x + ((n * a.di + hd0) * a.hi + hh0) * a.wi + hw0;
#pragma unroll
      for (int k = 0; k < N_X_PER; ++k) {
        xb[k][0] = xt[coff[k]];
        xb[k][1] = xt[coff[k] + 1];
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < N_X_PER; ++k) {
      const int c = xc[k];
      const int id = k7_src(d0 + (c & 255) - a.P, a.di, a.reflect), ih = k7_src(h0 + ((c >> 8) & 255) - a.P, a.hi, a.reflect);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int iw = k7_src(w0 + (c >> 16) + e - a.P, a.wi, a.reflect);
        const bool ok = c >= 0 && (id | ih | iw) >= 0;
        if (CG_PROBE(a.probe, 2)) { xb[k][e] = (float)(id + iw); continue; }
        xb[k][e] = x[ok ? ((n * a.di + id) * a.hi + ih) * a.wi + iw : 0];
        if (!ok) xb[k][e] = 0.f;
      }
    }
  };
  // BatchNorm statistics (round 5): each lane accumulates its outputs of channels 4g + jj over every
  // tile as sums shifted by its first value (sum d, sum d^2, d = v - K: no cancellation while the
  // values stay near K), merged once per block (Chan) — the round-4 per-tile mean / M2 passes cost three
  // barriers and two cross-lane reductions per tile (7.8 of 40 us, tools/bench_ops.py probe)
  const bool want_stats = stats || bn_part || acc1;
  float sK[4] = {0.f, 0.f, 0.f, 0.f}, sS1[4] = {0.f, 0.f, 0.f, 0.f}, sS2[4] = {0.f, 0.f, 0.f, 0.f};
  float sN = 0.f;
  float run_n = 0.f, run_mean = 0.f, run_m2 = 0.f;  // the block's merged statistics (threads tid < 16)
  // folded mode-2 pairs of this lane's channels 4g + jj, summed over its outputs of every tile
  float fp1[4] = {0.f, 0.f, 0.f, 0.f}, fp2[4] = {0.f, 0.f, 0.f, 0.f};
  float fsc[4] = {0.f, 0.f, 0.f, 0.f}, fsh[4] = {0.f, 0.f, 0.f, 0.f}, fmean[4] = {0.f, 0.f, 0.f, 0.f},
        finv[4] = {0.f, 0.f, 0.f, 0.f};
  if (fb.z) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int c = 4 * g + jj;
      fsc[jj] = fb.ss[c]; fsh[jj] = fb.ss[C + c]; fmean[jj] = fb.mi[c]; finv[jj] = fb.mi[C + c];
    }
  }
  const int t0 = blockIdx.x * tiles_per_block, t1 = min(ntiles, t0 + tiles_per_block);
  if (t0 < t1) load(t0);
  for (int tile = t0; tile < t1; ++tile) {
    int n, d0, h0, w0;
    tile_origin(tile, &n, &d0, &h0, &w0);
    lds_barrier();  // previous tile's reads of us / red done
#pragma unroll
    for (int k = 0; k < N_X_PER; ++k) {
      const int c = xc[k];
      if (c >= 0) {  // one 4-byte LDS store per pair (two lanes never write halves of one word)
        bf16x2_k v;
        v[0] = (__bf16)xb[k][0];
        v[1] = (__bf16)xb[k][1];
        *reinterpret_cast<bf16x2_k*>(xs + ((c & 255) * N_HH + ((c >> 8) & 255)) * N_HWP + (c >> 16)) = v;
      }
    }
    if (tile + 1 < t1) load(tile + 1);  // in flight during this tile's MFMAs
    lds_barrier();
    for (int i = tid; i < (CG_PROBE(a.probe, 4) ? 0 : N_ROWS * 2); i += 256) {  // unfold (row, half of ow): 8 shifted windows
      const int r = i >> 1, hf = i & 1;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(xs + r * N_HWP + 8 * hf);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(xs + r * N_HWP + 8 * hf + 8);
      const unsigned wv[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int sft = 0; sft < 8; ++sft) {
        u32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int m = sft / 2 + k;
          o[k] = (sft & 1) ? __builtin_amdgcn_alignbyte(wv[m + 1], wv[m], 2) : wv[m];
        }
        *reinterpret_cast<u32x4*>(us + r * N_US + (8 * hf + sft) * 8) = o;
      }
    }
    lds_barrier();
    f32x4 acc[N_TH];
#pragma unroll
    for (int r = 0; r < N_TH; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __bf16* ub = us + wave * N_HH * N_US;
#pragma unroll
    for (int ks = 0; ks < (CG_PROBE(a.probe, 1) ? 0 : N_PAIRS / 4); ++ks) {
      bf16x8_k av[N_TH];
#pragma unroll
      for (int r = 0; r < N_TH; ++r) av[r] = *reinterpret_cast<const bf16x8_k*>(ub + aoff[ks] + r * N_US);
      // transposed: D[channel][ow] (A = weights, B = the unfolded image), so a lane ends up with 4
      // consecutive channels of one voxel: 16-byte output stores and z loads
#pragma unroll
      for (int r = 0; r < N_TH; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[ks], av[r], acc[r], 0, 0, 0);
    }
    // lane holds out[c = 4g + jj][ow = w0 + r16] of row r (oh = h0 + r, od = d0 + wave)
    const int od = d0 + wave, ow = w0 + r16;
#pragma unroll
    for (int r = 0; r < N_TH; ++r) {
      const int oh = h0 + r;
      if (od < a.do_ && oh < a.ho && ow < a.wo && !CG_PROBE(a.probe, 8)) {
        const int o = (((n * a.do_ + od) * a.ho + oh) * a.wo + ow) * C + 4 * g;
        if constexpr (B16) {
          bf16x4_k h;
          h[0] = (__bf16)acc[r][0]; h[1] = (__bf16)acc[r][1]; h[2] = (__bf16)acc[r][2]; h[3] = (__bf16)acc[r][3];
          *reinterpret_cast<bf16x4_k*>(reinterpret_cast<__bf16*>(y) + o) = h;
        } else {
          *reinterpret_cast<f32x4*>(y + o) = acc[r];
        }
      }
    }
    if (fb.z) {  // every z of the tile's outputs loaded before the first is used
      const int vd = reflect_idx(od - fb.P, fb.zd), vw = reflect_idx(ow - fb.P, fb.zw);
      f32x4 zv[N_TH];
#pragma unroll
      for (int r = 0; r < N_TH; ++r) {
        const int vh = reflect_idx(h0 + r - fb.P, fb.zh);
        const bool ok = od < a.do_ && h0 + r < a.ho && ow < a.wo;
        const int zo = ok ? (((n * fb.zd + vd) * fb.zh + vh) * fb.zw + vw) * C + 4 * g : 0;
        if constexpr (B16) {
          const bf16x4_k h = *reinterpret_cast<const bf16x4_k*>(reinterpret_cast<const __bf16*>(fb.z) + zo);
          zv[r] = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
        } else {
          zv[r] = *reinterpret_cast<const f32x4*>(fb.z + zo);
        }
      }
#pragma unroll
      for (int r = 0; r < N_TH; ++r)
        if (od < a.do_ && h0 + r < a.ho && ow < a.wo) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const float gg = acc[r][jj] * act_grad(zv[r][jj] * fsc[jj] + fsh[jj], fb.act, fb.slope);
            fp1[jj] += gg;
            fp2[jj] += gg * (zv[r][jj] - fmean[jj]) * finv[jj];
          }
        }
    }
    if (want_stats && !CG_PROBE(a.probe, 16)) {
      if (tile == t0) {  // the shift: this lane's first output (row 0 of its first tile), 0 off the volume
        const bool ok0 = od < a.do_ && h0 < a.ho && ow < a.wo;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) sK[jj] = ok0 ? acc[0][jj] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < N_TH; ++r) {
        const bool ok = od < a.do_ && h0 + r < a.ho && ow < a.wo;
        sN += ok ? 1.f : 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float dv = ok ? acc[r][jj] - sK[jj] : 0.f;
          sS1[jj] += dv;
          sS2[jj] = fmaf(dv, dv, sS2[jj]);
        }
      }
    }
  }
  if (want_stats) {  // lane (n, mean, M2) -> Chan merge over the 16 voxel lanes, then over the 4 waves
    float mm[4], m2[4];
    float nn = sN;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      mm[jj] = nn > 0.f ? sK[jj] + sS1[jj] / nn : 0.f;
      m2[jj] = nn > 0.f ? fmaxf(sS2[jj] - sS1[jj] * sS1[jj] / nn, 0.f) : 0.f;
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const float no = __shfl_xor(nn, off, 64), nt = nn + no;
      const float wo = nt > 0.f ? no / nt : 0.f, wx = nt > 0.f ? nn * no / nt : 0.f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float mo = __shfl_xor(mm[jj], off, 64), qo = __shfl_xor(m2[jj], off, 64);
        const float dl = mo - mm[jj];
        mm[jj] += dl * wo;
        m2[jj] += qo + dl * dl * wx;
      }
      nn = nt;
    }
    float* rn = reinterpret_cast<float*>(us);  // [4 waves][16] x (n, mean, M2); us is dead after the last tile
    lds_barrier();
    if (r16 == 0) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        rn[(0 * 4 + wave) * C + 4 * g + jj] = nn;
        rn[(1 * 4 + wave) * C + 4 * g + jj] = mm[jj];
        rn[(2 * 4 + wave) * C + 4 * g + jj] = m2[jj];
      }
    }
    lds_barrier();
    if (tid < C) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float no = rn[(0 * 4 + w) * C + tid], mo = rn[(1 * 4 + w) * C + tid], qo = rn[(2 * 4 + w) * C + tid];
        const float nt = run_n + no;
        if (no > 0.f) {
          const float dl = mo - run_mean;
          run_mean += dl * (no / nt);
          run_m2 += qo + dl * dl * (run_n * no / nt);
          run_n = nt;
        }
      }
    }
  }
  if (stats && tid < C) {  // BatchNorm partials (sum, M2, count) per block, layout of conv.hip
    const long long sb = (long long)blockIdx.x * (2 * C + 1);
    stats[sb + tid] = run_mean * run_n;
    stats[sb + C + tid] = run_m2;
    if (tid == 0) stats[sb + 2 * C] = run_n;
  }
  if (acc1 && tid < C && run_n > 0.f) {  // or (sum, sum of squares) into fp64 accumulators (cgan3d_bn_fuse)
    double* r = acc1 + (long long)(blockIdx.x % reps1) * 2 * C;
    const double S = (double)run_mean * run_n;
    unsafeAtomicAdd(r + tid, S);
    unsafeAtomicAdd(r + C + tid, (double)run_m2 + S * (double)run_mean);
  }
  if (bn_part && tid < C) {  // the same partials into slot blockIdx.x of the channel-major slab
    bn_part[(long long)tid * gridDim.x + blockIdx.x] = run_mean * run_n;
    bn_part[(long long)(C + tid) * gridDim.x + blockIdx.x] = run_m2;
    if (tid == 0) bn_part[(long long)2 * C * gridDim.x + blockIdx.x] = run_n;
  }
  if (fb.z) {  // folded mode-2 pairs: voxel lanes -> row sums, waves -> LDS, into slot blockIdx.x
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      fp1[jj] = k7m_rowsum16(fp1[jj]);
      fp2[jj] = k7m_rowsum16(fp2[jj]);
    }
    lds_barrier();
    if (r16 == 0) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) red[wave][4 * g + jj] = fp1[jj];
    }
    lds_barrier();
    double* fr = fb.acc ? fb.acc + (long long)(blockIdx.x % fb.reps) * 2 * C : nullptr;
    if (tid < C) {
      const float q = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      if (fr) unsafeAtomicAdd(fr + tid, (double)q);
      else fb.part[(long long)tid * gridDim.x + blockIdx.x] = q;
    }
    lds_barrier();
    if (r16 == 0) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) red[wave][4 * g + jj] = fp2[jj];
    }
    lds_barrier();
    if (tid < C) {
      const float q = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      if (fr) unsafeAtomicAdd(fr + C + tid, (double)q);
      else fb.part[(long long)(C + tid) * gridDim.x + blockIdx.x] = q;
    }
  }
}

// ---- w2n tile: 4 (d) x 4 (h) x 16 (w) outputs; the 4 waves split the 100 input rows; the 16
// channels are staged in two halves of 8 (one 16-byte vector per halo voxel).  Persistent blocks:
// the weight table is staged once per block and each half's halo is loaded into registers while
// the previous half's MFMAs run.  X16: the halo comes from a bf16 shadow of x (cgan3d_epilogue
// x_bf16; one 16-byte granule per voxel and half, copied as it is) instead of fp32 x.
constexpr int W_TD = 4, W_TH = 4, W_TW = 16;
constexpr int W_HD = W_TD + 6, W_HH = W_TH + 6, W_HW = 24, W_HWU = W_TW + 6;
constexpr int W_ROWS = W_HD * W_HH;  // 100
constexpr int W_F4 = W_ROWS * W_HWU * 2, W_F4_PER = (W_F4 + 255) / 256;  // float4 per half
constexpr int W_G16 = W_ROWS * W_HWU, W_G16_PER = (W_G16 + 255) / 256;   // bf16 granules per half

template <bool X16>
__global__ __launch_bounds__(256, 2) void k7m_w2n_kernel(K7Args a, const float* __restrict__ x,
                                                         const __bf16* __restrict__ x16,
                                                         const float* __restrict__ w, float* __restrict__ y,
                                                         const float* __restrict__ bias, int act,
                                                         const float* __restrict__ minuend, float* __restrict__ out2,
                                                         int tiles_per_block, int ntiles) {
  constexpr int C = 16;
  __shared__ __attribute__((aligned(16))) __bf16 hs[W_ROWS * W_HW * 8];  // [row][iw][8 channels]
  constexpr int WP = 8 * C + 8;  // (td, th) block of the weight table, padded
  __shared__ __attribute__((aligned(16))) __bf16 wt[50 * WP];           // [td*7+th][tw8][c]; row 49 = 0
  __shared__ float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int odl = r16 >> 2, ohl = r16 & 3;  // this lane's B column: output row (od, oh)
  k7m_stage<(49 * 8 * C + 255) / 256>(
      w, 49 * 8 * C,
      [&](int i) -> long long {
        const int c = i & 15, tw = (i >> 4) & 7, p = i >> 7;
        return tw < K7 ? (long long)c * a.wc + p * K7 + tw : -1;
      },
      [&](int i, float v) { wt[(i >> 7) * WP + (i & 127)] = (__bf16)v; });
  for (int i = tid; i < WP; i += 256) wt[49 * WP + i] = (__bf16)0.f;  // off-band rows read this zero block
  for (int i = tid; i < W_ROWS * (W_HW - W_HWU) * 8; i += 256) {  // pad columns 22, 23: read with zero weights
    const int r = i / ((W_HW - W_HWU) * 8), j = i % ((W_HW - W_HWU) * 8);
    hs[(r * W_HW + W_HWU) * 8 + j] = (__bf16)0.f;
  }
  constexpr int NPER = X16 ? W_G16_PER : W_F4_PER, NTOT = X16 ? W_G16 : W_F4;
  int hc[NPER];  // this thread's staged vectors: packed (hd, hh, hw, q), -1 past the halo
#pragma unroll
  for (int k = 0; k < NPER; ++k) {
    const int i = tid + 256 * k, q = X16 ? 0 : i & 1, v = X16 ? i : i >> 1, hw = v % W_HWU, r = v / W_HWU;
    hc[k] = i < NTOT ? ((r / W_HH) | ((r % W_HH) << 8) | (hw << 16) | (q << 24)) : -1;
  }
  f32x4 xv[X16 ? 1 : W_F4_PER];
  bf16x8_k xb[X16 ? W_G16_PER : 1];
  auto tile_origin = [&](int tile, int* n, int* d0, int* h0, int* w0) {
    int r = tile;
    const int tw_ = r % a.tiles_w; r /= a.tiles_w;
    const int th_ = r % a.tiles_h; r /= a.tiles_h;
    const int td_ = r % a.tiles_d; *n = r / a.tiles_d;
    *d0 = td_ * W_TD; *h0 = th_ * W_TH; *w0 = tw_ * W_TW;
  };
  auto load = [&](int tile, int half) {
    int n, d0, h0, w0;
    tile_origin(tile, &n, &d0, &h0, &w0);
    const f32x4* xp = reinterpret_cast<const f32x4*>(x);
    const bf16x8_k* xq = reinterpret_cast<const bf16x8_k*>(x16);
#pragma unroll
    for (int k = 0; k < NPER; ++k) {
      const int c = hc[k];
      const int id = k7_src(d0 + (c & 255) - a.P, a.di, a.reflect),
                ih = k7_src(h0 + ((c >> 8) & 255) - a.P, a.hi, a.reflect),
                iw = k7_src(w0 + ((c >> 16) & 255) - a.P, a.wi, a.reflect);
      const bool ok = c >= 0 && (id | ih | iw) >= 0;
      const int vox = ((n * a.di + id) * a.hi + ih) * a.wi + iw;
      if constexpr (X16) {
        xb[k] = xq[ok ? vox * 2 + half : 0];
        if (!ok) xb[k] = bf16x8_k{};
      } else {
        xv[k] = xp[ok ? vox * (C / 4) + half * 2 + (c >> 24) : 0];
        if (!ok) xv[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < NPER; ++k) {
      const int c = hc[k];
      if (c < 0) continue;
      const int row = (c & 255) * W_HH + ((c >> 8) & 255);
      if constexpr (X16) {
        *reinterpret_cast<bf16x8_k*>(hs + (row * W_HW + ((c >> 16) & 255)) * 8) = xb[k];
        continue;
      }
      bf16x4_k u;
      u[0] = (__bf16)xv[k][0]; u[1] = (__bf16)xv[k][1]; u[2] = (__bf16)xv[k][2]; u[3] = (__bf16)xv[k][3];
      *reinterpret_cast<bf16x4_k*>(hs + (row * W_HW + ((c >> 16) & 255)) * 8 + 4 * (c >> 24)) = u;
    }
  };
  const int t0 = blockIdx.x * tiles_per_block, t1 = min(ntiles, t0 + tiles_per_block);
  if (t0 < t1) load(t0, 0);
  for (int tile = t0; tile < t1; ++tile) {
    f32x4 acc[2];  // independent accumulators: back-to-back MFMAs do not wait on each other
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      lds_barrier();  // every wave done reading hs (and red) of the previous half / tile
      store();
      if (half == 0) load(tile, 1);
      else if (tile + 1 < t1) load(tile + 1, 0);
      lds_barrier();
      {
        // software-pipelined: row prl + 1's four fragments are read from LDS while row prl's two
        // MFMAs run (the LDS latency is otherwise exposed on every row)
        bf16x8_k av[2][2], bv[2][2];
        auto fetch = [&](int prl, bf16x8_k (&ar)[2], bf16x8_k (&br)[2]) {
          const int pr = wave * 25 + prl;
          const int id = pr / W_HH, ih = pr - id * W_HH;
          const int td = id - odl, th = ih - ohl;
          const bool band = td >= 0 && td < K7 && th >= 0 && th < K7;
          const __bf16* wrow = wt + (band ? td * K7 + th : 49) * WP + half * 8;
          const __bf16* hrow = hs + (pr * W_HW + r16) * 8;
#pragma unroll
          for (int sq = 0; sq < 2; ++sq) {
            const int tw = 4 * sq + g;
            ar[sq] = *reinterpret_cast<const bf16x8_k*>(hrow + tw * 8);
            br[sq] = *reinterpret_cast<const bf16x8_k*>(wrow + tw * C);
          }
        };
        auto mma = [&](const bf16x8_k (&ar)[2], const bf16x8_k (&br)[2]) {
#pragma unroll
          for (int sq = 0; sq < 2; ++sq)
            acc[sq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[sq], br[sq], acc[sq], 0, 0, 0);
        };
        fetch(0, av[0], bv[0]);
#pragma unroll 1
        for (int prl = 0; prl < 24; prl += 2) {  // ping-pong buffers (compile-time indices)
          fetch(prl + 1, av[1], bv[1]);
          __builtin_amdgcn_sched_barrier(0);
          mma(av[0], bv[0]);
          __builtin_amdgcn_sched_barrier(0);
          fetch(prl + 2, av[0], bv[0]);
          __builtin_amdgcn_sched_barrier(0);
          mma(av[1], bv[1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        mma(av[0], bv[0]);
      }
    }
    acc[0] += acc[1];
    // combine the 4 waves: lane holds out[ow = 4g + jj][(od, oh) = r16]
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) red[wave][(4 * g + jj) * 16 + r16] = acc[0][jj];
    lds_barrier();
    int n, d0, h0, w0;
    tile_origin(tile, &n, &d0, &h0, &w0);
    const int m = tid >> 4, nn = tid & 15;  // ow_l = m, (odl, ohl) = nn
    const int od = d0 + (nn >> 2), oh = h0 + (nn & 3), ow = w0 + m;
    if (od < a.do_ && oh < a.ho && ow < a.wo) {
      float v = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid] + (bias ? bias[0] : 0.f);
      if (act == CGAN3D_ACT_TANH) v = tanhf(v);
      const int o = ((n * a.do_ + od) * a.ho + oh) * a.wo + ow;
      y[o] = v;
      if (out2) out2[o] = minuend[o] - v;
    }
  }
}

// ---- streamed-plane w2n (16 -> 1 from the bf16 shadow, the generator's last conv): the
// contraction is split as  out[d][h][w] = sum_td P[d + td - 3][h][w][td]  with
//   P[q][h][w][td] = sum_{th, tw, c} X[q][h + th - 3][w + tw - 3][c] * W[c][td][th][tw]
// a GEMM per (input plane q, output row pair): M = 16 w, N = (h of the pair, td) = 2 x 7 of 16
// columns, K = (th, tw, c) = 7 x (8 tw x 16 c).  The A fragment of a K-step is 8 consecutive
// channels of one staged voxel (16 bytes straight from the plane staged in LDS: no unfolding); the
// B fragment of staged row r and output pair (h, h + 1) holds W[.][td][r - h][.] in its first 8
// columns and W[.][td][r - h - 1][.] in the next 8, so it depends on r - h only and the 32 of them
// (r - h = 0..7, 4 tw pairs) stay in registers for the whole launch; every A fragment feeds the
// MFMAs of each output pair it reaches (64 per plane and wave, none off-band).
// A block = 16 x 16 output columns (h, w) x a chunk of TDc output planes, 8 waves: wave = (4
// output rows, half of K = tw pairs 0-1 or 2-3), two waves per SIMD, so one wave's MFMAs run while
// the other waits on LDS or issues its DMAs.  The block streams the TDc + 6 input planes (22 x 23
// staged voxels each: the (h, w) halo re-read is 1.98x, against 2.78x for a 4 x 64 tile) through a
// ring of 4 LDS buffers filled by LDS-DMA (global_load_lds, 16 bytes per lane, no staging
// registers) three planes ahead, with the minuend rows of the output plane a step finishes; lane
// (g, h, td) adds its P values into its wave's ring of the 7 output planes still open (eight LDS
// reads, then eight writes), laid out [h][w % 4][w / 4][plane slot, 9 apart] so neither the adds
// (td picks the slot) nor the row reads of the flush share a bank.  Output plane d is finished
// (both K halves' rings summed, bias, tanh, opt_hat) at the top of step d + 7, after the barrier
// that follows its last input plane; the flush zeroes the slots for the plane 8 later.  Every
// store instruction is issued by the whole wave (lanes past the volume write a sink), so the vmcnt
// wait for a plane counts exactly the DMAs and stores issued after it.
__device__ u32x4 k7s_zero;    // zero-initialised device global: the source of out-of-volume granules
__device__ float k7s_sink[64];  // target of the stores of lanes past the volume

namespace k7s {
constexpr int NT = 512;                  // threads per block (8 waves)
constexpr int SH = 16;                   // output rows per block (4 per wave pair)
constexpr int WB = 16;                   // output columns per block (one M tile)
constexpr int ROWS = SH + 6, COLS = WB + 7;  // 22 halo columns + one zero column (read by tw = 7)
constexpr int RB = COLS * 32;            // staged row bytes (16 bf16 channels per voxel)
constexpr int GRAN = ROWS * COLS * 2;    // 16-byte granules of a plane
constexpr int GPT = (GRAN + NT - 1) / NT;  // LDS-DMA instructions per wave per plane
constexpr int MOFF = GPT * NT * 16;      // minuend granules after the plane (waves 0-3 x 64 lanes;
constexpr int BUF = MOFF + 4 * 64 * 16;  // 16 of them used) — bytes per ring buffer
constexpr int NBUF = 4;                  // planes in flight: 3 ahead of the one computed
constexpr int RING = 4 * 4 * 4 * 9;      // per-wave ring floats: [h][w % 4][w / 4][9]
constexpr int FL = 7;                    // output plane s - FL is flushed at step s
}  // namespace k7s

template <int N>
__device__ __forceinline__ void k7s_wait_vm(int n) {  // s_waitcnt vmcnt(n) for n in [N, N + 6]
  switch (n - N) {
    case 0: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 1) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 2) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 3) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 4) : "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 5) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N + 6) : "memory"); break;
  }
}

__global__ __launch_bounds__(512, 1) void k7s_w2n_kernel(K7Args a, const __bf16* __restrict__ x16,
                                                         const float* __restrict__ w, float* __restrict__ y,
                                                         const float* __restrict__ bias, int act,
                                                         const float* __restrict__ minuend, float* __restrict__ out2,
                                                         int tdc) {
  using namespace k7s;
  extern __shared__ __attribute__((aligned(16))) unsigned char k7s_lds[];
  unsigned char* bufs = k7s_lds;  // [NBUF][BUF]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = wave & 3, kh = wave >> 2;  // row quad, K half (the flushing waves are kh == 0)
  const int g = lane >> 4, r16 = lane & 15;
  float* rings = reinterpret_cast<float*>(k7s_lds + NBUF * BUF);
  float* ring = rings + wave * RING;
  int bid = blockIdx.x;
  const int wt_ = bid % a.tiles_w; bid /= a.tiles_w;
  const int ht_ = bid % a.tiles_h; bid /= a.tiles_h;
  const int dt_ = bid % a.tiles_d;
  const int n = bid / a.tiles_d;
  const int d0 = dt_ * tdc, h0 = ht_ * SH, w0 = wt_ * WB;
  // weights: B fragment (t0 = r - h, j) of lane (g, col = r16): column col = 8 hsel + td holds
  // W[c0 .. c0 + 7][td][t0 - hsel][tw], tw = 2 (2 kh + j) + (g >> 1), c0 = 8 (g & 1); zero off the
  // band.  Staged once as bf16 [tap][16 channels] in the last ring buffer (first filled after the
  // loop's first barrier): coalesced global reads, then one ds_read_b128 per fragment.
  bf16x8_k bw[8][2];
  {
    __bf16* wl = reinterpret_cast<__bf16*>(bufs + (NBUF - 1) * BUF);
    for (int i = tid; i < 16 * KT7; i += NT) {
      const int c = i / KT7, t = i - c * KT7;
      wl[t * 16 + c] = (__bf16)w[(long long)c * a.wc + t];
    }
    __syncthreads();
    const int hsel = r16 >> 3, td = r16 & 7, c0 = 8 * (g & 1);
#pragma unroll
    for (int t0 = 0; t0 < 8; ++t0)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int th = t0 - hsel, tw = 2 * (2 * kh + j) + (g >> 1);
        const bool ok = td < 7 && th >= 0 && th < 7 && tw < 7;
        const bf16x8_k v = *reinterpret_cast<const bf16x8_k*>(wl + (ok ? (td * 7 + th) * 7 + tw : 0) * 16 + c0);
        bw[t0][j] = ok ? v : bf16x8_k{};
      }
    for (int i = lane; i < RING; i += 64) ring[i] = 0.f;  // slots are added into, zeroed again by the flush
  }
  // this lane's plane granules (lane-linear LDS image: granule i of the plane at byte 16 i, i = k *
  // NT + wave * 64 + lane): the (h, w) part of the source offset, -1 = zero (past a partial tile,
  // the tw = 7 pad column, or past the plane's granules).  Reflect padding (the launcher's
  // condition): every plane index is in range.
  int hw[GPT];
#pragma unroll
  for (int k = 0; k < GPT; ++k) {
    const int i = k * NT + wave * 64 + lane;
    const int q = i & 1, u = (i >> 1) % COLS, r = (i >> 1) / COLS;
    const int ih = k7_src(h0 - a.P + r, a.hi, 1);
    const int iw = u < WB + 6 ? k7_src(w0 - a.P + u, a.wi, 1) : -1;
    hw[k] = (i < GRAN && (ih | iw) >= 0) ? (ih * a.wi + iw) * 2 + q : -1;
  }
  const int nplanes = tdc + 6;
  const u32x4* xg = reinterpret_cast<const u32x4*>(x16);
  const float* mbase = out2 ? minuend : y;  // any valid address when there is no minuend
  // plane s into buffer s % NBUF (GPT instructions per wave, dummy sources past the chunk) and, by
  // the flushing waves, the minuend rows of output plane s - FL (one more): the vmcnt waits below
  // count them exactly
  auto issue = [&](int s) {
    const int sp = s < nplanes ? s : nplanes - 1;
    const int id = k7_src(d0 - a.P + sp, a.di, 1);
    const u32x4* src = xg + (long long)(n * a.di + id) * a.hi * a.wi * 2;
    unsigned char* dst = bufs + (s % NBUF) * BUF;
#pragma unroll
    for (int k = 0; k < GPT; ++k)
      __builtin_amdgcn_global_load_lds((const void*)(hw[k] >= 0 ? src + hw[k] : &k7s_zero),
                                       (__attribute__((address_space(3))) void*)(dst + (k * NT + wave * 64) * 16),
                                       16, 0, 0);
    if (kh == 0) {  // minuend granule lane (16 per wave: row 4 q4 + lane / 4, 4 floats); W % 4 == 0 (launcher)
      const int df = s - FL, od = d0 + df, oh = h0 + 4 * q4 + (lane >> 2), ow = w0 + 4 * (lane & 3);
      const bool mok = lane < 16 && out2 && df >= 0 && df < tdc && od < a.do_ && oh < a.ho && ow < a.wo;
      const float* ms = mok ? mbase + (((long long)n * a.do_ + od) * a.ho + oh) * a.wo + ow
                            : reinterpret_cast<const float*>(&k7s_zero);
      __builtin_amdgcn_global_load_lds((const void*)ms,
                                       (__attribute__((address_space(3))) void*)(dst + MOFF + q4 * 64 * 16), 16, 0, 0);
    }
  };
  const int nst = out2 ? 2 : 1;  // store instructions of a flushing wave at a step that finishes a plane
  auto stores_at = [&](int k) { return (k >= FL && k - FL < tdc) ? nst : 0; };
  const float b0 = bias ? bias[0] : 0.f;
  const int td = r16 & 7, hsel = r16 >> 3;
  for (int s = 0; s < NBUF - 1; ++s) issue(s);
  for (int s = 0; s <= nplanes; ++s) {
    // plane s (and the minuend rows it carries) are in: everything issued after them may still be
    // in flight (the two later DMA batches and the stores of the three steps since; in order), then
    // a barrier so every wave's DMA and ring adds are visible to every wave and every wave has
    // finished reading the buffer refilled next
    if (kh == 0)
      k7s_wait_vm<(GPT + 1) * (NBUF - 2)>((GPT + 1) * (NBUF - 2) + stores_at(s - 3) + stores_at(s - 2) + stores_at(s - 1));
    else
      k7s_wait_vm<GPT * (NBUF - 2)>(GPT * (NBUF - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s < nplanes) issue(s + NBUF - 1);  // NBUF - 1 planes ahead, into the buffer of plane s - 1
    const int df = s - FL;  // output plane whose last input plane (s - 1) both K halves have added
    if (kh == 0 && df >= 0 && df < tdc) {
      const int fh = lane >> 4, fw = lane & 15;
      const int od = d0 + df, oh = h0 + 4 * q4 + fh, ow = w0 + fw;
      const int si = ((fh * 4 + (fw & 3)) * 4 + (fw >> 2)) * 9 + (df & 7);
      float* s0 = ring + si;
      float* s1 = rings + (wave + 4) * RING + si;
      float v = *s0 + *s1 + b0;
      *s0 = 0.f;
      *s1 = 0.f;
      if (act == CGAN3D_ACT_TANH) v = tanhf(v);
      const bool ok = od < a.do_ && oh < a.ho && ow < a.wo;
      const long long o = (((long long)n * a.do_ + od) * a.ho + oh) * a.wo + ow;
      *(ok ? y + o : k7s_sink + lane) = v;
      if (out2) {
        const float* mrow = reinterpret_cast<const float*>(bufs + (s % NBUF) * BUF + MOFF + q4 * 64 * 16);
        *(ok ? out2 + o : k7s_sink + lane) = mrow[fh * 16 + fw] - v;
      }
    }
    if (s == nplanes) break;
    const unsigned char* pb = bufs + (s % NBUF) * BUF + 4 * q4 * RB + r16 * 32 + 16 * (g & 1) + 2 * kh * 64;
    f32x4 acc[2];
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) acc[hp] = f32x4{0.f, 0.f, 0.f, 0.f};
    // row r + 1's two A fragments are read while row r's MFMAs run
    bf16x8_k av[2][2];
    auto fetch = [&](int r, bf16x8_k (&o)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j) o[j] = *reinterpret_cast<const bf16x8_k*>(pb + r * RB + (2 * j + (g >> 1)) * 32);
    };
    fetch(0, av[0]);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      if (r + 1 < 10) fetch(r + 1, av[(r + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int hp = 0; hp < 2; ++hp) {
          const int t0 = r - 2 * hp;
          if (t0 >= 0 && t0 < 8)
            acc[hp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[r & 1][j], bw[t0][j], acc[hp], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    // lane (g, hsel, td) holds this K half of P[s][h = 2 hp + hsel][w = 4g + jj][td]: output plane
    // dl = s - td (every read of the eight slots issued before the first write)
    const int dl = s - td;
    if (td < 7 && dl >= 0 && dl < tdc) {
      float* rb = ring + (hsel * 16 + g) * 9 + (dl & 7);
      float v[2][4];
#pragma unroll
      for (int hp = 0; hp < 2; ++hp)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[hp][jj] = rb[(hp * 32 + jj * 4) * 9];
#pragma unroll
      for (int hp = 0; hp < 2; ++hp)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) rb[(hp * 32 + jj * 4) * 9] = v[hp][jj] + acc[hp][jj];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing dummy DMAs land before the block exits
}

// ---- weight gradients.  Both roles are  dW[c][t] = sum_v X16[v][c] * X1[v + t']  with one
// operand on an exact tile (no halo, every voxel read once) and the single-channel one on a halo:
//  * first conv (MODE 0):  X16 = g on the output grid, X1[u] = x[reflect(u - P)], t' = t;
//  * last conv  (MODE 1):  X16 = reflect-padded x on the padded grid (di + 2P), X1[u] = g[u - 6]
//    (zero outside), t' = flip(t) = 342 - t  — the reflection moves to the 16-channel side so the
//    16-channel tensor is never re-read through a halo.
// M = 16 channels, N = taps (2 (td, th) pairs x 8 tw per 16-column tile, 25 tiles), K = the tile's
// voxels.  The four waves split the N tiles (no cross-wave reduction); A fragments come from the
// X16 tile staged channel-major in LDS, B fragments from 8 shifted bf16 copies of the X1 halo.  Each
// block loops over tiles (next tile's global loads in flight during the current tile's MFMAs) and
// writes one partial [c][t]; colsum_kernel adds the partials into dW.
constexpr int G_TD = 4, G_TH = 8, G_TW = 16, G_ROWS_IN = (G_TD + 6) * (G_TH + 6), G_VOX = G_TD * G_TH * G_TW;
constexpr int G_NT = 25;                // N tiles: pairs (2j, 2j+1) x tw 0..7
constexpr int G_COLS = 16 * KT7;        // partial row: [c][t]
constexpr int G_HW = G_TW + 6;          // X1 halo row length (22)
// shifted-copy row (bf16): w 0..15, unpadded.  With [row][tw][16] the ds_read_b128 lane groups
// (MI355X_MICROARCH.md, LDS table) of a B-fragment read cover 16 distinct 16-byte bank blocks:
// (pair half, w half) in {(0,0) tw 0-3, (1,0) tw 4-7, (0,1) tw 4-7, (1,1) tw 0-3} -> blocks 2tw + half.
constexpr int G_SXW = G_TW;
constexpr int G_X1 = G_ROWS_IN * G_HW;  // X1 halo values (3080)
constexpr int G_HWP = 24;               // xh row stride: 16-byte aligned halves, zero tail
constexpr int G_X1_PER = (G_X1 + 255) / 256;

template <int MODE>
__global__ __launch_bounds__(256, 2) void k7m_wg_kernel(K7Args a, const float* __restrict__ x,
                                                        const float* __restrict__ go, float* __restrict__ part,
                                                        int tiles_per_block, int ntiles,
                                                        const __bf16* __restrict__ x16src) {
  constexpr int SX_BYTES = G_ROWS_IN * 8 * G_SXW * 2;    // 53760
  constexpr int AS_BYTES = G_VOX * 16 * 2;               // 16384: [octet][c][8]
  __shared__ __attribute__((aligned(16))) unsigned char lds[SX_BYTES + AS_BYTES + G_ROWS_IN * G_HWP * 2];
  __bf16* sx = reinterpret_cast<__bf16*>(lds);                        // [row][tw][G_SXW]
  __bf16* as = reinterpret_cast<__bf16*>(lds + SX_BYTES);             // [octet][c][8]
  __bf16* xh = reinterpret_cast<__bf16*>(lds + SX_BYTES + AS_BYTES);  // [row][G_HWP]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            r16 = lane & 15;
  // the X16 grid (tiles run over it) and the source of X1
  const int gd = MODE ? a.di + 2 * a.P : a.do_, gh = MODE ? a.hi + 2 * a.P : a.ho, gw = MODE ? a.wi + 2 * a.P : a.wo;
  const int td_n = (gd + G_TD - 1) / G_TD, th_n = (gh + G_TH - 1) / G_TH, tw_n = (gw + G_TW - 1) / G_TW;

  // staging registers: X16 = 8 voxels (one octet along w) x 4 channels per thread, X1 = G_X1_PER values
  const int oct = tid >> 2, c4 = tid & 3;  // octet 0..63 -> (row, half) of the tile
  f32x4 xa[8];
  float xb[G_X1_PER];
  // this thread's X1 halo values: packed (hd, hh, hw), -1 past the halo (fixed over tiles)
  int x1c[G_X1_PER];
#pragma unroll
  for (int k = 0; k < G_X1_PER; ++k) {
    const int i = tid + 256 * k;
    const int hw = i % G_HW, row = i / G_HW;
    x1c[k] = i < G_X1 ? ((row / (G_TH + 6)) | ((row % (G_TH + 6)) << 8) | (hw << 16)) : -1;
  }
  // 32-bit element indices (k7m_ok bounds the tensor sizes)
  auto load = [&](int tile) {
    int tw_ = tile % tw_n, r = tile / tw_n;
    const int th_ = r % th_n; r /= th_n;
    const int td_ = r % td_n, n = r / td_n;
    const int d0 = td_ * G_TD, h0 = th_ * G_TH, w0 = tw_ * G_TW;
    {  // X16 octet: one (d, h) row, 8 consecutive w
      const int row = oct >> 1, wl = w0 + 8 * (oct & 1);
      const int vd = d0 + row / G_TH, vh = h0 + row % G_TH;
      int rowbase;  // element index of (n, d, h, w = 0) in the X16 source, -1 if the row is empty
      if (MODE) {
        const int id = k7_src(vd - a.P, a.di, a.reflect), ih = k7_src(vh - a.P, a.hi, a.reflect);
        rowbase = (vd < gd && vh < gh && (id | ih) >= 0) ? ((n * a.di + id) * a.hi + ih) * a.wi : -1;
      } else {
        rowbase = (vd < gd && vh < gh) ? ((n * a.do_ + vd) * a.ho + vh) * a.wo : -1;
      }
      const f32x4* p = reinterpret_cast<const f32x4*>(MODE ? x : go);
      const bf16x4_k* p16 = reinterpret_cast<const bf16x4_k*>(x16src);  // bf16 shadow of the same tensor
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int vw = wl + e;
        const int iw = MODE ? k7_src(vw - a.P, a.wi, a.reflect) : (vw < gw ? vw : -1);
        const bool ok = rowbase >= 0 && vw < gw && iw >= 0;
        const int idx = ok ? (rowbase + iw) * 4 + c4 : 0;
        if (p16) {  // exact: bf16 -> fp32 here, back to the same bf16 in store()
          const bf16x4_k h = p16[idx];
          xa[e] = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
        } else {
          xa[e] = p[idx];
        }
        if (!ok) xa[e] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const float* p = MODE ? go : x;
#pragma unroll
    for (int k = 0; k < G_X1_PER; ++k) {  // X1 halo value (hd, hh, hw)
      const int c = x1c[k], hd = c & 255, hh = (c >> 8) & 255, hw = c >> 16;
      int src;
      if (MODE) {  // g[u - 6], zero outside
        const int ud = d0 + hd - (K7 - 1), uh = h0 + hh - (K7 - 1), uw = w0 + hw - (K7 - 1);
        const bool ok = c >= 0 && (unsigned)ud < (unsigned)a.do_ && (unsigned)uh < (unsigned)a.ho &&
                        (unsigned)uw < (unsigned)a.wo;
        src = ok ? ((n * a.do_ + ud) * a.ho + uh) * a.wo + uw : -1;
      } else {   // x[reflect(u - P)]
        const int id = k7_src(d0 + hd - a.P, a.di, a.reflect), ih = k7_src(h0 + hh - a.P, a.hi, a.reflect),
                  iw = k7_src(w0 + hw - a.P, a.wi, a.reflect);
        src = (c >= 0 && (id | ih | iw) >= 0) ? ((n * a.di + id) * a.hi + ih) * a.wi + iw : -1;
      }
      xb[k] = p[src >= 0 ? src : 0];
      if (src < 0) xb[k] = 0.f;
    }
  };
  auto store = [&]() {  // staged registers -> LDS (X16 channel-major, X1 as bf16)
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      bf16x8_k u;
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = (__bf16)xa[e][cc];
      *reinterpret_cast<bf16x8_k*>(as + (oct * 16 + 4 * c4 + cc) * 8) = u;
    }
#pragma unroll
    for (int k = 0; k < G_X1_PER; ++k) {
      const int c = x1c[k];
      if (c >= 0) xh[((c & 255) * (G_TH + 6) + ((c >> 8) & 255)) * G_HWP + (c >> 16)] = (__bf16)xb[k];
    }
  };
  for (int r = tid; r < G_ROWS_IN; r += 256) {  // row tails (read by the shifted copies, never stored)
    xh[r * G_HWP + G_HW] = (__bf16)0.f;
    xh[r * G_HWP + G_HW + 1] = (__bf16)0.f;
  }

  f32x4 acc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int boff[7];  // sx offset of this lane's B column in the wave's N tiles (j = wave + 4 jl)
#pragma unroll
  for (int jl = 0; jl < 7; ++jl) {
    const int pair = min(2 * (wave + 4 * jl) + (r16 >> 3), 48);  // past tap 342: dropped at the store
    const int td = pair / K7, th = pair - td * K7;
    boff[jl] = ((td * (G_TH + 6) + th) * 8 + (r16 & 7)) * G_SXW;
  }
  const int t0 = blockIdx.x * tiles_per_block, t1 = min(ntiles, t0 + tiles_per_block);
  if (t0 < t1) load(t0);
  for (int tile = t0; tile < t1; ++tile) {
    lds_barrier();  // previous tile's reads of sx / as done
    store();
    if (tile + 1 < t1) load(tile + 1);  // in flight during this tile's MFMAs
    lds_barrier();
    for (int i = tid; i < G_ROWS_IN * 2; i += 256) {  // shifted copies of (row, half): 8 tw
      const int r = i >> 1, hf = i & 1;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(xh + r * G_HWP + 8 * hf);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(xh + r * G_HWP + 8 * hf + 8);
      const unsigned w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int tw = 0; tw < 8; ++tw) {
        u32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int m = tw / 2 + k;
          o[k] = (tw & 1) ? __builtin_amdgcn_alignbyte(w[m + 1], w[m], 2) : w[m];
        }
        *reinterpret_cast<u32x4*>(sx + ((r * 8 + tw) * G_SXW + 8 * hf)) = o;
      }
    }
    lds_barrier();
    // K-step ks = 32 voxels = tile rows 2ks, 2ks+1 (16 w each); lane group g: row 2ks + (g >> 1), w 8 (g & 1)
    // K-step ks = 32 voxels = tile rows 2ks, 2ks+1; lane group g: row 2ks + (g >> 1), w 8 (g & 1).
    // Two fragment sets in registers: K-step ks + 1's reads are in flight during ks's MFMAs.
    bf16x8_k av[2], bv[2][7];
    auto frag = [&](int ks, int buf) {
      av[buf] = *reinterpret_cast<const bf16x8_k*>(as + ((ks * 4 + g) * 16 + r16) * 8);
      const int row = 2 * ks + (g >> 1), dl = row / G_TH, hl = row % G_TH, wl = 8 * (g & 1);
      const __bf16* sb = sx + ((dl * (G_TH + 6) + hl) * 8 * G_SXW + wl);
#pragma unroll
      for (int jl = 0; jl < 7; ++jl) bv[buf][jl] = *reinterpret_cast<const bf16x8_k*>(sb + boff[jl]);
    };
    frag(0, 0);
#pragma unroll
    for (int ks = 0; ks < G_VOX / 32; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < G_VOX / 32) frag(ks + 1, cur ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jl = 0; jl < 6; ++jl)
        acc[jl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[cur], bv[cur][jl], acc[jl], 0, 0, 0);
      if (wave == 0) acc[6] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[cur], bv[cur][6], acc[6], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // lane holds dW[c = 4g + jj][column r16 of tile j]
  float* pb = part + (long long)blockIdx.x * G_COLS;
#pragma unroll
  for (int jl = 0; jl < 7; ++jl) {
    const int j = wave + 4 * jl;
    if (j >= G_NT) break;
    const int pair = 2 * j + (r16 >> 3), tw = r16 & 7;
    if (pair < 49 && tw < K7) {
      const int tp = pair * K7 + tw;
      const int t = MODE ? KT7 - 1 - tp : tp;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) pb[(4 * g + jj) * KT7 + t] = acc[jl][jj];
    }
  }
}

// dW[c * wc + t] += sum_r part[r][c * T + t] over the nrows partial rows, in a fixed order (round 6:
// the row-split atomics this replaced made the weight gradients order-dependent).  Block = 64 columns
// x 16 row groups; group k sums rows k, k + 16, ... with 8 independent partial sums (8 loads in
// flight), the groups are combined in group order in LDS and one thread per column adds the result
// into dW (the only writer of that element in the launch).
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int nrows, int ncols, int T,
                                                     float* dw, long long wc) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, k = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int cc = col < ncols ? col : 0;
  float s8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = 0.f;
  for (int r0 = k; r0 < nrows; r0 += 128)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = r0 + 16 * j;
      const float v = part[(long long)(r < nrows ? r : k) * ncols + cc];
      s8[j] += r < nrows ? v : 0.f;
    }
  red[k][lane] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  __syncthreads();
  if (k == 0 && col < ncols) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += red[q][lane];
    const int c = col / T, t = col - c * T;
    dw[c * wc + t] += v;
  }
}

void colsum_launch(const float* part, int nrows, int ncols, int T, float* dw, long long wc, hipStream_t s) {
  ::cg::launch(colsum_kernel, dim3((unsigned)((ncols + 63) / 64)), dim3(1024), 0, s, part, nrows, ncols, T, dw, wc);
}

// tiles of the wgrad X16 grid (output grid, or the padded input grid for the last conv)
static int g_k7wg_blocks = 512;  // cgan3d_set_tuning key 20: most blocks of a k7 weight grad (its partial rows)
void k7wg_blocks_set(int v) { g_k7wg_blocks = v > 0 ? v : 512; }

static void k7m_wg_split(const cgan3d_conv_geom* g, bool wide_in, int* grid, int* per, int* ntiles) {
  const int gd = wide_in ? g->di + 2 * g->pad : g->do_, gh = wide_in ? g->hi + 2 * g->pad : g->ho,
            gw = wide_in ? g->wi + 2 * g->pad : g->wo;
  *ntiles = g->n * ((gd + G_TD - 1) / G_TD) * ((gh + G_TH - 1) / G_TH) * ((gw + G_TW - 1) / G_TW);
  *per = (*ntiles + g_k7wg_blocks - 1) / g_k7wg_blocks;
  *grid = (*ntiles + *per - 1) / *per;
}


static K7Args k7m_args(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, int td, int th, int tw) {
  K7Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.P = P; a.reflect = reflect; a.flip = flip; a.wc = wc;
  a.tiles_d = (g->do_ + td - 1) / td; a.tiles_h = (g->ho + th - 1) / th; a.tiles_w = (g->wo + tw - 1) / tw;
  a.probe = g_probe;
  return a;
}

static void k7m_n2w_split(const K7Args& a, int* grid, int* per, int* ntiles) {
  *ntiles = a.n * a.tiles_d * a.tiles_h * a.tiles_w;
  *per = (*ntiles + g_k7wg_blocks - 1) / g_k7wg_blocks;
  *grid = (*ntiles + *per - 1) / *per;
}

long long k7m_n2w_blocks(const cgan3d_conv_geom* g) {
  const K7Args a = k7m_args(g, 0, 0, 0, 0, N_TD, N_TH, N_TW);
  int grid, per, nt;
  k7m_n2w_split(a, &grid, &per, &nt);
  return grid;
}

void k7m_n2w_launch(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, const float* x,
                    const float* w, float* y, float* stats, float* bn_part, hipStream_t s, const Epi* fold,
                    const BnFuse* fz, bool out16) {
  const K7Args a = k7m_args(g, P, reflect, flip, wc, N_TD, N_TH, N_TW);
  int grid, per, nt;
  k7m_n2w_split(a, &grid, &per, &nt);
  K7Fold fb{};
  double* acc1 = nullptr;
  int reps1 = 1;
  if (fold) {
    const int f = fold->bn_fold;
    const bool acc = fold->fz.acc_mode == 4;
    fb = K7Fold{fold->bn_z, fold->bn_ss, fold->bn_mi, acc ? nullptr : fold->bn_part, acc ? fold->fz.acc_out : nullptr,
                acc ? fold->fz.reps : 1, fold->bn_act, fold->bn_slope, f, g->do_ - 2 * f, g->ho - 2 * f, g->wo - 2 * f};
  } else if (fz && fz->acc_mode == 3) {
    acc1 = fz->acc_out;
    reps1 = fz->reps;
  }
  // the streamed-plane kernel (conv_k7p.hip) takes the step's statistics modes (none, fp64 accumulators,
  // folded accumulators); the slab forms stay here
  if (!stats && !bn_part && k7p_n2w_try(g, P, reflect, flip, wc, x, w, y, fold ? &fb : nullptr, fz, out16, s)) return;
  ::cg::launch(out16 ? k7m_n2w_kernel<true> : k7m_n2w_kernel<false>, dim3(grid), dim3(256), 0, s, a, x, w, y, stats,
               bn_part, per, nt, fb, acc1, reps1);
}

static int g_k7s = 0;  // cgan3d_set_tuning key 13: output planes per streamed-w2n block (0 auto, -1 off)
void k7s_set(int v) { g_k7s = v; }

void k7m_w2n_launch(const cgan3d_conv_geom* g, int P, int reflect, long long wc, const float* x, const float* w,
                    float* y, const Epi& e, hipStream_t s) {
  if (e.x16 && g_k7s >= 0 && reflect && g->di == g->do_ && g->hi == g->ho && g->wi == g->wo && P == 3 &&
      std::min(g->di, std::min(g->hi, g->wi)) >= 4 && g->wo % 4 == 0) {
    // streamed-plane kernel: output-plane chunks of 16 planes, or 8 when 16 leaves CUs idle
    K7Args a = k7m_args(g, P, reflect, 0, wc, 1, k7s::SH, k7s::WB);
    int tdc = g_k7s > 0 ? g_k7s : 16;
    auto blocks = [&](int t) { return (long long)g->n * ((g->do_ + t - 1) / t) * a.tiles_h * a.tiles_w; };
    if (g_k7s == 0 && blocks(16) < 256) tdc = 8;
    a.tiles_d = (g->do_ + tdc - 1) / tdc;
    const size_t lds = (size_t)k7s::NBUF * k7s::BUF + 8 * k7s::RING * sizeof(float);
    static bool attr = false;  // > 64 KB of dynamic LDS must be allowed explicitly
    if (!attr) {
      attr = hipFuncSetAttribute((const void*)k7s_w2n_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds) == hipSuccess;
    }
    ::cg::launch(k7s_w2n_kernel, dim3((unsigned)blocks(tdc)), dim3(k7s::NT), lds, s, a, e.x16, w, y, e.bias, e.act,
                 e.minuend, e.out2, tdc);
    return;
  }
  const K7Args a = k7m_args(g, P, reflect, 0, wc, W_TD, W_TH, W_TW);
  int grid, per, nt;
  k7m_n2w_split(a, &grid, &per, &nt);
  if (e.x16)
    ::cg::launch(k7m_w2n_kernel<true>, dim3(grid), dim3(256), 0, s, a, x, e.x16, w, y, e.bias, e.act, e.minuend,
                 e.out2, per, nt);
  else
    ::cg::launch(k7m_w2n_kernel<false>, dim3(grid), dim3(256), 0, s, a, x, e.x16, w, y, e.bias, e.act, e.minuend,
                 e.out2, per, nt);
}

long long k7m_wgrad_ws_floats(const cgan3d_conv_geom* g) {
  int grid, per, nt, grid2;
  k7m_wg_split(g, true, &grid, &per, &nt);
  k7m_wg_split(g, false, &grid2, &per, &nt);
  // the streamed-plane kernel's partial rows (conv_k7p.hip) share the workspace
  const long long p1 = k7p_wg_blocks(g, true), p2 = k7p_wg_blocks(g, false);
  return std::max<long long>(std::max(grid, grid2), std::max(p1, p2)) * G_COLS;
}

// weight grad of a k7 conv with one single-channel side; dw already zeroed (or accumulating)
void k7m_wgrad_launch(const cgan3d_conv_geom* g, bool wide_in, long long wc, const float* x, const float* go, float* dw,
                      float* ws, hipStream_t s, const __bf16* wide16) {
  if (k7p_wgrad_try(g, wide_in, wc, x, go, dw, ws, s, wide16)) return;
  const K7Args a = k7m_args(g, g->pad, g->reflect, 0, wc, G_TD, G_TH, G_TW);
  int grid, per, ntiles;
  k7m_wg_split(g, wide_in, &grid, &per, &ntiles);
  if (wide_in) ::cg::launch(k7m_wg_kernel<1>, dim3(grid), dim3(256), 0, s, a, x, go, ws, per, ntiles, wide16);
  else ::cg::launch(k7m_wg_kernel<0>, dim3(grid), dim3(256), 0, s, a, x, go, ws, per, ntiles, wide16);
  colsum_launch(ws, grid, G_COLS, KT7, dw, wc, s);
}

}  // namespace cg
