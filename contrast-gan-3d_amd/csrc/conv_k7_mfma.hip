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

// ---- n2w tile: 4 (d) x 8 (h) x 16 (w) outputs, wave = one d-slice (8 rows of 16 voxels)
constexpr int N_TD = 4, N_TH = 8, N_TW = 16;
constexpr int N_HD = N_TD + 6, N_HH = N_TH + 6, N_HW = 24;  // x halo (23 used: ow 0..15 + tw 0..7)
constexpr int N_ROWS = N_HD * N_HH;
constexpr int N_PAIRS = 52;                                 // 49 (td, th) pairs padded to 13 K-steps

__global__ __launch_bounds__(256) void k7m_n2w_kernel(K7Args a, const float* __restrict__ x,
                                                      const float* __restrict__ w, float* __restrict__ y,
                                                      float* stats) {
  constexpr int C = 16;
  __shared__ __attribute__((aligned(16))) float xs[N_ROWS * N_HW];
  __shared__ __attribute__((aligned(16))) __bf16 us[N_ROWS * N_TW * 8];  // [row][ow][8 taps]
  __shared__ __attribute__((aligned(16))) __bf16 wt[N_PAIRS * C * 8];    // [pair][c][tw8]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int n, d0, h0, w0;
  {
    int bid = blockIdx.x;
    const int tw_ = bid % a.tiles_w; bid /= a.tiles_w;
    const int th_ = bid % a.tiles_h; bid /= a.tiles_h;
    const int td_ = bid % a.tiles_d; n = bid / a.tiles_d;
    d0 = td_ * N_TD; h0 = th_ * N_TH; w0 = tw_ * N_TW;
  }
  k7m_stage<(N_PAIRS * C * 8 + 255) / 256>(
      w, N_PAIRS * C * 8,
      [&](int i) -> long long {
        const int tw = i & 7, c = (i >> 3) & 15, p = i >> 7;
        if (p >= 49 || tw >= K7) return -1;
        const int t = p * K7 + tw;
        return (long long)c * a.wc + (a.flip ? KT7 - 1 - t : t);
      },
      [&](int i, float v) { wt[i] = (__bf16)v; });
  k7m_stage<(N_ROWS * N_HW + 255) / 256>(
      x, N_ROWS * N_HW,
      [&](int i) -> long long {
        const int hw = i % N_HW, r = i / N_HW, hh = r % N_HH, hd = r / N_HH;
        if (hw >= N_TW + 7) return -1;
        const int id = k7_src(d0 + hd - a.P, a.di, a.reflect);
        const int ih = k7_src(h0 + hh - a.P, a.hi, a.reflect);
        const int iw = k7_src(w0 + hw - a.P, a.wi, a.reflect);
        return (id | ih | iw) >= 0 ? ((long long)(n * a.di + id) * a.hi + ih) * a.wi + iw : -1;
      },
      [&](int i, float v) { xs[i] = v; });
  __syncthreads();
  for (int i = tid; i < N_ROWS * N_TW; i += 256) {
    const int ow = i % N_TW, r = i / N_TW;
    const float* src = xs + r * N_HW + ow;
    bf16x8_k u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = (__bf16)src[j];
    *reinterpret_cast<bf16x8_k*>(us + i * 8) = u;
  }
  __syncthreads();

  const int g = lane >> 4, r16 = lane & 15;
  f32x4 acc[N_TH];
#pragma unroll
  for (int r = 0; r < N_TH; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ks = 0; ks < N_PAIRS / 4; ++ks) {
    const int p = 4 * ks + g;
    const bf16x8_k bv = *reinterpret_cast<const bf16x8_k*>(wt + (p * C + r16) * 8);
    const int pa = p < 49 ? p : 48;  // zero weights past 49: any finite A
    const int td = pa / K7, th = pa - td * K7;
    const __bf16* ub = us + (((wave + td) * N_HH + th) * N_TW + r16) * 8;
#pragma unroll
    for (int r = 0; r < N_TH; ++r) {
      const bf16x8_k av = *reinterpret_cast<const bf16x8_k*>(ub + r * N_TW * 8);
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[r], 0, 0, 0);
    }
  }

  // lane holds out[ow = 4g + jj][c = r16] of row r (oh = h0 + r, od = d0 + wave)
  const int od = d0 + wave;
  float s1 = 0.f;
  int cntl = 0;
#pragma unroll
  for (int r = 0; r < N_TH; ++r) {
    const int oh = h0 + r;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int ow = w0 + 4 * g + jj;
      if (od < a.do_ && oh < a.ho && ow < a.wo) {
        y[((((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow) * C) + r16] = acc[r][jj];
        s1 += acc[r][jj];
        ++cntl;
      }
    }
  }
  if (stats) {  // BatchNorm partials (sum, M2, count) per block, layout of conv.hip
    __shared__ float red[4][C];
    __shared__ float bmean[C];
    __shared__ int bcnt;
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    if (tid == 0) bcnt = 0;
    __syncthreads();
    if (r16 == 0) atomicAdd(&bcnt, cntl);  // count over the 4 g-groups of each wave
    if (g == 0) red[wave][r16] = s1;
    __syncthreads();
    const long long sb = (long long)blockIdx.x * (2 * C + 1);
    if (tid < C) {
      const float S = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      bmean[tid] = bcnt ? S / bcnt : 0.f;
      stats[sb + tid] = S;
    }
    __syncthreads();
    const float m = bmean[r16];
    float q = 0.f;
#pragma unroll
    for (int r = 0; r < N_TH; ++r) {
      const int oh = h0 + r;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int ow = w0 + 4 * g + jj;
        const float dv = (od < a.do_ && oh < a.ho && ow < a.wo) ? acc[r][jj] - m : 0.f;
        q += dv * dv;
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    __syncthreads();
    if (g == 0) red[wave][r16] = q;
    __syncthreads();
    if (tid < C) stats[sb + C + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    if (tid == 0) stats[sb + 2 * C] = (float)bcnt;
  }
}

// ---- w2n tile: 4 (d) x 4 (h) x 16 (w) outputs; the 4 waves split the 100 input rows; the 16
// channels are staged in two halves of 8 (one 16-byte vector per halo voxel)
constexpr int W_TD = 4, W_TH = 4, W_TW = 16;
constexpr int W_HD = W_TD + 6, W_HH = W_TH + 6, W_HW = 24;
constexpr int W_ROWS = W_HD * W_HH;  // 100

__global__ __launch_bounds__(256) void k7m_w2n_kernel(K7Args a, const float* __restrict__ x,
                                                      const float* __restrict__ w, float* __restrict__ y,
                                                      const float* __restrict__ bias, int act,
                                                      const float* __restrict__ minuend, float* __restrict__ out2) {
  constexpr int C = 16;
  __shared__ __attribute__((aligned(16))) __bf16 hs[W_ROWS * W_HW * 8];  // [row][iw][8 channels]
  constexpr int WP = 8 * C + 8;  // (td, th) block of the weight table, padded: lanes of one B read
                                 // hit 16 different blocks, 4 banks apart instead of 64
  __shared__ __attribute__((aligned(16))) __bf16 wt[49 * WP];           // [td*7+th][tw8][c]
  __shared__ float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int n, d0, h0, w0;
  {
    int bid = blockIdx.x;
    const int tw_ = bid % a.tiles_w; bid /= a.tiles_w;
    const int th_ = bid % a.tiles_h; bid /= a.tiles_h;
    const int td_ = bid % a.tiles_d; n = bid / a.tiles_d;
    d0 = td_ * W_TD; h0 = th_ * W_TH; w0 = tw_ * W_TW;
  }
  k7m_stage<(49 * 8 * C + 255) / 256>(
      w, 49 * 8 * C,
      [&](int i) -> long long {
        const int c = i & 15, tw = (i >> 4) & 7, p = i >> 7;
        return tw < K7 ? (long long)c * a.wc + p * K7 + tw : -1;
      },
      [&](int i, float v) { wt[(i >> 7) * WP + (i & 127)] = (__bf16)v; });
  const int g = lane >> 4, r16 = lane & 15;
  const int odl = r16 >> 2, ohl = r16 & 3;  // this lane's B column: output row (od, oh)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int half = 0; half < 2; ++half) {
    if (half) __syncthreads();  // all waves done reading the first half
    k7m_stage<(W_ROWS * W_HW * 2 + 255) / 256>(
        reinterpret_cast<const f32x4*>(x), W_ROWS * W_HW * 2,
        [&](int i) -> long long {  // float4 index
          const int q = i & 1, v = i >> 1, hw = v % W_HW, r = v / W_HW, hh = r % W_HH, hd = r / W_HH;
          if (hw >= W_TW + 7) return -1;
          const int id = k7_src(d0 + hd - a.P, a.di, a.reflect);
          const int ih = k7_src(h0 + hh - a.P, a.hi, a.reflect);
          const int iw = k7_src(w0 + hw - a.P, a.wi, a.reflect);
          return (id | ih | iw) >= 0 ? (((long long)(n * a.di + id) * a.hi + ih) * a.wi + iw) * (C / 4) + half * 2 + q
                                     : -1;
        },
        [&](int i, f32x4 val) {
          __bf16* d = hs + (i >> 1) * 8 + 4 * (i & 1);
          d[0] = (__bf16)val[0]; d[1] = (__bf16)val[1]; d[2] = (__bf16)val[2]; d[3] = (__bf16)val[3];
        });
    __syncthreads();
#pragma unroll 1
    for (int pr = wave * 25; pr < wave * 25 + 25; ++pr) {
      const int id = pr / W_HH, ih = pr - id * W_HH;
      const int td = id - odl, th = ih - ohl;
      const bool band = td >= 0 && td < K7 && th >= 0 && th < K7;
      const __bf16* wrow = wt + (band ? td * K7 + th : 0) * WP + half * 8;
      const __bf16* hrow = hs + (pr * W_HW + r16) * 8;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int tw = 4 * s + g;
        const bf16x8_k av = *reinterpret_cast<const bf16x8_k*>(hrow + tw * 8);
        bf16x8_k bv = *reinterpret_cast<const bf16x8_k*>(wrow + tw * C);
        if (!band) bv = bf16x8_k{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
      }
    }
  }
  // combine the 4 waves: lane holds out[ow = 4g + jj][(od, oh) = r16]
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) red[wave][(4 * g + jj) * 16 + r16] = acc[jj];
  __syncthreads();
  {
    const int m = tid >> 4, nn = tid & 15;  // ow_l = m, (odl, ohl) = nn
    const int od = d0 + (nn >> 2), oh = h0 + (nn & 3), ow = w0 + m;
    if (od < a.do_ && oh < a.ho && ow < a.wo) {
      float v = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid] + (bias ? bias[0] : 0.f);
      if (act == CGAN3D_ACT_TANH) v = tanhf(v);
      const long long o = ((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow;
      y[o] = v;
      if (out2) out2[o] = minuend[o] - v;
    }
  }
}

// ---- weight gradients: M = the 16 channels, N = taps (2 (td, th) pairs x 8 tw per 16-column
// tile, 25 tiles), K = voxels.  The channel operand comes straight from global memory (8 strided
// floats per lane, rounded to bf16); the single-channel operand is staged as 8 shifted bf16 copies
// so that every B fragment is one aligned ds_read_b128.  Blocks loop over output tiles (4 x 8 x 16)
// with the 25 accumulators resident, combine their waves in LDS and write one partial per block;
// k7m_colsum_kernel adds the partials into dW.
constexpr int G_TD = 4, G_TH = 8, G_TW = 16, G_ROWS_IN = (G_TD + 6) * (G_TH + 6), G_OROWS = G_TD * G_TH;
constexpr int G_NT = 25;                // N tiles: pairs (2j, 2j+1) x tw 0..7
constexpr int G_COLS = 16 * KT7;        // partial row: [c][t]

__device__ __forceinline__ void k7m_tile(const K7Args& a, int tile, int* n, int* d0, int* h0, int* w0) {
  const int tw_ = tile % a.tiles_w; tile /= a.tiles_w;
  const int th_ = tile % a.tiles_h; tile /= a.tiles_h;
  const int td_ = tile % a.tiles_d; *n = tile / a.tiles_d;
  *d0 = td_ * G_TD; *h0 = th_ * G_TH; *w0 = tw_ * G_TW;
}

// combine the 4 waves' accumulators and write this block's partial [c][t].  Column n of N-tile
// j holds tap (pair, tw) = (2j + (n >> 3), n & 7) when TD_TILES is false (25 tiles), and
// (td, th, tw) = (j >> 2, 2 (j & 3) + (n >> 3), n & 7) when it is true (28 tiles).
template <int NT, bool TD_TILES>
__device__ __forceinline__ void k7m_wg_store(f32x4 (&acc)[NT], float* red, float* part) {
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
  for (int i = tid; i < NT * 256; i += 256) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) atomicAdd(&red[j * 256 + (4 * g + jj) * 16 + r16], acc[j][jj]);
  __syncthreads();
  float* pb = part + (long long)blockIdx.x * G_COLS;
  for (int i = tid; i < NT * 256; i += 256) {
    const int j = i >> 8, c = (i >> 4) & 15, col = i & 15, tw = col & 7;
    int pair;
    if (TD_TILES) {
      const int th = 2 * (j & 3) + (col >> 3);
      pair = th < K7 ? (j >> 2) * K7 + th : 99;
    } else {
      pair = 2 * j + (col >> 3);
    }
    if (pair < 49 && tw < K7) pb[c * KT7 + pair * K7 + tw] = red[i];
  }
}

// dW[c, t] = sum_o x[src(o + t - P)] * g[o, c]   (first conv; x single-channel, g 16 channels)
__global__ __launch_bounds__(256) void k7m_wg_n2w_kernel(K7Args a, const float* __restrict__ x,
                                                         const float* __restrict__ go, float* __restrict__ part,
                                                         int ntiles) {
  constexpr int HW = G_TW + 8;  // x halo row: ow 0..15 + tw 0..7
  constexpr int SXW = G_TW + 8;  // shifted-copy row (bf16), padded: the 8 tw copies of a row fall
                                 // on distinct banks
  __shared__ __attribute__((aligned(16))) unsigned char lds[8 * G_ROWS_IN * SXW * 2 + G_ROWS_IN * HW * 4];
  __bf16* sx = reinterpret_cast<__bf16*>(lds);                           // [row][tw][SXW]
  float* xs = reinterpret_cast<float*>(lds + 8 * G_ROWS_IN * SXW * 2);  // [row][24]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            r16 = lane & 15;
  f32x4 acc[G_NT];
#pragma unroll
  for (int j = 0; j < G_NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int n, d0, h0, w0;
    k7m_tile(a, tile, &n, &d0, &h0, &w0);
    __syncthreads();
    k7m_stage<(G_ROWS_IN * HW + 255) / 256>(
        x, G_ROWS_IN * HW,
        [&](int i) -> long long {
          const int hw = i % HW, r = i / HW, hh = r % (G_TH + 6), hd = r / (G_TH + 6);
          if (hw >= G_TW + 6) return -1;
          const int id = k7_src(d0 + hd - a.P, a.di, a.reflect);
          const int ih = k7_src(h0 + hh - a.P, a.hi, a.reflect);
          const int iw = k7_src(w0 + hw - a.P, a.wi, a.reflect);
          return (id | ih | iw) >= 0 ? ((long long)(n * a.di + id) * a.hi + ih) * a.wi + iw : -1;
        },
        [&](int i, float v) { xs[i] = v; });
    __syncthreads();
    for (int i = tid; i < 8 * G_ROWS_IN * 2; i += 256) {  // (tw, row, half of 16)
      const int hf = i & 1, r = (i >> 1) % G_ROWS_IN, tw = (i >> 1) / G_ROWS_IN;
      const float* src = xs + r * HW + tw + 8 * hf;
      bf16x8_k u;
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = (__bf16)src[e];
      *reinterpret_cast<bf16x8_k*>(sx + ((r * 8 + tw) * SXW + 8 * hf)) = u;
    }
    __syncthreads();
    // K-steps of 32 outputs = 2 output rows x 16; wave takes K-steps wave, wave+4, ...
    constexpr int KS = G_OROWS / 2 / 4;  // K-steps per wave per tile
    float gv[KS][8];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {  // issue every load of the wave's K-steps first
      const int orow = 2 * (wave + 4 * kk) + (g >> 1), owl = 8 * (g & 1);
      const int od = d0 + orow / G_TH, oh = h0 + orow % G_TH;
      const bool rv = od < a.do_ && oh < a.ho;
      const long long vb = (((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + w0 + owl) * 16 + r16;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rv && w0 + owl + e < a.wo;
        gv[kk][e] = go[ok ? vb + e * 16 : 0];
        if (!ok) gv[kk][e] = 0.f;
      }
    }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int ks = wave + 4 * kk;
      const int orow = 2 * ks + (g >> 1), odl = orow / G_TH, ohl = orow % G_TH, owl = 8 * (g & 1);
      bf16x8_k av;
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = (__bf16)gv[kk][e];
#pragma unroll
      for (int j = 0; j < G_NT; ++j) {
        const int pair = 2 * j + (r16 >> 3), tw = r16 & 7;
        const int pa = pair < 49 ? pair : 48;
        const int td = pa / K7, th = pa - td * K7;
        const bf16x8_k bv = *reinterpret_cast<const bf16x8_k*>(
            sx + ((((odl + td) * (G_TH + 6) + ohl + th) * 8 + tw) * SXW + owl));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  k7m_wg_store<G_NT, false>(acc, reinterpret_cast<float*>(lds), part);
}

// dW[c, t] = sum_i x[src(i), c] * g[i - t]   (last conv; x 16 channels on the input halo, g single-
// channel on the output tile); K = the 32 halo columns of one input row
__global__ __launch_bounds__(256) void k7m_wg_w2n_kernel(K7Args a, const float* __restrict__ x,
                                                         const float* __restrict__ go, float* __restrict__ part,
                                                         int ntiles) {
  constexpr int Q = 32;  // halo columns per input row (22 used)
  __shared__ __attribute__((aligned(16))) unsigned char lds[28 * 256 * 4];
  constexpr int QP = Q + 8;  // padded row: a B read's 8 tw copies fall on distinct banks
  __bf16* sd = reinterpret_cast<__bf16*>(lds);                   // [orow][tw][QP]: g[orow][q - tw]
  float* gs = reinterpret_cast<float*>(lds + 8 * G_OROWS * QP * 2);  // [orow][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            r16 = lane & 15;
  constexpr int NT = 28;  // N tiles (td, th pair (0,1) (2,3) (4,5) (6,-)) x tw 0..7
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int n, d0, h0, w0;
    k7m_tile(a, tile, &n, &d0, &h0, &w0);
    __syncthreads();
    for (int i = tid; i < G_OROWS * G_TW; i += 256) {
      const int owl = i % G_TW, r = i / G_TW, od = d0 + r / G_TH, oh = h0 + r % G_TH, ow = w0 + owl;
      gs[i] = (od < a.do_ && oh < a.ho && ow < a.wo) ? go[((long long)(n * a.do_ + od) * a.ho + oh) * a.wo + ow] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < 8 * G_OROWS * (Q / 8); i += 256) {
      const int q8 = i % (Q / 8), r = (i / (Q / 8)) % G_OROWS, tw = i / (Q / 8 * G_OROWS);
      bf16x8_k u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ow = 8 * q8 + e - tw;
        u[e] = (__bf16)((ow >= 0 && ow < G_TW) ? gs[r * G_TW + ow] : 0.f);
      }
      *reinterpret_cast<bf16x8_k*>(sd + ((r * 8 + tw) * QP + 8 * q8)) = u;
    }
    __syncthreads();
    // this lane's 8 halo columns (fixed over the rows)
    int swc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = 8 * g + e;
      swc[e] = q < G_TW + 6 ? k7_src(w0 + q - a.P, a.wi, a.reflect) : -1;
    }
    constexpr int RB = 5;  // rows per batch: 5 x 8 loads in flight per lane
    static_assert((G_ROWS_IN / 4) % RB == 0, "row batches");
    for (int rb0 = wave; rb0 < G_ROWS_IN; rb0 += 4 * RB) {
      float xv[RB][8];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int r = rb0 + 4 * b, id = r / (G_TH + 6), ih = r % (G_TH + 6);
        const int sd_ = k7_src(d0 + id - a.P, a.di, a.reflect);
        const int sh_ = k7_src(h0 + ih - a.P, a.hi, a.reflect);
        const long long rowb = ((long long)(n * a.di + sd_) * a.hi + sh_) * a.wi;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool ok = (sd_ | sh_ | swc[e]) >= 0;
          xv[b][e] = x[ok ? (rowb + swc[e]) * 16 + r16 : 0];
          if (!ok) xv[b][e] = 0.f;
        }
      }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int r = rb0 + 4 * b, id = r / (G_TH + 6), ih = r % (G_TH + 6);
        bf16x8_k av;
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = (__bf16)xv[b][e];
        // taps reaching an output row of this tile from input row (id, ih): td in [id-3, id],
        // th in [ih-7, ih] (intersected with 0..6); branch per td (scalar), 4 th-pair tiles each
        const int thl = ih - (G_TH - 1) > 0 ? ih - (G_TH - 1) : 0, thh = ih < K7 - 1 ? ih : K7 - 1;
        const int th0 = r16 >> 3, tw = r16 & 7;  // this lane's column: th = 2q + th0, tw
#pragma unroll
        for (int td = 0; td < K7; ++td) {
          const int odl = id - td;
          if (odl < 0 || odl >= G_TD) continue;
          bf16x8_k bv[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // all four B reads before the MFMAs
            const int thq = 2 * q + th0, ohl = ih - thq;
            const bool mine = thq >= thl && thq <= thh;
            bv[q] = *reinterpret_cast<const bf16x8_k*>(sd + (((mine ? odl * G_TH + ohl : 0) * 8 + tw) * QP + 8 * g));
            if (!mine) bv[q] = bf16x8_k{};
          }
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[td * 4 + q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[q], acc[td * 4 + q], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();
  k7m_wg_store<NT, true>(acc, reinterpret_cast<float*>(lds), part);
}

// dW[c * wc + t] += sum_b part[b][c * 343 + t]; grid (cols / 256, row splits)
__global__ __launch_bounds__(256) void k7m_colsum_kernel(const float* __restrict__ part, int nrows, int rows_per,
                                                         float* dw, long long wc) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= G_COLS) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(nrows, r0 + rows_per);
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += part[(long long)r * G_COLS + col];
  const int c = col / KT7, t = col - c * KT7;
  atomicAdd(dw + c * wc + t, s);
}

static int k7m_wg_grid(int ntiles) { return ntiles < 512 ? ntiles : 512; }

static K7Args k7m_args(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, int td, int th, int tw) {
  K7Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.P = P; a.reflect = reflect; a.flip = flip; a.wc = wc;
  a.tiles_d = (g->do_ + td - 1) / td; a.tiles_h = (g->ho + th - 1) / th; a.tiles_w = (g->wo + tw - 1) / tw;
  return a;
}

long long k7m_n2w_blocks(const cgan3d_conv_geom* g) {
  const K7Args a = k7m_args(g, 0, 0, 0, 0, N_TD, N_TH, N_TW);
  return (long long)a.n * a.tiles_d * a.tiles_h * a.tiles_w;
}

void k7m_n2w_launch(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, const float* x,
                    const float* w, float* y, float* stats, hipStream_t s) {
  const K7Args a = k7m_args(g, P, reflect, flip, wc, N_TD, N_TH, N_TW);
  hipLaunchKernelGGL(k7m_n2w_kernel, dim3((unsigned)(a.n * a.tiles_d * a.tiles_h * a.tiles_w)), dim3(256), 0, s, a,
                     x, w, y, stats);
}

void k7m_w2n_launch(const cgan3d_conv_geom* g, int P, int reflect, long long wc, const float* x, const float* w,
                    float* y, const Epi& e, hipStream_t s) {
  const K7Args a = k7m_args(g, P, reflect, 0, wc, W_TD, W_TH, W_TW);
  hipLaunchKernelGGL(k7m_w2n_kernel, dim3((unsigned)(a.n * a.tiles_d * a.tiles_h * a.tiles_w)), dim3(256), 0, s, a,
                     x, w, y, e.bias, e.act, e.minuend, e.out2);
}

long long k7m_wgrad_ws_floats(const cgan3d_conv_geom* g) {
  const K7Args a = k7m_args(g, 0, 0, 0, 0, G_TD, G_TH, G_TW);
  return (long long)k7m_wg_grid(a.n * a.tiles_d * a.tiles_h * a.tiles_w) * G_COLS;
}

// weight grad of a k7 conv with one single-channel side; dw already zeroed (or accumulating)
void k7m_wgrad_launch(const cgan3d_conv_geom* g, bool wide_in, long long wc, const float* x, const float* go, float* dw,
                      float* ws, hipStream_t s) {
  const K7Args a = k7m_args(g, g->pad, g->reflect, 0, wc, G_TD, G_TH, G_TW);
  const int ntiles = a.n * a.tiles_d * a.tiles_h * a.tiles_w;
  const int grid = k7m_wg_grid(ntiles);
  if (wide_in) hipLaunchKernelGGL(k7m_wg_w2n_kernel, dim3(grid), dim3(256), 0, s, a, x, go, ws, ntiles);
  else hipLaunchKernelGGL(k7m_wg_n2w_kernel, dim3(grid), dim3(256), 0, s, a, x, go, ws, ntiles);
  const int rows_per = 32;
  hipLaunchKernelGGL(k7m_colsum_kernel, dim3((G_COLS + 255) / 256, (grid + rows_per - 1) / rows_per), dim3(256), 0, s,
                     ws, grid, rows_per, dw, wc);
}

}  // namespace cg
