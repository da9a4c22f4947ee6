// Halo-tiled direct convolution, bf16 MFMA (gfx950) — the generator's 32/64-channel convs.
//
// ResNetBlock convs (model/blocks.py:68-85; k3 s1 p1, 64 -> 64), the 32 -> 64 downsampling conv
// and both ConvTranspose3d upsampling layers (generator.py:40-47,61-77), their input-grads, and the
// critic's 32/64-channel layers.  conv_gemm.hip re-gathers every input row once per tap through
// L1/L2; here each 4x4x4 output tile loads its input halo ONCE:
//
//  * halo [Ez][Ey][Ex][cin(+8 pad)] bf16 in LDS, converted from the fp32 NDHWC activations while
//    staging (one pass of coalesced float4 loads);
//  * the packed weights (bf16, [tap][cout][cin], 16-byte granules XOR-swizzled by cout so the
//    MFMA B-fragment reads are conflict-free) stream through a 3-slot LDS ring by LDS-DMA
//    (global_load_lds_dwordx4), two taps ahead, with counted vmcnt waits and raw s_barrier so the
//    DMAs stay in flight across barriers (cdna_hip_programming.md §5 "Pipelining across barriers");
//  * per tap each wave (one z-slice = 16 output voxels) runs cin/32 x (BN/16)
//    v_mfma_f32_16x16x32_bf16 whose A fragments are b128 reads of the halo at the tap's offset.
//
// Stride-2 transposed launches keep conv.hip's parity classes; a class's valid taps map a tile of
// class coordinates j to gathered coordinates j + off(t), so its halo is tile + (max-min) offset.
// Epilogue (bias, act, mask, residual, BatchNorm partial statistics) as in conv_gemm.hip.
#include "common.h"

namespace cg {

typedef __bf16 bf16x8_h __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_h __attribute__((ext_vector_type(4)));

struct HaloArgs {
  int n, di, hi, wi, do_, ho, wo, cin, cout, k, s, p, transposed;
  int cd, ch, cw;             // class-local grid (transposed s>1) or output grid
  int td, th, tw;             // tiles per dim (4 each)
  int nclass;
  int ez, ey, ex;             // halo extents
  int halo_bytes;
  int bn;                     // output channels per block
};

constexpr int HT = 4;  // tile edge (4 x 4 x 4 = 64 output voxels)


struct ClassTaps {
  int f, st, n;   // first tap, step, count
  int omin, omax; // gathered offset range (transposed) / tap range (forward)
};

__host__ __device__ inline ClassTaps class_info(int r, int k, int s, int p, int transposed) {
  ClassTaps c;
  if (transposed) {
    c.f = (r + p) % s; c.st = s; c.n = c.f < k ? (k - c.f + s - 1) / s : 0;
    // off(t) = (r + p - t)/s decreases with t
    c.omax = c.n ? (r + p - c.f) / s : 0;
    c.omin = c.n ? (r + p - (c.f + s * (c.n - 1))) / s : 0;
  } else {
    c.f = 0; c.st = 1; c.n = k; c.omin = 0; c.omax = k - 1;
  }
  return c;
}

// halo extent along one dim for a 4-wide tile
__host__ __device__ inline int halo_extent(const ClassTaps& c, int s, int transposed) {
  return transposed ? HT + c.omax - c.omin : (HT - 1) * s + c.omax + 1;
}

__device__ __attribute__((aligned(16))) float g_halo_zero[4];  // source of the absent epilogue operands

// Epilogue of the halo-tiled kernels: lane holds tile rows wave*16 + 4g + jj (row_out: output
// voxel of each of the 64 tile rows, -1 outside) for channel co0 + t*16 + r16; bias, activation,
// mask, residual, store, BatchNorm statistics (block-major partials, or slab modes 1 / 2).
// smemf: >= 8 * 16 * NT floats of LDS the caller no longer needs.
template <int NT>
__device__ __forceinline__ void halo_epilogue(const HaloArgs& a, f32x4 (&acc)[NT], const int* row_out, int co0,
                                              float* y, const Epi& ep, float* smemf) {
  constexpr int BN = 16 * NT;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  // ---- epilogue: lane holds tile rows wave*16 + 4g + jj for channel co0 + t*16 + r16
  float vals[NT][4];
  bool rowv[4];
  int rowo[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    rowo[jj] = row_out[wave * 16 + 4 * g + jj];
    rowv[jj] = rowo[jj] >= 0;
  }
  // residual / BatchNorm-input / mask / bias operands: every load issued before the first use,
  // unconditionally (clamped offsets, absent operands read from a zero dummy through an opaque
  // pointer: a select between load addresses, or a load under a condition, becomes a branch with a
  // wait of its own)
  const bool mode2 = ep.bn_mode == 2 || ep.fz.acc_mode == 4;  // (sum g, sum g*xhat): slab or accumulators
  const bool has_res = ep.residual != nullptr, has_mask = ep.mask_src != nullptr, has_bias = ep.bias != nullptr;
  uintptr_t pr = has_res ? (uintptr_t)ep.residual : (uintptr_t)g_halo_zero;
  uintptr_t pz = mode2 ? (uintptr_t)ep.bn_z : (uintptr_t)g_halo_zero;
  uintptr_t pm = has_mask ? (uintptr_t)ep.mask_src : (uintptr_t)g_halo_zero;
  uintptr_t pb = has_bias ? (uintptr_t)ep.bias : (uintptr_t)g_halo_zero;
  asm volatile("" : "+s"(pr), "+s"(pz), "+s"(pm), "+s"(pb));
  float resv[NT][4], zv[NT][4], mv[NT][4], bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = co0 + t * 16 + r16;
    bv[t] = reinterpret_cast<const float*>(pb)[has_bias && c < a.cout ? c : 0];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const long long o = (rowv[jj] && c < a.cout) ? (long long)rowo[jj] * a.cout + c : 0;
      resv[t][jj] = reinterpret_cast<const float*>(pr)[has_res ? o : 0];
      zv[t][jj] = reinterpret_cast<const float*>(pz)[mode2 ? o : 0];
      mv[t][jj] = reinterpret_cast<const float*>(pm)[has_mask ? o : 0];
    }
  }
  const bool relu = ep.act == CGAN3D_ACT_RELU, lrelu = ep.act == CGAN3D_ACT_LRELU;
  const float slope = ep.slope;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = co0 + t * 16 + r16;
    const bool cv = c < a.cout;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      float v = acc[t][jj] + bv[t];
      v = relu ? fmaxf(v, 0.f) : v;
      v = (lrelu & !(v > 0.f)) ? v * slope : v;
      v = (has_mask & !(mv[t][jj] > 0.f)) ? v * slope : v;
      v += resv[t][jj];
      if (rowv[jj] && cv) y[(long long)rowo[jj] * a.cout + c] = v;
      vals[t][jj] = (rowv[jj] && cv) ? v : 0.f;
    }
  }
  const bool acc3 = ep.fz.acc_mode == 3;
  // replica of the fp64 accumulators this block adds into (cgan3d_bn_fuse)
  double* const facc = ep.fz.acc_mode ? ep.fz.acc_out + (long long)(blockIdx.x % ep.fz.reps) * 2 * a.cout : nullptr;
  if (ep.stats || ep.bn_mode == 1 || acc3) {  // (sum, M2 about the block mean, count): block-major or slab
    lds_barrier();
    float* red = smemf;  // [4 waves][BN]
    __shared__ float bmean[64];
    const int cntv = __popcll(__ballot(row_out[lane] >= 0));  // valid tile rows (64 = one per lane)
    const long long sbase = (long long)blockIdx.x * (2 * a.cout + 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float sum = vals[t][0] + vals[t][1] + vals[t][2] + vals[t][3];
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      if (g == 0) red[wave * BN + t * 16 + r16] = sum;
    }
    lds_barrier();
    float S = 0.f;
    if (tid < BN) {
      S = red[tid] + red[BN + tid] + red[2 * BN + tid] + red[3 * BN + tid];
      bmean[tid] = cntv ? S / cntv : 0.f;
      if (co0 + tid < a.cout && !acc3) {
        if (ep.stats) ep.stats[sbase + co0 + tid] = S;
        else *bn_slot(ep, 0, a.cout, co0 + tid, blockIdx.x) = S;
      }
    }
    lds_barrier();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int cl = t * 16 + r16;
      const float m = bmean[cl];
      float q = 0.f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float d = (rowv[jj] && co0 + cl < a.cout) ? vals[t][jj] - m : 0.f;
        q += d * d;
      }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) red[wave * BN + cl] = q;
    }
    lds_barrier();
    if (tid < BN) {
      const float M2 = red[tid] + red[BN + tid] + red[2 * BN + tid] + red[3 * BN + tid];
      if (co0 + tid < a.cout) {
        if (acc3) {  // (sum, sum of squares) = (S, M2 + S * mean), fp64 adds into this block's replica
          if (cntv) {
            unsafeAtomicAdd(facc + co0 + tid, (double)S);
            unsafeAtomicAdd(facc + a.cout + co0 + tid, (double)M2 + (double)S * (double)S / cntv);
          }
        } else if (ep.stats) {
          ep.stats[sbase + a.cout + co0 + tid] = M2;
        } else {
          *bn_slot(ep, 1, a.cout, co0 + tid, blockIdx.x) = M2;
        }
      }
    }
    if (tid == 0 && blockIdx.y == 0 && !acc3) {
      if (ep.stats) ep.stats[sbase + 2 * a.cout] = (float)cntv;
      else *bn_slot(ep, 2, a.cout, 0, blockIdx.x) = (float)cntv;
    }
  }
  if (mode2) {  // fused BatchNorm backward statistics: this block's slot of the slab (or accumulators)
    float p1[NT], p2[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = co0 + t * 16 + r16;
      p1[t] = 0.f;
      p2[t] = 0.f;
      if (c < a.cout) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (rowv[jj]) bn_pair_z(ep, vals[t][jj], zv[t][jj], c, a.cout, &p1[t], &p2[t]);
      }
      p1[t] += __shfl_xor(p1[t], 16, 64);
      p1[t] += __shfl_xor(p1[t], 32, 64);
      p2[t] += __shfl_xor(p2[t], 16, 64);
      p2[t] += __shfl_xor(p2[t], 32, 64);
    }
    lds_barrier();
    float* red = smemf;  // [2][4 waves][BN]
    if (g == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        red[wave * BN + t * 16 + r16] = p1[t];
        red[(4 + wave) * BN + t * 16 + r16] = p2[t];
      }
    }
    lds_barrier();
    if (tid < BN && co0 + tid < a.cout) {
      const float q0 = red[tid] + red[BN + tid] + red[2 * BN + tid] + red[3 * BN + tid];
      const float q1 = red[4 * BN + tid] + red[5 * BN + tid] + red[6 * BN + tid] + red[7 * BN + tid];
      if (facc) {
        unsafeAtomicAdd(facc + co0 + tid, (double)q0);
        unsafeAtomicAdd(facc + a.cout + co0 + tid, (double)q1);
      } else {
        *bn_slot(ep, 0, a.cout, co0 + tid, blockIdx.x) = q0;
        *bn_slot(ep, 1, a.cout, co0 + tid, blockIdx.x) = q1;
      }
    }
  }
}

template <int CIN, int NT>  // NT = BN/16 output-channel tiles per wave
__global__ __launch_bounds__(256) void conv_halo_kernel(HaloArgs a, const float* __restrict__ x,
                                                        const __bf16* __restrict__ wpk, float* y, Epi ep) {
  constexpr int BN = 16 * NT;
  constexpr int ROW = CIN + 8;                 // halo row (elements), 16 B pad
  constexpr int NG = CIN / 8;                  // 16-byte granules per weight row
  constexpr int SLOT = BN * CIN;               // bf16 elements per tap slab
  constexpr int DMA_PER_TAP = (SLOT * 2 + 4095) / 4096;  // global_load_lds_dwordx4 per thread per tap
  static_assert(SLOT * 2 % 1024 == 0 && DMA_PER_TAP <= 2, "slab must be 2, 4 or 8 KB");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __bf16* wring = reinterpret_cast<__bf16*>(smem);                // [3][SLOT]
  __bf16* halo = reinterpret_cast<__bf16*>(smem + 3 * SLOT * 2);  // [E][ROW]
  __shared__ int tq[3][64];                                        // per-tap halo offsets
  __shared__ int tlin[64];
  __shared__ int row_out[64];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles = a.td * a.th * a.tw;
  int bid = blockIdx.x;
  const int cls = bid / (a.n * tiles);
  bid -= cls * a.n * tiles;
  const int nb = bid / tiles;
  bid -= nb * tiles;
  const int tz = bid / (a.th * a.tw), ty = (bid / a.tw) % a.th, tx = bid % a.tw;
  const int co0 = blockIdx.y * BN;
  const int s = a.s;
  int r3[3] = {0, 0, 0};
  if (a.transposed) { r3[0] = cls / (s * s); r3[1] = (cls / s) % s; r3[2] = cls % s; }
  const ClassTaps cz = class_info(r3[0], a.k, s, a.p, a.transposed);
  const ClassTaps cy = class_info(r3[1], a.k, s, a.p, a.transposed);
  const ClassTaps cx = class_info(r3[2], a.k, s, a.p, a.transposed);
  const int ntap = cz.n * cy.n * cx.n;
  // gathered-grid origin of the halo
  int oz, oy, ox;
  if (a.transposed) { oz = tz * HT + cz.omin; oy = ty * HT + cy.omin; ox = tx * HT + cx.omin; }
  else { oz = tz * HT * s - a.p; oy = ty * HT * s - a.p; ox = tx * HT * s - a.p; }
  const int se = a.transposed ? 1 : s;

  // ---- tap table: halo offsets and packed-weight slab index
  if (tid < ntap) {
    const int mw = tid % cx.n, mh = (tid / cx.n) % cy.n, md = tid / (cx.n * cy.n);
    const int t0 = cz.f + cz.st * md, t1 = cy.f + cy.st * mh, t2 = cx.f + cx.st * mw;
    if (a.transposed) {
      tq[0][tid] = (r3[0] + a.p - t0) / s - cz.omin;
      tq[1][tid] = (r3[1] + a.p - t1) / s - cy.omin;
      tq[2][tid] = (r3[2] + a.p - t2) / s - cx.omin;
    } else {
      tq[0][tid] = t0; tq[1][tid] = t1; tq[2][tid] = t2;
    }
    tlin[tid] = (t0 * a.k + t1) * a.k + t2;
  }
  if (tid < 64) {  // output voxel of tile row tid = (z, y, x) = (tid>>4, (tid>>2)&3, tid&3)
    const int jz = tz * HT + (tid >> 4), jy = ty * HT + ((tid >> 2) & 3), jx = tx * HT + (tid & 3);
    int od = jz, oh = jy, ow = jx;
    if (a.transposed) { od = jz * s + r3[0]; oh = jy * s + r3[1]; ow = jx * s + r3[2]; }
    const bool ok = jz < a.cd && jy < a.ch && jx < a.cw;
    row_out[tid] = ok ? ((nb * a.do_ + od) * a.ho + oh) * a.wo + ow : -1;
  }
  __syncthreads();

  // ---- weight ring: slab of tap j (channels co0..co0+BN) -> slot j % 3 by LDS-DMA
  auto issue = [&](int j) {
    const __bf16* src = wpk + ((long long)tlin[j] * a.cout + co0) * CIN;
    __bf16* dst = wring + (j % 3) * SLOT;
#pragma unroll
    for (int q = 0; q < DMA_PER_TAP; ++q) {
      const int byte = (q * 256 + tid) * 16;
      if (byte >= SLOT * 2) break;  // 2 KB slabs: waves 2-3 idle (wave-uniform)
      // LDS destination = wave-uniform base + lane * 16 (M0 holds the base)
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const char*>(src) + byte),
                                       (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(dst) + (q * 256 + wave * 64) * 16),
                                       16, 0, 0);
    }
  };
  if (ntap > 0) issue(0);
  if (ntap > 1) issue(1);

  // ---- halo: fp32 NDHWC -> bf16 LDS (zero outside the gathered volume); with a bf16 shadow of
  // x (ep.x16) 16-byte granules are copied as they are.  Batches of HB items per thread: every load
  // of a batch is issued (unconditionally, from a clamped address; outside items selected to zero)
  // before the first LDS store — round 3 stored each item right after its own load under a branch,
  // one round trip per item (12 per thread for the 32 -> 64 layer's 9^3 x 4-granule halo).
  {
    constexpr int HB = 8;
    const int nvox = a.ez * a.ey * a.ex;
    // v -> (hz, hy, hx) by multiply-high with block-uniform magic numbers (exact: v * ex < 2^32):
    // the runtime divisions were most of the kernel's VALU (SQ counters, profiles/r04_pmc_sq_step.json)
    const unsigned mex = 0xffffffffu / (unsigned)a.ex + 1u, mey = 0xffffffffu / (unsigned)a.ey + 1u;
    auto coords = [&](int v, int* o) -> bool {
      const unsigned q = __umulhi((unsigned)v, mex), hz = __umulhi(q, mey);
      const int hx = v - (int)q * a.ex, hy = (int)q - (int)hz * a.ey;
      const int iz = oz + (int)hz, iy = oy + hy, ix = ox + hx;
      *o = ((nb * a.di + iz) * a.hi + iy) * a.wi + ix;  // 32-bit: halo_setup bounds the volume
      return iz >= 0 && iz < a.di && iy >= 0 && iy < a.hi && ix >= 0 && ix < a.wi;
    };
    if (ep.x16) {
      constexpr int C8 = CIN / 8;
      const int total = nvox * C8;
      for (int i0 = 0; i0 < total; i0 += 256 * HB) {
        bf16x8_h val[HB];
#pragma unroll
        for (int u = 0; u < HB; ++u) {
          const int i = i0 + u * 256 + tid, ic = min(i, total - 1);
          const int v = ic / C8, c8 = ic - v * C8;
          int o;
          const bool ok = coords(v, &o) && i < total;
          const bf16x8_h t = *reinterpret_cast<const bf16x8_h*>(ep.x16 + (ok ? (long long)o * CIN + 8 * c8 : 0));
          val[u] = ok ? t : bf16x8_h{};
        }
#pragma unroll
        for (int u = 0; u < HB; ++u) {
          const int i = i0 + u * 256 + tid;
          if (i < total) {
            const int v = i / C8, c8 = i - v * C8;
            *reinterpret_cast<bf16x8_h*>(halo + v * ROW + 8 * c8) = val[u];
          }
        }
      }
    } else {
      constexpr int C4 = CIN / 4;
      const int total = nvox * C4;
      for (int i0 = 0; i0 < total; i0 += 256 * HB) {
        f32x4 val[HB];
#pragma unroll
        for (int u = 0; u < HB; ++u) {
          const int i = i0 + u * 256 + tid, ic = min(i, total - 1);
          const int v = ic / C4, c4 = ic - v * C4;
          int o;
          const bool ok = coords(v, &o) && i < total;
          const f32x4 t = *reinterpret_cast<const f32x4*>(x + (ok ? (long long)o * CIN + 4 * c4 : 0));
          val[u] = ok ? t : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < HB; ++u) {
          const int i = i0 + u * 256 + tid;
          if (i < total) {
            const int v = i / C4, c4 = i - v * C4;
            __bf16* d = halo + v * ROW + 4 * c4;
            d[0] = (__bf16)val[u][0]; d[1] = (__bf16)val[u][1]; d[2] = (__bf16)val[u][2]; d[3] = (__bf16)val[u][3];
          }
        }
      }
    }
  }
  // the halo stores and tap tables must be visible before the first MFMA; the weight DMAs are
  // waited for per tap below
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;
  // this lane's output voxel (A row): z = wave, y = r16 >> 2, x = r16 & 3
  const int lane_vox = ((wave * se) * a.ey + ((r16 >> 2) * se)) * a.ex + (r16 & 3) * se;

  for (int j = 0; j < ntap; ++j) {
    if (j + 2 < ntap) issue(j + 2);
    // wait for tap j's DMA: leave the (up to) two younger taps in flight
    if (j + 2 < ntap) {
      if constexpr (DMA_PER_TAP == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (j + 1 < ntap) {
      if constexpr (DMA_PER_TAP == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const __bf16* ws = wring + (j % 3) * SLOT;
    const int voff = (tq[0][j] * a.ey + tq[1][j]) * a.ex + tq[2][j];
    const __bf16* arow = halo + (lane_vox + voff) * ROW;
#pragma unroll
    for (int ks = 0; ks < CIN / 32; ++ks) {
      const bf16x8_h av = *reinterpret_cast<const bf16x8_h*>(arow + ks * 32 + 8 * g);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = t * 16 + r16;  // channel within the block
        const int gr = (ks * 4 + g) ^ (col & (NG - 1));
        const bf16x8_h bv = *reinterpret_cast<const bf16x8_h*>(ws + col * CIN + gr * 8);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[t], 0, 0, 0);
      }
    }
    // every wave has read slot j % 3 before tap j + 3 may overwrite it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  halo_epilogue<NT>(a, acc, row_out, co0, y, ep, reinterpret_cast<float*>(smem));
}

// ---- ResNet-block convs (k3 s1 p1, 64 -> 64) and their input-grads: one 4x4x4 output tile x
// all 64 output channels per block, the 27 taps split over the 4 waves (K split), so each tap's
// work is 4 M tiles x 4 N tiles x 2 K steps = 32 MFMAs per wave between no barriers at all:
//  * the input halo (6 x 6 x 6 voxels, x padded to 8) is staged once, bf16, 192-byte voxel rows
//    with 16-byte granules XOR-swizzled by (2 * row) & 7 — conflict-free A reads for every tap and
//    M tile (ds_read_b128 lane groups, MI355X_MICROARCH.md LDS table; found by exhaustive search);
//  * B fragments come straight from the packed weights in L2 (format 2), the next tap's eight in
//    flight during the current tap's MFMAs;
//  * the four waves' partial tiles are combined once through LDS (wave w keeps M tile w) and the
//    shared halo epilogue writes the tile.
constexpr int K3_HX = 8, K3_HY = 6, K3_HZ = 6, K3_VROW = 96;  // halo dims (x padded), elements per voxel row

template <bool TR, int NT>  // NT: 16-channel output tiles per block (blockIdx.y picks the channel block)
__global__ __launch_bounds__(256, 2) void conv_k3_kernel(HaloArgs a, const float* __restrict__ x,
                                                         const __bf16* __restrict__ wpk, float* y, Epi ep) {
  constexpr int CIN = 64, COUT = 64, KS = 2;
  const int co0 = blockIdx.y * 16 * NT;
  constexpr int HALO_BYTES = K3_HZ * K3_HY * K3_HX * K3_VROW * 2;  // 55296
  static_assert(HALO_BYTES >= 3 * 4 * NT * 256 * 4, "reduction buffer aliases the halo");
  __shared__ __attribute__((aligned(16))) unsigned char smem[HALO_BYTES];
  __shared__ int row_out[64];
  __bf16* halo = reinterpret_cast<__bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tiles = a.td * a.th * a.tw;
  int bid = blockIdx.x;
  const int nb = bid / tiles;
  bid -= nb * tiles;
  const int tz = bid / (a.th * a.tw), ty = (bid / a.tw) % a.th, tx = bid % a.tw;
  const int oz = tz * HT - 1, oy = ty * HT - 1, ox = tx * HT - 1;  // halo origin (pad 1 either way)
  if (tid < 64) {
    const int jz = tz * HT + (tid >> 4), jy = ty * HT + ((tid >> 2) & 3), jx = tx * HT + (tid & 3);
    row_out[tid] = (jz < a.do_ && jy < a.ho && jx < a.wo) ? ((nb * a.do_ + jz) * a.ho + jy) * a.wo + jx : -1;
  }
  // B fragments of one tap: N tile nt, K step ks -> lane (channel nt*16 + r16, granule ks*4 + g);
  // taps t, t+4 and t+8 in registers: two taps' loads in flight during a tap's MFMAs
  bf16x8_h bq[3][NT][KS];
  auto loadb = [&](int t, bf16x8_h (&b)[NT][KS]) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int col = co0 + nt * 16 + r16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        b[nt][ks] = *reinterpret_cast<const bf16x8_h*>(wpk + ((long long)t * COUT + col) * CIN +
                                                      8 * ((ks * 4 + g) ^ (col & 7)));
    }
  };
  loadb(wave, bq[0]);
  loadb(wave + 4, bq[1]);
  // ---- halo: fp32 NDHWC -> bf16 LDS, voxel (hz, hy, hx) row (hz*6 + hy)*8 + hx, granule swizzle;
  // every load of the thread issued before the first conversion
  constexpr int ST = K3_HZ * K3_HY * 6 * 16, ST_PER = (ST + 255) / 256;
  if (ep.x16) {  // bf16 shadow of the input: 16-byte granules copied as they are
    constexpr int SB = K3_HZ * K3_HY * 6 * 8, SB_PER = (SB + 255) / 256;
    bf16x8_h sb[SB_PER];
#pragma unroll
    for (int k = 0; k < SB_PER; ++k) {
      const int i = tid + 256 * k;
      const int g8 = i & 7, v = i >> 3;
      const int hx = v % 6, hy = (v / 6) % 6, hz = v / 36;
      const int iz = oz + hz, iy = oy + hy, ix = ox + hx;
      const bool ok = i < SB && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi &&
                      (unsigned)ix < (unsigned)a.wi;
      sb[k] = *reinterpret_cast<const bf16x8_h*>(
          ep.x16 + (ok ? (((long long)(nb * a.di + iz) * a.hi + iy) * a.wi + ix) * CIN + 8 * g8 : 0));
      if (!ok) sb[k] = bf16x8_h{};
    }
#pragma unroll
    for (int k = 0; k < SB_PER; ++k) {
      const int i = tid + 256 * k;
      if (i >= SB) break;
      const int g8 = i & 7, v = i >> 3;
      const int hx = v % 6, hy = (v / 6) % 6, hz = v / 36;
      const int row = hz * K3_HY + hy, vv = row * K3_HX + hx;
      *reinterpret_cast<bf16x8_h*>(halo + vv * K3_VROW + (g8 ^ ((row * 2) & 7)) * 8) = sb[k];
    }
  } else {
    f32x4 sv[ST_PER];
#pragma unroll
    for (int k = 0; k < ST_PER; ++k) {
      const int i = tid + 256 * k;
      const int c4 = i & 15, v = i >> 4;
      const int hx = v % 6, hy = (v / 6) % 6, hz = v / 36;
      const int iz = oz + hz, iy = oy + hy, ix = ox + hx;
      const bool ok = i < ST && (unsigned)iz < (unsigned)a.di && (unsigned)iy < (unsigned)a.hi &&
                      (unsigned)ix < (unsigned)a.wi;
      sv[k] = *reinterpret_cast<const f32x4*>(
          x + (ok ? (((long long)(nb * a.di + iz) * a.hi + iy) * a.wi + ix) * CIN + 4 * c4 : 0));
      if (!ok) sv[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < ST_PER; ++k) {
      const int i = tid + 256 * k;
      if (i >= ST) break;
      const int c4 = i & 15, v = i >> 4;
      const int hx = v % 6, hy = (v / 6) % 6, hz = v / 36;
      const int row = hz * K3_HY + hy, vv = row * K3_HX + hx;
      const int pg = (c4 >> 1) ^ ((row * 2) & 7);
      bf16x4_h u;
      u[0] = (__bf16)sv[k][0]; u[1] = (__bf16)sv[k][1]; u[2] = (__bf16)sv[k][2]; u[3] = (__bf16)sv[k][3];
      *reinterpret_cast<bf16x4_h*>(halo + vv * K3_VROW + pg * 8 + 4 * (c4 & 1)) = u;
    }
  }
  __syncthreads();

  f32x4 acc[4][NT];  // [M tile = tile z slice][N tile]
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ly = r16 >> 2, lx = r16 & 3;  // this lane's A row (y, x) inside an M tile
#pragma unroll
  for (int j = 0; j < 7; ++j) {  // taps t = wave + 4j (< 27); ring slot j % 3
    const int t = wave + 4 * j;
    if (t >= 27) break;  // wave-uniform
    if (t + 8 < 27) loadb(t + 8, bq[(j + 2) % 3]);
    const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
    const int dz = TR ? 2 - td : td, dy = TR ? 2 - th : th, dx = TR ? 2 - tw : tw;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = (m + dz) * K3_HY + ly + dy;
      const __bf16* arow = halo + (row * K3_HX + lx + dx) * K3_VROW;
      const int sw = (row * 2) & 7;
      bf16x8_h av[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) av[ks] = *reinterpret_cast<const bf16x8_h*>(arow + 8 * ((ks * 4 + g) ^ sw));
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], bq[j % 3][nt][ks], acc[m][nt], 0, 0, 0);
    }
  }
  // ---- combine the waves' K partials: wave w keeps M tile w, ships the other three
  __syncthreads();  // halo reads done: the buffer becomes the reduction area [m][slot][nt][256]
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    if (m == wave) continue;  // wave-uniform
    const int slot = wave < m ? wave : wave - 1;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      *reinterpret_cast<f32x4*>(red + (((m * 3 + slot) * NT + nt) * 256) + lane * 4) = acc[m][nt];
  }
  __syncthreads();
  f32x4 mine[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    mine[nt] = acc[0][nt];
#pragma unroll
    for (int m = 1; m < 4; ++m)
      if (m == wave) mine[nt] = acc[m][nt];
#pragma unroll
    for (int slot = 0; slot < 3; ++slot)
      mine[nt] += *reinterpret_cast<const f32x4*>(red + (((wave * 3 + slot) * NT + nt) * 256) + lane * 4);
  }
  __syncthreads();  // reduction area free for the epilogue's scratch
  halo_epilogue<NT>(a, mine, row_out, co0, y, ep, red);
}

// bf16 [tap][b][a] with 16-byte granules of a XOR-swizzled by (b mod granules-per-row)
__global__ __launch_bounds__(256) void pack_halo_kernel(const float* __restrict__ w, __bf16* __restrict__ wp, int T,
                                                        int cin, int cout, long long sa, long long sb) {
  const long long total = (long long)T * cout * cin;
  const int ng = cin / 8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int ai = (int)(i % cin);
    const long long r = i / cin;
    const int b = (int)(r % cout), t = (int)(r / cout);
    const int gsw = (ai / 8) ^ (b & (ng - 1));
    wp[r * cin + gsw * 8 + (ai & 7)] = (__bf16)w[ai * sa + b * sb + t];
  }
}

constexpr int g_halo_min_blocks = 512;

static bool halo_setup(const cgan3d_conv_geom* g, HaloArgs* a) {
  if (g->prec != CGAN3D_PREC_BF16 || g->reflect) return false;
  if (!(g->cin == 32 || g->cin == 64) || g->cout % 16 || g->k > 4 || g->stride < 1 || g->stride > 2) return false;
  if ((long long)g->n * g->di * g->hi * g->wi >= (1LL << 31)) return false;  // 32-bit voxel index (halo staging)
  a->n = g->n; a->di = g->di; a->hi = g->hi; a->wi = g->wi; a->do_ = g->do_; a->ho = g->ho; a->wo = g->wo;
  a->cin = g->cin; a->cout = g->cout; a->k = g->k; a->s = g->stride; a->p = g->pad; a->transposed = g->transposed;
  if (g->transposed && g->stride > 1) {
    if (g->do_ % g->stride || g->ho % g->stride || g->wo % g->stride) return false;
    a->cd = g->do_ / g->stride; a->ch = g->ho / g->stride; a->cw = g->wo / g->stride;
    a->nclass = g->stride * g->stride * g->stride;
  } else {
    a->cd = g->do_; a->ch = g->ho; a->cw = g->wo; a->nclass = 1;
  }
  a->td = (a->cd + HT - 1) / HT; a->th = (a->ch + HT - 1) / HT; a->tw = (a->cw + HT - 1) / HT;
  // largest halo over the classes (all classes share the allocation)
  int ez = 0, ey = 0, ex = 0;
  for (int r = 0; r < (g->transposed ? g->stride : 1); ++r) {
    ClassTaps c = class_info(r, g->k, g->stride, g->pad, g->transposed);
    const int e = halo_extent(c, g->stride, g->transposed);
    ez = std::max(ez, e);
  }
  ey = ex = ez;
  a->ez = ez; a->ey = ey; a->ex = ex;
  a->bn = g->cout % 64 == 0 ? 64 : (g->cout % 32 == 0 ? 32 : 16);
  // small grids: split the output channels over more blocks (more waves in flight per CU)
  const long long tiles = (long long)a->nclass * a->n * a->td * a->th * a->tw;
  while (a->bn > 32 && tiles * (g->cout / a->bn) < g_halo_min_blocks) a->bn /= 2;
  const int slot = a->bn * g->cin * 2;
  if (slot != 2048 && slot != 4096 && slot != 8192) return false;
  a->halo_bytes = ez * ey * ex * (g->cin + 8) * 2;
  if (3 * slot + a->halo_bytes > 96 * 1024) return false;
  if (g->k * g->k * g->k > 64) return false;
  return true;
}

// k3 s1 p1 64 -> 64, forward or input-grad (the input-grad of a stride-1 conv is a stride-1 conv)
static bool k3_tile_ok(const cgan3d_conv_geom* g) {
  return g->cin == 64 && g->cout == 64 && g->k == 3 && g->stride == 1 && g->pad == 1 && !g->reflect;
}

bool halo_format_ok(const cgan3d_conv_geom* g) {
  HaloArgs a;
  return s2_kind(g) || halo_setup(g, &a);
}

bool halo_ok(const cgan3d_conv_geom* g) { return g->w_packed == 2 && halo_format_ok(g); }

// the geometry's launch goes to conv_k3m_kernel when its epilogue allows (k3m_ok)
bool k3m_route(const cgan3d_conv_geom* g) {
  HaloArgs a;
  return g->w_packed == 2 && !s2_kind(g) && halo_setup(g, &a) && k3_tile_ok(g) && k3m_geom_ok(g);
}

long long halo_mblocks(const cgan3d_conv_geom* g) {
  if (s2_kind(g)) return s2_blocks(g);
  HaloArgs a;
  if (!halo_setup(g, &a)) return 0;
  return (long long)a.nclass * a.n * a.td * a.th * a.tw;
}

int halo_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st) {
  if (s2_kind(g)) return s2_launch(g, x, reinterpret_cast<const __bf16*>(w), y, e, st);  // conv_s2.hip
  HaloArgs a;
  if (!halo_setup(g, &a)) {
    set_error("conv_halo: geometry not supported");
    return CGAN3D_EINVAL;
  }
  if (k3_tile_ok(g) && k3m_ok(g, e))  // ResNet-block shape with a bf16 input: operands in LDS (conv_k3m.hip)
    return k3m_launch(g, reinterpret_cast<const __bf16*>(w), y, e, st);
  if (t64_ok(g, e))  // 64 -> 32 stride-2 transposed, all parity classes per block (conv_t64.hip)
    return t64_launch(g, reinterpret_cast<const __bf16*>(w), y, e, st);
  if (f64_ok(g, e))  // 32 -> 64 stride-2, operands resident in LDS (conv_f64.hip)
    return f64_launch(g, reinterpret_cast<const __bf16*>(w), y, e, st);
  if (k3_tile_ok(g)) {  // ResNet-block shape: whole-tile K-split kernel
    const long long tiles = (long long)a.n * a.td * a.th * a.tw;
    // small grids: the 64 output channels split over 2 blocks per tile
    const int split = tiles < g_halo_min_blocks ? 2 : 1;
    const dim3 grid1((unsigned)tiles, split);
    const __bf16* wp = reinterpret_cast<const __bf16*>(w);
#define CG_K3(N) (g->transposed ? ::cg::launch((conv_k3_kernel<true, N>), grid1, dim3(256), 0, st, a, x, wp, y, e) \
                                : ::cg::launch((conv_k3_kernel<false, N>), grid1, dim3(256), 0, st, a, x, wp, y, e))
    if (split == 4) CG_K3(1);
    else if (split == 2) CG_K3(2);
    else CG_K3(4);
#undef CG_K3
    return CGAN3D_OK;
  }
  dim3 grid((unsigned)(a.nclass * a.n * a.td * a.th * a.tw), g->cout / a.bn);
  const size_t lds = 3 * (size_t)a.bn * g->cin * 2 + a.halo_bytes;
  const __bf16* wp = reinterpret_cast<const __bf16*>(w);
#define CG_HL(CI, NT) ::cg::launch((conv_halo_kernel<CI, NT>), grid, dim3(256), lds, st, a, x, wp, y, e)
  if (g->cin == 64) {
    if (a.bn == 64) CG_HL(64, 4); else if (a.bn == 32) CG_HL(64, 2); else return CGAN3D_EINVAL;
  } else {
    if (a.bn == 64) CG_HL(32, 4); else if (a.bn == 32) CG_HL(32, 2); else return CGAN3D_EINVAL;
  }
#undef CG_HL
  return CGAN3D_OK;
}

int halo_pack(const cgan3d_conv_geom* g, const float* w, void* wp, hipStream_t st) {
  const int T = g->k * g->k * g->k;
  const long long total = (long long)T * g->cout * g->cin;
  int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
  ::cg::launch(pack_halo_kernel, dim3(blocks), dim3(256), 0, st, w, reinterpret_cast<__bf16*>(wp), T, g->cin,
                     g->cout, (long long)g->w_sa, (long long)g->w_sb);
  return CGAN3D_OK;
}

}  // namespace cg
