// Streamed-plane 1 -> 16 k7 convolution on bf16 MFMA (round 6): the generator's first conv forward
// (model/generator.py:31-38, 1 -> 16, reflect pad 3) and its last conv's input-grad onto the padded grid
// (generator.py:78-85: the transposed map of 16 -> 1, flipped taps, zero pad 6), replacing k7m_n2w's
// per-tile unfold for the bf16 step's statistics modes.
//
// The contraction is split by input plane:  out[d][h][w][c] = sum_td P[d + td][h][w][c][td]  with
//   P[q][h][w][c][td] = sum_{th, tw} x[q][h + th][w + tw] * W[c][td][th][tw]
// a 16 x 16 MFMA tile per (input plane q, output row h, td): M = the 16 channels (A = weights, in
// registers for the whole launch), N = 16 output columns w, K = (th 0..7, tw 0..7) in two 32-deep steps
// (th 7 and tw 7 carry zero weights).  The B fragment of (row h, K-step kk) is the single-channel plane
// itself: lane (w, g) holds x[q][h + 4 kk + g][w .. w + 7] — eight consecutive floats read straight from
// the plane staged in LDS (two copies, the second shifted by one element, so every lane's window starts
// 8-byte aligned: four ds_read_b64), converted to bf16 in registers.  Each fragment then feeds the seven
// MFMAs of td = 0..6, one per open output plane (the k7m_n2w kernel read one fragment per MFMA and built
// an 8x unfolded LDS image per tile).
//
// A block = 16 output rows x 16 columns x a chunk of TDc output planes; 4 waves, wave = 4 rows, each
// holding the 7 open output planes of its rows in registers (4 x 7 accumulator tiles): the plane loop is
// unrolled by 7 so the ring slot (d mod 7) of every MFMA is static.  The TDc + 6 input planes stream
// through a ring of 4 LDS buffers filled by LDS-DMA (global_load_lds, one dword per lane, per-lane
// sources: reflect / zero padding resolved in the source address) three planes ahead, waited for with
// exact vmcnt counts (every store and z load of a flush is issued by the whole wave: lanes past the
// volume use a sink).  Output plane d is complete after input plane d + 6: the flush at that step stores
// its 4 rows (bf16 or fp32), adds its BatchNorm statistics (mode 1: per-lane shifted sums, merged per
// block, fp64 accumulators; mode 2: the reflect-folded mode-2 pairs from z at the mirrored voxel, as
// k7m_n2w) and zeroes the slot for plane d + 7.  MFMAs of (plane, td) pairs whose output plane lies
// outside the chunk are skipped (uniform branches), so the MFMA work is exactly the convolution's.
#include "k7.h"

namespace cg {

namespace k7p {
constexpr int NT = 256;              // 4 waves
constexpr int SH = 16, WB = 16;      // output rows / columns per block (4 rows per wave)
constexpr int ROWS = SH + 6;         // staged input rows
constexpr int POS = 24;              // staged positions per copy row (bf16): windows start at 0, 4, .., 16
constexpr int ROWB = 4 * POS * 2;    // staged row bytes: 6 groups of 4 positions x 4 shifted copies (192:
                                     // rows 16 dwords apart mod 32, for the weight grad's two-row lane groups)
constexpr int PLANEB = (ROWS + 1) * ROWB;  // bytes per ring buffer: + one zero row (read by th = 7 only)
constexpr int NBUF = 3;              // ring: the plane computed, the plane written, one free
constexpr int TASKS = ROWS * (POS / 4);  // staging tasks per plane: (row, group of 4 positions) = 132
constexpr int RINGB = NBUF * PLANEB > 14 * 64 * 16 ? NBUF * PLANEB : 14 * 64 * 16;  // also the weight image
// n2w, wave-private staging (round 6b): a wave stages the 10 input rows its 4 output rows read through th <= 6
// (row 10, read only with the zero weights of th = 7, is never staged: it keeps finite stale values), into
// two buffers of its own — the plane loop then needs no workgroup barrier
constexpr int WROWS = 11, WTASKS = 10 * (POS / 4), WNB = 2;
constexpr int WPLANE = WROWS * ROWB, WREG = WNB * WPLANE;
constexpr int NRINGB = 4 * WREG > 14 * 64 * 16 ? 4 * WREG : 14 * 64 * 16;
}  // namespace k7p

typedef __bf16 bf16x8_p __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_p __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_p __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_p __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned k7p_pack(float a, float b) {  // two floats -> a bf16 pair (RNE)
  bf16x4_p h;
  h[0] = (__bf16)a;
  h[1] = (__bf16)b;
  return reinterpret_cast<const u32x2_p&>(h)[0];
}

// MODE 0: no statistics; 1: BatchNorm (sum, sum of squares) of the output into fp64 accumulators
// (cgan3d_bn_fuse mode 3); 2: the reflect-folded mode-2 pairs into fp64 accumulators (K7Fold, acc).
// B16: y (and mode 2's z) in bf16.
template <int MODE, bool B16>
__global__ __launch_bounds__(256, 2) void k7p_n2w_kernel(K7Args a, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* __restrict__ y, int tdc,
                                                         K7Fold fb, double* acc1, int reps1) {
  using namespace k7p;
  constexpr int C = 16;
  constexpr unsigned OOB = 0x80000000u;  // past every buffer: loads return 0, stores are dropped
  __shared__ __attribute__((aligned(16))) unsigned char ring[NRINGB];
  __shared__ __attribute__((aligned(16))) float coef[4 * C];  // mode 2: scale, shift, mean, invstd
  __shared__ float red[8 * 4 * C];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  int bid = blockIdx.x;
  const int wt_ = bid % a.tiles_w; bid /= a.tiles_w;
  const int ht_ = bid % a.tiles_h; bid /= a.tiles_h;
  const int dt_ = bid % a.tiles_d;
  const int n = bid / a.tiles_d;
  const int d0 = dt_ * tdc, h0 = ht_ * SH, w0 = wt_ * WB;
  const int tdl = min(tdc, a.do_ - d0);  // output planes of this chunk
  const int nsteps = tdl + 6;            // input planes streamed

  // staging task of this lane (lane < WTASKS): the wave's row r (block row 4 wave + r), positions 4 m ..
  // 4 m + 3 of every copy, from the eight source values x[q][h0 - P + 4 wave + r][w0 - P - 1 + 4 m + i],
  // i = 0..7 (byte offsets inside the plane, reflect / zero padding resolved here: OOB = zero)
  const bool stager = lane < WTASKS;
  const int tr = lane / (POS / 4), tm = lane - tr * (POS / 4);
  unsigned soff[8];
  {
    const int ih = k7_src(h0 - a.P + 4 * wave + tr, a.hi, a.reflect);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // window position p = 4 m + i holds x[w0 - P - 1 + p] (lane w reads positions w + 1 .. w + 8)
      const int iw = k7_src(w0 - a.P - 1 + 4 * tm + i, a.wi, a.reflect);
      soff[i] = (stager && (ih | iw) >= 0) ? 4u * (unsigned)(ih * a.wi + iw) : OOB;
    }
  }
  const int pbytes = a.hi * a.wi * 4;
  float sv[8];  // the staged values of the next plane, in flight during the current step
  auto load = [&](int sp) {
    const int id = sp < nsteps ? k7_src(d0 - a.P + sp, a.di, a.reflect) : -1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (long long)(n * a.di + max(id, 0)) * a.hi * a.wi), (short)0, id >= 0 ? pbytes : 0, 0x00020000);
    if (CG_PROBE(a.probe, 2)) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, soff[i], 0, 0));
  };
  auto store = [&](int sp) {  // the eight values -> four shifted bf16 copies (copy c: positions p = x[.. + c + p])
    if (!stager || CG_PROBE(a.probe, 2)) return;
    const unsigned d0_ = k7p_pack(sv[0], sv[1]), d1 = k7p_pack(sv[2], sv[3]), d2 = k7p_pack(sv[4], sv[5]),
                   d3 = k7p_pack(sv[6], sv[7]);
    const unsigned a01 = __builtin_amdgcn_alignbyte(d1, d0_, 2), a12 = __builtin_amdgcn_alignbyte(d2, d1, 2),
                   a23 = __builtin_amdgcn_alignbyte(d3, d2, 2);
    // row layout [group k][copy c][4 positions]: a task's four copies are 32 contiguous bytes
    unsigned char* rb = ring + wave * WREG + (sp % WNB) * WPLANE + tr * ROWB + tm * 32;
    *reinterpret_cast<u32x4_p*>(rb) = u32x4_p{d0_, d1, a01, a12};
    *reinterpret_cast<u32x4_p*>(rb + 16) = u32x4_p{d1, d2, a12, a23};
  };
  load(0);  // in flight during the weight staging

  // A fragments: lane (c = r16, g) of (td, kk) holds W[c][td][th = 4 kk + g][tw = 0..7] (zero for th, tw = 7).
  // Staged once per block through LDS (the ring's first buffers, before any plane lands there): coalesced
  // loads of the [c][343] weights, each value scattered as bf16 into its fragment slot of a zeroed image
  // [td][kk][lane][8], then one 16-byte read per fragment (per-lane scattered loads of the 98 taps took
  // the texture path ~10 us per launch)
  bf16x8_p wa[7][2];
  {
    __bf16* wi = reinterpret_cast<__bf16*>(ring);  // 14 x 64 x 8 bf16 = 14 KB
    for (int i = tid; i < 14 * 64; i += NT) reinterpret_cast<u32x4_p*>(wi)[i] = u32x4_p{0u, 0u, 0u, 0u};
    __syncthreads();
    for (int i = tid; i < C * KT7; i += NT) {
      const int c = i / KT7, t = i - c * KT7;
      const int tt = a.flip ? KT7 - 1 - t : t;  // this value is W[c][t], used at tap tt
      const int td = tt / 49, rem = tt - td * 49, th = rem / K7, tw = rem - th * K7;
      wi[((td * 2 + (th >> 2)) * 64 + (th & 3) * 16 + c) * 8 + tw] = (__bf16)w[(long long)c * a.wc + t];
    }
    __syncthreads();
#pragma unroll
    for (int td = 0; td < 7; ++td)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wa[td][kk] = reinterpret_cast<const bf16x8_p*>(wi)[(td * 2 + kk) * 64 + lane];
    __syncthreads();  // the image is dead before the first plane is staged over it
  }
  for (int i = lane; i < WREG / 16; i += 64)  // this wave's buffers zeroed once (the unstaged row stays finite)
    reinterpret_cast<u32x4_p*>(ring + wave * WREG)[i] = u32x4_p{0u, 0u, 0u, 0u};
  if (MODE == 2 && tid < C) {
    coef[tid] = fb.ss[tid]; coef[C + tid] = fb.ss[C + tid];
    coef[2 * C + tid] = fb.mi[tid]; coef[3 * C + tid] = fb.mi[C + tid];
  }
  store(0);
  load(1);
  __syncthreads();  // coef: the last workgroup barrier before the epilogue

  // this lane's fragment base (bytes): row 4 wave + g, window positions j = w + 1 .. w + 8 = copy j & 3 of
  // groups j >> 2 and (j >> 2) + 1 (a 16-lane group's 8-byte reads then cover all 32 banks of each access)
  const int jw = r16 + 1;
  const int fbase = wave * WREG + g * ROWB + (4 * (jw >> 2) + (jw & 3)) * 8;
  f32x4 acc[4][7];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // outputs: a buffer over the whole tensor (rows / columns past the volume get OOB offsets: dropped)
  const int ow = w0 + r16;
  const int oh0 = h0 + 4 * wave;
  const long long ybytes = (long long)a.n * a.do_ * a.ho * a.wo * C * (B16 ? 2 : 4);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, (int)ybytes, 0x00020000);
  // byte offset of this lane's 4 channels of row 0 at output plane d0 (OOB past the volume's columns); rows
  // add a uniform stride and a uniform row count bounds them (one register instead of four)
  const unsigned ybase = ow < a.wo
      ? (unsigned)((((long long)(n * a.do_ + d0) * a.ho + oh0) * a.wo + ow) * C + 4 * g) * (B16 ? 2u : 4u) : OOB;
  const unsigned yrow = (unsigned)(a.wo * C * (B16 ? 2 : 4));
  const int nrows = __builtin_amdgcn_readfirstlane(min(max(a.ho - oh0, 0), 4));
  const unsigned ypl = (unsigned)(a.ho * a.wo * C * (B16 ? 2 : 4));  // bytes per output plane
  // statistics (mode 1: per-lane sums shifted by the lane's first output; valid rows only)
  float sK[4] = {0.f, 0.f, 0.f, 0.f}, sS1[4] = {0.f, 0.f, 0.f, 0.f}, sS2[4] = {0.f, 0.f, 0.f, 0.f};
  float sN = 0.f;
  float fp1[4] = {0.f, 0.f, 0.f, 0.f}, fp2[4] = {0.f, 0.f, 0.f, 0.f};
  const int nval = ow < a.wo ? nrows : 0;  // valid rows of this lane (0..4; all lanes of a full tile: 4)

  for (int s0 = 0; s0 < nsteps; s0 += 7) {
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int s = s0 + u;
      if (s >= nsteps) break;
      // plane s is in this wave's LDS (its own writes, in order); no barrier.  The scheduling fence keeps
      // the compiler from hoisting the next step's reads into this one (live ranges past 256 VGPRs)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // every step issues the same vector-memory instructions (staging loads past the chunk read an empty
      // buffer, stores of a step without a flush get OOB offsets): the compiler's vmcnt wait for the
      // staged values then skips the previous flush's stores instead of waiting for everything
      store(s + 1);
      load(s + 2);
      const bool fl = s >= 6 && s - 6 < tdl;
      const int od = min(max(d0 + s - 6, 0), a.do_ - 1);
      bf16x4_p zh[4];
      f32x4 zf[4];
      auto zload = [&]() {
        const int vd = reflect_idx(od - fb.P, fb.zd), vw = reflect_idx(min(ow, a.wo - 1) - fb.P, fb.zw);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int vh = reflect_idx(min(oh0 + r, a.ho - 1) - fb.P, fb.zh);
          const int zo = (((n * fb.zd + vd) * fb.zh + vh) * fb.zw + vw) * C + 4 * g;
          if constexpr (B16) zh[r] = *reinterpret_cast<const bf16x4_p*>(reinterpret_cast<const __bf16*>(fb.z) + zo);
          else zf[r] = *reinterpret_cast<const f32x4*>(fb.z + zo);
        }
      };
      if (MODE == 2 && B16) zload();  // before the MFMAs: they cover the latency (every step: static counts)
      const unsigned char* pb = ring + (s % WNB) * WPLANE + fbase;
      const int tlo = max(0, s - (tdl - 1)), thi = min(6, s);  // td whose output plane s - td is in the chunk
      const unsigned tmask = __builtin_amdgcn_readfirstlane(((2u << thi) - 1u) & ~((1u << tlo) - 1u));
      const int slot0 = u;  // slot of td: (u - td) mod 7
      bf16x8_p fr[4][2];  // (row, kk): x[q][row + 4 kk + g][w + 1 .. w + 8 positions]
      auto fread = [&](int r) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const unsigned char* p = pb + (r + 4 * kk) * ROWB;
          const u32x2_p lo = CG_PROBE(a.probe, 4) ? u32x2_p{0x3f003f00u, 0x3f003f00u} : *reinterpret_cast<const u32x2_p*>(p),
                        hi = CG_PROBE(a.probe, 4) ? lo : *reinterpret_cast<const u32x2_p*>(p + 32);
          const u32x4_p q4 = {lo[0], lo[1], hi[0], hi[1]};
          fr[r][kk] = reinterpret_cast<const bf16x8_p&>(q4);
        }
      };
      // modes 0 / 1 read all eight fragments first (the second half's reads in flight during the first
      // half's MFMAs); mode 2 per half (its z values hold the registers)
      if (MODE != 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) fread(r);
      }
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        if (MODE == 2) {
          fread(2 * half);
          fread(2 * half + 1);
        }
#pragma unroll
        for (int td = 0; td < 7; ++td) {
          if (!((tmask >> td) & 1u) || CG_PROBE(a.probe, 1)) continue;
          const int slot = (slot0 - td + 7) % 7;
#pragma unroll
          for (int rr = 0; rr < 2; ++rr) {
            const int r = 2 * half + rr;
            // the first contribution to a slot (td = 0) starts from zero: no slot is cleared at a flush
            acc[r][slot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                wa[td][0], fr[r][0], td == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[r][slot], 0, 0, 0);
            acc[r][slot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[td][1], fr[r][1], acc[r][slot], 0, 0, 0);
          }
        }
      }
      {  // output plane od is complete after this step when fl: slot (u + 1) % 7
        const int f = (u + 1) % 7;
        const unsigned po = (unsigned)(s - 6) * ypl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const f32x4 v = acc[r][f];
          const unsigned o = (!fl || ybase == OOB || r >= nrows) ? OOB : ybase + r * yrow + po;
          if (CG_PROBE(a.probe, 8)) {
          } else if constexpr (B16) {
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_p{k7p_pack(v[0], v[1]), k7p_pack(v[2], v[3])}, ys, o, 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4_p&>(v), ys, o, 0, 0);
          }
        }
        if (fl) {
          f32x4 cs, chf, cm, ci;
          if (MODE == 2 && !B16) zload();
          if (MODE == 2) {
            cs = *reinterpret_cast<const f32x4*>(coef + 4 * g);
            chf = *reinterpret_cast<const f32x4*>(coef + C + 4 * g);
            cm = *reinterpret_cast<const f32x4*>(coef + 2 * C + 4 * g);
            ci = *reinterpret_cast<const f32x4*>(coef + 3 * C + 4 * g);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const f32x4 v = acc[r][f];
            if (MODE == 1) {
              if (s == 6 && r == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) sK[j] = v[j];
              }
              if (r < nval) {  // rows past the volume are the last ones of a lane
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  const float dv = v[j] - sK[j];
                  sS1[j] += dv;
                  sS2[j] = fmaf(dv, dv, sS2[j]);
                }
              }
            }
            if (MODE == 2 && r < nval) {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const float z = B16 ? (float)zh[r][j] : zf[r][j];
                const float gg = v[j] * act_grad(z * cs[j] + chf[j], fb.act, fb.slope);
                fp1[j] += gg;
                fp2[j] += gg * (z - cm[j]) * ci[j];
              }
            }
          }
        }
      }
    }
  }
  if (MODE == 1) sN = (float)(nval * tdl);
  __syncthreads();
  if (MODE == 1) {  // lane (n, mean, M2) -> Chan merge over the 16 voxel lanes, the 4 waves, then fp64 adds
    float mm[4], m2[4];
    float nn = sN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mm[j] = nn > 0.f ? sK[j] + sS1[j] / nn : 0.f;
      m2[j] = nn > 0.f ? fmaxf(sS2[j] - sS1[j] * sS1[j] / nn, 0.f) : 0.f;
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const float no = __shfl_xor(nn, off, 64), nt = nn + no;
      const float wo = nt > 0.f ? no / nt : 0.f, wx = nt > 0.f ? nn * no / nt : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float mo = __shfl_xor(mm[j], off, 64), qo = __shfl_xor(m2[j], off, 64);
        const float dl = mo - mm[j];
        mm[j] += dl * wo;
        m2[j] += qo + dl * dl * wx;
      }
      nn = nt;
    }
    if (r16 == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[(0 * 4 + wave) * C + 4 * g + j] = nn;
        red[(1 * 4 + wave) * C + 4 * g + j] = mm[j];
        red[(2 * 4 + wave) * C + 4 * g + j] = m2[j];
      }
    }
    __syncthreads();
    if (tid < C && acc1) {
      float run_n = 0.f, run_mean = 0.f, run_m2 = 0.f;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) {
        const float no = red[(0 * 4 + wv) * C + tid], mo = red[(1 * 4 + wv) * C + tid], qo = red[(2 * 4 + wv) * C + tid];
        const float nt = run_n + no;
        if (no > 0.f) {
          const float dl = mo - run_mean;
          run_mean += dl * (no / nt);
          run_m2 += qo + dl * dl * (run_n * no / nt);
          run_n = nt;
        }
      }
      if (run_n > 0.f) {
        double* rp = acc1 + (long long)(blockIdx.x % reps1) * 2 * C;
        const double S = (double)run_mean * run_n;
        unsafeAtomicAdd(rp + tid, S);
        unsafeAtomicAdd(rp + C + tid, (double)run_m2 + S * (double)run_mean);
      }
    }
  }
  if (MODE == 2) {  // folded mode-2 pairs: voxel lanes -> row sums, waves -> LDS, fp64 adds
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        fp1[j] += __shfl_xor(fp1[j], m, 64);
        fp2[j] += __shfl_xor(fp2[j], m, 64);
      }
    }
    if (r16 == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[wave * C + 4 * g + j] = fp1[j];
        red[4 * C + wave * C + 4 * g + j] = fp2[j];
      }
    }
    __syncthreads();
    if (tid < 2 * C) {
      const int c = tid & 15, k = tid >> 4;
      const float q = red[k * 4 * C + c] + red[k * 4 * C + C + c] + red[k * 4 * C + 2 * C + c] + red[k * 4 * C + 3 * C + c];
      double* fr = fb.acc + (long long)(blockIdx.x % fb.reps) * 2 * C;
      unsafeAtomicAdd(fr + k * C + c, (double)q);
    }
  }
}

// ---- streamed-plane weight gradient of the 1 <-> 16 k7 convs (round 6): both roles are
//   dW[c][tap(t)] = sum_{v in grid} A16(v)[c] * X1(v + t - P)
// first conv (MODE 0): grid = the output grid, A16 = dL/dz (bf16 shadow), X1 = x reflect-padded by 3;
// last conv (MODE 1): grid = the reflect-padded input grid, A16(v) = y16[reflect(v - 3)] (the conv's
// input shadow), X1 = the output gradient g zero-padded by 6, tap = 342 - t (k7m_wg_kernel's split).
// MFMA D[c][n] (16 x 16 x 32): K = 32 grid voxels (2 rows x 16 w), A = A16 (channel-major fragments by
// ds_read_b64_tr_b16 from NDHWC bf16 rows), N = (th parity j, tw) of a th pair tt, B = eight
// consecutive X1 values of row h + 2 tt + j at w + tw: the X1 plane staged as in k7p_n2w (four shifted
// bf16 copies, two ds_read_b64 per fragment).  The block streams the X1 planes of its chunk; each
// X1 plane s pairs with the A16 planes s - td (td = 0..6), whose fragments stay in registers for the
// seven steps they are used (the plane loop unrolled by 7, as k7p_n2w's output planes): per step and
// K-step a wave reads one new A16 fragment and four X1 fragments for 28 MFMAs into its 28
// accumulator tiles (td, tt).  The waves' tiles are summed in LDS in wave order (deterministic) and each
// block writes one partial [c][343] row; colsum_kernel adds the rows into dW.
namespace k7g {
constexpr int AROW = 16 * 32;              // A16 staged row: 16 voxels x 32 bytes (quads 2 / 3 swapped per row)
constexpr int APL = 16 * AROW;             // A16 plane (16 rows): 8 KB
constexpr int NA = 2;                      // A16 staging buffers
}  // namespace k7g

template <int MODE>
__global__ __launch_bounds__(256, 2) void k7p_wg_kernel(K7Args a, const float* __restrict__ x1,
                                                        const __bf16* __restrict__ a16, int ad, int ah, int aw,
                                                        float* __restrict__ part, int tdc) {
  using namespace k7p;
  using namespace k7g;
  constexpr int C = 16;
  constexpr unsigned OOB = 0x80000000u;
  // wave-private staging (as k7p_n2w): per wave two X1 planes of its 10 rows (+ one never-staged row) and
  // two A16 planes of its 4 rows; the block's bytes are then reused by the epilogue's reduction (28 KB)
  constexpr int WAPL = 4 * AROW;                       // A16 rows of a wave: 2 KB
  constexpr int WSZ = WNB * WPLANE + WNB * WAPL;       // per wave: 8.2 KB
  __shared__ __attribute__((aligned(16))) unsigned char lds[4 * WSZ > 28 * 1024 ? 4 * WSZ : 28 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  // grid (the A16 side) tile: a.do_ / a.ho / a.wo are the grid dims; a.di / a.hi / a.wi and a.P / a.reflect
  // the X1 source's
  int bid = blockIdx.x;
  const int wt_ = bid % a.tiles_w; bid /= a.tiles_w;
  const int ht_ = bid % a.tiles_h; bid /= a.tiles_h;
  const int dt_ = bid % a.tiles_d;
  const int n = bid / a.tiles_d;
  const int d0 = dt_ * tdc, h0 = ht_ * SH, w0 = wt_ * WB;
  const int tdl = min(tdc, a.do_ - d0);
  const int nsteps = tdl + 6;

  unsigned char* xr = lds + wave * WSZ;                 // this wave's X1 buffers
  unsigned char* ar = xr + WNB * WPLANE;               // and A16 buffers
  // X1 staging (as k7p_n2w: the wave's rows 4 wave + 0..9)
  const bool stager = lane < WTASKS;
  const int tr = lane / (POS / 4), tm = lane - tr * (POS / 4);
  unsigned soff[8];
  {
    const int ih = k7_src(h0 - a.P + 4 * wave + tr, a.hi, a.reflect);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int iw = k7_src(w0 - a.P - 1 + 4 * tm + i, a.wi, a.reflect);
      soff[i] = (stager && (ih | iw) >= 0) ? 4u * (unsigned)(ih * a.wi + iw) : OOB;
    }
  }
  const int pbytes = a.hi * a.wi * 4;
  float sv[8];
  auto xload = [&](int sp) {
    const int id = sp < nsteps ? k7_src(d0 - a.P + sp, a.di, a.reflect) : -1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x1 + (long long)(n * a.di + max(id, 0)) * a.hi * a.wi), (short)0, id >= 0 ? pbytes : 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, soff[i], 0, 0));
  };
  auto xstore = [&](int sp) {
    if (!stager) return;
    const unsigned e0 = k7p_pack(sv[0], sv[1]), e1 = k7p_pack(sv[2], sv[3]), e2 = k7p_pack(sv[4], sv[5]),
                   e3 = k7p_pack(sv[6], sv[7]);
    const unsigned a01 = __builtin_amdgcn_alignbyte(e1, e0, 2), a12 = __builtin_amdgcn_alignbyte(e2, e1, 2),
                   a23 = __builtin_amdgcn_alignbyte(e3, e2, 2);
    unsigned char* rb = xr + (sp % WNB) * WPLANE + tr * ROWB + tm * 32;
    *reinterpret_cast<u32x4_p*>(rb) = u32x4_p{e0, e1, a01, a12};
    *reinterpret_cast<u32x4_p*>(rb + 16) = u32x4_p{e1, e2, a12, a23};
  };
  // A16 staging: lane = voxel (the wave's row lane >> 4, w lane & 15) of the plane, 32 bytes, slot
  // w ^ 4 (w >> 3) (the two 8-voxel halves of a row land 32 banks apart for the transposed reads)
  const int av = lane & 15, arow = 4 * wave + (lane >> 4);
  unsigned aoff;  // byte offset of this voxel's source row position inside its source plane, OOB past the grid
  {
    const int gh = h0 + arow, gw = w0 + av;
    const bool ok = gh < a.ho && gw < a.wo;
    int sh = gh, sw = gw;
    if (MODE == 1) { sh = reflect_idx(gh - 3, ah); sw = reflect_idx(gw - 3, aw); }
    aoff = ok ? (unsigned)((sh * aw + sw) * C * 2) : OOB;
  }
  const int apb = ah * aw * C * 2;
  u32x4_p av0, av1;
  auto aload = [&](int sp) {  // grid plane d0 + sp (sp < tdl)
    const int gd = d0 + sp;
    const int sd = MODE == 1 ? reflect_idx(gd - 3, ad) : gd;
    const bool ok = sp < tdl;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a16 + ((long long)n * ad + (ok ? sd : 0)) * ah * aw * C), (short)0, ok ? apb : 0, 0x00020000);
    av0 = __builtin_amdgcn_raw_buffer_load_b128(rs, aoff, 0, 0);
    av1 = __builtin_amdgcn_raw_buffer_load_b128(rs, aoff == OOB ? OOB : aoff + 16, 0, 0);
  };
  auto astore = [&](int sp) {
    unsigned char* b = ar + (sp % WNB) * WAPL + (lane >> 4) * AROW + ((av ^ ((av >> 3) << 2)) * 32);
    *reinterpret_cast<u32x4_p*>(b) = av0;
    *reinterpret_cast<u32x4_p*>(b + 16) = av1;
  };
  for (int i = lane; i < WNB * WPLANE / 16; i += 64)  // the wave's X1 buffers zeroed (the unstaged row stays finite)
    reinterpret_cast<u32x4_p*>(xr)[i] = u32x4_p{0u, 0u, 0u, 0u};
  xload(0);
  aload(0);
  xstore(0);
  astore(0);
  xload(1);
  aload(1);

  // A fragment read (K-step kq of wave's rows, from A16 staging buffer): lane (q, p) = (r16 >> 2, r16 & 3)
  // supplies voxel (row 4 wave + 2 kq + (g >> 1), w = 8 (g & 1) + q [+ 4]) channels 4 p .. 4 p + 3
  const int aq = r16 >> 2, ap = r16 & 3;
  auto aslot = [&](int w_) { return (w_ ^ ((w_ >> 3) << 2)) * 32; };
  const int abase0 = (g >> 1) * AROW + aslot(8 * (g & 1) + aq) + ap * 8;
  const int abase1 = (g >> 1) * AROW + aslot(8 * (g & 1) + aq + 4) + ap * 8;
  typedef short s16x4_p __attribute__((ext_vector_type(4)));
  auto afrag = [&](int buf, int kq) -> bf16x8_p {
    const unsigned char* base = ar + buf * WAPL + 2 * kq * AROW;
    const s16x4_p lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_p*)(base + abase0));
    const s16x4_p hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_p*)(base + abase1));
    typedef short s16x8_p __attribute__((ext_vector_type(8)));
    const s16x8_p v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return reinterpret_cast<const bf16x8_p&>(v);
  };
  // B fragment (K-step kq, th pair tt): lane (n = (j, tw), g): X1 row 4 wave + 2 kq + (g >> 1) + 2 tt + j,
  // positions 8 (g & 1) + tw + 1 .. + 8
  const int bj = r16 >> 3, btw = r16 & 7;
  const int bp0 = 8 * (g & 1) + btw + 1;
  const int bbase = ((g >> 1) + bj) * ROWB + (4 * (bp0 >> 2) + (bp0 & 3)) * 8;

  f32x4 acc[7][4];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8_p aw_[7][2];  // A fragments of the A16 planes still in use: slot d mod 7, K-step

  for (int s0 = 0; s0 < nsteps; s0 += 7) {
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int s = s0 + u;
      if (s >= nsteps) break;
      // X1 plane s and A16 plane s are in this wave's LDS (its own writes, in order): no barrier
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      xstore(s + 1);
      astore(s + 1);
      xload(s + 2);
      aload(s + 2);
      if (s < tdl) {  // A16 plane s: its fragments into register slot u
        aw_[u][0] = afrag(s % WNB, 0);
        aw_[u][1] = afrag(s % WNB, 1);
      }
      const unsigned char* xb = xr + (s % WNB) * WPLANE + bbase;
      const int tlo = max(0, s - (tdl - 1)), thi = min(6, s);  // A16 plane s - td in the chunk
      const unsigned tmask = __builtin_amdgcn_readfirstlane(((2u << thi) - 1u) & ~((1u << tlo) - 1u));
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {
        bf16x8_p bf[4];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const unsigned char* p = xb + (2 * kq + 2 * tt) * ROWB;
          const u32x2_p lo = *reinterpret_cast<const u32x2_p*>(p), hi = *reinterpret_cast<const u32x2_p*>(p + 32);
          const u32x4_p q4 = {lo[0], lo[1], hi[0], hi[1]};
          bf[tt] = reinterpret_cast<const bf16x8_p&>(q4);
        }
#pragma unroll
        for (int td = 0; td < 7; ++td) {
          if (!((tmask >> td) & 1u)) continue;
          const int slot = (u - td + 7) % 7;
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            acc[td][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw_[slot][kq], bf[tt], acc[td][tt], 0, 0, 0);
        }
      }
    }
  }
  // the four waves' tiles summed in LDS in wave order, then this block's partial row [c][t]
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // 7 x 4 x 256 floats = 28 KB
  float* red2 = red + 16 * 256;
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int td = 0; td < 7; ++td)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int ti = td * 4 + tt;
          float* q = (ti < 16 ? red + ti * 256 : red2 + (ti - 16) * 256) + lane * 4;
          f32x4 v = acc[td][tt];
          if (wv > 0) v += *reinterpret_cast<const f32x4*>(q);
          *reinterpret_cast<f32x4*>(q) = v;
        }
    }
    __syncthreads();
  }
  // tile (td, tt): lane l holds D[c = 4 (l >> 4) + jj][n = l & 15], n = (j, tw): tap (td, 2 tt + j, tw)
  float* pb = part + (long long)blockIdx.x * (C * KT7);
  for (int i = tid; i < 28 * 256; i += NT) {
    const int ti = i >> 8, e = i & 255, l = e >> 2, jj = e & 3;
    const int td = ti >> 2, tt = ti & 3, c = 4 * (l >> 4) + jj, nn = l & 15, j = nn >> 3, tw = nn & 7;
    const int th = 2 * tt + j;
    if (th < K7 && tw < K7) {
      const int t = (td * K7 + th) * K7 + tw;
      const float v = ti < 16 ? red[i] : red2[i - 16 * 256];
      pb[c * KT7 + (MODE ? KT7 - 1 - t : t)] = v;
    }
  }
}

static int g_k7p = 0;  // cgan3d_set_tuning key 21: output planes per k7p block (0 auto, -1: k7m_n2w)
void k7p_set(int v) { g_k7p = v; }

// 1 if the streamed-plane kernel took the launch (else the caller runs k7m_n2w)
int k7p_n2w_try(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, const float* x, const float* w,
                float* y, const K7Fold* fold, const BnFuse* fz, bool out16, hipStream_t s) {
  if (g_k7p < 0) return 0;
  const bool fold_acc = fold && fold->acc && !fold->part;
  if (fold && !fold_acc) return 0;
  if (!fold && fz && fz->acc_mode != 0 && fz->acc_mode != 3) return 0;
  // 32-bit element offsets inside the kernel except the output (64-bit): bound the input
  if ((long long)g->n * g->di * g->hi * g->wi >= (1LL << 31)) return 0;
  // buffer descriptors: the output (bytes) and one input plane must fit their 31-bit ranges
  if ((long long)g->n * g->do_ * g->ho * g->wo * 16 * (out16 ? 2 : 4) >= (1LL << 31)) return 0;
  K7Args a;
  a.n = g->n; a.di = g->di; a.hi = g->hi; a.wi = g->wi; a.do_ = g->do_; a.ho = g->ho; a.wo = g->wo;
  a.P = P; a.reflect = reflect; a.flip = flip; a.wc = wc;
  a.tiles_h = (g->ho + k7p::SH - 1) / k7p::SH;
  a.tiles_w = (g->wo + k7p::WB - 1) / k7p::WB;
  a.probe = g_probe;
  const long long cols = (long long)g->n * a.tiles_h * a.tiles_w;
  int tdc = g_k7p;
  if (tdc <= 0) {  // auto: about two blocks per CU
    tdc = (int)std::max<long long>(4, (g->do_ * cols + 511) / 512);
    tdc = std::min(tdc, g->do_);
  }
  a.tiles_d = (g->do_ + tdc - 1) / tdc;
  const long long blocks = cols * a.tiles_d;
  if (blocks >= (1LL << 31)) return 0;
  const bool m1 = !fold && fz && fz->acc_mode == 3;
  K7Fold fb = fold ? *fold : K7Fold{};
  double* acc1 = m1 ? fz->acc_out : nullptr;
  const int reps1 = m1 ? fz->reps : 1;
#define K7P_LAUNCH(M, B)                                                                                     \
  ::cg::launch(k7p_n2w_kernel<M, B>, dim3((unsigned)blocks), dim3(k7p::NT), 0, s, a, x, w, y, tdc, fb, acc1, reps1)
  if (fold) {
    if (out16) K7P_LAUNCH(2, true); else K7P_LAUNCH(2, false);
  } else if (m1) {
    if (out16) K7P_LAUNCH(1, true); else K7P_LAUNCH(1, false);
  } else {
    if (out16) K7P_LAUNCH(0, true); else K7P_LAUNCH(0, false);
  }
#undef K7P_LAUNCH
  return 1;
}

}  // namespace cg

namespace cg {

static int k7p_wg_split(const cgan3d_conv_geom* g, bool wide_in, K7Args* a, int* tdc) {
  // grid = the 16-channel operand's voxels: the output grid (first conv) or the padded input grid (last)
  const int gd = wide_in ? g->di + 2 * g->pad : g->do_, gh = wide_in ? g->hi + 2 * g->pad : g->ho,
            gw = wide_in ? g->wi + 2 * g->pad : g->wo;
  a->n = g->n;
  a->do_ = gd; a->ho = gh; a->wo = gw;
  if (wide_in) { a->di = g->do_; a->hi = g->ho; a->wi = g->wo; a->P = 2 * g->pad; a->reflect = 0; a->flip = 1; }
  else { a->di = g->di; a->hi = g->hi; a->wi = g->wi; a->P = g->pad; a->reflect = g->reflect; a->flip = 0; }
  a->wc = 0;
  a->probe = g_probe;
  a->tiles_h = (gh + k7p::SH - 1) / k7p::SH;
  a->tiles_w = (gw + k7p::WB - 1) / k7p::WB;
  const long long cols = (long long)g->n * a->tiles_h * a->tiles_w;
  int t = g_k7p > 0 ? g_k7p : (int)std::max<long long>(4, (gd * cols + 511) / 512);
  t = std::min(t, gd);
  *tdc = t;
  a->tiles_d = (gd + t - 1) / t;
  return (int)(cols * a->tiles_d);
}

long long k7p_wg_blocks(const cgan3d_conv_geom* g, bool wide_in) {
  K7Args a;
  int tdc;
  return k7p_wg_split(g, wide_in, &a, &tdc);
}

int k7p_wgrad_try(const cgan3d_conv_geom* g, bool wide_in, long long wc, const float* x, const float* go, float* dw,
                  float* ws, hipStream_t s, const __bf16* wide16) {
  if (g_k7p < 0 || !wide16 || g->pad != 3 || !g->reflect) return 0;
  K7Args a;
  int tdc;
  const int blocks = k7p_wg_split(g, wide_in, &a, &tdc);
  // buffer descriptors over one X1 plane and one A16 plane (31-bit byte ranges)
  if ((long long)a.hi * a.wi * 4 >= (1LL << 31) || (long long)g->n * a.di * a.hi * a.wi >= (1LL << 31)) return 0;
  if (wide_in) {
    ::cg::launch(k7p_wg_kernel<1>, dim3(blocks), dim3(k7p::NT), 0, s, a, go, wide16, g->di, g->hi, g->wi, ws, tdc);
  } else {
    ::cg::launch(k7p_wg_kernel<0>, dim3(blocks), dim3(k7p::NT), 0, s, a, x, wide16, g->do_, g->ho, g->wo, ws, tdc);
  }
  colsum_launch(ws, blocks, 16 * KT7, KT7, dw, wc, s);
  return 1;
}

}  // namespace cg
