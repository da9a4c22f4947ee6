// Shared helpers for the cgan3d HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <memory>
#include <tuple>
#include <unordered_map>
#include <type_traits>
#include <vector>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/cgan3d.h"

namespace cg {

// ---- launch plans (cgan3d_plan_*, plan.hip): while a plan is being recorded on this host thread,
// every launch / memset / cross-stream wait the entry points issue is appended to it (kernel
// arguments copied by value) instead of being enqueued; cgan3d_plan_run re-issues the whole
// sequence from C++ on the recorded streams — the step's ~200 launches without the Python
// wrappers' per-launch cost, and with the side-stream concurrency a replayed hipGraph loses.
struct Plan {
  std::vector<std::function<hipError_t()>> ops;
  std::vector<hipEvent_t> events;  // owned (cross-stream waits)
  // Per stream, the completion-event slot of its last recorded op when that op is a kernel launch
  // (null otherwise).  A cross-stream wait on that stream binds the event to the launch itself
  // (hipExtLaunchKernel's stop event: the dispatch's own completion signal) instead of enqueueing
  // a separate marker packet behind it — see cgan3d_stream_wait.
  std::unordered_map<hipStream_t, std::shared_ptr<hipEvent_t>> tail;
  // (start, stop) timing events of the launches cgan3d_plan_time_filter selected at record time
  // (hipExtLaunchKernel's own dispatch events: the kernel's in-plan duration, no extra packets)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> timed;
  std::vector<std::pair<hipStream_t, const void*>> timed_what;  // (stream, kernel) of each timed launch
  void add(std::function<hipError_t()> op, hipStream_t st, std::shared_ptr<hipEvent_t> stop = nullptr) {
    ops.push_back(std::move(op));
    tail[st] = std::move(stop);
  }
};
extern thread_local Plan* g_rec;
// true when the launch of kernel k being recorded is one cgan3d_plan_time_filter selected (plan.hip)
bool plan_time_match(const void* k, hipStream_t st);

template <typename... KArgs, typename... Args>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t st, Args... args) {
  if (g_rec == nullptr) {
    hipLaunchKernelGGL(k, grid, block, lds, st, args...);
    return;
  }
  std::tuple<std::decay_t<KArgs>...> t(static_cast<std::decay_t<KArgs>>(args)...);
  auto stop = std::make_shared<hipEvent_t>(nullptr);
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (plan_time_match(reinterpret_cast<const void*>(k), st) && hipEventCreate(&t0) == hipSuccess) {
    if (hipEventCreate(&t1) == hipSuccess) {
      g_rec->events.push_back(t0);
      g_rec->events.push_back(t1);
      g_rec->timed.emplace_back(t0, t1);
      g_rec->timed_what.emplace_back(st, reinterpret_cast<const void*>(k));
    } else {
      (void)hipEventDestroy(t0);
      t0 = nullptr;
    }
  }
  g_rec->add([k, grid, block, lds, st, t, stop, t0, t1]() mutable {
    return std::apply([&](auto&... a) {
      void* argv[] = {static_cast<void*>(&a)...};
      if (t0 != nullptr) {  // a timed launch (then a bound cross-stream wait gets a marker behind it)
        hipError_t e = hipExtLaunchKernel(reinterpret_cast<const void*>(k), grid, block, argv, lds, st, t0, t1, 0);
        if (e == hipSuccess && *stop != nullptr) e = hipEventRecord(*stop, st);
        return e;
      }
      if (*stop != nullptr)
        return hipExtLaunchKernel(reinterpret_cast<const void*>(k), grid, block, argv, lds, st, nullptr, *stop, 0);
      return hipLaunchKernel(reinterpret_cast<const void*>(k), grid, block, argv, lds, st);
    }, t);
  }, st, stop);
}

inline hipError_t memset_async(void* p, int v, size_t bytes, hipStream_t st) {
  if (g_rec == nullptr) return hipMemsetAsync(p, v, bytes, st);
  g_rec->add([=]() { return hipMemsetAsync(p, v, bytes, st); }, st);
  return hipSuccess;
}

// Workgroup barrier for LDS hand-offs that leaves outstanding global loads in flight: hipcc's
// __syncthreads() waits vmcnt(0) first, which serialises a register-prefetch pipeline on the
// memory latency (cdna_hip_programming.md §5 "Pipelining across barriers").
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


// last-error slot, per host thread (the C-ABI is callable from any thread)
void set_error(const char* fmt, ...);

#define CG_CHECK_ARG(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::cg::set_error(__VA_ARGS__);      \
      return CGAN3D_EINVAL;              \
    }                                    \
  } while (0)

#define CG_LAUNCH_CHECK(what)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::cg::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));   \
      return CGAN3D_EHIP;                                                       \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// reflect index into [0, n) without edge repeat (torch "reflect"), valid for |overhang| < n
__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// taps of a geometry's kernel: k^3, or k^2 for the 2-D variants (cgan3d_conv_geom.planar)
inline int geom_taps(const cgan3d_conv_geom* g) { return g->planar ? g->k * g->k : g->k * g->k * g->k; }
// depth-axis kernel extent / stride / pad: the 2-D variants pass depth through (1, 1, 0)
inline int geom_kd(const cgan3d_conv_geom* g) { return g->planar ? 1 : g->k; }
inline int geom_sd(const cgan3d_conv_geom* g) { return g->planar ? 1 : g->stride; }
inline int geom_pd(const cgan3d_conv_geom* g) { return g->planar ? 0 : g->pad; }

// device-side view of cgan3d_bn_fuse (BatchNorm statistics into fp64 accumulators, include/cgan3d.h)
struct BnFuse {
  double* acc_out;
  int acc_mode, reps;
};

// device-side view of cgan3d_epilogue
// cgan3d_bn_pre (include/cgan3d.h), copied by value; mode 0: none
struct BnPre {
  int mode;
  const __bf16* z;
  const double* acc;
  int reps;
  double nvox;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float momentum, eps;
  float* ss;
  float* mi;
  float* dgamma;
  float* dbeta;
  int accumulate;
  int act;
  float slope;
  __bf16* out16;
  double* zero;
  int zero_n;
};

struct Epi {
  const float* bias;
  const float* residual;
  const float* mask_src;
  const float* minuend;
  float* out2;
  float* stats;
  int act;
  float slope;
  float* bn_part;
  int bn_mode;
  int bn_slots;
  const float* bn_z;
  const float* bn_ss;
  const float* bn_mi;
  int bn_act;
  float bn_slope;
  const __bf16* x16;  // optional bf16 shadow of the conv input
  int bn_fold;        // mode 2 over a reflect-padded k7 input-grad grid (cgan3d_epilogue.bn_fold)
  BnFuse fz;          // all-zero unless cgan3d_epilogue.fuse is given
  int out16;          // cgan3d_epilogue.out_bf16 bit 0: y and bn_z are bf16 (k7m n2w, S2T, conv_k3m launches)
  int res16;          // bit 1: the residual is bf16 (conv_k3m only)
  BnPre pre;          // the input's BatchNorm applied while staging (conv_k3m only)
};

// c ? v : 0 for a just-loaded v, by an integer mask: the compiler turns a select whose operand is a
// load into a branch around the load (CodeGenPrepare), and a load under a branch gets a vmcnt(0) of
// its own — serialising loads meant to be in flight together
__device__ __forceinline__ float keep_if(bool c, float v) {
  return __uint_as_float(__float_as_uint(v) & (c ? 0xffffffffu : 0u));
}

__device__ __forceinline__ float act_grad(float pre, int act, float slope) {
  if (act == CGAN3D_ACT_RELU) return pre > 0.f ? 1.f : 0.f;
  if (act == CGAN3D_ACT_LRELU) return pre > 0.f ? 1.f : slope;
  return 1.f;
}

// The fused BatchNorm statistic pair of an epilogue value v at output element o, channel c (C
// channels): (v, v^2) in mode 1, (g, g*xhat) of the layer whose dL/dy is v in mode 2.
__device__ __forceinline__ void bn_pair(const Epi& e, float v, long long o, int c, int C, float* p1, float* p2) {
  if (e.bn_mode == 1) {
    *p1 += v;
    *p2 += v * v;
  } else {
    const float z = e.bn_z[o];
    const float gg = v * act_grad(z * e.bn_ss[c] + e.bn_ss[C + c], e.bn_act, e.bn_slope);
    *p1 += gg;
    *p2 += gg * (z - e.bn_mi[c]) * e.bn_mi[C + c];
  }
}

// specialised k = 7 generator first/last conv kernels (conv_k7.hip); return 1 when they apply
int k7_try_fwd(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t s);
void k7s_set(int v);
void k7p_set(int v);
int k7_wgrad_handles(const cgan3d_conv_geom* g);
int k7m_wgrad_taken(const cgan3d_conv_geom* g);
int k7m_w2n_taken(const cgan3d_conv_geom* g);
int k7m_fold_ok(const cgan3d_conv_geom* g);
int k7m_n2w_ok(const cgan3d_conv_geom* g);
int k7_try_wgrad(const cgan3d_conv_geom* g, const float* x, const float* go, float* dw, float* ws, hipStream_t s,
                 const __bf16* wide16 = nullptr);
long long k7_wgrad_ws_floats(const cgan3d_conv_geom* g);
long long k7m_wgrad_ws_floats(const cgan3d_conv_geom* g);
void k7m_wgrad_launch(const cgan3d_conv_geom* g, bool wide_in, long long wc, const float* x, const float* go, float* dw,
                      float* ws, hipStream_t s, const __bf16* wide16 = nullptr);
long long k7_n2w_blocks(const cgan3d_conv_geom* g);
long long k7m_n2w_blocks(const cgan3d_conv_geom* g);
void k7m_n2w_launch(const cgan3d_conv_geom* g, int P, int reflect, int flip, long long wc, const float* x,
                    const float* w, float* y, float* stats, float* bn_part, hipStream_t s, const Epi* fold = nullptr,
                    const BnFuse* fz = nullptr, bool out16 = false);
void k7m_w2n_launch(const cgan3d_conv_geom* g, int P, int reflect, long long wc, const float* x, const float* w,
                    float* y, const Epi& e, hipStream_t s);
// implicit-GEMM forward / input-grad (conv_gemm.hip)
int gemm_blocks(const cgan3d_conv_geom* g, long long* mblocks);
bool wgrad_bf16_ok(const cgan3d_conv_geom* g);
bool wgrad_c1_ok(const cgan3d_conv_geom* g);
bool wgrad_k3_ok(const cgan3d_conv_geom* g);
// critic middle layers, K split over waves (conv_sk.hip): packed weights format 3
bool sk_format_ok(const cgan3d_conv_geom* g);
bool sk_ok(const cgan3d_conv_geom* g);
long long sk_blocks(const cgan3d_conv_geom* g);
// Phase probes (timing only, wrong results): kernels skip the phases set in g_probe (cgan3d_set_tuning
// key 90).  Compiled in only with -DCGAN3D_PROBES (make PROBES=1); the product library has neither
// the key nor the branches (CG_PROBE is constant false).
extern int g_probe;
#ifdef CGAN3D_PROBES
#define CG_PROBE(p, bit) (((p) & (bit)) != 0)
#else
#define CG_PROBE(p, bit) false
#endif
int sk_launch(const cgan3d_conv_geom* g, const float* x, const __bf16* wp, float* y, const Epi& e, hipStream_t st);
// critic first layer, single channel (conv_c1.hip)
bool c1_fwd_ok(const cgan3d_conv_geom* g);
bool c1_dgrad_ok(const cgan3d_conv_geom* g);
bool c1_wgrad_ok(const cgan3d_conv_geom* g);
int c1_fwd_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st);
int c1_dgrad_launch(const cgan3d_conv_geom* g, const float* dz, const float* w, float* dx, const Epi& e,
                    hipStream_t st);
int c1_wgrad_launch(const cgan3d_conv_geom* g, const float* x, const float* dz, float* dw, float* ws, hipStream_t st);
long long c1_wgrad_ws_floats(const cgan3d_conv_geom* g);
long long wgrad_k3_ws_floats(const cgan3d_conv_geom* g);
void wgrad_k3_set_chunks(int v);
void wgrad_k3m_set(int v);
bool wgrad_s2_ok(const cgan3d_conv_geom* g);
long long wgrad_s2_ws_floats(const cgan3d_conv_geom* g);
void wgrad_s2_set_blocks(int v);
int wgrad_s2_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, const __bf16* g16,
                    const __bf16* a16, float* dw, int accumulate, float* ws, hipStream_t st);
int wgrad_k3_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, const __bf16* g16,
                    const __bf16* a16, float* dw, int accumulate,
                    float* ws, hipStream_t st, bool defer_reduce = false);
int wgrad_k3_partials(const cgan3d_conv_geom* g);
int wgrad_c1_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw, hipStream_t st);
int wgrad_bf16_group_launch(const cgan3d_conv_geom* geoms, const float* const* gathered, const float* const* aligned,
                            float* const* ws, int n, hipStream_t st);
int wgrad_bf16_launch(const cgan3d_conv_geom* g, const float* gathered, const float* aligned, float* dw, float* dwp,
                      int accumulate, hipStream_t st);
long long wgrad_bf16_ws_floats(const cgan3d_conv_geom* g);
// ResNet-block convs with every operand in LDS, 32x32x16 MFMA (conv_k3m.hip)
bool k3m_ok(const cgan3d_conv_geom* g, const Epi& e);
bool k3m_geom_ok(const cgan3d_conv_geom* g);
bool k3m_route(const cgan3d_conv_geom* g);
int k3m_launch(const cgan3d_conv_geom* g, const __bf16* wp, float* y, const Epi& e, hipStream_t st);
bool t64_geom_ok(const cgan3d_conv_geom* g);
bool t64_ok(const cgan3d_conv_geom* g, const Epi& e);
int t64_launch(const cgan3d_conv_geom* g, const __bf16* wp, float* y, const Epi& e, hipStream_t st);
bool f64_geom_ok(const cgan3d_conv_geom* g);
bool f64_ok(const cgan3d_conv_geom* g, const Epi& e);
int f64_launch(const cgan3d_conv_geom* g, const __bf16* wp, float* y, const Epi& e, hipStream_t st);
void k3m_set(int v);
bool k3m_enabled();  // key 15: the LDS-resident ResNet-block and 32 <-> 64 level kernels
void k7wg_blocks_set(int v);
bool halo_ok(const cgan3d_conv_geom* g);         // w_packed == 2 and eligible
bool halo_format_ok(const cgan3d_conv_geom* g);  // eligible ignoring w_packed
long long halo_mblocks(const cgan3d_conv_geom* g);
int halo_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st);
// stride-2 16 <-> 32-channel convs (conv_s2.hip), part of the halo (format 2) family
int cu_count();  // compute units of the current device
long long c1_dgrad_blocks(const cgan3d_conv_geom* g);
int s2_kind(const cgan3d_conv_geom* g);
long long s2_blocks(const cgan3d_conv_geom* g);
int s2_launch(const cgan3d_conv_geom* g, const float* x, const __bf16* wp, float* y, const Epi& e, hipStream_t st);
int halo_pack(const cgan3d_conv_geom* g, const float* w, void* wp, hipStream_t st);
int gemm_launch(const cgan3d_conv_geom* g, const float* x, const float* w, float* y, const Epi& e, hipStream_t st);
// Adam over a flat arena (+ optional repack of packed weight copies, step tick) — conv_gemm.hip
void adam_launch(float* p, const float* g, float* m, float* v, long long n, float* hyper,
                 const cgan3d_pack_desc* descs, int ndesc, int tick, unsigned* ticket, hipStream_t st);

// mode-2 pair from a prefetched z
__device__ __forceinline__ void bn_pair_z(const Epi& e, float v, float z, int c, int C, float* p1, float* p2) {
  const float gg = v * act_grad(z * e.bn_ss[c] + e.bn_ss[C + c], e.bn_act, e.bn_slope);
  *p1 += gg;
  *p2 += gg * (z - e.bn_mi[c]) * e.bn_mi[C + c];
}

// dw[c * wc + t] += sum over the nrows partial rows part[r][c * T + t] (ncols = C x T columns), summed in
// a fixed order, one writer per element (conv_k7_mfma.hip; the k7 and critic first-layer weight grads)
void colsum_launch(const float* part, int nrows, int ncols, int T, float* dw, long long wc, hipStream_t s);

// ---- launch tickets: "last block out" of a launch, without any waiting.  Two uint32 words, zeroed
// once by the caller; each block takes a ticket when it is done and the last one (true in its
// thread 0) re-zeroes them.  Relaxed agent-scope atomics: no cache writeback / invalidate.  (A
// phase gate on top of this — later blocks spinning until earlier ones publish — measured 1.3-5x
// slower than two launches for BatchNorm finalize + apply)
__device__ __forceinline__ bool last_block_out(unsigned* ticket) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nblk = gridDim.x * gridDim.y * gridDim.z;
    if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
  }
  return false;
}

// torch.optim.Adam single-element update (no weight decay / amsgrad / maximize) at the 1-based
// `step`, then the optional WGAN weight clip (Trainer.py:136-138).  hyper = [lr, beta1, beta2, eps,
// step, clip]; shared by adam_kernel and the fused update + repack launch.
struct AdamK {
  float lr, b2, eps, clip, bc2s, wgt, step_size;
};
__device__ __forceinline__ AdamK adam_k(const float* hyper, float step) {
  AdamK k;
  const float b1 = hyper[1];
  k.lr = hyper[0]; k.b2 = hyper[2]; k.eps = hyper[3]; k.clip = hyper[5];
  k.bc2s = sqrtf(1.f - powf(k.b2, step));
  k.wgt = 1.f - b1;
  k.step_size = k.lr / (1.f - powf(b1, step));
  return k;
}
__device__ __forceinline__ void adam_vals(const AdamK& k, float gi, float& mi, float& vi, float& pi) {
  // no contraction: the float4 path (cgan3d_adam) and the per-element path with packed copies
  // (cgan3d_adam_pack) must leave the same bits whatever the compiler fuses in either context
#pragma clang fp contract(off)
  // torch lerp: weight < 0.5 ? self + w*(end-self) : end - (end-self)*(1-w)
  mi = k.wgt < 0.5f ? mi + k.wgt * (gi - mi) : gi - (gi - mi) * (1.f - k.wgt);
  vi = vi * k.b2 + (1.f - k.b2) * gi * gi;
  const float denom = sqrtf(vi) / k.bc2s + k.eps;
  pi = pi - k.step_size * (mi / denom);
  if (k.clip > 0.f) pi = fminf(fmaxf(pi, -k.clip), k.clip);
}
__device__ __forceinline__ float adam_elem(const AdamK& k, float* __restrict__ p, const float* __restrict__ g,
                                          float* __restrict__ m, float* __restrict__ v, long long i) {
  float mi = m[i], vi = v[i], pi = p[i];
  adam_vals(k, g[i], mi, vi, pi);
  m[i] = mi;
  v[i] = vi;
  p[i] = pi;
  return pi;
}

// out[i] = sum of padded[q] over the reflect-pad preimages q of interior voxel i
__device__ __forceinline__ int fold_src(int d, int D, int P, int* q) {  // padded rows mirroring onto d
  int n = 0;
  q[n++] = d + P;
  if (d >= 1 && d <= P) q[n++] = P - d;
  else if (d <= D - 2 && d >= D - 1 - P) q[n++] = 2 * (D - 1) - d + P;
  return n;
}

// lin -> (x, y, z, n) over extents (X, Y, Z, -): 32-bit divides whenever lin fits (a 64-bit divide
// is ~100 VALU instructions)
__device__ __forceinline__ void unflatten4(long long lin, int X, int Y, int Z, int& x, int& y, int& z, int& n) {
  if (lin < (1LL << 32)) {
    const unsigned l = (unsigned)lin, t1 = l / (unsigned)X, t2 = t1 / (unsigned)Y, t3 = t2 / (unsigned)Z;
    x = (int)(l - t1 * X); y = (int)(t1 - t2 * Y); z = (int)(t2 - t3 * Z); n = (int)t3;
  } else {
    long long t = lin / X;
    x = (int)(lin - t * X);
    y = (int)(t % Y); t /= Y;
    z = (int)(t % Z); n = (int)(t / Z);
  }
}

// slab slot b, channel c, pair member q of a fused BatchNorm slab
__device__ __forceinline__ float* bn_slot(const Epi& e, int q, int C, int c, int b) {
  return e.bn_part + ((long long)q * C + c) * e.bn_slots + b;
}

}  // namespace cg
