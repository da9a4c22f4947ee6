// Small device kernels of the step: fused Adam, reflect-pad fold, GP interpolation,
// plus the library's version / error plumbing.
#include <cstring>

#include "common.h"

namespace cg {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

__global__ void adam_tick_kernel(float* hyper) { hyper[4] += 1.f; }

// compute units of the current device (persistent-grid sizing), looked up once per device
int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int v = 0;
    cus[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return cus[dev];
}


// one thread per (voxel, V channels); 32-bit index math (element count < 2^31).  PD: the depth
// axis's pad (P, or 0 for the 2-D variants' planar grids, whose depth is not padded)
template <int V>
__global__ __launch_bounds__(256) void reflect_fold_kernel(const float* __restrict__ pad_in, float* __restrict__ out,
                                                           int N, int D, int H, int W, int C, int P, int PD) {
  typedef float fv __attribute__((ext_vector_type(V)));
  const int C4 = C / V;
  const int total = N * D * H * W * C4;
  const int Dp = D + 2 * PD, Hp = H + 2 * P, Wp = W + 2 * P;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    int t = i / C4;
    const int w = t % W; t /= W;
    const int h = t % H; t /= H;
    const int d = t % D, n = t / D;
    int qd[2], qh[2], qw[2];
    const int nd = fold_src(d, D, PD, qd), nh = fold_src(h, H, P, qh), nw = fold_src(w, W, P, qw);
    fv s = {};
    for (int a = 0; a < nd; ++a)
      for (int b = 0; b < nh; ++b)
        for (int e = 0; e < nw; ++e)
          s += *reinterpret_cast<const fv*>(pad_in + ((((long long)n * Dp + qd[a]) * Hp + qh[b]) * Wp + qw[e]) * C +
                                            V * c4);
    reinterpret_cast<fv*>(out)[i] = s;
  }
}

// reflect_fold + the fused BatchNorm backward statistics of its output (cgan3d_epilogue bn_gsum):
// V = 4 channels per thread, fixed for the whole grid-stride loop (256 % (C/4) == 0), so the
// channels' scale / shift / mean / invstd live in registers; z is read as float4; two items per
// iteration keep more loads in flight (HBM-bound: padded dL/dy in, dL/dy + z through)
__global__ __launch_bounds__(256) void reflect_fold_bn_kernel(const float* __restrict__ pad_in, float* __restrict__ out,
                                                              int N, int D, int H, int W, int C, int P, int PD, Epi ep) {
  __shared__ f32x4 r0[256], r1[256];
  const int C4 = C / 4, tid = threadIdx.x;
  const int total = N * D * H * W * C4;
  const int Dp = D + 2 * PD, Hp = H + 2 * P, Wp = W + 2 * P;
  const int c0 = (tid % C4) * 4;
  f32x4 sc, sf, mu, iv;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = ep.bn_ss[c0 + e]; sf[e] = ep.bn_ss[C + c0 + e]; mu[e] = ep.bn_mi[c0 + e]; iv[e] = ep.bn_mi[C + c0 + e];
  }
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  const int stride = gridDim.x * blockDim.x;
#pragma unroll 2
  for (int i = blockIdx.x * blockDim.x + tid; i < total; i += stride) {
    int t = i / C4;
    const int w = t % W; t /= W;
    const int h = t % H; t /= H;
    const int d = t % D, n = t / D;
    int qd[2], qh[2], qw[2];
    const int nd = fold_src(d, D, PD, qd), nh = fold_src(h, H, P, qh), nw = fold_src(w, W, P, qw);
    const f32x4 z = reinterpret_cast<const f32x4*>(ep.bn_z)[i];
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < nd; ++a)
      for (int b = 0; b < nh; ++b)
        for (int e = 0; e < nw; ++e)
          s += *reinterpret_cast<const f32x4*>(pad_in + ((((long long)n * Dp + qd[a]) * Hp + qh[b]) * Wp + qw[e]) * C + c0);
    reinterpret_cast<f32x4*>(out)[i] = s;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gg = s[e] * act_grad(z[e] * sc[e] + sf[e], ep.bn_act, ep.bn_slope);
      a0[e] += gg;
      a1[e] += gg * (z[e] - mu[e]) * iv[e];
    }
  }
  r0[tid] = a0;
  r1[tid] = a1;
  __syncthreads();
  if (tid < C4) {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = tid; k < 256; k += C4) { s0 += r0[k]; s1 += r1[k]; }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      *bn_slot(ep, 0, C, 4 * tid + e, blockIdx.x) = s0[e];
      *bn_slot(ep, 1, C, 4 * tid + e, blockIdx.x) = s1[e];
    }
  }
}

// interpolation = eps*real + (1-eps)*fake  (model/utils.py:27-28)
// idx (optional, device int32 [2 b]): sample s interpolates real row idx[s] and fake row idx[b + s] —
// the reference's resampling when |real| != |fake| (model/utils.py:21-25).  The rows are clamped to
// [0, n_real) / [0, n_fake) on the device: a bad index reads a valid row instead of past the batch
// (the host range-checks them, StepEngine.set_gp_indices)
__global__ __launch_bounds__(256) void interp_kernel(const float* __restrict__ real, const float* __restrict__ fake,
                                                     const float* __restrict__ eps, float* __restrict__ out,
                                                     long long ps, long long total, const int* __restrict__ idx, int b,
                                                     int n_real, int n_fake) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long s = i / ps, v = i - s * ps;
    const float e = eps[s];
    const long long ir = idx ? (long long)min(max(idx[s], 0), n_real - 1) * ps + v : i,
                    jf = idx ? (long long)min(max(idx[b + s], 0), n_fake - 1) * ps + v : i;
    out[i] = e * real[ir] + (1.f - e) * fake[jf];
  }
}

// dz = dy * (1 - y^2)   (tanh backward from its output, generator.py:85)
__global__ __launch_bounds__(256) void tanh_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                                       float* __restrict__ dz, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float t = y[i];
    dz[i] = dy[i] * (1.f - t * t);
  }
}

}  // namespace cg

using namespace cg;

extern "C" int cgan3d_tanh_backward(const float* y, const float* dy, float* dz, int64_t n, void* stream) {
  CG_CHECK_ARG(y && dy && dz && n > 0, "cgan3d_tanh_backward: bad args");
  int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  ::cg::launch(tanh_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, y, dy, dz, (long long)n);
  CG_LAUNCH_CHECK("tanh_bwd_kernel");
  return CGAN3D_OK;
}

extern "C" const char* cgan3d_version(void) { return "cgan3d 0.1.0 gfx950"; }
extern "C" const char* cgan3d_get_last_error(void) { return g_err; }

extern "C" int cgan3d_adam_tick(float* hyper, void* stream) {
  CG_CHECK_ARG(hyper, "cgan3d_adam_tick: null pointer");
  ::cg::launch(adam_tick_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, hyper);
  CG_LAUNCH_CHECK("adam_tick_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                           const float* hyper, void* stream) {
  CG_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && hyper, "cgan3d_adam: null pointer");
  CG_CHECK_ARG(n > 0, "cgan3d_adam: n must be positive");
  // torch.optim.Adam at step hyper[4] (advanced beforehand by cgan3d_adam_tick): the Adam phase
  // of adam_pack_kernel (conv_gemm.hip) with no packed copies and no tick
  adam_launch(param, grad, exp_avg, exp_avg_sq, (long long)n, const_cast<float*>(hyper), nullptr, 0, 0, nullptr,
              (hipStream_t)stream);
  CG_LAUNCH_CHECK("adam_pack_kernel");
  return CGAN3D_OK;
}

static int reflect_fold_launch(const float* padded, float* out, int n, int d, int h, int w, int c, int pad, int pad_d,
                               void* stream) {
  const long long total = (long long)n * d * h * w * c;
  CG_CHECK_ARG(total < (1LL << 31), "cgan3d_reflect_fold: volume too large");
  const bool v4 = c % 4 == 0;
  int blocks = (int)std::min<long long>((total / (v4 ? 4 : 1) + 255) / 256, 8192);
  if (v4)
    ::cg::launch(reflect_fold_kernel<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, padded, out, n, d, h, w,
                       c, pad, pad_d);
  else
    ::cg::launch(reflect_fold_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, padded, out, n, d, h, w,
                       c, pad, pad_d);
  CG_LAUNCH_CHECK("reflect_fold_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_reflect_fold(const float* padded, float* out, int32_t n, int32_t d, int32_t h, int32_t w,
                                   int32_t c, int32_t pad, void* stream) {
  CG_CHECK_ARG(padded && out, "cgan3d_reflect_fold: null pointer");
  CG_CHECK_ARG(n > 0 && d > 2 * pad && h > 2 * pad && w > 2 * pad && c > 0 && pad >= 0,
               "cgan3d_reflect_fold: dims must exceed 2*pad");
  return reflect_fold_launch(padded, out, n, d, h, w, c, pad, pad, stream);
}

extern "C" int32_t cgan3d_reflect_fold_slots(int32_t n, int32_t d, int32_t h, int32_t w, int32_t c) {
  const long long total = (long long)n * d * h * w * c;
  return (int32_t)std::max<long long>(1, std::min<long long>((total / 4 + 255) / 256, 4096));
}

static int reflect_fold_ex_launch(const float* padded, float* out, int n, int d, int h, int w, int c, int pad, int pad_d,
                                  const cgan3d_epilogue* ep, void* stream) {
  CG_CHECK_ARG(ep->bn_mode == 2, "cgan3d_reflect_fold_ex: only bn_mode 2");
  CG_CHECK_ARG(padded && out && ep->bn_part && ep->bn_z && ep->bn_ss && ep->bn_mi, "cgan3d_reflect_fold_ex: null pointer");
  CG_CHECK_ARG(c >= 4 && c % 4 == 0 && 256 % (c / 4) == 0, "cgan3d_reflect_fold_ex: channels must be 4k dividing 1024");
  const long long total = (long long)n * d * h * w * c;
  CG_CHECK_ARG(total < (1LL << 31), "cgan3d_reflect_fold_ex: volume too large");
  const int blocks = cgan3d_reflect_fold_slots(n, d, h, w, c);
  CG_CHECK_ARG(ep->bn_slots == blocks, "cgan3d_reflect_fold_ex: bn_slots %d, the launch has %d", ep->bn_slots, blocks);
  Epi e{};
  e.bn_part = ep->bn_part; e.bn_mode = 2; e.bn_slots = blocks; e.bn_z = ep->bn_z; e.bn_ss = ep->bn_ss;
  e.bn_mi = ep->bn_mi; e.bn_act = ep->bn_act; e.bn_slope = ep->bn_slope;
  ::cg::launch(reflect_fold_bn_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, padded, out, n, d, h, w, c,
                     pad, pad_d, e);
  CG_LAUNCH_CHECK("reflect_fold_bn_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_reflect_fold_ex(const float* padded, float* out, int32_t n, int32_t d, int32_t h, int32_t w,
                                      int32_t c, int32_t pad, const cgan3d_epilogue* ep, void* stream) {
  if (!ep || !ep->bn_mode) return cgan3d_reflect_fold(padded, out, n, d, h, w, c, pad, stream);
  CG_CHECK_ARG(n > 0 && d > 2 * pad && h > 2 * pad && w > 2 * pad && pad >= 0,
               "cgan3d_reflect_fold_ex: dims must exceed 2*pad");
  return reflect_fold_ex_launch(padded, out, n, d, h, w, c, pad, pad, ep, stream);
}

extern "C" int cgan3d_reflect_fold2d(const float* padded, float* out, int32_t n, int32_t h, int32_t w, int32_t c,
                                     int32_t pad, const cgan3d_epilogue* ep, void* stream) {
  CG_CHECK_ARG(padded && out, "cgan3d_reflect_fold2d: null pointer");
  CG_CHECK_ARG(n > 0 && h > 2 * pad && w > 2 * pad && c > 0 && pad >= 0, "cgan3d_reflect_fold2d: dims must exceed 2*pad");
  if (ep && ep->bn_mode) return reflect_fold_ex_launch(padded, out, n, 1, h, w, c, pad, 0, ep, stream);
  return reflect_fold_launch(padded, out, n, 1, h, w, c, pad, 0, stream);
}

extern "C" int cgan3d_gp_interpolate(const float* real, const float* fake, const float* eps, float* out, int32_t b,
                                     int64_t per_sample, void* stream) {
  CG_CHECK_ARG(real && fake && eps && out && b > 0 && per_sample > 0, "cgan3d_gp_interpolate: bad args");
  const long long total = (long long)b * per_sample;
  int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  ::cg::launch(interp_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, real, fake, eps, out,
                     (long long)per_sample, total, (const int*)nullptr, (int)b, (int)b, (int)b);
  CG_LAUNCH_CHECK("interp_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_gp_interpolate_idx(const float* real, const float* fake, const int32_t* idx, const float* eps,
                                         float* out, int32_t b, int64_t per_sample, int32_t n_real, int32_t n_fake,
                                         void* stream) {
  CG_CHECK_ARG(real && fake && idx && eps && out && b > 0 && per_sample > 0 && n_real > 0 && n_fake > 0,
               "cgan3d_gp_interpolate_idx: bad args");
  const long long total = (long long)b * per_sample;
  int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  ::cg::launch(interp_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, real, fake, eps, out,
                     (long long)per_sample, total, (const int*)idx, (int)b, (int)n_real, (int)n_fake);
  CG_LAUNCH_CHECK("interp_kernel");
  return CGAN3D_OK;
}

// Several device-to-device copies in one launch (a batch into the engine's input slots: the
// OPT / subopt patches, the segmentation mask, the GP interpolation weights).  Work unit = one
// 16-byte vector of a segment; a segment's tail (bytes % 16, or all of it when src/dst are not
// 16-byte aligned) is the extra last unit, copied bytewise by its thread.
namespace cg {
constexpr int COPY_SEGS = 8;
struct CopySegs {
  const unsigned char* src[COPY_SEGS];
  unsigned char* dst[COPY_SEGS];
  long long bytes[COPY_SEGS], n16[COPY_SEGS], start[COPY_SEGS + 1];
  int n;
};

__global__ __launch_bounds__(256) void copy_multi_kernel(CopySegs c) {
  const long long total = c.start[c.n];
  for (long long u = (long long)blockIdx.x * 256 + threadIdx.x; u < total; u += (long long)gridDim.x * 256) {
    int s = 0;
    while (s + 1 < c.n && u >= c.start[s + 1]) ++s;
    const long long k = u - c.start[s];
    if (k < c.n16[s]) {
      reinterpret_cast<uint4*>(c.dst[s])[k] = reinterpret_cast<const uint4*>(c.src[s])[k];
    } else {
      for (long long b = c.n16[s] * 16; b < c.bytes[s]; ++b) c.dst[s][b] = c.src[s][b];
    }
  }
}
}  // namespace cg

extern "C" int cgan3d_copy_multi(const void* const* src, void* const* dst, const int64_t* bytes, int32_t n,
                                 void* stream) {
  return cgan3d_copy_multi_ex(src, dst, bytes, n, 2048, stream);
}

extern "C" int cgan3d_copy_multi_ex(const void* const* src, void* const* dst, const int64_t* bytes, int32_t n,
                                    int32_t max_blocks, void* stream) {
  CG_CHECK_ARG(src && dst && bytes && n > 0 && n <= ::cg::COPY_SEGS && max_blocks > 0, "cgan3d_copy_multi: bad args");
  ::cg::CopySegs c{};
  c.n = n;
  c.start[0] = 0;
  for (int s = 0; s < n; ++s) {
    CG_CHECK_ARG(src[s] && dst[s] && bytes[s] >= 0, "cgan3d_copy_multi: bad segment");
    c.src[s] = static_cast<const unsigned char*>(src[s]);
    c.dst[s] = static_cast<unsigned char*>(dst[s]);
    c.bytes[s] = bytes[s];
    const bool aligned = !(reinterpret_cast<uintptr_t>(src[s]) & 15) && !(reinterpret_cast<uintptr_t>(dst[s]) & 15);
    c.n16[s] = aligned ? bytes[s] / 16 : 0;
    CG_CHECK_ARG(bytes[s] - c.n16[s] * 16 <= 4096, "cgan3d_copy_multi: unaligned segment over 4 KB");
    c.start[s + 1] = c.start[s] + c.n16[s] + (bytes[s] > c.n16[s] * 16 ? 1 : 0);
  }
  const long long total = c.start[n];
  if (total == 0) return CGAN3D_OK;
  const unsigned blocks = (unsigned)std::min<long long>((total + 255) / 256, max_blocks);
  ::cg::launch(::cg::copy_multi_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, c);
  CG_LAUNCH_CHECK("copy_multi_kernel");
  return CGAN3D_OK;
}

// Pinned host memory mapped into the device's address space (hipHostMallocMapped): kernels read it
// over PCIe through *dev, so a batch in such a buffer reaches HBM by a small copy / unpack kernel on
// the copy stream instead of a host-blocking SDMA transfer (tools/h2d_probe.py).
extern "C" int cgan3d_host_alloc(int64_t bytes, void** host, void** dev) {
  CG_CHECK_ARG(bytes > 0 && host && dev, "cgan3d_host_alloc: bad args");
  *host = nullptr;
  *dev = nullptr;
  if (hipHostMalloc(host, (size_t)bytes, hipHostMallocMapped) != hipSuccess || *host == nullptr) {
    set_error("cgan3d_host_alloc: hipHostMalloc(%lld) failed", (long long)bytes);
    return CGAN3D_EHIP;
  }
  if (hipHostGetDevicePointer(dev, *host, 0) != hipSuccess || *dev == nullptr) {
    (void)hipHostFree(*host);
    *host = nullptr;
    set_error("cgan3d_host_alloc: no device mapping");
    return CGAN3D_EHIP;
  }
  return CGAN3D_OK;
}

extern "C" int cgan3d_host_free(void* host) {
  if (host && hipHostFree(host) != hipSuccess) {
    set_error("cgan3d_host_free failed");
    return CGAN3D_EHIP;
  }
  return CGAN3D_OK;
}

// Zero `bytes` bytes at p (a gradient arena before an update): a memset recorded in launch plans.
extern "C" int cgan3d_zero(void* p, int64_t bytes, void* stream) {
  CG_CHECK_ARG(p && bytes > 0, "cgan3d_zero: bad args");
  if (::cg::memset_async(p, 0, (size_t)bytes, (hipStream_t)stream) != hipSuccess) {
    set_error("cgan3d_zero: memset failed");
    return CGAN3D_EHIP;
  }
  return CGAN3D_OK;
}
