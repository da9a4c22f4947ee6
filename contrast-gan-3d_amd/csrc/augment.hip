// Spatial augmentation of a patch batch on the GPU: the training transform of the reference
// (experiments/basic_conf.py:87-113, batchgenerators SpatialTransform_2 -> augment_spatial_2 with
// random_crop=False), restated from batchgenerators' published algorithm (the package is not part
// of the reference tree): per sample an optional elastic deformation (a random field smoothed by a
// Gaussian in Fourier space, scaled to a drawn magnitude), rotation and scaling of the
// zero-centred voxel grid, re-centring on the patch centre, then
//   data: cubic B-spline interpolation (scipy.ndimage.map_coordinates order 3, mode 'nearest':
//         the volume is edge-padded by 12 voxels and spline-prefiltered, taps clamped to the pad);
//   seg:  nearest-neighbour (order 0, mode 'constant', cval 0: round-half-up inside [0, n-1]).
// The host (cgan3d_amd/data/augment.py) draws the per-sample parameters; these kernels do the
// per-voxel work.  Samples with no transform drawn are copied unchanged (batchgenerators'
// centre crop of a same-size patch).
//
// Layout: [n][a0][a1][a2] float (C = 1), a2 fastest; seg uint8 of the same shape.
#include "common.h"

namespace cg {

constexpr int kAugPad = 12;   // scipy _prepad_for_spline_filter, mode 'nearest'
constexpr int kAugParams = 16;  // per sample: A[9] row-major, ctr[3], field slot (or -1 / -2), mag-scale[3]

__device__ __forceinline__ int aug_clamp(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

// edge-padded copy: coeff[s][p0][p1][p2] = x[s][clamp(p0 - 12)][clamp(p1 - 12)][clamp(p2 - 12)]
__global__ __launch_bounds__(256) void aug_pad_kernel(const float* __restrict__ x, int n, int a0, int a1, int a2,
                                                      float* __restrict__ c) {
  const int b0 = a0 + 2 * kAugPad, b1 = a1 + 2 * kAugPad, b2 = a2 + 2 * kAugPad;
  const long long tot = (long long)n * b0 * b1 * b2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    long long r = i;
    const int p2 = (int)(r % b2); r /= b2;
    const int p1 = (int)(r % b1); r /= b1;
    const int p0 = (int)(r % b0);
    const int s = (int)(r / b0);
    const int i0 = aug_clamp(p0 - kAugPad, a0), i1 = aug_clamp(p1 - kAugPad, a1), i2 = aug_clamp(p2 - kAugPad, a2);
    c[i] = x[(((long long)s * a0 + i0) * a1 + i1) * a2 + i2];
  }
}

// Cubic B-spline prefilter of one line in place (pole z = sqrt(3) - 2, gain 6), mirror-symmetric
// boundary with the exact causal initialisation; fp64 recursion.  One thread per line.
__global__ __launch_bounds__(256) void aug_prefilter_kernel(float* __restrict__ c, long long lines, int len,
                                                            long long stride, long long inner, long long outer_stride) {
  const long long l = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= lines) return;
  // line l = (outer, inner): start = outer * outer_stride + inner (inner < `inner` elements of stride 1)
  float* p = c + (l / inner) * outer_stride + (l % inner);
  const double z = 1.7320508075688772 - 2.0;
  const int n = len;
  // causal init: (c0 + z^(n-1) c_{n-1} + sum_{k=1}^{n-2} (z^k + z^(2n-2-k)) c_k) / (1 - z^(2n-2))
  double zn1 = 1.0;
  for (int k = 0; k < n - 1; ++k) zn1 *= z;  // z^(n-1)
  double acc = 6.0 * p[0] + zn1 * 6.0 * p[(long long)(n - 1) * stride];
  double zk = z, z2 = zn1 * zn1 / z;  // z^(2n-3)
  for (int k = 1; k < n - 1; ++k) {
    acc += (zk + z2) * 6.0 * p[(long long)k * stride];
    zk *= z;
    z2 /= z;
  }
  double prev = acc / (1.0 - zn1 * zn1);
  p[0] = (float)prev;
  // causal pass (stored in place as fp32; its last two values kept in fp64 for the anticausal init)
  double cm2 = prev, cm1 = prev;
  for (int i = 1; i < n; ++i) {
    const double v = 6.0 * p[(long long)i * stride] + z * prev;
    p[(long long)i * stride] = (float)v;
    cm2 = cm1;
    cm1 = v;
    prev = v;
  }
  double next = (z / (z * z - 1.0)) * (cm1 + z * cm2);
  p[(long long)(n - 1) * stride] = (float)next;
  for (int i = n - 2; i >= 0; --i) {
    next = z * (next - (double)p[(long long)i * stride]);
    p[(long long)i * stride] = (float)next;
  }
}

// circular convolution along one axis (the Fourier-space Gaussian of elastic_deform_coordinates_2):
// out[.., i, ..] = sum_m in[.., (i - m) mod len, ..] * k[m]; nf fields of a0*a1*a2 voxels, field
// f = 3 slot + d (the d-th offset field of elastic sample `slot`) convolved with its slot's kernel
// row for this axis, k[slot][axis][kst]
__global__ __launch_bounds__(256) void aug_circconv_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           int nf, int a0, int a1, int a2, int axis,
                                                           const float* __restrict__ k, int kst) {
  const long long vox = (long long)a0 * a1 * a2, tot = vox * nf;
  const int len = axis == 0 ? a0 : (axis == 1 ? a1 : a2);
  const long long st = axis == 0 ? (long long)a1 * a2 : (axis == 1 ? a2 : 1);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(i / vox);
    const long long v = i - (long long)f * vox;
    const int ci = (int)((v / st) % len);
    const long long base = i - (long long)ci * st;
    const float* kr = k + ((long long)(f / 3) * 3 + axis) * kst;
    float s = 0.f;
    for (int m = 0; m < len; ++m) {
      int j = ci - m;
      j += j < 0 ? len : 0;
      s += in[base + (long long)j * st] * kr[m];
    }
    out[i] = s;
  }
}

// per field: stats[2f] = max |f|, stats[2f+1] = mean f (fp64 block reduction, one block per field)
__global__ __launch_bounds__(1024) void aug_field_stats_kernel(const float* __restrict__ f, long long vox,
                                                               float* __restrict__ stats) {
  __shared__ double smax[1024], ssum[1024];
  const float* p = f + (long long)blockIdx.x * vox;
  double mx = 0.0, sm = 0.0;
  for (long long i = threadIdx.x; i < vox; i += blockDim.x) {
    const double v = p[i];
    mx = fmax(mx, fabs(v));
    sm += v;
  }
  smax[threadIdx.x] = mx;
  ssum[threadIdx.x] = sm;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + o]);
      ssum[threadIdx.x] += ssum[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[2 * blockIdx.x] = (float)smax[0];
    stats[2 * blockIdx.x + 1] = (float)(ssum[0] / (double)vox);
  }
}

__device__ __forceinline__ void bspline3_w(float t, float* w) {  // weights of taps floor-1 .. floor+2
  const float t2 = t * t, t3 = t2 * t;
  w[0] = (1.f - t) * (1.f - t) * (1.f - t) / 6.f;
  w[1] = (3.f * t3 - 6.f * t2 + 4.f) / 6.f;
  w[2] = (-3.f * t3 + 3.f * t2 + 3.f * t + 1.f) / 6.f;
  w[3] = t3 / 6.f;
}

// x_i = sum_j A_ij (g_j + e_j (f_j(v) - mean_j)) + ctr_i, g = zero-centred grid coordinate;
// data = cubic spline of the padded coefficients at x + 12 (taps clamped), seg = nearest inside
// [0, n-1]^3 else 0.  Field slot -2: unchanged copy (no transform drawn for the sample).
__global__ __launch_bounds__(256) void aug_sample_kernel(const float* __restrict__ coeff, const float* __restrict__ x,
                                                         const unsigned char* __restrict__ seg, int n, int a0, int a1,
                                                         int a2, const float* __restrict__ prm,
                                                         const float* __restrict__ fields,
                                                         const float* __restrict__ fstats, float* __restrict__ out,
                                                         unsigned char* __restrict__ seg_out) {
  const long long vox = (long long)a0 * a1 * a2, tot = vox * n;
  const int b0 = a0 + 2 * kAugPad, b1 = a1 + 2 * kAugPad, b2 = a2 + 2 * kAugPad;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(i / vox);
    const long long v = i - (long long)s * vox;
    const float* P = prm + kAugParams * s;
    const int slot = (int)P[12];
    if (slot == -2) {
      out[i] = x[i];
      seg_out[i] = seg[i];
      continue;
    }
    const int i2 = (int)(v % a2), i1 = (int)((v / a2) % a1), i0 = (int)(v / ((long long)a1 * a2));
    float g[3] = {i0 - 0.5f * (a0 - 1), i1 - 0.5f * (a1 - 1), i2 - 0.5f * (a2 - 1)};
    if (slot >= 0) {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float* fs = fstats + 2 * (3 * slot + d);
        g[d] += P[13 + d] / fs[0] * (fields[((long long)(3 * slot + d)) * vox + v] - fs[1]);
      }
    }
    float c[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) c[r] = P[3 * r] * g[0] + P[3 * r + 1] * g[1] + P[3 * r + 2] * g[2] + P[9 + r];
    // seg: order 0, constant 0 outside [0, n-1]
    const bool in = c[0] >= 0.f && c[0] <= (float)(a0 - 1) && c[1] >= 0.f && c[1] <= (float)(a1 - 1) && c[2] >= 0.f &&
                    c[2] <= (float)(a2 - 1);
    unsigned char sv = 0;
    if (in) {
      const int j0 = (int)floorf(c[0] + 0.5f), j1 = (int)floorf(c[1] + 0.5f), j2 = (int)floorf(c[2] + 0.5f);
      sv = seg[(((long long)s * a0 + j0) * a1 + j1) * a2 + j2];
    }
    seg_out[i] = sv;
    // data: cubic B-spline on the padded coefficients
    const float q0 = c[0] + kAugPad, q1 = c[1] + kAugPad, q2 = c[2] + kAugPad;
    const float f0 = a0 == 1 ? (float)kAugPad : floorf(q0), f1 = floorf(q1), f2 = floorf(q2);
    float w0[4], w1[4], w2[4];
    bspline3_w(q0 - f0, w0);
    bspline3_w(q1 - f1, w1);
    bspline3_w(q2 - f2, w2);
    if (a0 == 1) {  // 2-D patches (a0 = 1, not prefiltered along it): the plane itself, weight 1
      w0[0] = 0.f; w0[1] = 1.f; w0[2] = 0.f; w0[3] = 0.f;
    }
    const float* cb = coeff + (long long)s * b0 * b1 * b2;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k0 = aug_clamp((int)f0 - 1 + u, b0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k1 = aug_clamp((int)f1 - 1 + t, b1);
        const float* row = cb + ((long long)k0 * b1 + k1) * b2;
        float r = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) r += w2[e] * row[aug_clamp((int)f2 - 1 + e, b2)];
        acc += w0[u] * w1[t] * r;
      }
    }
    out[i] = acc;
  }
}

static int aug_blocks(long long n) { return (int)std::min<long long>((n + 255) / 256, 16384); }

// MirrorTransform (batchgenerators augment_mirroring): out[s][i] = x[s][i with axis d reversed for
// every set bit d of flags[s]]; seg likewise.  Out of place.
__global__ __launch_bounds__(256) void aug_mirror_kernel(const float* __restrict__ x, const unsigned char* __restrict__ seg,
                                                         int n, int a0, int a1, int a2, const int* __restrict__ flags,
                                                         float* __restrict__ out, unsigned char* __restrict__ seg_out) {
  const long long vox = (long long)a0 * a1 * a2, tot = vox * n;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(i / vox);
    const long long v = i - (long long)s * vox;
    int i2 = (int)(v % a2), i1 = (int)((v / a2) % a1), i0 = (int)(v / ((long long)a1 * a2));
    const int f = flags[s];
    if (f & 1) i0 = a0 - 1 - i0;
    if (f & 2) i1 = a1 - 1 - i1;
    if (f & 4) i2 = a2 - 1 - i2;
    const long long src = (long long)s * vox + ((long long)i0 * a1 + i1) * a2 + i2;
    out[i] = x[src];
    seg_out[i] = seg[src];
  }
}

}  // namespace cg

using namespace cg;

extern "C" int64_t cgan3d_augment_ws_floats(int32_t n, int32_t a0, int32_t a1, int32_t a2, int32_t n_elastic) {
  const long long padded = (long long)n * (a0 + 2 * kAugPad) * (a1 + 2 * kAugPad) * (a2 + 2 * kAugPad);
  const long long vox = (long long)a0 * a1 * a2;
  return padded + 2LL * 3 * n_elastic * vox + 6LL * n_elastic;
}

extern "C" int cgan3d_spatial_augment(const float* data, const uint8_t* seg, int32_t n, int32_t a0, int32_t a1,
                                      int32_t a2, const float* params, const float* noise, int32_t n_elastic,
                                      const float* gauss, float* data_out, uint8_t* seg_out, float* ws,
                                      void* stream) {
  CG_CHECK_ARG(data && seg && params && data_out && seg_out && ws && n > 0 && a0 >= 1 && a1 > 1 && a2 > 1,
               "cgan3d_spatial_augment: bad args");
  CG_CHECK_ARG(a0 > 1 || n_elastic == 0, "cgan3d_spatial_augment: 2-D patches (a0 = 1) take no elastic deformation");
  CG_CHECK_ARG(n_elastic >= 0 && n_elastic <= n && (n_elastic == 0 || (noise && gauss)),
               "cgan3d_spatial_augment: elastic samples need noise and Gaussian kernels");
  CG_CHECK_ARG(data_out != data && (const void*)seg_out != (const void*)seg, "cgan3d_spatial_augment: in place");
  hipStream_t st = (hipStream_t)stream;
  const int b0 = a0 + 2 * kAugPad, b1 = a1 + 2 * kAugPad, b2 = a2 + 2 * kAugPad;
  const long long padded = (long long)n * b0 * b1 * b2, vox = (long long)a0 * a1 * a2;
  float* coeff = ws;
  float* fa = ws + padded;
  float* fb = fa + 3LL * n_elastic * vox;
  float* fstats = fb + 3LL * n_elastic * vox;
  ::cg::launch(aug_pad_kernel, dim3(aug_blocks(padded)), dim3(256), 0, st, data, (int)n, (int)a0, (int)a1, (int)a2,
               coeff);
  CG_LAUNCH_CHECK("aug_pad_kernel");
  // prefilter along a2 (stride 1), a1 (stride b2), a0 (stride b1*b2)
  const long long l2 = (long long)n * b0 * b1, l1 = (long long)n * b0 * b2, l0 = (long long)n * b1 * b2;
  ::cg::launch(aug_prefilter_kernel, dim3((unsigned)((l2 + 255) / 256)), dim3(256), 0, st, coeff, l2, b2, 1LL, 1LL,
               (long long)b2);
  ::cg::launch(aug_prefilter_kernel, dim3((unsigned)((l1 + 255) / 256)), dim3(256), 0, st, coeff, l1, b1, (long long)b2,
               (long long)b2, (long long)b1 * b2);
  if (a0 > 1)  // a 2-D patch (a0 = 1) is sampled on its plane only
    ::cg::launch(aug_prefilter_kernel, dim3((unsigned)((l0 + 255) / 256)), dim3(256), 0, st, coeff, l0, b0,
                 (long long)b1 * b2, (long long)b1 * b2, (long long)b0 * b1 * b2);
  CG_LAUNCH_CHECK("aug_prefilter_kernel");
  if (n_elastic > 0) {  // separable circular Gaussian: noise -> fa (axis 0) -> fb (axis 1) -> fa (axis 2)
    const int kst = std::max(a0, std::max(a1, a2));
    const long long fv = 3LL * n_elastic * vox;
    for (int axis = 0; axis < 3; ++axis) {
      const float* src = axis == 0 ? noise : (axis == 1 ? fa : fb);
      float* dst = axis == 1 ? fb : fa;
      ::cg::launch(aug_circconv_kernel, dim3(aug_blocks(fv)), dim3(256), 0, st, src, dst, (int)(3 * n_elastic),
                   (int)a0, (int)a1, (int)a2, axis, gauss, kst);
    }
    CG_LAUNCH_CHECK("aug_circconv_kernel");
    ::cg::launch(aug_field_stats_kernel, dim3(3 * n_elastic), dim3(1024), 0, st, (const float*)fa, vox, fstats);
    CG_LAUNCH_CHECK("aug_field_stats_kernel");
  }
  ::cg::launch(aug_sample_kernel, dim3(aug_blocks((long long)n * vox)), dim3(256), 0, st, (const float*)coeff, data,
               (const unsigned char*)seg, (int)n, (int)a0, (int)a1, (int)a2, params, (const float*)fa,
               (const float*)fstats, data_out, (unsigned char*)seg_out);
  CG_LAUNCH_CHECK("aug_sample_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_mirror(const float* data, const uint8_t* seg, int32_t n, int32_t a0, int32_t a1, int32_t a2,
                             const int32_t* flags, float* data_out, uint8_t* seg_out, void* stream) {
  CG_CHECK_ARG(data && seg && flags && data_out && seg_out && n > 0 && a0 >= 1 && a1 >= 1 && a2 >= 1,
               "cgan3d_mirror: bad args");
  CG_CHECK_ARG(data_out != data && (const void*)seg_out != (const void*)seg, "cgan3d_mirror: in place");
  ::cg::launch(aug_mirror_kernel, dim3(aug_blocks((long long)n * a0 * a1 * a2)), dim3(256), 0, (hipStream_t)stream,
               data, (const unsigned char*)seg, (int)n, (int)a0, (int)a1, (int)a2, (const int*)flags, data_out,
               (unsigned char*)seg_out);
  CG_LAUNCH_CHECK("aug_mirror_kernel");
  return CGAN3D_OK;
}
