// Patch staging for the pinned-host -> HBM loader (cgan3d_amd/data/loader.py), replacing the
// per-sample numpy work of CCTADataLoader.generate_one (contrast_gan_3D/data/CCTADataLoader.py:
// 88-104): the host copies raw crops of the [W,H,D,(HU,label)] volumes into pinned memory; on the
// GPU one pass de-interleaves them into the scaled float patch ((HU - shift) / factor,
// data/Scaler.py:37-45) and the boolean centre-line mask (NumpyToTensor(cast_to="bool")).
#include "common.h"

namespace cg {

template <typename T>
__global__ __launch_bounds__(256) void unpack_patches_kernel(const T* __restrict__ src, long long nvox, float shift,
                                                             float factor, float* __restrict__ data,
                                                             unsigned char* __restrict__ seg) {
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvox; v += (long long)gridDim.x * blockDim.x) {
    const float hu = (float)src[2 * v], lab = (float)src[2 * v + 1];
    data[v] = (hu - shift) / factor;  // IEEE division, as the reference's float32 numpy
    seg[v] = lab != 0.f;
  }
}

// Four voxels per thread from 16-byte loads (int16 pairs: one load; float32 pairs: two), 16-byte data
// and 4-byte mask stores: the form for a source in mapped host memory, read over PCIe by a few blocks
// beside the step (cgan3d_unpack_patches_ex); the voxels past the last full quad by block 0.
template <typename T>
__global__ __launch_bounds__(256) void unpack4_patches_kernel(const T* __restrict__ src, long long nvox, float shift,
                                                              float factor, float* __restrict__ data,
                                                              unsigned char* __restrict__ seg) {
  const long long n4 = nvox >> 2;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    T v[8];
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    if constexpr (sizeof(T) == 2) {
      const uint4 u = s4[q];
      __builtin_memcpy(v, &u, 16);
    } else {
      const uint4 u0 = s4[2 * q], u1 = s4[2 * q + 1];
      __builtin_memcpy(v, &u0, 16);
      __builtin_memcpy(v + 4, &u1, 16);
    }
    float4 d;
    d.x = ((float)v[0] - shift) / factor;
    d.y = ((float)v[2] - shift) / factor;
    d.z = ((float)v[4] - shift) / factor;
    d.w = ((float)v[6] - shift) / factor;
    uchar4 m;
    m.x = (float)v[1] != 0.f;
    m.y = (float)v[3] != 0.f;
    m.z = (float)v[5] != 0.f;
    m.w = (float)v[7] != 0.f;
    reinterpret_cast<float4*>(data)[q] = d;
    reinterpret_cast<uchar4*>(seg)[q] = m;
  }
  if (blockIdx.x == 0)
    for (long long v = 4 * n4 + threadIdx.x; v < nvox; v += blockDim.x) {
      data[v] = ((float)src[2 * v] - shift) / factor;
      seg[v] = (float)src[2 * v + 1] != 0.f;
    }
}

}  // namespace cg

using namespace cg;

extern "C" int cgan3d_unpack_patches_ex(const void* src, int32_t src_dtype, int64_t nvox, float shift, float factor,
                                        float* data, uint8_t* seg, int32_t max_blocks, void* stream) {
  CG_CHECK_ARG(src && data && seg && nvox > 0 && factor != 0.f && max_blocks > 0, "cgan3d_unpack_patches_ex: bad args");
  CG_CHECK_ARG(src_dtype == 0 || src_dtype == 1, "cgan3d_unpack_patches_ex: src_dtype must be 0 (int16) or 1 (float32)");
  CG_CHECK_ARG(!(reinterpret_cast<uintptr_t>(src) & 15) && !(reinterpret_cast<uintptr_t>(data) & 15) &&
                   !(reinterpret_cast<uintptr_t>(seg) & 3),
               "cgan3d_unpack_patches_ex: src / data 16-byte and seg 4-byte aligned");
  const int blocks = (int)std::max<long long>(1, std::min<long long>((nvox / 4 + 255) / 256, max_blocks));
  if (src_dtype == 0)
    ::cg::launch(unpack4_patches_kernel<int16_t>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                 static_cast<const int16_t*>(src), (long long)nvox, shift, factor, data, seg);
  else
    ::cg::launch(unpack4_patches_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                 static_cast<const float*>(src), (long long)nvox, shift, factor, data, seg);
  CG_LAUNCH_CHECK("unpack4_patches_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_unpack_patches(const void* src, int32_t src_dtype, int64_t nvox, float shift, float factor,
                                     float* data, uint8_t* seg, void* stream) {
  CG_CHECK_ARG(src && data && seg && nvox > 0 && factor != 0.f, "cgan3d_unpack_patches: bad args");
  CG_CHECK_ARG(src_dtype == 0 || src_dtype == 1, "cgan3d_unpack_patches: src_dtype must be 0 (int16) or 1 (float32)");
  int blocks = (int)std::min<long long>((nvox + 255) / 256, 8192);
  if (src_dtype == 0)
    ::cg::launch(unpack_patches_kernel<int16_t>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const int16_t*>(src), (long long)nvox, shift, factor, data, seg);
  else
    ::cg::launch(unpack_patches_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const float*>(src), (long long)nvox, shift, factor, data, seg);
  CG_LAUNCH_CHECK("unpack_patches_kernel");
  return CGAN3D_OK;
}

// ---- whole-scan inference (eval/CCTAContrastCorrector.py, reference eval/CCTAContrastCorrector.py:
// 60-81, patchly GridSampler + Aggregator): overlapping grid patches of the corrected scan are
// averaged.  out / weight accumulate every patch (fp32 atomics: the squeezed last patch of a dim
// overlaps its neighbour within one batch); cgan3d_patch_normalize divides.
namespace cg {

__global__ __launch_bounds__(256) void patch_accumulate_kernel(const float* __restrict__ patch, int b, int p0, int p1,
                                                               int p2, const int* __restrict__ org, float* out,
                                                               float* weight, int s0, int s1, int s2) {
  const long long pv = (long long)p0 * p1 * p2, tot = pv * b;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i / pv);
    const long long v = i - (long long)k * pv;
    const int x2 = (int)(v % p2), x1 = (int)((v / p2) % p1), x0 = (int)(v / ((long long)p1 * p2));
    const long long o = ((long long)(org[3 * k] + x0) * s1 + (org[3 * k + 1] + x1)) * s2 + (org[3 * k + 2] + x2);
    atomicAdd(out + o, patch[i]);
    atomicAdd(weight + o, 1.f);
  }
}

__global__ __launch_bounds__(256) void patch_normalize_kernel(float* out, const float* __restrict__ weight, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = out[i] / weight[i];
}

}  // namespace cg

extern "C" int cgan3d_patch_accumulate(const float* patch, int32_t b, int32_t p0, int32_t p1, int32_t p2,
                                       const int32_t* origins, float* out, float* weight, int32_t s0, int32_t s1,
                                       int32_t s2, void* stream) {
  CG_CHECK_ARG(patch && origins && out && weight && b > 0 && p0 > 0 && p1 > 0 && p2 > 0 && p0 <= s0 && p1 <= s1 &&
               p2 <= s2, "cgan3d_patch_accumulate: bad args");
  const long long tot = (long long)b * p0 * p1 * p2;
  ::cg::launch(patch_accumulate_kernel, dim3((int)std::min<long long>((tot + 255) / 256, 16384)), dim3(256), 0,
               (hipStream_t)stream, patch, (int)b, (int)p0, (int)p1, (int)p2, (const int*)origins, out, weight,
               (int)s0, (int)s1, (int)s2);
  CG_LAUNCH_CHECK("patch_accumulate_kernel");
  return CGAN3D_OK;
}

extern "C" int cgan3d_patch_normalize(float* out, const float* weight, int64_t n, void* stream) {
  CG_CHECK_ARG(out && weight && n > 0, "cgan3d_patch_normalize: bad args");
  ::cg::launch(patch_normalize_kernel, dim3((int)std::min<long long>((n + 255) / 256, 16384)), dim3(256), 0,
               (hipStream_t)stream, out, weight, (long long)n);
  CG_LAUNCH_CHECK("patch_normalize_kernel");
  return CGAN3D_OK;
}
