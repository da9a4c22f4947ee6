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

}  // namespace cg

using namespace cg;

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
