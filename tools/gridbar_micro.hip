// Cost of a grid-wide barrier inside a persistent kernel against a kernel boundary, on the shape of
// the critic's layer chain: every phase reads another block's chunk of the previous phase's output
// (cross-XCD: block b reads block (b + 37) % NB) and writes its own chunk, then all blocks sync.
//   A: one launch per phase (the kernel boundary is the barrier)
//   B: one persistent launch, NB resident blocks, an agent-scope counter barrier between phases
//      (release: every wave drained + __syncthreads + one lane's release-add; acquire: that lane
//      spins with an acquire load and s_sleep, then __syncthreads) — cdna_hip_programming.md G16
// Every phase checks the values it reads (stale data from a missing fence counts as an error).
// build: hipcc -O3 --offload-arch=gfx950 tools/gridbar_micro.hip -o tools/gridbar_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ float val(int p, int b, int i) { return (float)((p * 131 + b * 7 + i) & 0xffff); }

__device__ __forceinline__ void phase_work(float4* buf, int p, int b, int NB, int chunk4, unsigned* err) {
  const int tid = threadIdx.x;
  if (p > 0) {  // read another block's chunk of phase p - 1
    const int o = (b + 37) % NB;
    const float4* src = buf + (size_t)((p - 1) & 1) * NB * chunk4 + (size_t)o * chunk4;
    unsigned bad = 0;
    for (int i = tid; i < chunk4; i += blockDim.x) {
      float4 v = src[i];
      bad += v.x != val(p - 1, o, 4 * i) || v.w != val(p - 1, o, 4 * i + 3);
    }
    if (bad) atomicAdd(err, bad);
  }
  float4* dst = buf + (size_t)(p & 1) * NB * chunk4 + (size_t)b * chunk4;
  for (int i = tid; i < chunk4; i += blockDim.x)
    dst[i] = make_float4(val(p, b, 4 * i), val(p, b, 4 * i + 1), val(p, b, 4 * i + 2), val(p, b, 4 * i + 3));
}

__global__ __launch_bounds__(256) void per_launch(float4* buf, int p, int chunk4, unsigned* err) {
  phase_work(buf, p, blockIdx.x, gridDim.x, chunk4, err);
}

// SPIN 0: acquire load per poll (an L2 invalidate each); 1: relaxed polls, one acquire fence after
template <int SPIN>
__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned target) {
  __syncthreads();  // every wave's stores issued; the release below waits for them (vmcnt) and writes back L2
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    if (SPIN == 0) {
      while (__hip_atomic_load(count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 20)) break;  // bounded: a stranded block cannot hang the GPU
      }
    } else {
      while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 20)) break;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  __syncthreads();
}

template <int SPIN>
__global__ __launch_bounds__(256) void persistent(float4* buf, int P, int chunk4, unsigned* err, unsigned* count) {
  for (int p = 0; p < P; ++p) {
    phase_work(buf, p, blockIdx.x, gridDim.x, chunk4, err);
    grid_barrier<SPIN>(count, (unsigned)(p + 1) * gridDim.x);
  }
}

int main(int argc, char** argv) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("CUs %d\n", prop.multiProcessorCount);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  unsigned *err, *count;
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&count, 4));
  const int P = 200;
  for (int NB : {256, 512}) {
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent<1>, 256, 0));
    if (occ * prop.multiProcessorCount < NB) { printf("NB %d not co-resident (occ %d)\n", NB, occ); continue; }
    for (int kb : {0, 4, 64}) {  // bytes per block per phase: 0 (barrier only), 4 KB, 64 KB
      const int chunk4 = kb * 1024 / 16;
      float4* buf;
      CK(hipMalloc(&buf, (size_t)2 * NB * (chunk4 > 0 ? chunk4 : 1) * 16));
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(err, 0, 4));
        CK(hipEventRecord(a, s));
        for (int p = 0; p < P; ++p) hipLaunchKernelGGL(per_launch, dim3(NB), dim3(256), 0, s, buf, p, chunk4, err);
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
        float ms_a;
        CK(hipEventElapsedTime(&ms_a, a, b));
        unsigned e_a;
        CK(hipMemcpy(&e_a, err, 4, hipMemcpyDeviceToHost));
        float ms_b[2];
        unsigned e_b[2], c[2];
        for (int spin = 0; spin < 2; ++spin) {
          CK(hipMemset(err, 0, 4));
          CK(hipMemset(count, 0, 4));
          CK(hipEventRecord(a, s));
          if (spin == 0) hipLaunchKernelGGL(persistent<0>, dim3(NB), dim3(256), 0, s, buf, P, chunk4, err, count);
          else hipLaunchKernelGGL(persistent<1>, dim3(NB), dim3(256), 0, s, buf, P, chunk4, err, count);
          CK(hipEventRecord(b, s));
          CK(hipStreamSynchronize(s));
          CK(hipEventElapsedTime(&ms_b[spin], a, b));
          CK(hipMemcpy(&e_b[spin], err, 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(&c[spin], count, 4, hipMemcpyDeviceToHost));
        }
        if (rep)
          printf("NB %3d, %2d KB/block/phase: per-launch %.2f us/phase (err %u) | persistent acquire-spin %.2f us "
                 "(err %u, count %u) | relaxed-spin %.2f us (err %u, count %u)\n",
                 NB, kb, 1e3 * ms_a / P, e_a, 1e3 * ms_b[0] / P, e_b[0], c[0], 1e3 * ms_b[1] / P, e_b[1], c[1]);
      }
      CK(hipFree(buf));
    }
  }
  return 0;
}
