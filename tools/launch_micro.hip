// Per-launch cost of back-to-back dependent kernels on one stream (events around N launches,
// queued behind a spin kernel so host enqueue is hidden), plain launches vs a captured hipGraph.
// build: hipcc -O3 --offload-arch=gfx950 tools/launch_micro.hip -o tools/launch_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin(long long cycles) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}
__global__ void tiny(float* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f; }
__global__ void touch(float* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1.f;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* buf;
    const int n = 1 << 22;
    CK(hipMalloc(&buf, n * 4));
    CK(hipMemset(buf, 0, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int N = 500;
    struct Case { const char* name; int grid; int kind; } cases[] = {
        {"tiny 1 block", 1, 0}, {"tiny 256 blocks", 256, 0}, {"tiny 2048 blocks", 2048, 0},
        {"touch 4M floats (16 MB rw)", n / 256, 1}, {"touch 256K floats (1 MB rw)", (1 << 18) / 256, 1}};
    for (auto& c : cases) {
        for (int rep = 0; rep < 2; ++rep) {
            auto issue = [&]() {
                for (int i = 0; i < N; ++i) {
                    if (c.kind == 0) hipLaunchKernelGGL(tiny, dim3(c.grid), dim3(256), 0, s, buf);
                    else hipLaunchKernelGGL(touch, dim3(c.grid), dim3(256), 0, s, buf, c.grid * 256);
                }
            };
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200000000LL);
            CK(hipEventRecord(a, s));
            issue();
            CK(hipEventRecord(b, s));
            CK(hipStreamSynchronize(s));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            // graph
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            issue();
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200000000LL);
            CK(hipEventRecord(a, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(b, s));
            CK(hipStreamSynchronize(s));
            float msg;
            CK(hipEventElapsedTime(&msg, a, b));
            if (rep == 1) printf("%-30s stream %.2f us/launch   graph %.2f us/launch\n", c.name, ms * 1e3 / N, msg * 1e3 / N);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    // cross-stream signalling after every launch: event record (+ a side stream waiting on it) vs
    // hipStreamWriteValue32 (+ hipStreamWaitValue32 on the side stream)
    hipStream_t side;
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    unsigned* flag;
    CK(hipMalloc(&flag, 4096));
    CK(hipMemset(flag, 0, 4096));
    for (unsigned fl : {(unsigned)hipEventDisableTiming, (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence)}) {
      hipEvent_t evs[N];
      for (int i = 0; i < N; ++i) CK(hipEventCreateWithFlags(&evs[i], fl));
      for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200000000LL);
        CK(hipEventRecord(a, s));
        for (int i = 0; i < N; ++i) {
          hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf);
          if (mode >= 1) CK(hipEventRecord(evs[i], s));
          if (mode == 2) { CK(hipStreamWaitEvent(side, evs[i], 0)); hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, side, buf + 64); }
        }
        CK(hipEventRecord(b, s));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("event flags %x mode %d (0 none, 1 record, 2 record+side wait+side kernel): %.2f us/launch\n", fl, mode, ms * 1e3 / N);
      }
      for (int i = 0; i < N; ++i) CK(hipEventDestroy(evs[i]));
    }
    for (int mode = 1; mode < 3; ++mode) {
      CK(hipMemset(flag, 0, 4096));
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200000000LL);
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf);
        CK(hipStreamWriteValue32(s, flag, i + 1, 0));
        if (mode == 2) { CK(hipStreamWaitValue32(side, flag, i + 1, hipStreamWaitValueGte, 0xffffffffu)); hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, side, buf + 64); }
      }
      CK(hipEventRecord(b, s));
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("write-value mode %d (1 write, 2 write+side wait+side kernel): %.2f us/launch\n", mode, ms * 1e3 / N);
    }
    return 0;
}
