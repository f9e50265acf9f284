// dispatch_probe.hip — graph-replayed cost of one kernel launch vs grid size / block size on
// MI355X (each thread stores one 16-byte value, so the work itself is negligible).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dispatch_probe.hip -o build/dispatch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int T>
__global__ __launch_bounds__(T) void k_touch(uint4* buf) {
  buf[(long long)blockIdx.x * T + threadIdx.x] = make_uint4(blockIdx.x, threadIdx.x, 1, 2);
}
template <int T>
__global__ __launch_bounds__(T) void k_nop(uint4* buf) {
  if (threadIdx.x == 9999) buf[0] = make_uint4(0, 0, 0, 0);
}

int main() {
  const int iters = 200;
  uint4* buf;
  CK(hipMalloc(&buf, 64 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_graph = [&](auto body) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < iters; ++i) body();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return best * 1e3f / iters;
  };
  printf("| blocks | store 64-thr us | store 256-thr us | store 1024-thr us | nop 256-thr us |\n|---:|---:|---:|---:|---:|\n");
  int grids[] = {1, 8, 16, 32, 64, 128, 256, 512, 1024, 2048};
  for (int P : grids) {
    float t64 = time_graph([&] { hipLaunchKernelGGL(k_touch<64>, dim3(P), dim3(64), 0, s, buf); });
    float t256 = time_graph([&] { hipLaunchKernelGGL(k_touch<256>, dim3(P), dim3(256), 0, s, buf); });
    float t1k = time_graph([&] { hipLaunchKernelGGL(k_touch<1024>, dim3(P), dim3(1024), 0, s, buf); });
    float tn = time_graph([&] { hipLaunchKernelGGL(k_nop<256>, dim3(P), dim3(256), 0, s, buf); });
    printf("| %d | %.2f | %.2f | %.2f | %.2f |\n", P, t64, t256, t1k, tn);
  }
  return 0;
}
