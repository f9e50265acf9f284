// graph_branch_probe.hip — do independent branches of a captured hipGraph run concurrently on
// MI355X (ROCm 7), and do two plain streams?  Each branch is one 1-block kernel that busy-waits
// ~T us on s_memrealtime (100 MHz), so concurrency shows up as total ~T instead of ~2T.
//   eager 1 stream : A ; B                       (~2T)
//   eager 2 streams: A on s1, B on s2            (~T if the queues run concurrently)
//   graph fork/join: capture s1 -> fork s2 -> A on s1, B on s2 -> join   (~T or ~2T?)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/graph_branch_probe.hip -o build/graph_branch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_spin(unsigned long long ticks, int* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(1);
    t = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = (int)(t - t0);
}

int main() {
  const unsigned long long ticks = 10000;  // 100 us at 100 MHz
  int* sink;
  CK(hipMalloc(&sink, 4096));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, fork, join;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  auto timed = [&](auto body) {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s1));
      body();
      CK(hipEventRecord(e1, s1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best * 1e3f;
  };
  const float one = timed([&] { hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, sink); });
  const float serial = timed([&] {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, sink);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, sink + 1);
  });
  const float two = timed([&] {
    CK(hipEventRecord(fork, s1));
    CK(hipStreamWaitEvent(s2, fork, 0));
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, sink);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, ticks, sink + 1);
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s1, join, 0));
  });
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
  CK(hipEventRecord(fork, s1));
  CK(hipStreamWaitEvent(s2, fork, 0));
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s1, ticks, sink);
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, ticks, sink + 1);
  CK(hipEventRecord(join, s2));
  CK(hipStreamWaitEvent(s1, join, 0));
  CK(hipStreamEndCapture(s1, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  const float graph = timed([&] { CK(hipGraphLaunch(ge, s1)); });
  // graph branch next to an eager kernel on another stream (the RCCL-outside-the-graph case)
  const float graph_vs_eager = timed([&] {
    CK(hipEventRecord(fork, s1));
    CK(hipStreamWaitEvent(s2, fork, 0));
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, ticks, sink + 2);
    CK(hipGraphLaunch(ge, s1));
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s1, join, 0));
  });
  printf("| case | us | (one spin kernel = %.1f us) |\n|---|---:|---|\n", one);
  printf("| eager, 2 kernels on one stream | %.1f | serial |\n", serial);
  printf("| eager, 2 streams | %.1f | %s |\n", two, two < 1.5f * one ? "concurrent" : "serialised");
  printf("| graph, fork/join branches (%zu nodes) | %.1f | %s |\n", nn, graph, graph < 1.5f * one ? "concurrent" : "serialised");
  printf("| graph (2 branches) + eager kernel on a 2nd stream | %.1f | %s |\n", graph_vs_eager,
         graph_vs_eager < 1.5f * one ? "all concurrent" : (graph_vs_eager < 2.5f * one ? "partly" : "serialised"));
  return 0;
}
