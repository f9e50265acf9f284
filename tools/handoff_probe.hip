// handoff_probe.hip — is one launch with an in-kernel producer->consumer hand-off cheaper than
// two dependent graph-captured launches on MI355X?
//
// Producer: P blocks each write `bytes/P` (bf16-sized payload, 16-byte stores).
// Consumer: P blocks each read a DIFFERENT block's share (crosses XCDs) and write it back.
//   two   : k_prod ; k_cons                       (graph edge between them)
//   fence : one launch, producers release (agent fence) + ticket, consumers spin then acquire
//   wt    : one launch, producers store write-through (agent-scope relaxed stores), consumers
//           load with agent-scope loads; ticket hand-off without fences
// Consumers have HIGHER block indices than every producer, so under in-order workgroup
// dispatch a spinning consumer never blocks a producer; the spin is also bounded (gives up
// after ~2^24 polls and flags an error) so a broken assumption cannot hang the GPU.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/handoff_probe.hip -o build/handoff_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void produce(uint4* buf, int blk, int per, int tid) {
  for (int i = tid; i < per; i += 256) buf[(long long)blk * per + i] = make_uint4(blk, i, 1, 2);
}

__global__ __launch_bounds__(256) void k_prod(uint4* buf, int per) { produce(buf, blockIdx.x, per, threadIdx.x); }

__global__ __launch_bounds__(256) void k_cons(const uint4* buf, uint4* out, int per, int P) {
  const int src = (blockIdx.x * 37 + 11) % P;
  for (int i = threadIdx.x; i < per; i += 256) {
    uint4 v = buf[(long long)src * per + i];
    v.x += 1;
    out[(long long)blockIdx.x * per + i] = v;
  }
}

__global__ __launch_bounds__(256) void k_empty() {}

__device__ bool wait_count(unsigned* cnt, unsigned target, unsigned* err) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    unsigned polls = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++polls < (1u << 24))
      __builtin_amdgcn_s_sleep(1);
    ok = polls < (1u << 24);
    if (!ok) atomicAdd(err, 1u);
  }
  __syncthreads();
  return ok;
}

__device__ void finish_waiter(unsigned* cnt, int P) {
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)P - 1) {  // every producer done and every consumer past the wait
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <bool WT>
__global__ __launch_bounds__(256) void k_fused(uint4* buf, uint4* out, int per, int P, unsigned* cnt, unsigned* err) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < P) {
    const int blk = blockIdx.x;
    if (WT) {
      for (int i = tid; i < per; i += 256) {
        unsigned* p = reinterpret_cast<unsigned*>(buf + (long long)blk * per + i);
        __hip_atomic_store(p + 0, (unsigned)blk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 1, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 3, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      produce(buf, blk, per, tid);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores issued to L2
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int c = blockIdx.x - P;
  if (!wait_count(cnt, (unsigned)P, err)) return;
  if (!WT) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // agent-scope acquire: L2 invalidate
  const int src = (c * 37 + 11) % P;
  for (int i = tid; i < per; i += 256) {
    uint4 v;
    if (WT) {
      unsigned* p = reinterpret_cast<unsigned*>(buf + (long long)src * per + i);
      v.x = __hip_atomic_load(p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.z = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v.w = __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      v = buf[(long long)src * per + i];
    }
    v.x += 1;
    out[(long long)c * per + i] = v;
  }
  finish_waiter(cnt, P);
}

int main(int argc, char** argv) {
  const int iters = 200;
  int sizes_kb[] = {128, 512, 2048, 8192};
  int blocks[] = {16, 64, 256};
  uint4 *buf, *out;
  unsigned *cnt, *err;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMalloc(&out, 64 << 20));
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&err, 64));
  CK(hipMemset(cnt, 0, 64));
  CK(hipMemset(err, 0, 64));
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
    return best * 1e3f / iters;  // us per iteration
  };
  printf("empty pair (2 launches): %.2f us\n", time_graph([&] {
           hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s);
           hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s);
         }));
  printf("empty single launch: %.2f us\n", time_graph([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s); }));
  printf("| KB | P | two launches us | fused fence us | fused write-through us |\n|---:|---:|---:|---:|---:|\n");
  for (int kb : sizes_kb)
    for (int P : blocks) {
      const int per = (kb << 10) / 16 / P;
      if (per < 1) continue;
      float t2 = time_graph([&] {
        hipLaunchKernelGGL(k_prod, dim3(P), dim3(256), 0, s, buf, per);
        hipLaunchKernelGGL(k_cons, dim3(P), dim3(256), 0, s, buf, out, per, P);
      });
      float tf = time_graph([&] {
        hipLaunchKernelGGL(k_fused<false>, dim3(2 * P), dim3(256), 0, s, buf, out, per, P, cnt, err);
      });
      float tw = time_graph([&] {
        hipLaunchKernelGGL(k_fused<true>, dim3(2 * P), dim3(256), 0, s, buf, out, per, P, cnt, err);
      });
      printf("| %d | %d | %.2f | %.2f | %.2f |\n", kb, P, t2, tf, tw);
    }
  unsigned herr = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("spin give-ups: %u\n", herr);
  return herr ? 3 : 0;
}
