// comm.hip — one-shot all-reduce for small buffers over peer-mapped HBM (gfx950, xGMI).
//
// RCCL's ring/tree all-reduce pays 2(P-1) latency-bound steps; for the small buffers of this
// framework (LeNet's 60k parameters, packed BN statistics of a K-AVG round, loss / count
// scalars) that latency is the whole cost.  The one-shot form: every rank
// exposes one IPC-shared region in its HBM, copies its input into it, tells every peer
// "epoch e is ready" with one system-scope store into the peer's flag slot, and then reads the
// P inputs straight over the fully connected xGMI links and sums them — one hop, no ring.
// The P inputs are summed in rank order on every rank, so all ranks get bit-identical sums.
//
// Region of rank r (hipMalloc, shared with hipIpcGetMemHandle):
//   [0, 256)                 uint32 flags[64]: flags[p] = last epoch peer p published
//   [256, 256 + cap)         slot 0   (double buffer selected by epoch parity)
//   [256 + cap, 256 + 2 cap) slot 1
// Local control block (not shared): epoch, block ticket, give-up counter.
//
// Two stream-ordered launches per call (both graph-capturable; the epoch lives on the device):
//   k_os_copyin : in -> own slot[(epoch + 1) & 1]
//   k_os_reduce : block 0 publishes epoch + 1 to every peer's flags[rank] (release, system
//                 scope); every block waits until all flags >= epoch + 1 (acquire), sums its
//                 range of the P slots into out; the last block to finish advances the epoch.
// Slot reuse is safe with two slots: a rank overwrites slot s again only two calls later,
// after every peer has published the call in between — which each peer does only after its
// reads of slot s (previous call, same stream) have completed.
// No deadlock: a waiting block only needs its peers' block 0 (the first block they dispatch)
// to run, never another block of its own grid.  The spin is bounded: after ~2^22 polls (~1 s)
// the block gives up, counts the failure in ctrl[2] and proceeds (wrong sums, no hang);
// the host checks the counter (kml_oneshot_errors).
#include "kml_common.h"

namespace {

constexpr int OS_MAX_RANKS = 8;
constexpr int OS_FLAGS_BYTES = 256;
constexpr unsigned OS_SPIN_LIMIT = 1u << 22;

struct OsPeers {
  const char* region[OS_MAX_RANKS];  // every rank's region, mapped into this process
};

// system-coherent 4-byte accesses: the slot bytes cross the xGMI link while other XCDs'
// L2s of the owner may still hold them, so stores write through (sc0 sc1) and peer loads
// bypass the caches — no L2 write-back / invalidate of whole XCD caches is needed
__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM));
}

__global__ __launch_bounds__(256) void k_os_copyin(const float* __restrict__ in, char* __restrict__ region,
                                                   const unsigned* __restrict__ ctrl, long long cap, long long n) {
  const unsigned e1 = ctrl[0] + 1u;
  float* dst = reinterpret_cast<float*>(region + OS_FLAGS_BYTES + (e1 & 1u) * cap);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) st_sys(dst + i, in[i]);
}

__global__ __launch_bounds__(256) void k_os_reduce(float* __restrict__ out, OsPeers peers, char* __restrict__ region,
                                                   unsigned* __restrict__ ctrl, int rank, int world, long long cap,
                                                   long long n, float scale) {
  __shared__ unsigned e1_sh;
  if (threadIdx.x == 0) e1_sh = __hip_atomic_load(ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned e1 = e1_sh;
  unsigned* flags = reinterpret_cast<unsigned*>(region);
  if (blockIdx.x == 0 && (int)threadIdx.x < world) {
    // this rank's slot for epoch e1 is complete (k_os_copyin finished: stream order)
    unsigned* peer_flags = reinterpret_cast<unsigned*>(const_cast<char*>(peers.region[threadIdx.x]));
    __hip_atomic_store(peer_flags + rank, e1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    unsigned polls = 0;
    for (int p = 0; p < world; ++p) {
      while (__hip_atomic_load(flags + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e1 > 0x7fffffffu &&
             polls < OS_SPIN_LIMIT) {  // wrap-safe "flag < e1"
        __builtin_amdgcn_s_sleep(2);
        ++polls;
      }
    }
    if (polls >= OS_SPIN_LIMIT) __hip_atomic_fetch_add(ctrl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const long long off = OS_FLAGS_BYTES + (long long)(e1 & 1u) * cap;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int p = 0; p < world; ++p)  // rank order on every rank: identical sums everywhere
      acc += ld_sys(reinterpret_cast<const float*>(peers.region[p] + off) + i);
    out[i] = acc * scale;
  }
  // the last block to finish advances the epoch (every block has read it at its start)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctrl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(ctrl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl, e1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

// ---- IPC regions ---------------------------------------------------------------------
KML_API int kml_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// region (flags + 2 slots of cap bytes) + zeroed local control block [epoch, ticket, errors]
KML_API int kml_oneshot_alloc(long long cap, void** region, void** ctrl) {
  if (cap <= 0 || cap % 16) return (int)hipErrorInvalidValue;
  *region = nullptr;
  *ctrl = nullptr;
  hipError_t e = hipMalloc(region, OS_FLAGS_BYTES + 2 * cap);
  if (e == hipSuccess) e = hipMemset(*region, 0, OS_FLAGS_BYTES);
  if (e == hipSuccess) e = hipMalloc(ctrl, 64);
  if (e == hipSuccess) e = hipMemset(*ctrl, 0, 64);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {  // nothing half-allocated survives a failure
    if (*region) (void)hipFree(*region);
    if (*ctrl) (void)hipFree(*ctrl);
    *region = *ctrl = nullptr;
  }
  return (int)e;
}

KML_API int kml_oneshot_free(void* region, void* ctrl) {
  hipError_t e = hipSuccess;
  if (region) e = hipFree(region);
  if (ctrl) {
    const hipError_t e2 = hipFree(ctrl);
    if (e == hipSuccess) e = e2;
  }
  return (int)e;
}

KML_API int kml_ipc_get_handle(void* ptr, void* handle_out) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), ptr);
}

KML_API int kml_ipc_open(const void* handle, void** ptr_out) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr_out, h, hipIpcMemLazyEnablePeerAccess);
}

KML_API int kml_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// give-up count of the bounded spins so far (host-side health check; synchronises)
KML_API int kml_oneshot_errors(const void* ctrl, unsigned* out) {
  return (int)hipMemcpy(out, reinterpret_cast<const unsigned*>(ctrl) + 2, sizeof(unsigned), hipMemcpyDeviceToHost);
}

// out = scale * sum over ranks of in (n floats, n * 4 <= cap); regions[world]: every rank's
// region as mapped in this process (own region at [rank]).  in and out may alias.
KML_API int kml_oneshot_allreduce(const float* in, float* out, const void* const* regions, void* region, void* ctrl,
                                  int rank, int world, long long cap, long long n, float scale, hipStream_t s) {
  if (world < 1 || world > OS_MAX_RANKS || rank < 0 || rank >= world || n < 0 || n * 4 > cap || cap % 16)
    return (int)hipErrorInvalidValue;
  OsPeers peers = {};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return (int)hipErrorInvalidValue;
    peers.region[p] = reinterpret_cast<const char*>(regions[p]);
  }
  if (peers.region[rank] != region) return (int)hipErrorInvalidValue;
  unsigned grid = (unsigned)((n + 1023) / 1024);
  if (grid < 1) grid = 1;
  if (grid > 128) grid = 128;
  hipLaunchKernelGGL(k_os_copyin, dim3(grid), dim3(256), 0, s, in, reinterpret_cast<char*>(region),
                     reinterpret_cast<const unsigned*>(ctrl), cap, n);
  hipLaunchKernelGGL(k_os_reduce, dim3(grid), dim3(256), 0, s, out, peers, reinterpret_cast<char*>(region),
                     reinterpret_cast<unsigned*>(ctrl), rank, world, cap, n, scale);
  KML_LAUNCH_CHECK();
}
