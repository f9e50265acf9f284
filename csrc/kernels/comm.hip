// comm.hip — peer-memory all-reduce over IPC-mapped HBM (gfx950, xGMI), graph-capturable.
//
// Every rank of a one-node group exposes ONE IPC-shared region in its HBM; every peer maps it,
// so on the fully connected xGMI mesh a rank reads any peer's bytes directly.
// Two algorithms share the region and the synchronisation protocol:
//
//   one-shot  (small buffers: LeNet's parameters, BN statistics, loss / count scalars)
//     copy-in   in -> own slot
//     reduce    barrier; read all P slots over xGMI, sum in rank order -> out
//     bytes read per rank: P * n     latency: ONE barrier
//
//   two-shot  (large buffers: the 87 MB ResNet-34 gradient; reduce-scatter + all-gather)
//     copy-in   in -> own slot (fp32, or rounded to bf16 = half the link bytes)
//     rs        barrier; rank r sums chunk r of all P slots (rank order) -> own slot chunk r + out
//     ag        barrier; rank r reads chunk q of peer q's slot for every q != r -> out
//     bytes read per rank: 2 (P-1)/P * n (the ring optimum)     latency: TWO barriers
//
// Chunk q is reduced by rank q alone and copied verbatim by the others, so every rank ends with
// bit-identical values (also with the bf16 wire: a rank's own chunk is widened from the same
// rounded bf16 it publishes).  Every launch takes a block cap: at the end of a step the whole
// chip may move bytes; beside a running backward the cap keeps the collective on a few CUs.
//
// Region of rank r (hipMalloc, shared with hipIpcGetMemHandle):
//   [0, 256)                 uint32 flags[64]: flags[p] = barrier sequence number peer p reached
//   [256, 256 + cap)         slot 0 (double buffer selected by call parity)
//   [256 + cap, 256 + 2 cap) slot 1
// Local control block (not shared), uint32: [0] seq (barriers passed) [1] block ticket
// [2] failures [3] calls.
//
// Barrier b of a call: block 0 of the launch stores seq + b into every peer's flags[rank]
// (release, system scope); thread 0 of every block polls its own flags until all P are
// >= seq + b (wrap-safe), then a system-scope acquire.  The last block of a call's final launch
// advances seq and calls (stream order makes the new values visible to the next launch).
// Slot reuse is safe with two slots: a rank rewrites slot s two calls later, after passing the
// next call's first barrier, which every peer enters only after its reads of slot s finished.
// No deadlock: a waiting block needs only its peers' block 0 (the first block they dispatch).
//
// Failure is loud, never a silent wrong sum: a wait is bounded by wall time (s_memrealtime,
// 100 MHz); on expiry the call writes NaN to its output range AND to the slot bytes peers would
// read from it, and counts the failure in ctrl[2].  A group with a failure is poisoned: every
// later call skips the waits (still publishing its flags) and writes NaN, so a late peer reads NaN
// rather than stale bytes; the host turns ctrl[2] != 0 into an error at its next check
// (kml_peer_errors).
//
// All payload bytes a peer reads are stored write-through at system scope (sc0 sc1) and read
// with system-scope loads (buffer_load ... sc0 sc1), so no L2 of either GPU can serve stale
// lines; the 16-byte forms keep the link traffic at full width.
#include "kml_common.h"

namespace {

constexpr int PC_MAX_RANKS = 8;
constexpr int PC_FLAGS_BYTES = 256;
constexpr int PC_BLOCK = 256;
constexpr int PC_AUX_SYS = 17;  // cache-policy bits sc0 | sc1: system-coherent access
enum { C_SEQ = 0, C_TICKET = 1, C_ERR = 2, C_CALLS = 3 };

struct PcPeers {
  const char* region[PC_MAX_RANKS];  // every rank's region, mapped into this process
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pc_rsrc(const char* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), (short)0, (int)bytes, 0x00020000);
}

// ---- wire formats: one 16-byte vector = 4 fp32 or 8 bf16 ---------------------------------
template <bool BF16>
struct Wire;
template <>
struct Wire<false> {
  static constexpr int VE = 4;
  __device__ static uint4 pack(const float (&x)[4]) {
    return make_uint4(__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3]));
  }
  __device__ static void unpack(uint4 w, float (&x)[4]) {
    x[0] = __uint_as_float(w.x);
    x[1] = __uint_as_float(w.y);
    x[2] = __uint_as_float(w.z);
    x[3] = __uint_as_float(w.w);
  }
};
template <>
struct Wire<true> {
  static constexpr int VE = 8;
  __device__ static uint4 pack(const float (&x)[8]) {
    return make_uint4(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]), pack_bf2(x[4], x[5]), pack_bf2(x[6], x[7]));
  }
  __device__ static void unpack(uint4 w, float (&x)[8]) {
    x[0] = lo_bf(w.x), x[1] = hi_bf(w.x), x[2] = lo_bf(w.y), x[3] = hi_bf(w.y);
    x[4] = lo_bf(w.z), x[5] = hi_bf(w.z), x[6] = lo_bf(w.w), x[7] = hi_bf(w.w);
  }
};

__device__ __forceinline__ uint4 ld_sys16(__amdgpu_buffer_rsrc_t r, long long off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, PC_AUX_SYS);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_sys16(__amdgpu_buffer_rsrc_t r, long long off, uint4 w) {
  __attribute__((ext_vector_type(4))) unsigned v = {w.x, w.y, w.z, w.w};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, PC_AUX_SYS);
}

// VE fp32 values of `in` starting at element e (zero beyond n); 16-byte loads when aligned
template <int VE>
__device__ __forceinline__ void load_in(const float* __restrict__ in, long long e, long long n, bool aligned,
                                        float (&x)[VE]) {
  if (aligned && e + VE <= n) {
#pragma unroll
    for (int j = 0; j < VE; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(in + e + j);
      x[j] = v.x, x[j + 1] = v.y, x[j + 2] = v.z, x[j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < VE; ++j) x[j] = (e + j < n) ? in[e + j] : 0.f;
  }
}

template <int VE>
__device__ __forceinline__ void store_out(float* __restrict__ out, long long e, long long n, bool aligned,
                                          const float (&x)[VE], float scale) {
  if (aligned && e + VE <= n) {
#pragma unroll
    for (int j = 0; j < VE; j += 4)
      *reinterpret_cast<float4*>(out + e + j) =
          make_float4(x[j] * scale, x[j + 1] * scale, x[j + 2] * scale, x[j + 3] * scale);
  } else {
#pragma unroll
    for (int j = 0; j < VE; ++j)
      if (e + j < n) out[e + j] = x[j] * scale;
  }
}

// Barrier `target` (= seq + b): block 0 publishes, every block's thread 0 waits; returns whether
// every peer arrived in time (false at once when the group is already poisoned).
__device__ bool pc_barrier(const PcPeers& peers, const char* region, unsigned* ctrl, int rank, int world,
                           unsigned target, unsigned long long limit_ticks) {
  __shared__ int ok_sh;
  if (blockIdx.x == 0 && (int)threadIdx.x < world) {
    // every payload byte this rank published before this launch was stored write-through
    // and completed in stream order; the release orders the flag after them
    unsigned* peer_flags = reinterpret_cast<unsigned*>(const_cast<char*>(peers.region[threadIdx.x]));
    __hip_atomic_store(peer_flags + rank, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    int ok = __hip_atomic_load(ctrl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    const unsigned* flags = reinterpret_cast<const unsigned*>(region);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < world && ok; ++p) {
      while ((int)(__hip_atomic_load(flags + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (!ok) __hip_atomic_fetch_add(ctrl + C_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // acquire at system scope: nothing this CU caches of the peers' regions survives
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok_sh = ok;
  }
  __syncthreads();
  return ok_sh != 0;
}

// the last block of a call's final launch advances the barrier sequence and the call count
// (and, when timing, stamps the collective's end)
__device__ void pc_finish_call(unsigned* ctrl, unsigned barriers, unsigned long long* stamp = nullptr) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctrl + C_TICKET, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      if (stamp) *stamp = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_store(ctrl + C_TICKET, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned s = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned c = __hip_atomic_load(ctrl + C_CALLS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl + C_CALLS, c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl + C_SEQ, s + barriers, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ const char* slot_of(const char* region, unsigned calls, long long cap) {
  return region + PC_FLAGS_BYTES + (long long)(calls & 1u) * cap;
}

// ---- K-AVG rounds on the two-shot: the model average fused into the collective -------------
// (parallel/kavg.py; reference merge ml/pkg/model/model.go:249-302, parallelSGD.go:26-54).  The
// state buffer's count slot (each rank's participation, 0 or 1) is also published in a word of
// the flags area per slot parity, so every block can form the divisor right after the call's
// first barrier without waiting for the rank that owns the count slot's chunk: the sum is taken
// in rank order like the payload, so every rank and every block gets the same divisor.  The
// epilogue then stores x * (1 / max(count, 1)) below the count slot (the raw sum at and above
// it, as the unfused all-reduce + kml_kavg_finish pair leaves them), refreshes the bf16 shadow of
// the parameter range and floors the int64 counters back into their arena — the finish pass
// over the whole state disappears.
constexpr int PC_KAVG_WORD = 32;  // flags-area words 32 / 33 (flags[p] uses words 0..7)

struct PcKavg {
  long long count_idx = -1;  // < 0: not a K-AVG call
  long long n_params = 0;    // shadow refreshed for [0, n_params)
  bf16_t* shadow = nullptr;
  long long* i64 = nullptr;  // int64 counters of [i64_off, i64_off + n_i64)
  long long i64_off = 0;
  int n_i64 = 0;
  int shadow_aligned = 0;    // 8-byte aligned shadow: 4-element packed stores
};

__device__ __forceinline__ unsigned* kavg_word(const char* region, unsigned calls) {
  return reinterpret_cast<unsigned*>(const_cast<char*>(region)) + PC_KAVG_WORD + (calls & 1u);
}

// after the call's first barrier: {1 / max(count, 1), count}, the count summed in rank order
template <int P>
__device__ float2 kavg_divisor(const PcPeers& peers, unsigned calls) {
  __shared__ float2 sh;
  if (threadIdx.x == 0) {
    float c = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p)
      c += __uint_as_float(
          __hip_atomic_load(kavg_word(peers.region[p], calls), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    sh = make_float2(1.f / fmaxf(c, 1.f), c);
  }
  __syncthreads();
  return sh;
}

// the K-AVG epilogue for 4 fp32 sums at element e (products rounded on their own: no FMA
// contraction into the counters' +1e-3, matching kml_kavg_finish bit for bit)
__device__ __forceinline__ void kavg_store(float* __restrict__ out, long long e, long long n, bool aligned,
                                           const float (&x)[4], float inv, const PcKavg& k) {
  float y[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) y[j] = (e + j < k.count_idx) ? __fmul_rn(x[j], inv) : x[j];
  store_out<4>(out, e, n, aligned, y, 1.f);
  if (k.shadow && e < k.n_params) {
    if (k.shadow_aligned && e + 4 <= k.n_params) {
      uint2 sv;
      sv.x = pack_bf2(y[0], y[1]);
      sv.y = pack_bf2(y[2], y[3]);
      *reinterpret_cast<uint2*>(k.shadow + e) = sv;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < k.n_params) k.shadow[e + j] = f2bf(y[j]);
    }
  }
  if (k.i64) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long q = e + j - k.i64_off;
      if (q >= 0 && q < k.n_i64) k.i64[q] = (long long)floorf(__fadd_rn(y[j], 1e-3f));
    }
  }
}

// in (n fp32) -> own slot as nvec wire vectors (zero padding beyond n)
template <bool BF16>
__global__ __launch_bounds__(PC_BLOCK) void k_pc_copyin(const float* __restrict__ in, char* __restrict__ region,
                                                        const unsigned* __restrict__ ctrl, long long cap, long long n,
                                                        long long nvec, int aligned, long long count_idx = -1) {
  using W = Wire<BF16>;
  constexpr int VE = W::VE;
  const unsigned calls = __hip_atomic_load(ctrl + C_CALLS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // a poisoned rank publishes NaN, so a late peer reading this slot cannot sum stale bytes
  const bool poisoned = __hip_atomic_load(ctrl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  const auto r = pc_rsrc(slot_of(region, calls, cap), cap);
  if (count_idx >= 0 && blockIdx.x == 0 && threadIdx.x == 0)  // K-AVG: this rank's count, per parity
    __hip_atomic_store(kavg_word(region, calls), __float_as_uint(poisoned ? __builtin_nanf("") : in[count_idx]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float x[VE];
    load_in<VE>(in, v * VE, n, aligned != 0, x);
    if (poisoned)
#pragma unroll
      for (int j = 0; j < VE; ++j) x[j] = __builtin_nanf("");
    st_sys16(r, v * 16, W::pack(x));
  }
}

// one-shot: out[0, n) = scale * sum over ranks (rank order) of the slots' first nvec vectors
template <bool BF16, int P>
__global__ __launch_bounds__(PC_BLOCK) void k_pc_oneshot(float* __restrict__ out, PcPeers peers, char* region,
                                                         unsigned* ctrl, int rank, long long cap, long long n,
                                                         long long nvec, float scale, int aligned,
                                                         unsigned long long limit) {
  using W = Wire<BF16>;
  constexpr int VE = W::VE;
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned calls = __hip_atomic_load(ctrl + C_CALLS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = pc_barrier(peers, region, ctrl, rank, P, seq + 1u, limit);
  __amdgpu_buffer_rsrc_t rs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) rs[p] = pc_rsrc(slot_of(peers.region[p], calls, cap), cap);
  const auto own = pc_rsrc(slot_of(region, calls, cap), cap);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float acc[VE];
    if (ok) {
      uint4 w[P];
#pragma unroll
      for (int p = 0; p < P; ++p) w[p] = ld_sys16(rs[p], v * 16);
      W::unpack(w[0], acc);
#pragma unroll
      for (int p = 1; p < P; ++p) {
        float x[VE];
        W::unpack(w[p], x);
#pragma unroll
        for (int j = 0; j < VE; ++j) acc[j] += x[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < VE; ++j) acc[j] = __builtin_nanf("");
      st_sys16(own, v * 16, W::pack(acc));  // a late peer reads NaN, never a stale slot
    }
    store_out<VE>(out, v * VE, n, aligned != 0, acc, scale);
  }
  pc_finish_call(ctrl, 1u);
}

// two-shot, reduce-scatter: chunk `rank` (cv vectors) summed over the P slots in rank order,
// published back into the own slot (write-through) and widened into out
template <bool BF16, int P, bool KAVG = false>
__global__ __launch_bounds__(PC_BLOCK) void k_pc_rs(float* __restrict__ out, PcPeers peers, char* region,
                                                    unsigned* ctrl, int rank, long long cap, long long n, long long cv,
                                                    float scale, int aligned, unsigned long long limit,
                                                    PcKavg kv = PcKavg{}) {
  using W = Wire<BF16>;
  constexpr int VE = W::VE;
  static_assert(!KAVG || !BF16, "K-AVG rounds use the fp32 wire");
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned calls = __hip_atomic_load(ctrl + C_CALLS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = pc_barrier(peers, region, ctrl, rank, P, seq + 1u, limit);
  float inv = 1.f;
  if constexpr (KAVG) inv = kavg_divisor<P>(peers, calls).x;
  __amdgpu_buffer_rsrc_t rs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) rs[p] = pc_rsrc(slot_of(peers.region[p], calls, cap), cap);
  const auto own = pc_rsrc(slot_of(region, calls, cap), cap);
  const long long base = (long long)rank * cv;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < cv; v += stride) {
    const long long g = base + v;  // global vector index
    float acc[VE];
    if (ok) {
      uint4 w[P];
#pragma unroll
      for (int p = 0; p < P; ++p) w[p] = ld_sys16(rs[p], g * 16);
      W::unpack(w[0], acc);
#pragma unroll
      for (int p = 1; p < P; ++p) {
        float x[VE];
        W::unpack(w[p], x);
#pragma unroll
        for (int j = 0; j < VE; ++j) acc[j] += x[j];
      }
      const uint4 red = W::pack(acc);
      st_sys16(own, g * 16, red);
      W::unpack(red, acc);  // the exact wire value every peer will read
    } else {
#pragma unroll
      for (int j = 0; j < VE; ++j) acc[j] = __builtin_nanf("");
      st_sys16(own, g * 16, W::pack(acc));  // peers gathering this chunk read NaN
    }
    if constexpr (KAVG)
      kavg_store(out, g * VE, n, aligned != 0, acc, inv, kv);
    else
      store_out<VE>(out, g * VE, n, aligned != 0, acc, scale);
  }
}

// two-shot, all-gather: every chunk q != rank copied from peer q's slot (its reduced chunk)
template <bool BF16, int P, bool KAVG = false>
__global__ __launch_bounds__(PC_BLOCK) void k_pc_ag(float* __restrict__ out, PcPeers peers, char* region,
                                                    unsigned* ctrl, int rank, long long cap, long long n, long long cv,
                                                    float scale, int aligned, unsigned long long limit,
                                                    PcKavg kv = PcKavg{}) {
  using W = Wire<BF16>;
  constexpr int VE = W::VE;
  static_assert(!KAVG || !BF16, "K-AVG rounds use the fp32 wire");
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned calls = __hip_atomic_load(ctrl + C_CALLS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = pc_barrier(peers, region, ctrl, rank, P, seq + 2u, limit);
  float inv = 1.f;
  if constexpr (KAVG) inv = kavg_divisor<P>(peers, calls).x;
  __amdgpu_buffer_rsrc_t rs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) rs[p] = pc_rsrc(slot_of(peers.region[p], calls, cap), cap);
  const long long total = (long long)(P - 1) * cv;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total; j += stride) {
    int q = (int)(j / cv);
    const long long v = j - (long long)q * cv;
    q += (q >= rank);
    const long long g = (long long)q * cv + v;
    float x[VE];
    if (ok) {
      uint4 w = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int p = 0; p < P; ++p)  // uniform-index select keeps the descriptors in SGPRs
        if (p == q) w = ld_sys16(rs[p], g * 16);
      W::unpack(w, x);
    } else {
#pragma unroll
      for (int jj = 0; jj < VE; ++jj) x[jj] = __builtin_nanf("");
    }
    if constexpr (KAVG)
      kavg_store(out, g * VE, n, aligned != 0, x, inv, kv);
    else
      store_out<VE>(out, g * VE, n, aligned != 0, x, scale);
  }
  pc_finish_call(ctrl, 2u);
}

// ---- sharded data-parallel update (ZeRO-1 over peer memory) ------------------------------
// Every rank's flat fp32 gradient, fp32 master and bf16 shadow are IPC-exportable hipMalloc
// buffers that every peer maps; nothing is staged.  Chunk q = elements [q*C, min((q+1)C, n)),
// C a multiple of 64, updated by rank q alone:
//   rs   barrier(seq+1); rank r sums chunk r of the P gradients in rank order (fp32, read in
//        place over xGMI) and either applies SGD to its master / momentum chunk and writes its
//        bf16 shadow chunk (fused), or stores the sum into its own gradient chunk (any optimizer
//        then runs on the chunk range)
//   ag   barrier(seq+2); rank r copies chunk q of peer q's bf16 shadow into its own, q != r
//   gm   barrier(seq+1); rank r copies chunk q of peer q's fp32 master (K-AVG, checkpoint, epoch
//        end: the only times a full fp32 master is read)
// Link bytes per rank per step: 4(P-1)/P n (gradient) + 2(P-1)/P n (shadow) — the fp32-exact
// gradient at 3/4 of an fp32 all-reduce, and 1/P of the optimizer pass.
// Reuse is safe single-buffered: a rank rewrites its gradient (next backward) only after its ag
// barrier, which every peer enters after its rs reads finished; it rewrites its shadow chunk
// only after the next rs barrier, which every peer enters after its ag reads finished.  The
// buffers are written with plain stores by ordinary kernels: the kernel boundary before the
// publishing launch writes the XCD L2s back, and peers read with system-scope loads.
struct ZsPeers {
  const char* flags[PC_MAX_RANKS];   // every rank's barrier region
  const char* data[PC_MAX_RANKS];    // every rank's gradient / shadow / master buffer
};

// Ranks that share one GPU (packed workers) must not spin in every block of a work kernel while
// a peer still needs CUs to reach the barrier: there the barrier is a one-block launch of its
// own (k_zs_wait) and the work kernel that follows only reads the poison flag (`split`).
__device__ __forceinline__ bool zs_enter(const ZsPeers& peers, char* region, unsigned* ctrl, int rank, int world,
                                         unsigned target, unsigned long long limit, int split) {
  if (split) return __hip_atomic_load(ctrl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
  PcPeers fl;
  for (int p = 0; p < world; ++p) fl.region[p] = peers.flags[p];
  return pc_barrier(fl, region, ctrl, rank, world, target, limit);
}

__global__ __launch_bounds__(64) void k_zs_wait(ZsPeers peers, char* region, unsigned* ctrl, int rank, int world,
                                                unsigned bar, unsigned long long limit, unsigned long long* stamp) {
  if (stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // collective start (timing)
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  PcPeers fl;
  for (int p = 0; p < world; ++p) fl.region[p] = peers.flags[p];
  (void)pc_barrier(fl, region, ctrl, rank, world, seq + bar, limit);
}

template <int P, bool SGD>
__global__ __launch_bounds__(PC_BLOCK) void k_zs_rs(ZsPeers peers, char* region, unsigned* ctrl, int rank,
                                                    long long lo, long long hi, float* __restrict__ own_grad,
                                                    float* __restrict__ master, float* __restrict__ mom,
                                                    bf16_t* __restrict__ shadow, const float* __restrict__ lr_ptr,
                                                    float wd, float momentum, float dampening, int nesterov,
                                                    const float* __restrict__ first_ptr, float grad_scale,
                                                    float* __restrict__ adv_ctr, float adv_batch, float adv_n,
                                                    unsigned long long limit, int split) {
  if (adv_ctr && blockIdx.x == 0 && threadIdx.x == 0) {  // data-sampler counter (see k_sgd)
    adv_ctr[1] += 1.f;
    float st = adv_ctr[2] + adv_batch;
    if (st >= adv_n) st -= adv_n;
    adv_ctr[2] = st;
  }
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = zs_enter(peers, region, ctrl, rank, P, seq + 1u, limit, split);
  const long long nv = (hi - lo) >> 2;  // fp32x4 vectors of this rank's chunk
  __amdgpu_buffer_rsrc_t rs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) rs[p] = pc_rsrc(peers.data[p] + lo * 4, (hi - lo) * 4);
  float lr = 0.f;
  int first = 0;
  if constexpr (SGD) {
    lr = *lr_ptr;
    first = first_ptr ? (*first_ptr != 0.f) : 0;
  }
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < nv; v += stride) {
    float acc[4];
    if (ok) {
      uint4 w[P];
#pragma unroll
      for (int p = 0; p < P; ++p)  // own gradient: local bytes, plain (L2-cached) loads
        w[p] = p == rank ? *reinterpret_cast<const uint4*>(own_grad + lo + v * 4) : ld_sys16(rs[p], v * 16);
      Wire<false>::unpack(w[0], acc);
#pragma unroll
      for (int p = 1; p < P; ++p) {
        float x[4];
        Wire<false>::unpack(w[p], x);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += x[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_nanf("");
    }
    const long long e = lo + v * 4;
    if constexpr (SGD) {
      const float4 W = *reinterpret_cast<const float4*>(master + e);
      float wv[4] = {W.x, W.y, W.z, W.w}, mv[4] = {0.f, 0.f, 0.f, 0.f};
      if (mom) {
        const float4 M = *reinterpret_cast<const float4*>(mom + e);
        mv[0] = M.x, mv[1] = M.y, mv[2] = M.z, mv[3] = M.w;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // the k_sgd recurrence, op for op
        float d = acc[k] * grad_scale + wd * wv[k];
        if (mom) {
          mv[k] = first ? d : momentum * mv[k] + (1.f - dampening) * d;
          d = nesterov ? d + momentum * mv[k] : mv[k];
        }
        wv[k] -= lr * d;
      }
      *reinterpret_cast<float4*>(master + e) = make_float4(wv[0], wv[1], wv[2], wv[3]);
      if (mom) *reinterpret_cast<float4*>(mom + e) = make_float4(mv[0], mv[1], mv[2], mv[3]);
      uint2 s;
      s.x = pack_bf2(wv[0], wv[1]);
      s.y = pack_bf2(wv[2], wv[3]);
      *reinterpret_cast<uint2*>(shadow + e) = s;
    } else {
      *reinterpret_cast<float4*>(own_grad + e) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
  }
}

// all-gather of chunks: chunk q of peer q's buffer -> own buffer, q != rank (16-byte vectors;
// `ve` elements per vector, `esz` bytes per element).  Barrier `bar` of the call; `finish` =
// barriers this call passes (the last launch of a call advances the sequence).
template <int P>
__global__ __launch_bounds__(PC_BLOCK) void k_zs_gather(ZsPeers peers, char* region, unsigned* ctrl, int rank,
                                                        char* __restrict__ own, long long n, long long chunk, int esz,
                                                        unsigned bar, unsigned finish, unsigned long long limit,
                                                        int split, unsigned long long* stamp) {
  const unsigned seq = __hip_atomic_load(ctrl + C_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = zs_enter(peers, region, ctrl, rank, P, seq + bar, limit, split);
  const long long cv = chunk * esz / 16;  // vectors per (full) chunk
  const long long total = (long long)(P - 1) * cv;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total; j += stride) {
    int q = (int)(j / cv);
    const long long v = j - (long long)q * cv;
    q += (q >= rank);
    const long long off = (long long)q * chunk * esz + v * 16;  // byte offset in the buffer
    if (off >= n * esz) continue;                                // the last chunk is short
    uint4 w;
    if (ok) {
      w = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int p = 0; p < P; ++p)  // uniform-index select keeps the descriptors in SGPRs
        if (p == q) w = ld_sys16(pc_rsrc(peers.data[p] + (long long)p * chunk * esz, chunk * esz), v * 16);
    } else {
      const unsigned nan = esz == 2 ? 0x7FC07FC0u : 0x7FC00000u;
      w = make_uint4(nan, nan, nan, nan);
    }
    *reinterpret_cast<uint4*>(own + off) = w;
  }
  if (finish) pc_finish_call(ctrl, finish, stamp);
}

// side-stream HBM streamer for the interference probe: `passes` copies of n 16-byte vectors
__global__ __launch_bounds__(PC_BLOCK) void k_stream_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          long long n, int passes) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (int it = 0; it < passes; ++it)
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
      uint4 v = src[i];
      v.x += (unsigned)it;
      dst[i] = v;
    }
}

template <bool BF16, int P>
hipError_t launch_all(const float* in, float* out, const PcPeers& peers, char* region, unsigned* ctrl, int rank,
                      long long cap, long long n, float scale, int algo, int max_blocks, unsigned long long limit,
                      hipStream_t s) {
  constexpr int VE = Wire<BF16>::VE;
  const int aligned = ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
  auto grid_for = [&](long long items) {
    long long g = (items + PC_BLOCK - 1) / PC_BLOCK;
    if (g > max_blocks) g = max_blocks;
    if (g < 1) g = 1;
    return (unsigned)g;
  };
  if (algo == 0) {
    const long long nvec = (n + VE - 1) / VE;
    if (nvec * 16 > cap) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pc_copyin<BF16>, dim3(grid_for(nvec)), dim3(PC_BLOCK), 0, s, in, region, ctrl, cap, n, nvec,
                       aligned);
    hipLaunchKernelGGL((k_pc_oneshot<BF16, P>), dim3(grid_for(nvec)), dim3(PC_BLOCK), 0, s, out, peers, region, ctrl,
                       rank, cap, n, nvec, scale, aligned, limit);
  } else {
    const long long cv = ((n + VE - 1) / VE + P - 1) / P;  // vectors per chunk
    const long long nvec = cv * P;
    if (nvec * 16 > cap) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pc_copyin<BF16>, dim3(grid_for(nvec)), dim3(PC_BLOCK), 0, s, in, region, ctrl, cap, n, nvec,
                       aligned);
    hipLaunchKernelGGL((k_pc_rs<BF16, P>), dim3(grid_for(cv)), dim3(PC_BLOCK), 0, s, out, peers, region, ctrl, rank,
                       cap, n, cv, scale, aligned, limit);
    hipLaunchKernelGGL((k_pc_ag<BF16, P>), dim3(grid_for((long long)(P - 1) * cv)), dim3(PC_BLOCK), 0, s, out, peers,
                       region, ctrl, rank, cap, n, cv, scale, aligned, limit);
  }
  return hipGetLastError();
}

template <int P>
hipError_t launch_kavg(float* state, const PcPeers& peers, char* region, unsigned* ctrl, int rank, long long cap,
                       long long n, const PcKavg& kv, int max_blocks, unsigned long long limit, hipStream_t s) {
  const int aligned = (((uintptr_t)state) & 15) == 0;
  auto grid_for = [&](long long items) {
    long long g = (items + PC_BLOCK - 1) / PC_BLOCK;
    if (g > max_blocks) g = max_blocks;
    if (g < 1) g = 1;
    return (unsigned)g;
  };
  const long long cv = ((n + 3) / 4 + P - 1) / P;
  const long long nvec = cv * P;
  if (nvec * 16 > cap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pc_copyin<false>, dim3(grid_for(nvec)), dim3(PC_BLOCK), 0, s, state, region, ctrl, cap, n, nvec,
                     aligned, kv.count_idx);
  hipLaunchKernelGGL((k_pc_rs<false, P, true>), dim3(grid_for(cv)), dim3(PC_BLOCK), 0, s, state, peers, region, ctrl,
                     rank, cap, n, cv, 1.f, aligned, limit, kv);
  hipLaunchKernelGGL((k_pc_ag<false, P, true>), dim3(grid_for((long long)(P - 1) * cv)), dim3(PC_BLOCK), 0, s, state,
                     peers, region, ctrl, rank, cap, n, cv, 1.f, aligned, limit, kv);
  return hipGetLastError();
}

template <bool BF16>
hipError_t launch_world(int world, const float* in, float* out, const PcPeers& peers, char* region, unsigned* ctrl,
                        int rank, long long cap, long long n, float scale, int algo, int max_blocks,
                        unsigned long long limit, hipStream_t s) {
  switch (world) {
#define PC_CASE(P) \
  case P:          \
    return launch_all<BF16, P>(in, out, peers, region, ctrl, rank, cap, n, scale, algo, max_blocks, limit, s);
    PC_CASE(1) PC_CASE(2) PC_CASE(3) PC_CASE(4) PC_CASE(5) PC_CASE(6) PC_CASE(7) PC_CASE(8)
#undef PC_CASE
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace

// ---- IPC regions ---------------------------------------------------------------------
KML_API int kml_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// region (flags + 2 slots of cap bytes) + zeroed local control block
KML_API int kml_peer_alloc(long long cap, void** region, void** ctrl) {
  if (cap <= 0 || cap % 16 || cap >= (1ll << 31)) return (int)hipErrorInvalidValue;
  *region = nullptr;
  *ctrl = nullptr;
  hipError_t e = hipMalloc(region, PC_FLAGS_BYTES + 2 * cap);
  if (e == hipSuccess) e = hipMemset(*region, 0, PC_FLAGS_BYTES);
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

KML_API int kml_peer_free(void* region, void* ctrl) {
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

// failed (timed-out) waits so far; non-zero = the group is poisoned (synchronises)
KML_API int kml_peer_errors(const void* ctrl, unsigned* out) {
  return (int)hipMemcpy(out, reinterpret_cast<const unsigned*>(ctrl) + C_ERR, sizeof(unsigned),
                        hipMemcpyDeviceToHost);
}

// out = scale * sum over ranks of in (n fp32; in and out may alias).
// regions[world]: every rank's region as mapped here (own at [rank]).  algo 0 = one-shot,
// 1 = two-shot.  wire_bf16: the slots carry bf16 (half the link bytes; sums stay fp32).
// max_blocks caps every launch's grid; timeout_s bounds each barrier wait.
KML_API int kml_peer_allreduce(const float* in, float* out, const void* const* regions, void* region, void* ctrl,
                               int rank, int world, long long cap, long long n, float scale, int algo, int wire_bf16,
                               int max_blocks, double timeout_s, hipStream_t s) {
  if (world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || n < 0 || cap % 16 || max_blocks < 1 ||
      (algo != 0 && algo != 1) || !(timeout_s > 0.0))
    return (int)hipErrorInvalidValue;
  if (n == 0) return (int)hipSuccess;
  PcPeers peers = {};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return (int)hipErrorInvalidValue;
    peers.region[p] = reinterpret_cast<const char*>(regions[p]);
  }
  if (peers.region[rank] != region) return (int)hipErrorInvalidValue;
  const double ticks = timeout_s * 1.0e8;  // s_memrealtime runs at 100 MHz
  const unsigned long long limit = ticks > 1.8e19 ? ~0ull : (unsigned long long)ticks;
  hipError_t e = wire_bf16
                     ? launch_world<true>(world, in, out, peers, reinterpret_cast<char*>(region),
                                          reinterpret_cast<unsigned*>(ctrl), rank, cap, n, scale, algo, max_blocks,
                                          limit, s)
                     : launch_world<false>(world, in, out, peers, reinterpret_cast<char*>(region),
                                           reinterpret_cast<unsigned*>(ctrl), rank, cap, n, scale, algo, max_blocks,
                                           limit, s);
  return (int)e;
}

// ---- sharded update (ZeRO-1) entry points ------------------------------------------------
// IPC-exportable buffer (hipMalloc base, zeroed): a flat gradient / master / shadow peers map
KML_API int kml_ipc_alloc(long long bytes, void** out) {
  *out = nullptr;
  if (bytes <= 0) return (int)hipErrorInvalidValue;
  hipError_t e = hipMalloc(out, (size_t)bytes);
  if (e == hipSuccess) e = hipMemset(*out, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess && *out) {
    (void)hipFree(*out);
    *out = nullptr;
  }
  return (int)e;
}

KML_API int kml_ipc_free(void* p) { return (int)(p ? hipFree(p) : hipSuccess); }

namespace {
bool zs_peers(ZsPeers& zp, const void* const* flags, const void* const* data, int world) {
  zp = {};
  for (int p = 0; p < world; ++p) {
    if (!flags[p] || !data[p]) return false;
    zp.flags[p] = reinterpret_cast<const char*>(flags[p]);
    zp.data[p] = reinterpret_cast<const char*>(data[p]);
  }
  return true;
}
unsigned long long zs_limit(double timeout_s) {
  const double ticks = timeout_s * 1.0e8;
  return ticks > 1.8e19 ? ~0ull : (unsigned long long)ticks;
}
unsigned zs_grid(long long items, int max_blocks) {
  long long g = (items + PC_BLOCK - 1) / PC_BLOCK;
  if (g > max_blocks) g = max_blocks;
  if (g < 1) g = 1;
  return (unsigned)g;
}
}  // namespace

// One K-AVG round in place on the flat state buffer (after kml_kavg_pack): the two-shot SUM with
// the average, the bf16 shadow refresh of [0, n_params) and the int64 counter unpack fused into
// its epilogues (see PcKavg).  Same result as kml_peer_allreduce(two-shot, fp32) + kml_kavg_finish.
KML_API int kml_peer_kavg(float* state, const void* const* regions, void* region, void* ctrl, int rank, int world,
                          long long cap, long long n, long long count_idx, long long n_params, bf16_t* shadow,
                          long long* i64, long long i64_off, int n_i64, int max_blocks, double timeout_s,
                          hipStream_t s) {
  if (world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || n <= 0 || cap % 16 || max_blocks < 1 ||
      !(timeout_s > 0.0) || count_idx < 0 || count_idx >= n || n_params < 0 || n_params > count_idx ||
      n_i64 < 0 || (n_i64 > 0 && (!i64 || i64_off < 0 || i64_off + n_i64 > count_idx)))
    return (int)hipErrorInvalidValue;
  PcPeers peers = {};
  for (int p = 0; p < world; ++p) {
    if (!regions[p]) return (int)hipErrorInvalidValue;
    peers.region[p] = reinterpret_cast<const char*>(regions[p]);
  }
  if (peers.region[rank] != region) return (int)hipErrorInvalidValue;
  PcKavg kv;
  kv.count_idx = count_idx;
  kv.n_params = shadow ? n_params : 0;
  kv.shadow = shadow;
  kv.i64 = n_i64 > 0 ? i64 : nullptr;
  kv.i64_off = i64_off;
  kv.n_i64 = n_i64;
  kv.shadow_aligned = (((uintptr_t)shadow) & 7) == 0;
  const unsigned long long limit = zs_limit(timeout_s);
  switch (world) {
#define PK_CASE(P) \
  case P:          \
    return (int)launch_kavg<P>(state, peers, reinterpret_cast<char*>(region), reinterpret_cast<unsigned*>(ctrl), rank, \
                               cap, n, kv, max_blocks, limit, s);
    PK_CASE(1) PK_CASE(2) PK_CASE(3) PK_CASE(4) PK_CASE(5) PK_CASE(6) PK_CASE(7) PK_CASE(8)
#undef PK_CASE
    default:
      return (int)hipErrorInvalidValue;
  }
}


// reduce-scatter of the flat fp32 gradients: rank's chunk [lo, hi) summed over the group in rank
// order.  fused_sgd: the sum goes straight into the SGD update of master / mom (may be null) and
// the bf16 shadow chunk (lr, first flag on device; advance counter as k_sgd); else it is stored
// into the own gradient chunk.  grads[world] / flags[world]: every rank's buffers as mapped here.
KML_API int kml_zs_reduce_scatter(const void* const* flags, const void* const* grads, void* region, void* ctrl,
                                  int rank, int world, long long lo, long long hi, int fused_sgd, float* master,
                                  float* mom, bf16_t* shadow, const float* lr_ptr, float wd, float momentum,
                                  float dampening, int nesterov, const float* first_ptr, float grad_scale,
                                  float* adv_ctr, float adv_batch, float adv_n, int max_blocks, double timeout_s,
                                  int split, unsigned long long* stamp, hipStream_t s) {
  ZsPeers zp;
  if (world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || lo < 0 || hi < lo || (lo & 3) ||
      (hi & 3) || max_blocks < 1 || !(timeout_s > 0.0) || !zs_peers(zp, flags, grads, world) ||
      zp.flags[rank] != region || (fused_sgd && (!master || !shadow || !lr_ptr)))
    return (int)hipErrorInvalidValue;
  float* own = const_cast<float*>(reinterpret_cast<const float*>(grads[rank]));
  const unsigned g = zs_grid((hi - lo) / 4, max_blocks);
  const unsigned long long lim = zs_limit(timeout_s);
  if (split)
    hipLaunchKernelGGL(k_zs_wait, dim3(1), dim3(64), 0, s, zp, reinterpret_cast<char*>(region),
                       reinterpret_cast<unsigned*>(ctrl), rank, world, 1u, lim, stamp);
  switch (world) {
#define ZS_CASE(P)                                                                                                   \
  case P:                                                                                                            \
    if (fused_sgd)                                                                                                   \
      hipLaunchKernelGGL((k_zs_rs<P, true>), dim3(g), dim3(PC_BLOCK), 0, s, zp, reinterpret_cast<char*>(region),     \
                         reinterpret_cast<unsigned*>(ctrl), rank, lo, hi, own, master, mom, shadow, lr_ptr, wd,      \
                         momentum, dampening, nesterov, first_ptr, grad_scale, adv_ctr, adv_batch, adv_n, lim,       \
                         split);                                                                                     \
    else                                                                                                             \
      hipLaunchKernelGGL((k_zs_rs<P, false>), dim3(g), dim3(PC_BLOCK), 0, s, zp, reinterpret_cast<char*>(region),    \
                         reinterpret_cast<unsigned*>(ctrl), rank, lo, hi, own, master, mom, shadow, lr_ptr, wd,      \
                         momentum, dampening, nesterov, first_ptr, grad_scale, adv_ctr, adv_batch, adv_n, lim,       \
                         split);                                                                                     \
    break;
    ZS_CASE(1) ZS_CASE(2) ZS_CASE(3) ZS_CASE(4) ZS_CASE(5) ZS_CASE(6) ZS_CASE(7) ZS_CASE(8)
#undef ZS_CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  KML_LAUNCH_CHECK();
}

// all-gather of chunks (n elements of esz = 2 or 4 bytes, chunk elements per rank, chunk*esz a
// multiple of 16): barrier `bar` (2 after a reduce-scatter of the same call, 1 standalone);
// `finish` barriers close the call.
KML_API int kml_zs_all_gather(const void* const* flags, const void* const* bufs, void* region, void* ctrl, int rank,
                              int world, long long n, long long chunk, int esz, int bar, int finish, int max_blocks,
                              double timeout_s, int split, unsigned long long* stamp, hipStream_t s) {
  ZsPeers zp;
  if (world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || n < 0 || chunk <= 0 ||
      (esz != 2 && esz != 4) || (chunk * esz) % 16 || chunk * world < n || bar < 1 || finish < 0 ||
      max_blocks < 1 || !(timeout_s > 0.0) || !zs_peers(zp, flags, bufs, world) || zp.flags[rank] != region)
    return (int)hipErrorInvalidValue;
  char* own = const_cast<char*>(reinterpret_cast<const char*>(bufs[rank]));
  const unsigned g = zs_grid((long long)(world - 1) * chunk * esz / 16, max_blocks);
  const unsigned long long lim = zs_limit(timeout_s);
  if (split)
    hipLaunchKernelGGL(k_zs_wait, dim3(1), dim3(64), 0, s, zp, reinterpret_cast<char*>(region),
                       reinterpret_cast<unsigned*>(ctrl), rank, world, (unsigned)bar, lim, nullptr);
  switch (world) {
#define ZS_CASE(P)                                                                                                   \
  case P:                                                                                                            \
    hipLaunchKernelGGL((k_zs_gather<P>), dim3(g), dim3(PC_BLOCK), 0, s, zp, reinterpret_cast<char*>(region),         \
                       reinterpret_cast<unsigned*>(ctrl), rank, own, n, chunk, esz, (unsigned)bar, (unsigned)finish,  \
                       lim, split, stamp);                                                                           \
    break;
    ZS_CASE(1) ZS_CASE(2) ZS_CASE(3) ZS_CASE(4) ZS_CASE(5) ZS_CASE(6) ZS_CASE(7) ZS_CASE(8)
#undef ZS_CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  KML_LAUNCH_CHECK();
}

// Fresh fp32 master values of the parameters the forward / backward read in fp32 (BN / LN affine,
// biases: nn master_of): under the ZeRO-1 layout a rank's master is current only on the chunks it
// owns, so after the step's last all-gather every listed element owned elsewhere is re-read from
// its owner's master (system-scope loads: nothing this GPU caches of a peer survives).  Element e
// of segment k belongs to rank (e - s0[k]) / ch[k].  Runs after the step's final gather in stream
// order: the owners' updates are complete (that gather's barrier), and no owner rewrites its
// master before this rank publishes the next step's READY.
struct FreshArgs {
  const char* bufs[PC_MAX_RANKS];   // every rank's master (fp32, flat index e at byte 4 e)
  long long s0[4], s1[4], ch[4];
  int nseg, rank;
};

__global__ __launch_bounds__(256) void k_zs_fresh(const int* __restrict__ idx, long long n, FreshArgs f) {
  float* own = reinterpret_cast<float*>(const_cast<char*>(f.bufs[f.rank]));
  for (long long j = (long long)blockIdx.x * 256 + threadIdx.x; j < n; j += (long long)gridDim.x * 256) {
    const long long e = idx[j];
    int q = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < f.nseg && e >= f.s0[k] && e < f.s1[k]) q = (int)((e - f.s0[k]) / f.ch[k]);
    if (q < 0 || q == f.rank) continue;
    unsigned v = 0u;
#pragma unroll
    for (int p = 0; p < PC_MAX_RANKS; ++p)  // uniform-index select keeps the descriptors in SGPRs
      if (p == q) v = __builtin_amdgcn_raw_buffer_load_b32(pc_rsrc(f.bufs[p], 0x7fffffff), (int)(e * 4), 0, PC_AUX_SYS);
    own[e] = __uint_as_float(v);
  }
}

KML_API int kml_zs_fresh(const int* idx, long long n, const void* const* bufs, int rank, int world,
                         const long long* segs, int nseg, hipStream_t s) {
  if (n < 0 || world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || nseg < 1 || nseg > 4 || !bufs ||
      !segs || (n > 0 && !idx))
    return (int)hipErrorInvalidValue;
  if (n == 0 || world == 1) return (int)hipSuccess;
  FreshArgs f{};
  for (int p = 0; p < world; ++p) {
    if (!bufs[p]) return (int)hipErrorInvalidValue;
    f.bufs[p] = static_cast<const char*>(bufs[p]);
  }
  for (int k = 0; k < nseg; ++k) {
    f.s0[k] = segs[3 * k];
    f.s1[k] = segs[3 * k + 1];
    f.ch[k] = segs[3 * k + 2];
    if (f.ch[k] <= 0 || f.s1[k] < f.s0[k] || f.s1[k] * 4 >= (1LL << 31)) return (int)hipErrorInvalidValue;
  }
  f.nseg = nseg;
  f.rank = rank;
  long long g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_zs_fresh, dim3((unsigned)g), dim3(256), 0, s, idx, n, f);
  KML_LAUNCH_CHECK();
}

// standalone barrier `bar` past the current sequence (one-block launch).  gather_master closes
// with it (all-gather with finish = 2, then bar = 0): no rank leaves the call — and overwrites
// its own master chunk with a local step, a broadcast or a restore — while a peer may still be
// reading that chunk over xGMI.
KML_API int kml_zs_barrier(const void* const* flags, void* region, void* ctrl, int rank, int world, int bar,
                           double timeout_s, hipStream_t s) {
  ZsPeers zp;
  if (world < 1 || world > PC_MAX_RANKS || rank < 0 || rank >= world || bar < 0 || !(timeout_s > 0.0) ||
      !zs_peers(zp, flags, flags, world) || zp.flags[rank] != region)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_zs_wait, dim3(1), dim3(64), 0, s, zp, reinterpret_cast<char*>(region),
                     reinterpret_cast<unsigned*>(ctrl), rank, world, (unsigned)bar, zs_limit(timeout_s), nullptr);
  KML_LAUNCH_CHECK();
}

// device wall-clock stamp (100 MHz ticks) into buf[idx]: brackets the collectives inside a
// captured step so their time is known without events or a host sync
__global__ void k_stamp(unsigned long long* buf, int idx) {
  if (threadIdx.x == 0) buf[idx] = __builtin_amdgcn_s_memrealtime();
}

KML_API int kml_stamp(void* buf, int idx, hipStream_t s) {
  if (!buf || idx < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, reinterpret_cast<unsigned long long*>(buf), idx);
  KML_LAUNCH_CHECK();
}

// interference probe: `passes` copies of `bytes` (multiple of 16) on `blocks` workgroups
KML_API int kml_stream_copy(const void* src, void* dst, long long bytes, int blocks, int passes, hipStream_t s) {
  if (bytes <= 0 || bytes % 16 || blocks < 1 || passes < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stream_copy, dim3(blocks), dim3(PC_BLOCK), 0, s, reinterpret_cast<const uint4*>(src),
                     reinterpret_cast<uint4*>(dst), bytes / 16, passes);
  KML_LAUNCH_CHECK();
}
