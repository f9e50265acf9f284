// kml_sgd.h — the fused SGD element update (torch.optim.SGD semantics: weight decay, momentum,
// dampening, nesterov, first step after a reset) shared by k_sgd (optim.hip) and the update
// "rider" blocks a grouped conv-backward launch can carry (conv_igemm.hip k_conv_pair), so both
// paths produce bit-identical masters, momenta and bf16 shadows.
#pragma once
#include "kml_common.h"

// elements [0, n) of one flat range, visited by virtual thread t0 of `stride` (float4 body, then
// the scalar tail); lr and first already resolved from device memory by the caller
__device__ __forceinline__ void kml_sgd_range(float* __restrict__ w, const float* __restrict__ g,
                                              float* __restrict__ mom, bf16_t* __restrict__ shadow, float lr, float wd,
                                              float momentum, float dampening, int nesterov, int first,
                                              float grad_scale, long long n, long long t0, long long stride) {
  const long long n4 = n >> 2;
  for (long long i = t0; i < n4; i += stride) {
    float4 W = reinterpret_cast<float4*>(w)[i];
    const float4 G = reinterpret_cast<const float4*>(g)[i];
    float wv[4] = {W.x, W.y, W.z, W.w}, gv[4] = {G.x, G.y, G.z, G.w};
    float mv[4] = {0, 0, 0, 0};
    if (mom && momentum != 0.f) {
      const float4 Mv = reinterpret_cast<float4*>(mom)[i];
      mv[0] = Mv.x; mv[1] = Mv.y; mv[2] = Mv.z; mv[3] = Mv.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = gv[k] * grad_scale + wd * wv[k];
      if (mom && momentum != 0.f) {
        mv[k] = first ? d : momentum * mv[k] + (1.f - dampening) * d;
        d = nesterov ? d + momentum * mv[k] : mv[k];
      }
      wv[k] -= lr * d;
    }
    reinterpret_cast<float4*>(w)[i] = make_float4(wv[0], wv[1], wv[2], wv[3]);
    if (mom && momentum != 0.f) reinterpret_cast<float4*>(mom)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
    if (shadow) {
      uint2 s;
      s.x = pack_bf2(wv[0], wv[1]);
      s.y = pack_bf2(wv[2], wv[3]);
      reinterpret_cast<uint2*>(shadow)[i] = s;
    }
  }
  // scalar tail
  for (long long i = (n4 << 2) + t0; i < n; i += stride) {
    float d = g[i] * grad_scale + wd * w[i];
    if (mom && momentum != 0.f) {
      mom[i] = first ? d : momentum * mom[i] + (1.f - dampening) * d;
      d = nesterov ? d + momentum * mom[i] : mom[i];
    }
    w[i] -= lr * d;
    if (shadow) shadow[i] = f2bf(w[i]);
  }
}

// ---- peer-shard collective slices carried as riders (parallel/peer.py ShardRider) ---------------
// At N > 1 the sharded update (ZeRO-1 over IPC-mapped HBM, comm.hip k_zs_*) of the parameters
// whose gradients are final early in the backward (ResNet: layer4 + fc, then layer3) runs as extra
// blocks of later backward launches on the SAME queue, instead of after the backward or on a
// side stream (which slowed every dispatch of the latency-bound chain: profiles/r5/zero1_staged.md):
//   RS slice   publish READY, wait until every rank is READY, sum this rank's chunk of every rank's
//              fp32 gradient (system-scope loads, rank order) and apply the fused SGD to the master /
//              momentum / bf16 shadow chunk (shadow stored write-through at system scope); the block
//              that finishes the phase's last slice publishes DONE
//   AG slice   wait until every rank is DONE, copy the peers' bf16 shadow chunks into the own shadow
// Progress is a per-rank monotonic counter: word KML_ZS_PROGRESS + r of every peer's flags area
// holds rank r's value (base + offset; base = ctrl word KML_ZS_BASE, advanced by the step's last
// slice).  Waits are bounded (s_memrealtime); on expiry the group is poisoned (ctrl word 2) and the
// slice writes NaN, as every comm.hip wait does.
constexpr int KML_ZS_MAX = 8;
constexpr int KML_ZS_PROGRESS = 48;  // flags-area words 48..55 (comm.hip uses 0..7 and 32..33)
enum { KML_ZS_ERR = 2, KML_ZS_BASE = 4 };  // ctrl words (comm.hip: 0 seq, 1 ticket, 2 errors, 3 calls)
enum { KML_RIDER_SGD = 0, KML_RIDER_ZS_RS = 1, KML_RIDER_ZS_AG = 2 };

struct KmlZsRider {
  const char* flags[KML_ZS_MAX];  // every rank's flags area (this process's mappings)
  const char* data[KML_ZS_MAX];   // RS: every rank's fp32 gradient at the segment; AG: every rank's bf16 shadow there
  unsigned* own_flags;            // this rank's flags area (its progress words are read here)
  unsigned* ctrl;                 // this rank's control block
  int rank, world;
  long long a, b;     // RS: this rank's chunk [a, b) of the segment; AG: chunk elements, segment elements
  long long v0, v1;   // this slice's 16-byte vectors (RS: of the own chunk; AG: of the P - 1 peer chunks)
  int ready;          // progress offset published before the wait (RS slices), 0: none
  int wait;           // progress offset every rank must have reached before this slice reads
  int done;           // progress offset published by the block that completes done_blocks, 0: none
  int done_blocks;    // rider blocks of the whole phase (all its slices), 0: no completion count
  int done_word;      // ctrl word counting the phase's finished blocks
  int advance;        // added to the base by that block (the step's last phase)
  unsigned long long limit;  // wait bound, s_memrealtime ticks (100 MHz)
};

// one SGD range (kind SGD) or one peer-shard slice (kinds ZS_*) carried by extra blocks of another
// launch (blocks == 0: none); the ZS kinds use w / mom / shadow / lr / first / coefficients for the
// fused SGD of the own chunk (RS: offset to the segment, indexed like zs.data) or the own shadow (AG)
struct KmlSgdRider {
  float* w;
  const float* g;
  float* mom;
  bf16_t* shadow;
  const float* lr_ptr;     // device lr (graph-captured steps follow set_lr)
  const float* first_ptr;  // device first-step flag, or null (no momentum)
  float wd, momentum, dampening, grad_scale;
  int nesterov;
  int blocks;
  long long n;
  int kind;
  KmlZsRider zs;
};

// The rider armed for the next rider-capable launch of this process (kml_rider_set; defined in
// util.hip, consumed — and cleared — by k_conv_pair's and k_bn_bwd_apply_v's launchers)
extern KmlSgdRider g_kml_rider;

extern "C" int kml_rider_flush(hipStream_t s);   // util.hip: an armed rider as its own launch

// take the armed rider (blocks = 0: none) and disarm it
static inline KmlSgdRider kml_rider_take() {
  const KmlSgdRider r = g_kml_rider;
  g_kml_rider.blocks = 0;
  return r;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t kml_zs_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
constexpr int KML_ZS_SYS = 17;  // buffer cache-policy bits sc0 | sc1: system-coherent access

// thread 0: store `value` into rank r's progress word of every peer's flags area, relaxed at system
// scope, no release (a system release writes back the XCD's L2 — the running conv tiles' working
// set — and cost ~10 us per host launch).  What a flag hands over is already in memory: READY the
// gradients of launches that completed before this one (a kernel boundary writes the L2s back: the
// next launch's blocks on other XCDs read them), DONE the shadow chunk, stored write-through at
// system scope and drained by every storing wave before the phase count reached this block
template <bool RELEASE = false>
__device__ __forceinline__ void kml_zs_publish(const KmlZsRider& z, unsigned value) {
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int p = 0; p < KML_ZS_MAX; ++p)
    if (p < z.world)
      __hip_atomic_store(reinterpret_cast<unsigned*>(const_cast<char*>(z.flags[p])) + KML_ZS_PROGRESS + z.rank, value,
                         RELEASE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// every thread: true once every rank's progress reached `target` in time (false at once when the
// group is poisoned); thread 0 polls.  No acquire fence: every peer byte a slice reads is a
// system-scope (sc0 sc1) load that no cache of this GPU serves (a system acquire would invalidate
// the L2 under the running conv tiles in every rider block)
__device__ inline bool kml_zs_wait(const KmlZsRider& z, unsigned target) {
  __shared__ int kml_zs_ok;
  if (threadIdx.x == 0) {
    int ok = __hip_atomic_load(z.ctrl + KML_ZS_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < z.world && ok; ++p) {
      while ((int)(__hip_atomic_load(z.own_flags + KML_ZS_PROGRESS + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                   target) < 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > z.limit) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (!ok) __hip_atomic_fetch_add(z.ctrl + KML_ZS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    kml_zs_ok = ok;
  }
  __syncthreads();
  return kml_zs_ok != 0;
}

// end of a rider block: count it toward its phase; the block completing the phase resets the
// counter, publishes DONE (after every block's write-through stores drained) and advances the base.
// Relaxed atomics only: an agent-scope release / acquire writes back / invalidates the XCD's L2
// (the conv tiles' working set) and, taken by every rider block, cost the host launches more than
// the slice's own traffic (profiles/r6/shardride.md).  What DONE hands over was stored write-through
// at system scope and drained (vmcnt(0)) by every wave before its block counted itself; the counter
// and the base are atomics the memory side serialises, read by later launches or this phase's last
// block only.
__device__ inline void kml_zs_finish(const KmlZsRider& z, unsigned base) {
  if (z.done_blocks <= 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's system-scope stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(z.ctrl + z.done_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)z.done_blocks - 1u) {
      __hip_atomic_store(z.ctrl + z.done_word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (z.done) kml_zs_publish(z, base + (unsigned)z.done);
      if (z.advance) __hip_atomic_fetch_add(z.ctrl + KML_ZS_BASE, (unsigned)z.advance, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// RS slice, block b of r.blocks: the own chunk's vectors [v0, v1) summed over the ranks in rank
// order (own gradient: plain loads; peers': system-scope loads) and the fused SGD applied op for op
// as k_sgd / k_zs_rs do; the bf16 shadow chunk stored write-through at system scope (peers gather it)
__device__ inline void kml_zs_rs_run(const KmlSgdRider& r, int b) {
  const KmlZsRider& z = r.zs;
  const unsigned base = __hip_atomic_load(z.ctrl + KML_ZS_BASE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (z.ready && b == 0) kml_zs_publish(z, base + (unsigned)z.ready);   // block 0 of each RS slice
  const bool ok = kml_zs_wait(z, base + (unsigned)z.wait);
  const float lr = *r.lr_ptr;
  const int first = r.first_ptr ? (*r.first_ptr != 0.f) : 0;
  const bool mom = r.mom != nullptr && r.momentum != 0.f;
  const auto shr = kml_zs_rsrc(r.shadow);
  const long long stride = (long long)r.blocks * blockDim.x;
  for (long long v = z.v0 + (long long)b * blockDim.x + threadIdx.x; v < z.v1; v += stride) {
    const long long e = z.a + v * 4;  // element of the segment
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (ok) {
      uint4 w[KML_ZS_MAX];
#pragma unroll
      for (int p = 0; p < KML_ZS_MAX; ++p) {
        if (p >= z.world) break;
        if (p == z.rank) {
          w[p] = *reinterpret_cast<const uint4*>(z.data[p] + e * 4);
        } else {
          const auto rv = __builtin_amdgcn_raw_buffer_load_b128(kml_zs_rsrc(z.data[p]), (int)(e * 4), 0, KML_ZS_SYS);
          w[p] = make_uint4(rv[0], rv[1], rv[2], rv[3]);
        }
      }
#pragma unroll
      for (int p = 0; p < KML_ZS_MAX; ++p) {
        if (p >= z.world) break;
        acc[0] += __uint_as_float(w[p].x);
        acc[1] += __uint_as_float(w[p].y);
        acc[2] += __uint_as_float(w[p].z);
        acc[3] += __uint_as_float(w[p].w);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_nanf("");
    }
    const float4 W = *reinterpret_cast<const float4*>(r.w + e);
    float wv[4] = {W.x, W.y, W.z, W.w}, mv[4] = {0.f, 0.f, 0.f, 0.f};
    if (mom) {
      const float4 M = *reinterpret_cast<const float4*>(r.mom + e);
      mv[0] = M.x, mv[1] = M.y, mv[2] = M.z, mv[3] = M.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // the k_sgd recurrence, op for op
      float d = acc[k] * r.grad_scale + r.wd * wv[k];
      if (mom) {
        mv[k] = first ? d : r.momentum * mv[k] + (1.f - r.dampening) * d;
        d = r.nesterov ? d + r.momentum * mv[k] : mv[k];
      }
      wv[k] -= lr * d;
    }
    *reinterpret_cast<float4*>(r.w + e) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    if (mom) *reinterpret_cast<float4*>(r.mom + e) = make_float4(mv[0], mv[1], mv[2], mv[3]);
    __attribute__((ext_vector_type(2))) unsigned sv = {pack_bf2(wv[0], wv[1]), pack_bf2(wv[2], wv[3])};
    __builtin_amdgcn_raw_buffer_store_b64(sv, shr, (int)(e * 2), 0, KML_ZS_SYS);
  }
  kml_zs_finish(z, base);
}

// AG slice, block b: 16-byte vectors [v0, v1) of the P - 1 peer chunks of the segment's bf16 shadow
// (chunk q of peer q), system-scope loads, plain stores into the own shadow
__device__ inline void kml_zs_ag_run(const KmlSgdRider& r, int b) {
  const KmlZsRider& z = r.zs;
  const unsigned base = __hip_atomic_load(z.ctrl + KML_ZS_BASE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = kml_zs_wait(z, base + (unsigned)z.wait);
  const long long cv = z.a * 2 / 16;  // vectors per chunk
  char* own = reinterpret_cast<char*>(r.shadow);
  const long long stride = (long long)r.blocks * blockDim.x;
  for (long long j = z.v0 + (long long)b * blockDim.x + threadIdx.x; j < z.v1; j += stride) {
    int q = (int)((unsigned)j / (unsigned)cv);  // 16-byte vector counts stay far below 2^32
    const long long v = j - (long long)q * cv;
    q += (q >= z.rank);
    const long long off = (long long)q * z.a * 2 + v * 16;  // byte offset in the segment
    if (off >= z.b * 2) continue;                            // the last chunk is short
    uint4 w = make_uint4(0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u);
    if (ok) {
#pragma unroll
      for (int p = 0; p < KML_ZS_MAX; ++p)  // uniform-index select keeps the descriptors in SGPRs
        if (p == q) {
          const auto rv = __builtin_amdgcn_raw_buffer_load_b128(kml_zs_rsrc(z.data[p]), (int)off, 0, KML_ZS_SYS);
          w = make_uint4(rv[0], rv[1], rv[2], rv[3]);
        }
    }
    *reinterpret_cast<uint4*>(own + off) = w;
  }
  kml_zs_finish(z, base);
}

// block `b` of the rider's `blocks` (256 threads each)
__device__ __forceinline__ void kml_sgd_rider_run(const KmlSgdRider& r, int b) {
  if (r.kind == KML_RIDER_ZS_RS) {
    kml_zs_rs_run(r, b);
    return;
  }
  if (r.kind == KML_RIDER_ZS_AG) {
    kml_zs_ag_run(r, b);
    return;
  }
  const float lr = *r.lr_ptr;
  const int first = r.first_ptr ? (*r.first_ptr != 0.f) : 0;
  kml_sgd_range(r.w, r.g, r.mom, r.shadow, lr, r.wd, r.momentum, r.dampening, r.nesterov, first, r.grad_scale, r.n,
                (long long)b * blockDim.x + threadIdx.x, (long long)r.blocks * blockDim.x);
}
