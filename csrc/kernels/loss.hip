// loss.hip — softmax cross-entropy (mean reduction) for gfx950.
//
// forward : one wave64 per row.  Online max/sum-exp over the row (bf16 or fp32
//           logits, 16 B loads), writes the row's log-sum-exp, loss and whether the
//           argmax equals the label (the reference's validation "correct" count,
//           function_resnet34.py:86-89).  Rows whose label == ignore_index contribute 0.
// reduce  : one block folds per-row results into [mean loss, correct, valid] — inside the
//           forward launch when a ticket counter is given: rows are stored write-through
//           (sc1), every wave drains, one relaxed agent-scope ticket per block, and the last
//           block reads all rows with sc1 loads (CDNA guide §6 G16 fan-in, no fences); else as
//           a second launch.  Fixed summation order either way (deterministic).
// backward: dlogits = grad_out * (softmax - onehot) / valid, recomputed from the saved
//           log-sum-exp (no [B, C] probability tensor is kept).
#include "kml_common.h"

namespace {

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// [mean loss, correct, valid] of B rows, by one block of 1024 threads (or fewer) in a fixed order
template <bool SC1>
__device__ void ce_fold(const float* __restrict__ rowloss, const float* __restrict__ rowcorrect, float* __restrict__ out,
                        int B) {
  float l = 0.f, c = 0.f, v = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const float rc = SC1 ? ld_sc1(rowcorrect + i) : rowcorrect[i];
    if (rc >= 0.f) { l += SC1 ? ld_sc1(rowloss + i) : rowloss[i]; c += rc; v += 1.f; }
  }
  l = wave_sum(l); c = wave_sum(c); v = wave_sum(v);
  __shared__ float sh[3][16];
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) { sh[0][w] = l; sh[1][w] = c; sh[2][w] = v; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float L = 0, Cc = 0, V = 0;
    for (int i = 0; i < nw; ++i) { L += sh[0][i]; Cc += sh[1][i]; V += sh[2][i]; }
    out[0] = V > 0 ? L / V : 0.f;
    out[1] = Cc;
    out[2] = V;
  }
}

// bf16 rows with C % 8 == 0 (16-byte aligned): 8 logits per lane per load; the running
// max is updated once per 8-element chunk (one rescale v_exp per chunk instead of a
// dependent exp + branch per element), exponentials in the base-2 domain (v_exp_f32).
constexpr float LOG2E_CE = 1.4426950408889634f;
__device__ __forceinline__ void unpack8f(const uint4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
// (m2, s): running max of x*log2e and sum of 2^(x*log2e - m2); argmax over the lane's elements
__device__ __forceinline__ void row_pass_vec(const bf16_t* __restrict__ x, int C, int lane, float& m2, float& s,
                                             float& vmax, int& amax) {
  m2 = -INFINITY; s = 0.f; vmax = -INFINITY; amax = 0;
  const uint4* x8 = reinterpret_cast<const uint4*>(x);
  const int n8 = (C + 7) / 8;   // the row is padded to a multiple of 8 (ld); pad columns masked
  for (int c8 = lane; c8 < n8; c8 += 64) {
    float f[8];
    unpack8f(x8[c8], f);
    if (c8 * 8 + 8 > C) {
#pragma unroll
      for (int k = 0; k < 8; ++k) if (c8 * 8 + k >= C) f[k] = -INFINITY;
    }
    float cm = f[0];
    int ci = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) if (f[k] > cm) { cm = f[k]; ci = k; }
    if (cm > vmax) { vmax = cm; amax = c8 * 8 + ci; }
    const float mn = fmaxf(m2, cm * LOG2E_CE);
    float add = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) add += __builtin_amdgcn_exp2f(fmaf(f[k], LOG2E_CE, -mn));
    s = (m2 == -INFINITY ? 0.f : s * __builtin_amdgcn_exp2f(m2 - mn)) + add;
    m2 = mn;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_ce_fwd(const T* __restrict__ logits, const long long* __restrict__ labels,
                                                float* __restrict__ lse, float* __restrict__ rowloss,
                                                float* __restrict__ rowcorrect, int B, int C, int ld,
                                                long long ignore, unsigned* __restrict__ ticket,
                                                float* __restrict__ out3) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row < B) {
    const T* x = logits + (long long)row * ld;
    float m = -INFINITY, s = 0.f;
    int amax = 0;
    float vmax = -INFINITY;
    if (sizeof(T) == 2 && (ld & 7) == 0) {
      float m2;
      row_pass_vec(reinterpret_cast<const bf16_t*>(x), C, lane, m2, s, vmax, amax);
      m = m2 * 0.69314718055994531f;   // back to natural-log units for the combine below
    } else {
      for (int c = lane; c < C; c += 64) {
        const float v = ldf<T>(x + c);
        if (v > vmax) { vmax = v; amax = c; }
        if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
        else s += __expf(v - m);
      }
    }
    // combine (m, s) across the wave
  #pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
      const float mn = fmaxf(m, mo);
      s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
      m = mn;
      const float vo = __shfl_xor(vmax, o, 64);
      const int ao = __shfl_xor(amax, o, 64);
      if (vo > vmax || (vo == vmax && ao < amax)) { vmax = vo; amax = ao; }
    }
    if (lane == 0) {
      const long long y = labels[row];
      const float l = m + __logf(s);
      lse[row] = l;
      const bool skip = (y == ignore || y < 0 || y >= C);
      const float rl = skip ? 0.f : l - ldf<T>(x + y);
      const float rc = skip ? -1.f : ((amax == (int)y) ? 1.f : 0.f);
      if (ticket) { st_sc1(rowloss + row, rl); st_sc1(rowcorrect + row, rc); }
      else { rowloss[row] = rl; rowcorrect[row] = rc; }
    }
  }
  if (!ticket) return;
  // in-launch fold: drain the sc1 row stores, one ticket per block, the last block folds
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (last) ce_fold<true>(rowloss, rowcorrect, out3, B);
}

// out[0] = sum loss / valid, out[1] = correct count, out[2] = valid rows
__global__ __launch_bounds__(1024) void k_ce_reduce(const float* __restrict__ rowloss,
                                                    const float* __restrict__ rowcorrect, float* __restrict__ out,
                                                    int B) {
  ce_fold<false>(rowloss, rowcorrect, out, B);
}

template <typename T>
__global__ __launch_bounds__(256) void k_ce_bwd(const T* __restrict__ logits, const long long* __restrict__ labels,
                                                const float* __restrict__ lse, const float* __restrict__ red,
                                                const float* __restrict__ grad_out, T* __restrict__ dlogits, int B,
                                                int C, int ld, long long ignore) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const long long y = labels[row];
  const bool skip = (y == ignore || y < 0 || y >= C);
  const float valid = red[2];
  const float g = (grad_out ? *grad_out : 1.f) / fmaxf(valid, 1.f);
  const float l = lse[row];
  const T* x = logits + (long long)row * ld;
  T* d = dlogits + (long long)row * ld;
  if constexpr (sizeof(T) == 2) {
    if ((ld & 7) == 0) {   // 16-byte loads / stores, base-2 exponentials; pad columns -> 0
      const uint4* x8 = reinterpret_cast<const uint4*>(x);
      uint4* d8 = reinterpret_cast<uint4*>(d);
      const float l2 = l * LOG2E_CE;
      for (int c8 = lane; c8 < ld / 8; c8 += 64) {
        float f[8];
        unpack8f(x8[c8], f);
        unsigned o[4];
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const int c = c8 * 8 + k;
          const float a = (skip || c >= C) ? 0.f
                          : (__builtin_amdgcn_exp2f(fmaf(f[k], LOG2E_CE, -l2)) - (c == y ? 1.f : 0.f)) * g;
          const float b = (skip || c + 1 >= C) ? 0.f
                          : (__builtin_amdgcn_exp2f(fmaf(f[k + 1], LOG2E_CE, -l2)) - (c + 1 == y ? 1.f : 0.f)) * g;
          o[k / 2] = pack_bf2(a, b);
        }
        d8[c8] = make_uint4(o[0], o[1], o[2], o[3]);
      }
      return;
    }
  }
  for (int c = lane; c < ld; c += 64) {
    float v = (skip || c >= C) ? 0.f : (__expf(ldf<T>(x + c) - l) - (c == y ? 1.f : 0.f)) * g;
    if constexpr (sizeof(T) == 2) d[c] = f2bf(v); else d[c] = v;
  }
}

// k_ce_bwd (bf16 vector path) that also produces the column sums of dlogits — the bias
// gradient of the Linear that produced the logits (its own column-sum pass is skipped).  A
// block owns CE_BIAS_ROWS rows: each wave sums its 4 rows (in row order) into its own LDS row
// ([4][ld] fp32, ld <= 4096), the 4 wave rows are combined into one partial row
// part[block][CP] (write-through stores); the last block to arrive (agent-scope ticket) sums
// the G = ceil(B / 16) partial rows in block order — one thread per float4 column, all G loads
// in flight at once — and stores (acc = 0) or adds (acc = 1) them into dbias: deterministic,
// one writer per element, no zeroed buffer needed.
constexpr int CE_BIAS_ROWS = 16;

__global__ __launch_bounds__(256) void k_ce_bwd_bias(const bf16_t* __restrict__ logits,
                                                     const long long* __restrict__ labels,
                                                     const float* __restrict__ lse, const float* __restrict__ red,
                                                     const float* __restrict__ grad_out, bf16_t* __restrict__ dlogits,
                                                     float* __restrict__ dbias, int B, int C, int ld,
                                                     long long ignore, float* __restrict__ part,
                                                     unsigned* __restrict__ ticket, int acc) {
  extern __shared__ float colsh[];  // [4][ld]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float valid = red[2];
  const float g = (grad_out ? *grad_out : 1.f) / fmaxf(valid, 1.f);
  float* mine = colsh + w * ld;
  for (int r = 0; r < CE_BIAS_ROWS / 4; ++r) {
    const int row = blockIdx.x * CE_BIAS_ROWS + w * (CE_BIAS_ROWS / 4) + r;
    const bool have = row < B;
    const long long y = have ? labels[row] : -1;
    const bool skip = !have || (y == ignore || y < 0 || y >= C);
    const float l = have ? lse[row] : 0.f;
    const float l2 = l * LOG2E_CE;
    const uint4* x8 = reinterpret_cast<const uint4*>(logits + (long long)(have ? row : 0) * ld);
    uint4* d8 = reinterpret_cast<uint4*>(dlogits + (long long)(have ? row : 0) * ld);
    for (int c8 = lane; c8 < ld / 8; c8 += 64) {
      float f[8];
      unpack8f(x8[c8], f);
      unsigned o[4];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        const int c = c8 * 8 + k;
        const float a = (skip || c >= C) ? 0.f
                        : (__builtin_amdgcn_exp2f(fmaf(f[k], LOG2E_CE, -l2)) - (c == y ? 1.f : 0.f)) * g;
        const float b = (skip || c + 1 >= C) ? 0.f
                        : (__builtin_amdgcn_exp2f(fmaf(f[k + 1], LOG2E_CE, -l2)) - (c + 1 == y ? 1.f : 0.f)) * g;
        o[k / 2] = pack_bf2(a, b);
        // the bf16 gradient the Linear would column-sum; each lane owns its columns, so the
        // running sum over the wave's rows needs no barrier
        mine[c] = r ? mine[c] + lo_bf(o[k / 2]) : lo_bf(o[k / 2]);
        mine[c + 1] = r ? mine[c + 1] + hi_bf(o[k / 2]) : hi_bf(o[k / 2]);
      }
      if (have) d8[c8] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  __syncthreads();
  // partial row of this block, published write-through (sc1): no release fence
  // (CDNA guide §6 G16 R1); the row is padded to CP (multiple of 4) for 16-byte access
  const int CP = (C + 3) & ~3;
  float* mine_row = part + (long long)blockIdx.x * CP;
  for (int c = threadIdx.x; c < CP; c += 256) {
    const float v = c < C ? (colsh[c] + colsh[ld + c]) + (colsh[2 * ld + c] + colsh[3 * ld + c]) : 0.f;
    __hip_atomic_store(mine_row + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // graph-replay safe
    }
  }
  __syncthreads();
  if (!last) return;
  // last block: column sums of the G partial rows in block order, 16 loads per batch
  const int G = (int)gridDim.x;
  const int C4 = CP / 4;
  for (int j = threadIdx.x; j < C4; j += 256) {
    const float4* col = reinterpret_cast<const float4*>(part) + j;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int g0 = 0; g0 < G; g0 += 16) {
      float4 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = g0 + k < G ? col[(long long)(g0 + k) * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        t.x += v[k].x; t.y += v[k].y; t.z += v[k].z; t.w += v[k].w;
      }
    }
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * j + e;
      if (c < C) dbias[c] = acc ? dbias[c] + tv[e] : tv[e];
    }
  }
}

}  // namespace

// dtype: 0 = bf16 logits, 1 = fp32 logits.  ws = [3*B] fp32 workspace (lse, rowloss, rowcorrect).
// ticket: a zeroed device counter (reset by the kernel) -> one launch; null -> fold in a 2nd launch.
// ld: row stride of the logits (>= C; a row padded to 16 bytes keeps the vector path, the
// pad columns are ignored in the forward and written as 0 in the gradient)
KML_API int kml_ce_fwd(const void* logits, const long long* labels, float* ws, float* out3, int B, int C, int ld,
                       long long ignore, int dtype, unsigned* ticket, hipStream_t s) {
  if (B < 1 || ld < C) return (int)hipErrorInvalidValue;
  dim3 g((B + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(k_ce_fwd<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)logits, labels, ws, ws + B, ws + 2 * B,
                       B, C, ld, ignore, ticket, out3);
  else
    hipLaunchKernelGGL(k_ce_fwd<float>, g, dim3(256), 0, s, (const float*)logits, labels, ws, ws + B, ws + 2 * B, B,
                       C, ld, ignore, ticket, out3);
  if (!ticket) hipLaunchKernelGGL(k_ce_reduce, dim3(1), dim3(1024), 0, s, ws + B, ws + 2 * B, out3, B);
  KML_LAUNCH_CHECK();
}

// dbias (optional; bf16 logits, ld % 8 == 0, ld <= 4096): column sums of dlogits, stored
// (accumulate = 0) or added (1); needs part = [ceil(B/16)][roundup(C, 4)] fp32 scratch and a
// zeroed ticket
KML_API int kml_ce_bwd(const void* logits, const long long* labels, const float* ws, const float* out3,
                       const float* grad_out, void* dlogits, int B, int C, int ld, long long ignore, int dtype,
                       float* dbias, float* part, unsigned* ticket, int accumulate, hipStream_t s) {
  if (ld < C) return (int)hipErrorInvalidValue;
  dim3 g((B + 3) / 4);
  if (dbias) {
    if (dtype != 0 || ld % 8 || ld > 4096 || !part || !ticket) return (int)hipErrorInvalidValue;
    const size_t shm = (size_t)4 * ld * sizeof(float);
    hipLaunchKernelGGL(k_ce_bwd_bias, dim3((B + CE_BIAS_ROWS - 1) / CE_BIAS_ROWS), dim3(256), shm, s, (const bf16_t*)logits, labels,
                       ws, out3, grad_out, (bf16_t*)dlogits, dbias, B, C, ld, ignore, part, ticket, accumulate);
    KML_LAUNCH_CHECK();
  }
  if (dtype == 0)
    hipLaunchKernelGGL(k_ce_bwd<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)logits, labels, ws, out3, grad_out,
                       (bf16_t*)dlogits, B, C, ld, ignore);
  else
    hipLaunchKernelGGL(k_ce_bwd<float>, g, dim3(256), 0, s, (const float*)logits, labels, ws, out3, grad_out,
                       (float*)dlogits, B, C, ld, ignore);
  KML_LAUNCH_CHECK();
}
