// bn.hip — BatchNorm2d (NHWC, bf16 activations, fp32 statistics) for gfx950.
//
// Training forward is split as   conv(+stats epilogue)  ->  bn_apply
// so the per-channel sum / sum-of-squares come for free from the producing GEMM
// (conv_igemm.hip).  kml_bn_stats exists for inputs that were not produced by our
// conv (user models).  bn_apply fuses: normalisation, affine, optional residual
// add and optional ReLU, plus the running-stat update (momentum, unbiased var) and
// the saved mean / inv-std used by backward.
//
// Backward is two streaming passes:
//   bn_bwd_reduce : dz = dy * [y > 0] (if ReLU);  dbeta += sum dz,  dgamma += sum dz*xhat
//                   (accumulated straight into the flat fp32 gradient buffer)
//   bn_bwd_apply  : dx = gamma*rstd*(dz - (dbeta + xhat*dgamma)/M), and optionally
//                   dres = dz (gradient of the residual branch).
// All loads are 16 B per lane (8 channels), C % 8 == 0.
//
// Reference parity: torch.nn.BatchNorm2d semantics (momentum 0.1, eps 1e-5, biased
// batch variance for normalisation, unbiased for the running estimate), which the
// reference gets from cuDNN through torchvision resnet34 (function_resnet34.py:101).
#include "kml_common.h"
#include "kml_sgd.h"

#include <cstdlib>
#include <cstring>

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]); v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]); v.w = pack_bf2(f[6], f[7]);
  return v;
}

// column sums over an [M][C] bf16 matrix: out[0..C) += sum x, out[C..2C) += sum x^2
// Each thread owns one 8-channel chunk; threads sharing a chunk are reduced in LDS.
__global__ __launch_bounds__(TPB) void k_bn_stats(const bf16_t* __restrict__ x, float* __restrict__ stats,
                                                  long long M, int C) {
  const int CH = C / 8;                 // chunks per row
  const int rows_per_iter = TPB / CH;   // CH <= 256 assumed (C <= 2048)
  const int tid = threadIdx.x;
  const int chunk = tid % CH, rsub = tid / CH;
  float s1[8] = {0}, s2[8] = {0};
  if (rsub < rows_per_iter) {
    for (long long r = (long long)blockIdx.x * rows_per_iter + rsub; r < M;
         r += (long long)gridDim.x * rows_per_iter) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + r * C + chunk * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s1[i] += f[i]; s2[i] += f[i] * f[i]; }
    }
  }
  __shared__ float red[TPB][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = s1[i]; red[tid][8 + i] = s2[i]; }
  __syncthreads();
  if (tid < CH) {
    float a1[8] = {0}, a2[8] = {0};
    for (int rr = 0; rr < rows_per_iter; ++rr) {
      const int t = rr * CH + tid;
#pragma unroll
      for (int i = 0; i < 8; ++i) { a1[i] += red[t][i]; a2[i] += red[t][8 + i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(stats + tid * 8 + i, a1[i]);
      atomicAdd(stats + C + tid * 8 + i, a2[i]);
    }
  }
}


// partial-row variant: block b writes its [sum | sumsq] row into part[b][2C] (plain
// stores); bn_apply(stats_rows = gridDim) sums the rows — no zeroing, no atomics.
__global__ __launch_bounds__(TPB) void k_bn_stats_part(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                       long long M, int C, int rows_per_block) {
  const int CH = C / 8;
  const int rows_per_iter = TPB / CH;
  const int tid = threadIdx.x;
  const int chunk = tid % CH, rsub = tid / CH;
  float s1[8] = {0}, s2[8] = {0};
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  if (rsub < rows_per_iter) {
#pragma unroll 2
    for (long long r = r0 + rsub; r < r1; r += rows_per_iter) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + r * C + chunk * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s1[i] += f[i]; s2[i] += f[i] * f[i]; }
    }
  }
  __shared__ float red[TPB][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = s1[i]; red[tid][8 + i] = s2[i]; }
  __syncthreads();
  if (tid < CH) {
    float a1[8] = {0}, a2[8] = {0};
    for (int rr = 0; rr < rows_per_iter; ++rr) {
      const int t = rr * CH + tid;
#pragma unroll
      for (int i = 0; i < 8; ++i) { a1[i] += red[t][i]; a2[i] += red[t][8 + i]; }
    }
    float* row = part + (long long)blockIdx.x * 2 * C;
#pragma unroll
    for (int i = 0; i < 8; ++i) { row[tid * 8 + i] = a1[i]; row[C + tid * 8 + i] = a2[i]; }
  }
}

// Rows g0, g0+S, ... < G of one float4 column, summed in that order with 16 loads in
// flight per thread: the rows were just written by the producing kernel (other XCDs), so
// every batch of loads is a full memory round trip and the batch depth sets the latency.
// Loads past the last row re-read row G-1 (clamped, never branched around: a branch per
// load would serialise the batch) and are selected out of the sum.
__device__ __forceinline__ float4 sum_rows_strided(const float4* __restrict__ p4, int g0, int G, int S, int Q) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int U = 16;
  for (int g = g0; g < G; g += U * S) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p4[(long long)min(g + u * S, G - 1) * Q];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = g + u * S < G;
      acc.x += in ? v[u].x : 0.f; acc.y += in ? v[u].y : 0.f;
      acc.z += in ? v[u].z : 0.f; acc.w += in ? v[u].w : 0.f;
    }
  }
  return acc;
}

// Sum G rows of a [G][W4*4] fp32 partial matrix into out[W4*4] (LDS), column groups of
// float4 x row slices with independent loads in flight; scratch: TPB float4 of LDS.
template <int NT>
__device__ void sum_partial_rows(const float* __restrict__ part, int G, int W, float* out, float4* scratch) {
  const int Q = W / 4;
  const int QT = Q < NT ? Q : NT;
  const int S = NT / QT;
  for (int q0 = 0; q0 < Q; q0 += QT) {
    const int q = q0 + (int)(threadIdx.x % QT);
    const int sl = threadIdx.x / QT;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < Q && sl < S) acc = sum_rows_strided(reinterpret_cast<const float4*>(part) + q, sl, G, S, Q);
    scratch[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < QT && q < Q) {
      float4 t4 = scratch[threadIdx.x];
      for (int k = 1; k < S; ++k) {
        const float4 v = scratch[k * QT + threadIdx.x];
        t4.x += v.x; t4.y += v.y; t4.z += v.z; t4.w += v.w;
      }
      reinterpret_cast<float4*>(out)[q] = t4;
    }
    __syncthreads();
  }
}

// sum_partial_rows split in two so its first batch of loads can be ISSUED before the
// caller's data loads (vmcnt retires in issue order: a row sum issued after the data
// would wait for the data's HBM round trip).  Single pass over the columns (W/4 <= NT);
// rows beyond the first batch of 16 per slice are summed in finish().
struct EarlyRows {
  float4 v[16];
  int q, sl, S, Q;
  __device__ __forceinline__ void issue(const float* __restrict__ part, int G, int W, int nt) {
    Q = W / 4;
    S = nt / Q;
    q = (int)threadIdx.x % Q;
    sl = (int)threadIdx.x / Q;
    const float4* p4 = reinterpret_cast<const float4*>(part) + q;
    if (sl < S) {
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p4[(long long)min(sl + u * S, G - 1) * Q];
    }
  }
  __device__ __forceinline__ void finish(const float* __restrict__ part, int G, float* out, float4* scratch) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sl < S) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const bool in = sl + u * S < G;
        acc.x += in ? v[u].x : 0.f; acc.y += in ? v[u].y : 0.f;
        acc.z += in ? v[u].z : 0.f; acc.w += in ? v[u].w : 0.f;
      }
      if (sl + 16 * S < G) {
        const float4 r = sum_rows_strided(reinterpret_cast<const float4*>(part) + q, sl + 16 * S, G, S, Q);
        acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
      }
    }
    scratch[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < Q) {
      float4 t4 = scratch[threadIdx.x];
      for (int k = 1; k < S; ++k) {
        const float4 w = scratch[k * Q + threadIdx.x];
        t4.x += w.x; t4.y += w.y; t4.z += w.z; t4.w += w.w;
      }
      reinterpret_cast<float4*>(out)[threadIdx.x] = t4;
    }
    __syncthreads();
  }
};

// y = act((x - mean) * rstd * gamma + beta [+ res])
// mode 0: training (stats = [sum, sumsq] over M rows); mode 1: eval (running stats)
template <int NT>
__global__ __launch_bounds__(NT) void k_bn_apply(
    const bf16_t* __restrict__ x, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
    float* __restrict__ save_mean, float* __restrict__ save_rstd, float* __restrict__ run_mean,
    float* __restrict__ run_var, long long M, int C, float eps, float momentum, int relu, int mode,
    int stats_rows) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // scale[C], shift[C], (sums[2C], scratch)
  float* scale = sh;
  float* shift = sh + C;
  // first iteration's operands in flight while the statistics are summed (the prologue and
  // this load are two dependent memory round trips otherwise)
  const long long n8 = M * C / 8;
  const long long i0 = blockIdx.x * (long long)NT + threadIdx.x;
  uint4 x0 = make_uint4(0, 0, 0, 0), r0 = make_uint4(0, 0, 0, 0);
  if (i0 < n8) {
    x0 = reinterpret_cast<const uint4*>(x)[i0];
    if (res) r0 = reinterpret_cast<const uint4*>(res)[i0];
  }
  const float* st = stats;
  if (mode == 0 && stats_rows > 0) {  // per-wave partial rows written by the conv epilogue
    float* sums = sh + 2 * C;
    sum_partial_rows<NT>(stats, stats_rows, 2 * C, sums, reinterpret_cast<float4*>(sh + 4 * C));
    st = sums;
  }
  for (int c = threadIdx.x; c < C; c += NT) {
    float mean, var;
    if (mode == 0) {
      mean = st[c] / (float)M;
      var = fmaxf(st[C + c] / (float)M - mean * mean, 0.f);
    } else {
      mean = run_mean[c];
      var = run_var[c];
    }
    const float rstd = rsqrtf(var + eps);
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    scale[c] = g * rstd;
    shift[c] = bb - mean * g * rstd;
    if (mode == 0 && blockIdx.x == 0) {
      if (save_mean) { save_mean[c] = mean; save_rstd[c] = rstd; }
      if (run_mean) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
      }
    }
  }
  __syncthreads();
  const int CH = C / 8;
  for (long long i = i0; i < n8; i += (long long)gridDim.x * NT) {
    const int c0 = (int)(i % CH) * 8;
    float f[8];
    unpack8(i == i0 ? x0 : reinterpret_cast<const uint4*>(x)[i], f);
    float r[8];
    if (res) unpack8(i == i0 ? r0 : reinterpret_cast<const uint4*>(res)[i], r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = f[k] * scale[c0 + k] + shift[c0 + k];
      if (res) v += r[k];
      if (relu) v = fmaxf(v, 0.f);
      f[k] = v;
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

// dz = dy * [y>0];  dbeta += sum dz;  dgamma += sum dz * (x - mean) * rstd
__global__ __launch_bounds__(TPB) void k_bn_bwd_reduce(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, long long M, int C) {
  const int CH = C / 8;
  const int rows_per_iter = TPB / CH;
  const int tid = threadIdx.x;
  const int chunk = tid % CH, rsub = tid / CH;
  float sd[8] = {0}, sx[8] = {0}, mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { mu[i] = mean[chunk * 8 + i]; rs[i] = rstd[chunk * 8 + i]; }
  if (rsub < rows_per_iter) {
    for (long long r = (long long)blockIdx.x * rows_per_iter + rsub; r < M;
         r += (long long)gridDim.x * rows_per_iter) {
      const long long off = r * C + chunk * 8;
      float d[8], xv[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + off), d);
      unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
      if (y) {
        float yv[8];
        unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) { sd[i] += d[i]; sx[i] += d[i] * (xv[i] - mu[i]) * rs[i]; }
    }
  }
  __shared__ float red[TPB][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = sd[i]; red[tid][8 + i] = sx[i]; }
  __syncthreads();
  if (tid < CH) {
    float a1[8] = {0}, a2[8] = {0};
    for (int rr = 0; rr < rows_per_iter; ++rr) {
      const int t = rr * CH + tid;
#pragma unroll
      for (int i = 0; i < 8; ++i) { a1[i] += red[t][i]; a2[i] += red[t][8 + i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(dbeta + tid * 8 + i, a1[i]);
      atomicAdd(dgamma + tid * 8 + i, a2[i]);
    }
  }
}

// Two-level deterministic variant of k_bn_bwd_reduce: every block reduces a contiguous
// row range into part[block][2C] (no atomics), then the last block to arrive (ticket)
// sums the partials in block order and adds them into dbeta/dgamma.  Gives ~8x more
// blocks than the atomic version without same-address atomic contention (which crosses
// XCD L2s), and bitwise-reproducible gradients.
template <int RMODE>  // 0: partials + last-arriver reduce, 1: atomics, 2: partials only
__global__ __launch_bounds__(TPB) void k_bn_bwd_reduce2(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ part, unsigned* __restrict__ counter, long long M, int C,
    int rows_per_block) {
  const int CH = C / 8;
  const int rows_per_iter = TPB / CH;
  const int tid = threadIdx.x;
  const int chunk = tid % CH, rsub = tid / CH;
  float sd[8] = {0}, sx[8] = {0}, mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { mu[i] = mean[chunk * 8 + i]; rs[i] = rstd[chunk * 8 + i]; }
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  if (rsub < rows_per_iter) {
#pragma unroll 2
    for (long long r = r0 + rsub; r < r1; r += rows_per_iter) {
      const long long off = r * C + chunk * 8;
      float d[8], xv[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + off), d);
      unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
      if (y) {
        float yv[8];
        unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) { sd[i] += d[i]; sx[i] += d[i] * (xv[i] - mu[i]) * rs[i]; }
    }
  }
  __shared__ float red[TPB][17];
  __shared__ unsigned last;
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = sd[i]; red[tid][8 + i] = sx[i]; }
  __syncthreads();
  if (RMODE == 1) {
    // memory-side fp32 atomics: no agent-scope release (which would write back the
    // XCD's whole dirty L2 per block) — the fast default
    if (tid < CH) {
      float a1[8] = {0}, a2[8] = {0};
      for (int rr = 0; rr < rows_per_iter; ++rr) {
        const int t = rr * CH + tid;
#pragma unroll
        for (int i = 0; i < 8; ++i) { a1[i] += red[t][i]; a2[i] += red[t][8 + i]; }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        atomicAdd(dbeta + tid * 8 + i, a1[i]);
        atomicAdd(dgamma + tid * 8 + i, a2[i]);
      }
    }
    return;
  }
  float* mine = part + (long long)blockIdx.x * 2 * C;
  if (tid < CH) {
    float a1[8] = {0}, a2[8] = {0};
    for (int rr = 0; rr < rows_per_iter; ++rr) {
      const int t = rr * CH + tid;
#pragma unroll
      for (int i = 0; i < 8; ++i) { a1[i] += red[t][i]; a2[i] += red[t][8 + i]; }
    }
    float4* o = reinterpret_cast<float4*>(mine);
    o[tid * 2] = make_float4(a1[0], a1[1], a1[2], a1[3]);
    o[tid * 2 + 1] = make_float4(a1[4], a1[5], a1[6], a1[7]);
    o[CH * 2 + tid * 2] = make_float4(a2[0], a2[1], a2[2], a2[3]);
    o[CH * 2 + tid * 2 + 1] = make_float4(a2[4], a2[5], a2[6], a2[7]);
  }
  if (RMODE == 2) return;  // the apply kernel sums the partials (kernel boundary = visibility)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned l = (t == gridDim.x - 1) ? 1u : 0u;
    if (l) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  // last arriver: sum G partial rows of 2C floats, float4 groups x row slices
  const int Q = C / 2;                       // float4 groups per partial row
  const int S = Q >= TPB ? 1 : TPB / Q;      // row slices
  const int G = gridDim.x;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int q = tid % (Q < TPB ? Q : TPB); q < Q; q += TPB) {
    const int sl = Q >= TPB ? 0 : tid / Q;
    if (sl >= S) break;
    acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int g = sl; g < G; g += S) {
      const float4 v = reinterpret_cast<const float4*>(part + (long long)g * 2 * C)[q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (S == 1) {
      float* dst = q < Q / 2 ? dbeta + q * 4 : dgamma + (q - Q / 2) * 4;
      dst[0] += acc.x; dst[1] += acc.y; dst[2] += acc.z; dst[3] += acc.w;
    }
  }
  if (S == 1) return;
  // S > 1: combine slices through LDS (reuse red as [S][Q] float4 = 4*TPB floats)
  float4* r4 = reinterpret_cast<float4*>(&red[0][0]);
  __syncthreads();
  if (tid < S * Q) r4[tid] = acc;
  __syncthreads();
  if (tid < Q) {
    float4 t4 = r4[tid];
    for (int sl = 1; sl < S; ++sl) {
      const float4 v = r4[sl * Q + tid];
      t4.x += v.x; t4.y += v.y; t4.z += v.z; t4.w += v.w;
    }
    float* dst = tid < Q / 2 ? dbeta + tid * 4 : dgamma + (tid - Q / 2) * 4;
    dst[0] += t4.x; dst[1] += t4.y; dst[2] += t4.z; dst[3] += t4.w;
  }
}

__global__ __launch_bounds__(TPB) void k_bn_bwd_apply(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ dgamma, const float* __restrict__ dbeta, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dres, long long M, int C) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // a[C], b[C], mu[C], rs[C]
  float* ka = sh;          // gamma*rstd
  float* kb = sh + C;      // dbeta/M
  float* kc = sh + 2 * C;  // dgamma/M
  float* mu = sh + 3 * C;
  float* rs = sh + 4 * C;
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += TPB) {
    const float g = gamma ? gamma[c] : 1.f;
    ka[c] = g * rstd[c];
    kb[c] = dbeta[c] * invM;
    kc[c] = dgamma[c] * invM;
    mu[c] = mean[c];
    rs[c] = rstd[c];
  }
  __syncthreads();
  const long long n8 = M * C / 8;
  const int CH = C / 8;
  for (long long i = blockIdx.x * (long long)TPB + threadIdx.x; i < n8; i += (long long)gridDim.x * TPB) {
    const int c0 = (int)(i % CH) * 8;
    float d[8], xv[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], d);
    unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
    if (y) {
      float yv[8];
      unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
    }
    if (dres) reinterpret_cast<uint4*>(dres)[i] = pack8(d);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float xh = (xv[k] - mu[c]) * rs[c];
      o[k] = ka[c] * (d[k] - kb[c] - xh * kc[c]);
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(o);
  }
}

// bn_bwd_apply with the dgamma/dbeta reduction fused in: every block sums the G
// per-block partials [G][2C] (dbeta | dgamma) of k_bn_bwd_reduce2<2> in a fixed order
// (deterministic; no atomics, no fences — the kernel boundary makes them visible);
// block 0 also adds the sums into the parameter gradients.
template <int NT>
__global__ __launch_bounds__(NT) void k_bn_bwd_apply_fin(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ part, int G, float* __restrict__ dgamma, float* __restrict__ dbeta,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, long long M, int C, int acc) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // red4 scratch [4*NT], ka kb kc mu rs [C]
  float4* red4 = reinterpret_cast<float4*>(sh);
  float* ka = sh + 4 * NT;
  float* kb = ka + C;
  float* kc = ka + 2 * C;
  float* mu = ka + 3 * C;
  float* rs = ka + 4 * C;
  const float invM = 1.f / (float)M;
  // first iteration's operands in flight while the partial rows are summed
  const long long n8 = M * C / 8;
  const long long i0 = blockIdx.x * (long long)NT + threadIdx.x;
  uint4 dy0 = make_uint4(0, 0, 0, 0), x0 = dy0, y0 = dy0;
  if (i0 < n8) {
    dy0 = reinterpret_cast<const uint4*>(dy)[i0];
    x0 = reinterpret_cast<const uint4*>(x)[i0];
    if (y) y0 = reinterpret_cast<const uint4*>(y)[i0];
  }
  // sum the G partial rows of 2C floats: float4 column groups x row slices (several
  // independent loads in flight per thread), slices combined through LDS
  const int Q = C / 2;                         // float4 groups per partial row
  const int QT = Q < NT ? Q : NT;            // groups handled per pass
  const int S = NT / QT;                      // row slices per pass
  for (int q0 = 0; q0 < Q; q0 += QT) {
    const int q = q0 + (int)(threadIdx.x % QT);
    const int sl = threadIdx.x / QT;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < Q) acc = sum_rows_strided(reinterpret_cast<const float4*>(part) + q, sl, G, S, Q);
    red4[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < QT && q < Q) {
      float4 t4 = red4[threadIdx.x];
      for (int k = 1; k < S; ++k) {
        const float4 v = red4[k * QT + threadIdx.x];
        t4.x += v.x; t4.y += v.y; t4.z += v.z; t4.w += v.w;
      }
      const float vals[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = 4 * q + k;               // [dbeta (C) | dgamma (C)]
        if (col < C) kb[col] = vals[k];
        else kc[col - C] = vals[k];
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < C; c += NT) {
    const float sb = kb[c], sg = kc[c];
    if (blockIdx.x == 0) {  // one writer: store (overwrite) or add (accumulate)
      dbeta[c] = acc ? dbeta[c] + sb : sb;
      dgamma[c] = acc ? dgamma[c] + sg : sg;
    }
    const float gm = gamma ? gamma[c] : 1.f;
    ka[c] = gm * rstd[c];
    kb[c] = sb * invM;
    kc[c] = sg * invM;
    mu[c] = mean[c];
    rs[c] = rstd[c];
  }
  __syncthreads();
  const int CH = C / 8;
  for (long long i = i0; i < n8; i += (long long)gridDim.x * NT) {
    const int c0 = (int)(i % CH) * 8;
    float d[8], xv[8];
    unpack8(i == i0 ? dy0 : reinterpret_cast<const uint4*>(dy)[i], d);
    unpack8(i == i0 ? x0 : reinterpret_cast<const uint4*>(x)[i], xv);
    if (y) {
      float yv[8];
      unpack8(i == i0 ? y0 : reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
    }
    if (dres) reinterpret_cast<uint4*>(dres)[i] = pack8(d);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float xh = (xv[k] - mu[c]) * rs[c];
      o[k] = ka[c] * (d[k] - kb[c] - xh * kc[c]);
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(o);
  }
}

// Channel-transposed coefficient slots: channel c at (c % 8) * TSTRIDE + c / 8.  The apply loops
// read slot k * TSTRIDE + j (j consecutive across lanes: conflict-free for any stride); the
// per-channel writes (lane = channel; ds_write_b32 banks are (a / 4) mod 32 per 32-lane half) are
// conflict-free when TSTRIDE = 4 (mod 32): a half's 32 (c % 8, c / 8) pairs then map onto 32
// distinct banks.  The unpadded C / 8 stride put them on 8 and was most of these kernels' LDS
// bank conflicts (k_bn_bwd_apply_v 44 %, k_bn_apply_v 38 %; profiles/r6/bn_lds.md).
__host__ __device__ constexpr int bn_tstride(int ch8) { return ch8 + (((4 - ch8) % 32) + 32) % 32; }
__host__ __device__ constexpr int bn_tslots(int C) { return 8 * bn_tstride(C >> 3); }

// ---------------------------------------------------------------------------------------
// Register-resident apply kernels (the default).  Each thread owns V 16-byte chunks
// i0, i0 + T, ..., T = grid * NT a multiple of C/8, so all its chunks hold the SAME 8
// channels: their scale / shift (or the backward coefficients) are read from LDS once,
// into registers, and no per-element channel division or LDS read remains.  All V chunks
// of every operand are loaded up front — before the statistics prologue — so the data
// round trip overlaps the partial-row reduction instead of following it, and a thread
// never waits on more than one memory round trip.  Out-of-range chunks load a clamped
// (valid) index and skip the store (no branch around a load: straight-line vmcnt).
// ---------------------------------------------------------------------------------------
struct BnApArgs {
  const bf16_t* x;
  const float* stats;
  const float* gamma;
  const float* beta;
  const bf16_t* res;
  bf16_t* y;
  float* save_mean;
  float* save_rstd;
  float* run_mean;
  float* run_var;
  long long M;
  int C;
  float eps, momentum;
  int relu, mode, stats_rows;
};

// one block (bid of nblk) of the apply; k_bn_apply_v runs it over its grid, k_bn_apply_pair over
// a shared one
template <int NT, int V, bool PIPE>
__device__ __forceinline__ void bn_apply_body(const BnApArgs& p, int bid, int nblk, float* sh) {
  const bf16_t* __restrict__ x = p.x;
  const float* __restrict__ stats = p.stats;
  const float* __restrict__ gamma = p.gamma;
  const float* __restrict__ beta = p.beta;
  const bf16_t* __restrict__ res = p.res;
  bf16_t* __restrict__ y = p.y;
  float* __restrict__ save_mean = p.save_mean;
  float* __restrict__ save_rstd = p.save_rstd;
  float* __restrict__ run_mean = p.run_mean;
  float* __restrict__ run_var = p.run_var;
  const long long M = p.M;
  const int C = p.C, relu = p.relu, mode = p.mode, stats_rows = p.stats_rows;
  const float eps = p.eps, momentum = p.momentum;
  // sh: scale[TS], shift[TS], (sums[2C], scratch)
  const int TS = bn_tslots(C), TSTR = bn_tstride(C >> 3);
  float* scale = sh;
  float* shift = sh + TS;
  const int n8 = (int)(M * C / 8);
  const int T = nblk * NT;
  const int i0 = bid * NT + (int)threadIdx.x;
  const bool parts = mode == 0 && stats_rows > 0;
  const bool early = parts && C / 2 <= NT;
  EarlyRows er;
  if (early) er.issue(stats, stats_rows, 2 * C, NT);
  uint4 xv[V], rv[V];
#pragma unroll
  for (int v = 0; v < V; ++v) xv[v] = reinterpret_cast<const uint4*>(x)[min(i0 + v * T, n8 - 1)];
  if (res) {
#pragma unroll
    for (int v = 0; v < V; ++v) rv[v] = reinterpret_cast<const uint4*>(res)[min(i0 + v * T, n8 - 1)];
  }
  const float* st = stats;
  if (parts) {
    float* sums = sh + 2 * TS;
    if (early) er.finish(stats, stats_rows, sums, reinterpret_cast<float4*>(sh + 2 * TS + 2 * C));
    else sum_partial_rows<NT>(stats, stats_rows, 2 * C, sums, reinterpret_cast<float4*>(sh + 2 * TS + 2 * C));
    st = sums;
  }
  for (int c = threadIdx.x; c < C; c += NT) {
    float mean, var;
    if (mode == 0) {
      mean = st[c] / (float)M;
      var = fmaxf(st[C + c] / (float)M - mean * mean, 0.f);
    } else {
      mean = run_mean[c];
      var = run_var[c];
    }
    const float rstd = rsqrtf(var + eps);
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    // channel-transposed slots (bn_tstride): the 8-channel reads below hit consecutive words
    // across consecutive lanes, these writes 64 distinct banks
    const int tslot = (c & 7) * TSTR + (c >> 3);
    scale[tslot] = g * rstd;
    shift[tslot] = bb - mean * g * rstd;
    if (mode == 0 && bid == 0) {
      if (save_mean) { save_mean[c] = mean; save_rstd[c] = rstd; }
      if (run_mean) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
      }
    }
  }
  __syncthreads();
  const int CH8 = C >> 3, j8 = i0 % CH8;
  float sc[8], sf[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = scale[k * TSTR + j8]; sf[k] = shift[k * TSTR + j8]; }
  // grid-stride batches of V chunks (large tensors); T % (C/8) == 0 keeps the channels.
  // PIPE (the host's choice when a thread has more than one batch): each chunk's register is
  // refilled with the next batch's chunk right after its store, so the next batch's loads are in
  // flight while this batch is still being stored (ResNet-50's 56x56 BNs +6-9 %); single-batch
  // launches (every ResNet-34 BN) keep the plain loop, whose code measured faster there
  if constexpr (PIPE) {
    for (int base = i0; base < n8; base += V * T) {
      const int nb = base + V * T;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float f[8], r[8];
        unpack8(xv[v], f);
        if (res) unpack8(rv[v], r);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float o = f[k] * sc[k] + sf[k];
          if (res) o += r[k];
          if (relu) o = fmaxf(o, 0.f);
          f[k] = o;
        }
        const int i = base + v * T;
        if (i < n8) reinterpret_cast<uint4*>(y)[i] = pack8(f);
        if (nb < n8) {
          xv[v] = reinterpret_cast<const uint4*>(x)[min(nb + v * T, n8 - 1)];
          if (res) rv[v] = reinterpret_cast<const uint4*>(res)[min(nb + v * T, n8 - 1)];
        }
      }
    }
  } else {
    for (int base = i0, it = 0; base < n8; base += V * T, ++it) {
      if (it > 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) xv[v] = reinterpret_cast<const uint4*>(x)[min(base + v * T, n8 - 1)];
        if (res) {
#pragma unroll
          for (int v = 0; v < V; ++v) rv[v] = reinterpret_cast<const uint4*>(res)[min(base + v * T, n8 - 1)];
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float f[8], r[8];
        unpack8(xv[v], f);
        if (res) unpack8(rv[v], r);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float o = f[k] * sc[k] + sf[k];
          if (res) o += r[k];
          if (relu) o = fmaxf(o, 0.f);
          f[k] = o;
        }
        const int i = base + v * T;
        if (i < n8) reinterpret_cast<uint4*>(y)[i] = pack8(f);
      }
    }
  }
}

template <int NT, int V, bool PIPE>
__global__ __launch_bounds__(NT) void k_bn_apply_v(BnApArgs p) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  bn_apply_body<NT, V, PIPE>(p, (int)blockIdx.x, (int)gridDim.x, sh);
}

// Two independent BN applies in one launch (kml_bn_apply_pair): blocks [0, n1) run the first
// over a grid of n1, the rest the second over n2 — a downsampling block's main-branch BN and its
// projection's BN, which follow one paired conv launch (k_conv_fwd_pair).
template <int NT, int V1, int V2>
__global__ __launch_bounds__(NT) void k_bn_apply_pair(BnApArgs p1, BnApArgs p2, int n1, int n2) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int b = (int)blockIdx.x;
  if (b < n1) bn_apply_body<NT, V1, false>(p1, b, n1, sh);
  else bn_apply_body<NT, V2, false>(p2, b - n1, n2, sh);
}

struct BnbArgs {
  const bf16_t* dy;
  const bf16_t* y;
  const bf16_t* x;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* part;
  int G;
  float* dgamma;
  float* dbeta;
  bf16_t* dx;
  bf16_t* dres;
  long long M;
  int C, acc;
};

// one block (bid of nblk) of the backward apply; k_bn_bwd_apply_v runs it over its grid (after
// its rider blocks split off), k_bn_bwd_apply_pair over a shared one
template <int NT, int V, bool PIPE>
__device__ __forceinline__ void bn_bwd_apply_body(const BnbArgs& p, int bid, int nblk, float* sh) {
  const bf16_t* __restrict__ dy = p.dy;
  const bf16_t* __restrict__ y = p.y;
  const bf16_t* __restrict__ x = p.x;
  const float* __restrict__ mean = p.mean;
  const float* __restrict__ rstd = p.rstd;
  const float* __restrict__ gamma = p.gamma;
  const float* __restrict__ part = p.part;
  float* __restrict__ dgamma = p.dgamma;
  float* __restrict__ dbeta = p.dbeta;
  bf16_t* __restrict__ dx = p.dx;
  bf16_t* __restrict__ dres = p.dres;
  const long long M = p.M;
  const int G = p.G, C = p.C, acc = p.acc;
  // sh: red4 scratch [4*NT], ka kb kc mu rs [C]
  float4* red4 = reinterpret_cast<float4*>(sh);
  float* ka = sh + 4 * NT;
  float* kb = ka + C;
  float* kc = ka + 2 * C;
  float* mu = ka + 3 * C;
  float* rs = ka + 4 * C;
  const float invM = 1.f / (float)M;
  const int n8 = (int)(M * C / 8);
  const int T = nblk * NT;
  const int i0 = bid * NT + (int)threadIdx.x;
  const bool early = C / 2 <= NT;
  EarlyRows er;
  if (early) er.issue(part, G, 2 * C, NT);
  uint4 dv[V], xv[V], yv[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int i = min(i0 + v * T, n8 - 1);
    dv[v] = reinterpret_cast<const uint4*>(dy)[i];
    xv[v] = reinterpret_cast<const uint4*>(x)[i];
  }
  if (y) {
#pragma unroll
    for (int v = 0; v < V; ++v) yv[v] = reinterpret_cast<const uint4*>(y)[min(i0 + v * T, n8 - 1)];
  }
  // the G partial rows [dbeta (C) | dgamma (C)] summed in a fixed order (deterministic)
  // kb | kc are contiguous: kb[0..C) kc[0..C)
  if (early) er.finish(part, G, kb, red4);
  else sum_partial_rows<NT>(part, G, 2 * C, kb, red4);
  // per-channel coefficients into channel-transposed slots (c % 8) * C/8 + c / 8 of a second
  // area (kb | kc stay readable by other channels' threads until the barrier): the 8-channel
  // reads below hit consecutive words across consecutive lanes (no LDS bank conflicts)
  float* tco = ka + 5 * C;  // [5][TS]: ka, kb/M, kc/M, mu, rs transposed (bn_tstride)
  const int TS = bn_tslots(C), TSTR = bn_tstride(C >> 3);
  for (int c = threadIdx.x; c < C; c += NT) {
    const float sb = kb[c], sg = kc[c];
    if (bid == 0) {  // one writer: store (overwrite) or add (accumulate)
      dbeta[c] = acc ? dbeta[c] + sb : sb;
      dgamma[c] = acc ? dgamma[c] + sg : sg;
    }
    const float gm = gamma ? gamma[c] : 1.f;
    const int tslot = (c & 7) * TSTR + (c >> 3);
    tco[tslot] = gm * rstd[c];
    tco[TS + tslot] = sb * invM;
    tco[2 * TS + tslot] = sg * invM;
    tco[3 * TS + tslot] = mean[c];
    tco[4 * TS + tslot] = rstd[c];
  }
  __syncthreads();
  const int CH8 = C >> 3, j8 = i0 % CH8;
  float a8[8], b8[8], g8[8], m8[8], r8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int t = k * TSTR + j8;
    a8[k] = tco[t]; b8[k] = tco[TS + t]; g8[k] = tco[2 * TS + t];
    m8[k] = tco[3 * TS + t]; r8[k] = tco[4 * TS + t];
  }
  if constexpr (PIPE) {   // as k_bn_apply_v
    for (int base = i0; base < n8; base += V * T) {
      const int nb = base + V * T;   // the next batch's chunk v is loaded right after chunk v is stored
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float d[8], xf[8];
        unpack8(dv[v], d);
        unpack8(xv[v], xf);
        if (y) {
          float yf[8];
          unpack8(yv[v], yf);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] = yf[k] > 0.f ? d[k] : 0.f;
        }
        const int i = base + v * T;
        if (dres && i < n8) reinterpret_cast<uint4*>(dres)[i] = pack8(d);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xf[k] - m8[k]) * r8[k];
          o[k] = a8[k] * (d[k] - b8[k] - xh * g8[k]);
        }
        if (i < n8) reinterpret_cast<uint4*>(dx)[i] = pack8(o);
        if (nb < n8) {
          const int inext = min(nb + v * T, n8 - 1);
          dv[v] = reinterpret_cast<const uint4*>(dy)[inext];
          xv[v] = reinterpret_cast<const uint4*>(x)[inext];
          if (y) yv[v] = reinterpret_cast<const uint4*>(y)[inext];
        }
      }
    }
  } else {
    for (int base = i0, it = 0; base < n8; base += V * T, ++it) {
      if (it > 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int i = min(base + v * T, n8 - 1);
          dv[v] = reinterpret_cast<const uint4*>(dy)[i];
          xv[v] = reinterpret_cast<const uint4*>(x)[i];
        }
        if (y) {
#pragma unroll
          for (int v = 0; v < V; ++v) yv[v] = reinterpret_cast<const uint4*>(y)[min(base + v * T, n8 - 1)];
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float d[8], xf[8];
        unpack8(dv[v], d);
        unpack8(xv[v], xf);
        if (y) {
          float yf[8];
          unpack8(yv[v], yf);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] = yf[k] > 0.f ? d[k] : 0.f;
        }
        const int i = base + v * T;
        if (dres && i < n8) reinterpret_cast<uint4*>(dres)[i] = pack8(d);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xf[k] - m8[k]) * r8[k];
          o[k] = a8[k] * (d[k] - b8[k] - xh * g8[k]);
        }
        if (i < n8) reinterpret_cast<uint4*>(dx)[i] = pack8(o);
      }
    }
  }
}

template <int NT, int V, bool PIPE>
__global__ __launch_bounds__(NT) void k_bn_bwd_apply_v(BnbArgs p, KmlSgdRider rider) {
  // optimizer-update rider (kml_sgd.h): the last rider.blocks blocks of the grid
  if ((int)blockIdx.x >= (int)gridDim.x - rider.blocks) {
    kml_sgd_rider_run(rider, (int)blockIdx.x - ((int)gridDim.x - rider.blocks));
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float sh[];
  bn_bwd_apply_body<NT, V, PIPE>(p, (int)blockIdx.x, (int)gridDim.x - rider.blocks, sh);
}

// Two independent BN backward applies in one launch (kml_bn_bwd_pair): a downsampling block's
// projection BN and its first BN, both ready once the second conv's backward has run.
template <int NT, int V1, int V2>
__global__ __launch_bounds__(NT) void k_bn_bwd_apply_pair(BnbArgs p1, BnbArgs p2, int n1, int n2) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int b = (int)blockIdx.x;
  if (b < n1) bn_bwd_apply_body<NT, V1, false>(p1, b, n1, sh);
  else bn_bwd_apply_body<NT, V2, false>(p2, b - n1, n2, sh);
}

// Fold G partial rows [G][W] into ceil(G / R) rows (fixed order: deterministic), so the
// apply kernels' per-block prologue stays small when a large conv (ResNet-50 at 56x56:
// 3136 M-tiles) left thousands of rows.  grid = (ceil(W / 4 / 64), ceil(G / R)).
__global__ __launch_bounds__(256) void k_rows_fold(const float* __restrict__ part, float* __restrict__ out, int G,
                                                   int W, int R) {
  const int Q = W / 4;
  const int q = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;                 // 4 row slices
  const int r0 = blockIdx.y * R, r1 = min(G, r0 + R);
  __shared__ float4 red[256];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < Q) {
    const float4* p4 = reinterpret_cast<const float4*>(part) + q;
    for (int r = r0 + sl; r < r1; r += 4) {
      const float4 v = p4[(long long)r * Q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < 64 && q < Q) {
    float4 t = red[threadIdx.x];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 v = red[k * 64 + threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    reinterpret_cast<float4*>(out)[(long long)blockIdx.y * Q + q] = t;
  }
}

// chunks per thread for the register-resident kernels: about 256 blocks, at most VMAX;
// past VMAX the grid grows to at most 1024 blocks and the kernel grid-strides
static int pick_v(long long n8, int vmax) {
  long long v = (n8 + 256LL * TPB - 1) / (256LL * TPB);
  int r = 1;
  while (r < v && r < vmax) r *= 2;
  return r;
}
// (fewer, fuller blocks — V >= 2/4/8 chunks per thread, or a grid cap below 1024 — measured
// slower on ResNet-34: profiles/r5/bn_fold_ab.md, profiles/r5/r50/bn_grid_cap_probe.txt)
static unsigned v_grid(long long n8, int V) {
  constexpr long long GRID_CAP = 1024;
  long long g = (n8 + (long long)TPB * V - 1) / ((long long)TPB * V);
  if (g > GRID_CAP) g = GRID_CAP;
  return (unsigned)(g < 1 ? 1 : g);
}

// G partial rows of W floats above this many bytes are folded by k_rows_fold first
constexpr long long FOLD_BYTES = 512 * 1024;   // ResNet-50 56x56 rows fold; ResNet-34 never (a fold launch costs ~5 us)
constexpr int FOLD_R = 32;

static bool reg_ok(long long M, int C) {
  return C % 8 == 0 && (TPB % (C / 8)) == 0 && M * C / 8 < (1LL << 30);
}

// relu backward alone: dx = dy * [y > 0]  (bf16, x8)
// (bn_bwd_apply_partial below reuses k_bn_bwd_apply_fin with partials from a conv epilogue)
__global__ void k_relu_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                           bf16_t* __restrict__ dx, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float d[8], yv[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], d);
    unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
    reinterpret_cast<uint4*>(dx)[i] = pack8(d);
  }
}

__global__ void k_relu_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k], 0.f);
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

// blocks for k_bn_bwd_reduce2: ~4 row iterations per thread, at most 1024 blocks
int bwd_blocks(long long M, int C, int* rows_per_block) {
  const int rpi = TPB / (C / 8);
  long long rpb = (long long)rpi * 4;
  long long g = (M + rpb - 1) / rpb;
  if (g > 1024) { rpb = ((M + 1023) / 1024 + rpi - 1) / rpi * rpi; g = (M + rpb - 1) / rpb; }
  *rows_per_block = (int)rpb;
  return (int)g;
}

int fin_blocks(long long M, int C, int* rows_per_block) {
  const int rpi = TPB / (C / 8);
  long long gmax = 32768 / (2 * C);   // <= 128 KB of partials read per apply block
  if (gmax > 256) gmax = 256;
  if (gmax < 8) gmax = 8;
  long long rpb = (long long)rpi * 4;
  long long g = (M + rpb - 1) / rpb;
  if (g > gmax) { rpb = ((M + gmax - 1) / gmax + rpi - 1) / rpi * rpi; g = (M + rpb - 1) / rpb; }
  *rows_per_block = (int)rpb;
  return (int)g;
}

unsigned rows_grid(long long M, int C) {
  const int rpi = TPB / (C / 8);
  long long g = (M + rpi * 8 - 1) / (rpi * 8);  // >= 8 rows per thread
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Stem fusion: y = maxpool_{k,s,p}(relu(bn(x))) with the window argmax (uint8 row-major tap,
// the k_maxpool_fwd format, so kml_maxpool_bwd runs the backward).  The normalised map is
// never written: one pass reads x and writes the pooled map (for the ResNet stem a quarter
// of the BN output's bytes) instead of BN-apply (read x, write y) + max-pool (read y).
// Statistics prologue as k_bn_apply (partial rows of the conv epilogue summed per block,
// block 0 updates running / saved statistics).  Every value is rounded to bf16 before the
// comparison, so maxima and argmax equal the unfused pair's exactly.
template <int NT>
__global__ __launch_bounds__(NT) void k_bn_relu_maxpool(
    const bf16_t* __restrict__ x, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ y, unsigned char* __restrict__ idx,
    float* __restrict__ save_mean, float* __restrict__ save_rstd, float* __restrict__ run_mean,
    float* __restrict__ run_var, int B, int H, int W, int C, int OH, int OW, int k, int st, int pd, float eps,
    float momentum, int stats_rows, long long* __restrict__ counters, int n_counters) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // scale[C], shift[C], sums[2C], scratch
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < n_counters; i += NT) counters[i] += 1;  // BN num_batches_tracked
  float* scale = sh;
  float* shift = sh + C;
  const long long M = (long long)B * H * W;
  const float* sums = stats;
  if (stats_rows > 0) {  // same row-summation order as k_bn_apply_v: bit-identical statistics
    float* acc = sh + 2 * C;
    if (C / 2 <= NT) {
      EarlyRows er;
      er.issue(stats, stats_rows, 2 * C, NT);
      er.finish(stats, stats_rows, acc, reinterpret_cast<float4*>(sh + 4 * C));
    } else {
      sum_partial_rows<NT>(stats, stats_rows, 2 * C, acc, reinterpret_cast<float4*>(sh + 4 * C));
    }
    sums = acc;
  }
  for (int c = threadIdx.x; c < C; c += NT) {
    const float mean = sums[c] / (float)M;
    const float var = fmaxf(sums[C + c] / (float)M - mean * mean, 0.f);
    const float rstd = rsqrtf(var + eps);
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    scale[c] = g * rstd;
    shift[c] = bb - mean * g * rstd;
    if (blockIdx.x == 0) {
      if (save_mean) { save_mean[c] = mean; save_rstd[c] = rstd; }
      if (run_mean) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
      }
    }
  }
  __syncthreads();
  const int CH = C / 8;
  const long long total = (long long)B * OH * OW * CH;
  for (long long t = blockIdx.x * (long long)NT + threadIdx.x; t < total; t += (long long)gridDim.x * NT) {
    const int ch = (int)(t % CH);
    long long pix = t / CH;
    const int ow = (int)(pix % OW); pix /= OW;
    const int oh = (int)(pix % OH);
    const int b = (int)(pix / OH);
    float sc[8], sf[8], best[8];
    int bi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale[ch * 8 + i];
      sf[i] = shift[ch * 8 + i];
      best[i] = -INFINITY;
      bi[i] = 0;
    }
    for (int r = 0; r < k; ++r) {
      const int ih = oh * st - pd + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int q = 0; q < k; ++q) {
        const int iw = ow * st - pd + q;
        if ((unsigned)iw >= (unsigned)W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + ((long long)(b * H + ih) * W + iw) * C + ch * 8), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float v = bf2f(f2bf(fmaxf(f[i] * sc[i] + sf[i], 0.f)));
          if (v > best[i] || (v != v)) { best[i] = v; bi[i] = r * k + q; }
        }
      }
    }
    reinterpret_cast<uint4*>(y)[t] = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    reinterpret_cast<uint2*>(idx)[t] = packed;
  }
}

// k_bn_relu_maxpool specialised for the 3x3 window of the ResNet stem: each thread owns IPT
// output chunks per grid-stride round and issues ALL their window loads (IPT x 9 x 16 B, taps
// outside the image clamped to the centre and masked) before the statistics prologue
// finishes, so one memory round trip covers both (the generic kernel's per-tap loop
// serialised nine).  Same statistics order and rounding as k_bn_apply_v.
template <int NT, int IPT>
__global__ __launch_bounds__(NT) void k_bn_relu_maxpool3(
    const bf16_t* __restrict__ x, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ y, unsigned char* __restrict__ idx,
    float* __restrict__ save_mean, float* __restrict__ save_rstd, float* __restrict__ run_mean,
    float* __restrict__ run_var, int B, int H, int W, int C, int OH, int OW, int st, int pd, float eps,
    float momentum, int stats_rows, long long* __restrict__ counters, int n_counters) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < n_counters; i += NT) counters[i] += 1;  // BN num_batches_tracked
  float* scale = sh;
  float* shift = sh + C;
  const long long M = (long long)B * H * W;
  const int CH = C / 8;
  const long long total = (long long)B * OH * OW * CH;
  const long long T = (long long)gridDim.x * NT;
  const bool parts = stats_rows > 0;
  const bool early = parts && C / 2 <= NT;
  EarlyRows er;
  if (early) er.issue(stats, stats_rows, 2 * C, NT);
  uint4 v[IPT][9];
  unsigned okm[IPT];
  auto load = [&](long long base) {
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const long long t = min(base + j * T, total - 1);
      long long pix = t / CH;
      const int ch = (int)(t - pix * CH);
      const int ow = (int)(pix % OW); pix /= OW;
      const int oh = (int)(pix % OH);
      const int b = (int)(pix / OH);
      okm[j] = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int ih = oh * st - pd + r, iw = ow * st - pd + q;
          const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
          okm[j] |= ok ? (1u << (r * 3 + q)) : 0u;
          const int ih2 = ok ? ih : min(max(ih, 0), H - 1), iw2 = ok ? iw : min(max(iw, 0), W - 1);
          v[j][r * 3 + q] = *reinterpret_cast<const uint4*>(x + ((long long)(b * H + ih2) * W + iw2) * C + ch * 8);
        }
    }
  };
  const long long i0 = blockIdx.x * (long long)NT + threadIdx.x;
  load(i0);
  const float* sums = stats;
  if (parts) {
    float* acc = sh + 2 * C;
    if (early) er.finish(stats, stats_rows, acc, reinterpret_cast<float4*>(sh + 4 * C));
    else sum_partial_rows<NT>(stats, stats_rows, 2 * C, acc, reinterpret_cast<float4*>(sh + 4 * C));
    sums = acc;
  }
  for (int c = threadIdx.x; c < C; c += NT) {
    const float mean = sums[c] / (float)M;
    const float var = fmaxf(sums[C + c] / (float)M - mean * mean, 0.f);
    const float rstd = rsqrtf(var + eps);
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    scale[c] = g * rstd;
    shift[c] = bb - mean * g * rstd;
    if (blockIdx.x == 0) {
      if (save_mean) { save_mean[c] = mean; save_rstd[c] = rstd; }
      if (run_mean) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
      }
    }
  }
  __syncthreads();
  for (long long base = i0, it = 0; base < total; base += IPT * T, ++it) {
    if (it > 0) load(base);
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const long long t = base + j * T;
      if (t >= total) continue;
      const int ch = (int)(t % CH);
      // the chunk's 8 coefficients as two 16-byte reads each, once per output chunk (per-element
      // 4-byte reads of scale[ch * 8 + i] were 2-way bank conflicts: 38 % in profiles/r6/final/r34_pmc.md)
      float sc[8], sf[8];
      {
        const float4* s4 = reinterpret_cast<const float4*>(scale + ch * 8);
        const float4* f4 = reinterpret_cast<const float4*>(shift + ch * 8);
        const float4 a0 = s4[0], a1 = s4[1], b0 = f4[0], b1 = f4[1];
        sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
        sf[0] = b0.x; sf[1] = b0.y; sf[2] = b0.z; sf[3] = b0.w; sf[4] = b1.x; sf[5] = b1.y; sf[6] = b1.z; sf[7] = b1.w;
      }
      float best[8];
      int bi[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; bi[i] = 0; }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (!((okm[j] >> tap) & 1u)) continue;
        float f[8];
        unpack8(v[j][tap], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float o = bf2f(f2bf(fmaxf(f[i] * sc[i] + sf[i], 0.f)));
          if (o > best[i] || (o != o)) { best[i] = o; bi[i] = tap; }
        }
      }
      reinterpret_cast<uint4*>(y)[t] = pack8(best);
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      reinterpret_cast<uint2*>(idx)[t] = packed;
    }
  }
}

}  // namespace

// rows of partial statistics kml_bn_stats_part writes (<= 128 KB of partials for bn_apply to sum)
KML_API int kml_bn_stats_rows(long long M, int C) {
  int rpb;
  return fin_blocks(M, C, &rpb);
}

KML_API int kml_bn_stats_part(const bf16_t* x, float* part, long long M, int C, hipStream_t s) {
  if (C % 8 || C / 8 > TPB) return (int)hipErrorInvalidValue;
  int rpb;
  const int g = fin_blocks(M, C, &rpb);
  hipLaunchKernelGGL(k_bn_stats_part, dim3(g), dim3(TPB), 0, s, x, part, M, C, rpb);
  KML_LAUNCH_CHECK();
}

KML_API int kml_bn_stats(const bf16_t* x, float* stats, long long M, int C, hipStream_t s) {
  if (C % 8 || C / 8 > TPB) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_stats, dim3(rows_grid(M, C)), dim3(TPB), 0, s, x, stats, M, C);
  KML_LAUNCH_CHECK();
}

// Partial-row summation width: every block of the apply kernels sums all G rows of 2C
// floats before its elementwise pass.  At 256 threads a thread walks ceil(G / slices) rows
// in batches of 16 dependent-latency loads; past one batch, 1024-thread blocks (4x the
// slices, same grid) cut that prologue to one memory round trip.
static bool wide_sum(int G, int C) {
  const int Q = C / 2;  // float4 columns of a [2C] row
  const int slices = Q >= TPB ? 1 : TPB / Q;
  return C <= 1024 && (G + slices - 1) / slices > 16;
}

// kml_bn_bwd_pair: while g_bnb_rec is set, the single-batch register-path backward apply (no rider
// armed) records instead of launching; every other launch of the call runs as usual
struct BnbRec {
  BnbArgs p;
  int V = 0, grid = 0;
  size_t shm = 0;
  bool set = false;
};
static BnbRec* g_bnb_rec = nullptr;

static int launch_bwd_apply_fin(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean,
                                const float* rstd, const float* gamma, const float* part, int G, float* dgamma,
                                float* dbeta, bf16_t* dx, bf16_t* dres, long long M, int C, int acc,
                                hipStream_t s) {
  if (reg_ok(M, C)) {
    const long long n8 = M * C / 8;
    const int V = pick_v(n8, 4);
    const unsigned grid = v_grid(n8, V);
    const size_t shm = (4 * TPB + 5 * C + 5 * bn_tslots(C)) * sizeof(float);  // + transposed coefficients
    const bool pipe = n8 > (long long)grid * TPB * V;   // more than one batch per thread
    const BnbArgs p{dy, y, x, mean, rstd, gamma, part, G, dgamma, dbeta, dx, dres, M, C, acc};
    if (g_bnb_rec && g_kml_rider.blocks == 0 && !pipe) {   // kml_bn_bwd_pair: record, launch nothing
      *g_bnb_rec = BnbRec{p, V, (int)grid, shm, true};
      return 0;
    }
    const KmlSgdRider rider = kml_rider_take();
#define KML_BWD_V(VV)                                                                                          \
  do { if (pipe) hipLaunchKernelGGL((k_bn_bwd_apply_v<TPB, VV, true>), dim3(grid + rider.blocks), dim3(TPB), shm, s, p, \
                     rider);                                                                                    \
  else hipLaunchKernelGGL((k_bn_bwd_apply_v<TPB, VV, false>), dim3(grid + rider.blocks), dim3(TPB), shm, s, p, rider); \
  } while (0)
    if (V == 1) KML_BWD_V(1);
    else if (V == 2) KML_BWD_V(2);
    else KML_BWD_V(4);
#undef KML_BWD_V
    KML_LAUNCH_CHECK();
  }
  if (g_kml_rider.blocks > 0) (void)kml_rider_flush(s);   // an armed rider rides alone on these paths
  if (wide_sum(G, C)) {
    constexpr int NT = 1024;
    long long ab = (M * C / 8 + NT - 1) / NT;
    if (ab > 256) ab = 256;
    hipLaunchKernelGGL(k_bn_bwd_apply_fin<NT>, dim3((unsigned)ab), dim3(NT), (4 * NT + 5 * C) * sizeof(float), s,
                       dy, y, x, mean, rstd, gamma, part, G, dgamma, dbeta, dx, dres, M, C, acc);
    KML_LAUNCH_CHECK();
  }
  long long ab = (M * C / 8 + TPB - 1) / TPB;
  if (ab > 256) ab = 256;
  hipLaunchKernelGGL(k_bn_bwd_apply_fin<TPB>, dim3((unsigned)ab), dim3(TPB), (4 * TPB + 5 * C) * sizeof(float), s,
                     dy, y, x, mean, rstd, gamma, part, G, dgamma, dbeta, dx, dres, M, C, acc);
  KML_LAUNCH_CHECK();
}

// stats_rows > 0: stats is [stats_rows][2C] partial sums (conv epilogue), summed here
// fold rows [G][W] -> ws [ceil(G / FOLD_R)][W] when they are large; returns the rows to use
static const float* maybe_fold(const float* part, int& G, int W, float* ws, hipStream_t s) {
  if (!ws || (long long)G * W * 4 <= FOLD_BYTES) return part;
  const int NG = (G + FOLD_R - 1) / FOLD_R;
  hipLaunchKernelGGL(k_rows_fold, dim3((unsigned)((W / 4 + 63) / 64), (unsigned)NG), dim3(256), 0, s, part, ws, G, W,
                     FOLD_R);
  G = NG;
  return ws;
}

// rows of fp32 workspace (x 2C floats) kml_bn_apply / kml_bn_bwd_apply_partial may use to fold G rows
KML_API int kml_bn_fold_rows(int G, int C) {
  return (long long)G * 2 * C * 4 <= FOLD_BYTES ? 0 : (G + FOLD_R - 1) / FOLD_R;
}

// kml_bn_apply_pair: while g_bn_rec is set, kml_bn_apply records its register-path launch
struct BnRec {
  BnApArgs p;
  int V = 0, grid = 0;
  size_t shm = 0;
  bool ok = false;   // single-batch register path, no fold / wide-sum launch: pairable
};
static BnRec* g_bn_rec = nullptr;

KML_API int kml_bn_apply(const bf16_t* x, const float* stats, int stats_rows, const float* gamma, const float* beta,
                         const bf16_t* res, bf16_t* y, float* save_mean, float* save_rstd, float* run_mean,
                         float* run_var, long long M, int C, float eps, float momentum, int relu, int mode,
                         float* fold_ws, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  if (g_bn_rec) {   // recording: only the single-launch register path pairs
    g_bn_rec->ok = false;
    if (!reg_ok(M, C) || (mode == 0 && stats_rows > 0 && fold_ws && (long long)stats_rows * 2 * C * 4 > FOLD_BYTES))
      return 0;
  }
  if (mode == 0 && stats_rows > 0) stats = maybe_fold(stats, stats_rows, 2 * C, fold_ws, s);
  if (reg_ok(M, C)) {
    const long long n8 = M * C / 8;
    const int V = pick_v(n8, 8);
    const unsigned grid = v_grid(n8, V);
    const size_t shm = (2 * bn_tslots(C) + (stats_rows > 0 ? (2 * C + 4 * TPB) : 0)) * sizeof(float);
    const bool pipe = n8 > (long long)grid * TPB * V;   // more than one batch per thread
    const BnApArgs p{x, stats, gamma, beta, res, y, save_mean, save_rstd, run_mean, run_var, M, C, eps, momentum,
                     relu, mode, stats_rows};
    if (g_bn_rec) {   // kml_bn_apply_pair: record, launch nothing
      *g_bn_rec = BnRec{p, V, (int)grid, shm, !pipe && !(stats_rows > 0 && wide_sum(stats_rows, C))};
      return 0;
    }
#define KML_AP_V(VV)                                                                                           \
  do { if (pipe) hipLaunchKernelGGL((k_bn_apply_v<TPB, VV, true>), dim3(grid), dim3(TPB), shm, s, p);           \
  else hipLaunchKernelGGL((k_bn_apply_v<TPB, VV, false>), dim3(grid), dim3(TPB), shm, s, p); } while (0)
    if (V == 1) KML_AP_V(1);
    else if (V == 2) KML_AP_V(2);
    else if (V == 4) KML_AP_V(4);
    else KML_AP_V(8);
#undef KML_AP_V
    KML_LAUNCH_CHECK();
  }
  if (stats_rows > 0 && wide_sum(stats_rows, C)) {
    constexpr int NT = 1024;
    const size_t shm = (4 * C + 4 * NT) * sizeof(float);
    unsigned grid = kml_stream_grid(M * C / 8, NT);
    if (grid > 256) grid = 256;
    hipLaunchKernelGGL(k_bn_apply<NT>, dim3(grid), dim3(NT), shm, s, x, stats, gamma, beta, res, y, save_mean,
                       save_rstd, run_mean, run_var, M, C, eps, momentum, relu, mode, stats_rows);
    KML_LAUNCH_CHECK();
  }
  const size_t shm = (stats_rows > 0 ? (4 * C + 4 * TPB) : 2 * C) * sizeof(float);
  unsigned grid = kml_stream_grid(M * C / 8, TPB);
  if (stats_rows > 0 && grid > 256) grid = 256;  // every block re-sums the partials: fewer, fuller blocks
  hipLaunchKernelGGL(k_bn_apply<TPB>, dim3(grid), dim3(TPB), shm, s, x, stats, gamma, beta, res, y, save_mean,
                     save_rstd, run_mean, run_var, M, C, eps, momentum, relu, mode, stats_rows);
  KML_LAUNCH_CHECK();
}

// Two independent training BN applies (kml_bn_apply's arguments, stream excluded, as 64-bit values
// with the floats' bit patterns in the low words: q[11] M, q[13] eps, q[14] momentum) in one launch.
// Returns 0 when launched as a pair, 1 when either is not a single-batch register-path apply
// (nothing launched: the caller runs them with kml_bn_apply).
KML_API int kml_bn_apply_pair(const long long* q1, const long long* q2, hipStream_t s) {
  BnRec r[2];
  const long long* q[2] = {q1, q2};
  for (int i = 0; i < 2; ++i) {
    const long long* v = q[i];
    float eps, mom;
    const unsigned e = (unsigned)v[13], m = (unsigned)v[14];
    memcpy(&eps, &e, 4);
    memcpy(&mom, &m, 4);
    g_bn_rec = &r[i];
    const int rc = kml_bn_apply((const bf16_t*)v[0], (const float*)v[1], (int)v[2], (const float*)v[3],
                                (const float*)v[4], (const bf16_t*)v[5], (bf16_t*)v[6], (float*)v[7], (float*)v[8],
                                (float*)v[9], (float*)v[10], v[11], (int)v[12], eps, mom, (int)v[15], (int)v[16],
                                (float*)v[17], s);
    g_bn_rec = nullptr;
    if (rc) return rc;
    if (!r[i].ok) return 1;
  }
  const size_t shm = r[0].shm > r[1].shm ? r[0].shm : r[1].shm;
#define KML_BNP(A, B)                                                                                          \
  if (r[0].V == A && r[1].V == B) {                                                                            \
    hipLaunchKernelGGL((k_bn_apply_pair<TPB, A, B>), dim3((unsigned)(r[0].grid + r[1].grid)), dim3(TPB), shm, s, \
                       r[0].p, r[1].p, r[0].grid, r[1].grid);                                                  \
    KML_LAUNCH_CHECK();                                                                                        \
  }
  KML_BNP(1, 1) KML_BNP(1, 2) KML_BNP(2, 1) KML_BNP(2, 2)
#undef KML_BNP
  return 1;
}

// number of fp32 workspace floats kml_bn_bwd needs for the deterministic reduce
KML_API long long kml_bn_bwd_ws_floats(long long M, int C) {
  int rpb;
  const int g = bwd_blocks(M, C, &rpb);
  const long long a = (long long)g * 2 * C + (long long)((g + FOLD_R - 1) / FOLD_R) * 2 * C;  // + fold rows
  const long long b = (long long)fin_blocks(M, C, &rpb) * 2 * C;
  return a > b ? a : b;
}

// ws && !counter: partial sums + reduction fused into the apply kernel (default; deterministic)
// ws && counter : partials + in-kernel last-arriver reduce (agent-scope fences)
// !ws           : block partials + fp32 atomics
// (ws holds kml_bn_bwd_ws_floats(M, C) floats; *counter == 0 on entry and on exit).
extern "C" int kml_zero(void* p, long long bytes, hipStream_t s);  // util.hip

// accumulate: dgamma/dbeta += (1) or = (0) this pass's sums
KML_API int kml_bn_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean, const float* rstd,
                       const float* gamma, float* dgamma, float* dbeta, bf16_t* dx, bf16_t* dres, float* ws,
                       unsigned* counter, long long M, int C, int accumulate, hipStream_t s) {
  if (C % 8 || C / 8 > TPB) return (int)hipErrorInvalidValue;
  int rpb;
  if (ws && !counter) {  // default: partials, then the apply kernel reduces them (2 launches, no sync)
    // enough blocks to stream dy / y / x at full bandwidth (the old <= 128 KB-of-partials
    // cap left ResNet-50's 56x56 BNs on 64 blocks); large partial sets are folded first
    int gf = bwd_blocks(M, C, &rpb);
    hipLaunchKernelGGL(k_bn_bwd_reduce2<2>, dim3(gf), dim3(TPB), 0, s, dy, y, x, mean, rstd, dgamma, dbeta, ws,
                       nullptr, M, C, rpb);
    const float* part = maybe_fold(ws, gf, 2 * C, ws + (long long)gf * 2 * C, s);
    return launch_bwd_apply_fin(dy, y, x, mean, rstd, gamma, part, gf, dgamma, dbeta, dx, dres, M, C, accumulate, s);
  }
  const int g = bwd_blocks(M, C, &rpb);
  // these two variants reduce INTO dgamma / dbeta (the apply kernel reads them back)
  if (!accumulate) {  // zeroing kernels, not memset nodes (util.hip kml_zero)
    int e = kml_zero(dgamma, C * (long long)sizeof(float), s);
    if (!e) e = kml_zero(dbeta, C * (long long)sizeof(float), s);
    if (e) return e;
  }
  if (ws && counter) {  // deterministic: ordered partials + last-arriver reduce
    hipLaunchKernelGGL(k_bn_bwd_reduce2<0>, dim3(g), dim3(TPB), 0, s, dy, y, x, mean, rstd, dgamma, dbeta, ws,
                       counter, M, C, rpb);
  } else {              // fast: same partials, memory-side atomics
    hipLaunchKernelGGL(k_bn_bwd_reduce2<1>, dim3(g), dim3(TPB), 0, s, dy, y, x, mean, rstd, dgamma, dbeta,
                       nullptr, nullptr, M, C, rpb);
  }
  hipLaunchKernelGGL(k_bn_bwd_apply, dim3(kml_stream_grid(M * C / 8, TPB)), dim3(TPB), 5 * C * sizeof(float), s,
                     dy, y, x, mean, rstd, gamma, dgamma, dbeta, dx, dres, M, C);
  KML_LAUNCH_CHECK();
}

// BN backward when the dgamma/dbeta partial rows were produced by the dgrad epilogue that
// computed dy (conv_dgrad bnf_*): a single apply kernel, no reduction pass over dy/y/x.
KML_API int kml_bn_bwd_apply_partial(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean,
                                     const float* rstd, const float* gamma, const float* part, int G, float* dgamma,
                                     float* dbeta, bf16_t* dx, bf16_t* dres, long long M, int C, float* fold_ws,
                                     int accumulate, hipStream_t s) {
  if (C % 8 || C / 8 > TPB || G <= 0) return (int)hipErrorInvalidValue;
  part = maybe_fold(part, G, 2 * C, fold_ws, s);
  return launch_bwd_apply_fin(dy, y, x, mean, rstd, gamma, part, G, dgamma, dbeta, dx, dres, M, C, accumulate, s);
}

// Two independent training BN backwards with one apply launch.  q[0] selects the call: 0 =
// kml_bn_bwd (q[1..15] its arguments, stream excluded, as 64-bit values), 1 =
// kml_bn_bwd_apply_partial (q[1..16]).  Each call runs as usual (its reduction pass included)
// except that a single-batch register-path apply is recorded; two recorded applies launch as one
// k_bn_bwd_apply_pair, a lone one on its own.  Returns 0 or an error code.
static int bnb_call(const long long* q, hipStream_t s) {
  if (q[0] == 0)
    return kml_bn_bwd((const bf16_t*)q[1], (const bf16_t*)q[2], (const bf16_t*)q[3], (const float*)q[4],
                      (const float*)q[5], (const float*)q[6], (float*)q[7], (float*)q[8], (bf16_t*)q[9],
                      (bf16_t*)q[10], (float*)q[11], (unsigned*)q[12], q[13], (int)q[14], (int)q[15], s);
  if (q[0] == 1)
    return kml_bn_bwd_apply_partial((const bf16_t*)q[1], (const bf16_t*)q[2], (const bf16_t*)q[3],
                                    (const float*)q[4], (const float*)q[5], (const float*)q[6], (const float*)q[7],
                                    (int)q[8], (float*)q[9], (float*)q[10], (bf16_t*)q[11], (bf16_t*)q[12], q[13],
                                    (int)q[14], (float*)q[15], (int)q[16], s);
  return (int)hipErrorInvalidValue;
}

static int bnb_launch_one(const BnbRec& r, hipStream_t s) {
#define KML_BWD_ONE(VV) \
  if (r.V == VV) hipLaunchKernelGGL((k_bn_bwd_apply_v<TPB, VV, false>), dim3(r.grid), dim3(TPB), r.shm, s, r.p, KmlSgdRider{});
  KML_BWD_ONE(1) else KML_BWD_ONE(2) else KML_BWD_ONE(4) else return (int)hipErrorInvalidValue;
#undef KML_BWD_ONE
  KML_LAUNCH_CHECK();
}

KML_API int kml_bn_bwd_pair(const long long* q1, const long long* q2, hipStream_t s) {
  BnbRec r[2];
  const long long* q[2] = {q1, q2};
  for (int i = 0; i < 2; ++i) {
    g_bnb_rec = &r[i];
    const int rc = bnb_call(q[i], s);
    g_bnb_rec = nullptr;
    if (rc) return rc;
  }
  if (r[0].set && r[1].set) {
    const size_t shm = r[0].shm > r[1].shm ? r[0].shm : r[1].shm;
#define KML_BNBP(A, B)                                                                                             \
    if (r[0].V == A && r[1].V == B) {                                                                              \
      hipLaunchKernelGGL((k_bn_bwd_apply_pair<TPB, A, B>), dim3((unsigned)(r[0].grid + r[1].grid)), dim3(TPB), shm, s, \
                         r[0].p, r[1].p, r[0].grid, r[1].grid);                                                    \
      KML_LAUNCH_CHECK();                                                                                          \
    }
    KML_BNBP(1, 1) KML_BNBP(1, 2) KML_BNBP(2, 1) KML_BNBP(2, 2)
#undef KML_BNBP
  }
  for (int i = 0; i < 2; ++i) {
    if (!r[i].set) continue;
    const int rc = bnb_launch_one(r[i], s);
    if (rc) return rc;
  }
  return 0;
}

KML_API int kml_relu_fwd(const bf16_t* x, bf16_t* y, long long n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_relu_fwd, dim3(kml_stream_grid(n / 8, 256)), dim3(256), 0, s, x, y, n / 8);
  KML_LAUNCH_CHECK();
}

KML_API int kml_relu_bwd(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long long n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_relu_bwd, dim3(kml_stream_grid(n / 8, 256)), dim3(256), 0, s, dy, y, dx, n / 8);
  KML_LAUNCH_CHECK();
}

// Training forward of the ResNet stem's BN -> ReLU -> max-pool as one pass (k_bn_relu_maxpool):
// x [B][H][W][C] conv output, stats = [stats_rows][2C] partial rows (or final [2C] sums with
// stats_rows = 0), y [B][OH][OW][C] pooled output, idx its window argmax.
KML_API int kml_bn_relu_maxpool(const bf16_t* x, const float* stats, int stats_rows, const float* gamma,
                                const float* beta, bf16_t* y, unsigned char* idx, float* save_mean,
                                float* save_rstd, float* run_mean, float* run_var, int B, int H, int W, int C, int k,
                                int st, int pd, float eps, float momentum, float* fold_ws, long long* counters,
                                int n_counters, hipStream_t s) {
  if (n_counters < 0 || (n_counters > 0 && !counters)) return (int)hipErrorInvalidValue;
  if (C % 8 || k * k > 255 || k < 1 || st < 1 || pd < 0 || 2 * pd > k) return (int)hipErrorInvalidValue;
  if (stats_rows > 0) stats = maybe_fold(stats, stats_rows, 2 * C, fold_ws, s);
  const int OH = (H + 2 * pd - k) / st + 1, OW = (W + 2 * pd - k) / st + 1;
  const long long total = (long long)B * OH * OW * (C / 8);
  unsigned grid = kml_stream_grid(total, TPB);
  if (stats_rows > 0 && grid > 256) grid = 256;  // every block re-sums the partial rows
  const size_t shm = (stats_rows > 0 ? (4 * C + 4 * TPB) : 2 * C) * sizeof(float);
  if (k == 3 && stats_rows >= 128) {
    // many partial rows (ResNet stem: one per 128-pixel conv tile): 512-thread blocks sum
    // them in half the load batches (1024 threads would spill the window registers)
    constexpr int NT = 512;
    long long g3 = (total + NT - 1) / NT;
    if (g3 > 256) g3 = 256;
    const size_t shm3 = (4 * C + 4 * NT) * sizeof(float);
    hipLaunchKernelGGL((k_bn_relu_maxpool3<NT, 1>), dim3((unsigned)g3), dim3(NT), shm3, s, x, stats, gamma, beta,
                       y, idx, save_mean, save_rstd, run_mean, run_var, B, H, W, C, OH, OW, st, pd, eps, momentum,
                       stats_rows, counters, n_counters);
    KML_LAUNCH_CHECK();
  }
  if (k == 3) {
    constexpr int IPT = 2;
    long long g3 = (total + (long long)TPB * IPT - 1) / ((long long)TPB * IPT);
    if (g3 > 256) g3 = 256;
    hipLaunchKernelGGL((k_bn_relu_maxpool3<TPB, IPT>), dim3((unsigned)g3), dim3(TPB), shm, s, x, stats, gamma, beta,
                       y, idx, save_mean, save_rstd, run_mean, run_var, B, H, W, C, OH, OW, st, pd, eps, momentum,
                       stats_rows, counters, n_counters);
    KML_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_bn_relu_maxpool<TPB>, dim3(grid), dim3(TPB), shm, s, x, stats, gamma, beta, y, idx, save_mean,
                     save_rstd, run_mean, run_var, B, H, W, C, OH, OW, k, st, pd, eps, momentum, stats_rows, counters,
                     n_counters);
  KML_LAUNCH_CHECK();
}
