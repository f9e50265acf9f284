// optim.hip — fused multi-tensor optimizers over the flat parameter buffer (gfx950).
//
// All trainable parameters of a model live in ONE fp32 master buffer, their
// gradients in ONE fp32 buffer (the same buffer RCCL all-reduces) and their bf16
// compute copies in ONE shadow buffer.  Each optimizer step is therefore a single
// streaming launch over ~N floats: read w, g (+ state), write w, state and the bf16
// shadow the next forward consumes.  The data-parallel 1/world average is folded in
// as grad_scale, so the all-reduce needs no separate scaling pass.
//
// Learning rate and step count are read from device memory, so a hipGraph-captured
// training step follows an LR schedule / Adam bias correction without re-capture.
//
// Semantics follow torch.optim.SGD (momentum, dampening, nesterov, weight_decay) and
// torch.optim.Adam / AdamW (L2 vs decoupled decay), which is what the reference's user
// code configures (function_lenet.py:77-79, function_resnet34.py:62, function_vgg11.py:54).
// Optimizer-state reset at every K-AVG round (reference network.py:121-128) is a
// hipMemsetAsync of the state buffers (kml_memset).
#include "kml_common.h"
#include "kml_sgd.h"

namespace {

__global__ void k_sgd(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                      bf16_t* __restrict__ shadow, const float* __restrict__ lr_ptr, float lr_host, float wd,
                      float momentum, float dampening, int nesterov, const float* __restrict__ first_ptr,
                      int first_host, float grad_scale, long long n, float* __restrict__ adv_ctr,
                      float adv_batch, float adv_n) {
  // data-sampler counter advance (k_advance's job) folded into this launch: one thread, no
  // other block reads the counter, the next step's augment reads it after the launch boundary
  if (adv_ctr && blockIdx.x == 0 && threadIdx.x == 0) {
    adv_ctr[1] += 1.f;
    float st = adv_ctr[2] + adv_batch;
    if (st >= adv_n) st -= adv_n;
    adv_ctr[2] = st;
  }
  const float lr = lr_ptr ? *lr_ptr : lr_host;
  // first step after a reset (torch: momentum buffer := d, no dampening).  The flag lives
  // in device memory so a graph-captured step follows reset_state() between replays.
  const int first = first_ptr ? (*first_ptr != 0.f) : first_host;
  kml_sgd_range(w, g, mom, shadow, lr, wd, momentum, dampening, nesterov, first, grad_scale, n,
                blockIdx.x * (long long)blockDim.x + threadIdx.x, (long long)gridDim.x * blockDim.x);
}

__global__ void k_adam(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, bf16_t* __restrict__ shadow, const float* __restrict__ lr_ptr,
                       const float* __restrict__ step_ptr, float lr_host, float step_host, float b1, float b2,
                       float eps, float wd, int decoupled, float grad_scale, long long n) {
  const float lr = lr_ptr ? *lr_ptr : lr_host;
  const float t = step_ptr ? *step_ptr : step_host;
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const float step_size = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  // two float4 groups per thread and iteration, all eight loads issued before any math: the
  // 30-byte-per-parameter stream (4 reads, 3 writes, the bf16 shadow) keeps twice the bytes
  // in flight per wave (the one-group loop ran at ~78% of the achievable HBM rate)
  constexpr int U = 2;
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    float4 W[U], G[U], M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i < n4) {
        W[u] = reinterpret_cast<float4*>(w)[i];
        G[u] = reinterpret_cast<const float4*>(g)[i];
        M[u] = reinterpret_cast<float4*>(m)[i];
        V[u] = reinterpret_cast<float4*>(v)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n4) break;
      float wv[4] = {W[u].x, W[u].y, W[u].z, W[u].w}, gv[4] = {G[u].x, G[u].y, G[u].z, G[u].w};
      float mv[4] = {M[u].x, M[u].y, M[u].z, M[u].w}, vv[4] = {V[u].x, V[u].y, V[u].z, V[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gg = gv[k] * grad_scale;
        if (decoupled) wv[k] *= (1.f - lr * wd);
        else gg += wd * wv[k];
        mv[k] = b1 * mv[k] + (1.f - b1) * gg;
        vv[k] = b2 * vv[k] + (1.f - b2) * gg * gg;
        const float denom = sqrtf(vv[k]) * rbc2 + eps;
        wv[k] -= step_size * mv[k] / denom;
      }
      reinterpret_cast<float4*>(w)[i] = make_float4(wv[0], wv[1], wv[2], wv[3]);
      reinterpret_cast<float4*>(m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      reinterpret_cast<float4*>(v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
      if (shadow) {
        uint2 s;
        s.x = pack_bf2(wv[0], wv[1]);
        s.y = pack_bf2(wv[2], wv[3]);
        reinterpret_cast<uint2*>(shadow)[i] = s;
      }
    }
  }
  for (long long i = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gg = g[i] * grad_scale;
    float wi = w[i];
    if (decoupled) wi *= (1.f - lr * wd);
    else gg += wd * wi;
    m[i] = b1 * m[i] + (1.f - b1) * gg;
    v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
    wi -= step_size * m[i] / (sqrtf(v[i]) * rbc2 + eps);
    w[i] = wi;
    if (shadow) shadow[i] = f2bf(wi);
  }
}

__global__ void k_inc(float* p, float by) { if (threadIdx.x == 0 && blockIdx.x == 0) *p += by; }

// sum of squares of an fp32 vector into out[0] (atomic; out zeroed by caller)
__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ x, float* __restrict__ out, long long n) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    s += x[i] * x[i];
  s = wave_sum(s);
  __shared__ float sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, sh[0] + sh[1] + sh[2] + sh[3]);
}

// x *= min(1, max_norm / (sqrt(sumsq) + 1e-6))  — global-norm clipping, scale on device
__global__ void k_clip_scale(float* __restrict__ x, const float* __restrict__ sumsq, float max_norm, long long n) {
  const float nrm = sqrtf(*sumsq);
  const float c = fminf(1.f, max_norm / (nrm + 1e-6f));
  if (c >= 1.f) return;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] *= c;
}

}  // namespace

// NOTE: hipMemsetAsync is avoided on capturable paths (graph memset nodes raced with
// kernel nodes on this ROCm build); use kml_zero from util.hip.
KML_API int kml_memset(void* p, int value, long long bytes, hipStream_t s) {
  return (int)hipMemsetAsync(p, value, (size_t)bytes, s);
}

// max_blocks > 0 caps the grid (a range update running next to latency-bound backward
// kernels on a side stream should take a slice of the CUs, not all of them)
KML_API int kml_sgd(float* w, const float* g, float* mom, bf16_t* shadow, const float* lr_ptr, float lr, float wd,
                    float momentum, float dampening, int nesterov, const float* first_ptr, int first,
                    float grad_scale, long long n, int max_blocks, float* adv_ctr, float adv_batch, float adv_n,
                    hipStream_t s) {
  unsigned grid = kml_stream_grid((n + 3) / 4, 256);
  if (max_blocks > 0 && grid > (unsigned)max_blocks) grid = (unsigned)max_blocks;
  hipLaunchKernelGGL(k_sgd, dim3(grid), dim3(256), 0, s, w, g, mom, shadow, lr_ptr, lr, wd, momentum, dampening,
                     nesterov, first_ptr, first, grad_scale, n, adv_ctr, adv_batch, adv_n);
  KML_LAUNCH_CHECK();
}

// max_blocks > 0 caps the grid (a range update on a side stream beside the backward, as kml_sgd)
KML_API int kml_adam(float* w, const float* g, float* m, float* v, bf16_t* shadow, const float* lr_ptr,
                     const float* step_ptr, float lr, float step, float b1, float b2, float eps, float wd,
                     int decoupled, float grad_scale, long long n, int max_blocks, hipStream_t s) {
  unsigned grid = kml_stream_grid((n + 3) / 4, 256);
  if (max_blocks > 0 && grid > (unsigned)max_blocks) grid = (unsigned)max_blocks;
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, s, w, g, m, v, shadow, lr_ptr,
                     step_ptr, lr, step, b1, b2, eps, wd, decoupled, grad_scale, n);
  KML_LAUNCH_CHECK();
}

KML_API int kml_increment(float* p, float by, hipStream_t s) {
  hipLaunchKernelGGL(k_inc, dim3(1), dim3(64), 0, s, p, by);
  KML_LAUNCH_CHECK();
}

__global__ void k_zero1(float* p) { if (threadIdx.x == 0) *p = 0.f; }

KML_API int kml_clip_grad_norm(float* g, float* ws1, float max_norm, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_zero1, dim3(1), dim3(64), 0, s, ws1);
  hipLaunchKernelGGL(k_sumsq, dim3(kml_stream_grid(n, 256 * 4)), dim3(256), 0, s, g, ws1, n);
  hipLaunchKernelGGL(k_clip_scale, dim3(kml_stream_grid(n, 256)), dim3(256), 0, s, g, ws1, max_norm, n);
  KML_LAUNCH_CHECK();
}


// ---------------------------------------------------------------------------------------
// K-AVG model average over ONE persistent flat state buffer (reference: the TrainJob's
// merge, ml/pkg/model/model.go:249-302 + parallelSGD.go:26-54).  Layout of `state`:
//   [0, n_params)            fp32 master parameters (the optimizer's buffer)
//   [n_params, i64_off)      fp32 module buffers (BN running_mean / running_var)
//   [i64_off, i64_off+n_i64) int64 buffers (num_batches_tracked) carried as fp32
//   [count_idx]              1 if this rank contributes to the round, else 0
// pack:   i64 -> fp32 slots, count slot := participate (non-participants send zeros)
// <RCCL all-reduce SUM of the whole buffer on the caller's stream>
// finish: x *= 1/max(count, 1); bf16 shadow of the parameter range refreshed in the
//         same pass; int64 buffers := floor(average) (the reference's integer division)
// No host synchronisation: the divisor never leaves the device.
// ---------------------------------------------------------------------------------------
__global__ void k_kavg_pack(float* __restrict__ state, const long long* __restrict__ i64, long long i64_off,
                            int n_i64, long long count_idx, int participate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_i64) state[i64_off + i] = participate ? (float)i64[i] : 0.f;
  if (i == 0) state[count_idx] = participate ? 1.f : 0.f;
}

__global__ void k_kavg_finish(float* __restrict__ state, long long n_params, long long count_idx,
                              bf16_t* __restrict__ shadow, long long* __restrict__ i64, long long i64_off,
                              int n_i64) {
  const float inv = 1.f / fmaxf(state[count_idx], 1.f);
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long n4 = count_idx >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<float4*>(state)[i];
    v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
    reinterpret_cast<float4*>(state)[i] = v;
    const long long e = i << 2;
    if (shadow && e + 3 < n_params) {
      uint2 s;
      s.x = pack_bf2(v.x, v.y);
      s.y = pack_bf2(v.z, v.w);
      reinterpret_cast<uint2*>(shadow)[i] = s;
    } else if (shadow) {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int k = 0; k < 4; ++k)
        if (e + k < n_params) shadow[e + k] = f2bf(vv[k]);
    }
    if (i64) {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int k = 0; k < 4; ++k) {
        const long long j = e + k - i64_off;
        if (j >= 0 && j < n_i64) i64[j] = (long long)floorf(vv[k] + 1e-3f);
      }
    }
  }
  for (long long e = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; e < count_idx; e += stride) {
    const float v = state[e] * inv;
    state[e] = v;
    if (shadow && e < n_params) shadow[e] = f2bf(v);
    const long long j = e - i64_off;
    if (i64 && j >= 0 && j < n_i64) i64[j] = (long long)floorf(v + 1e-3f);
  }
}

// Staleness-1 K-AVG (parallel/kavg.py AsyncModelAverager), two passes per round instead of six:
// launch: flat := x, snap := x (one read, two writes; flat then goes into the async SUM);
// apply:  x := x + (flat / world - snap), the bf16 shadow of the parameter range refreshed in
// the same pass (same operation order as the torch div / sub / add it replaces).
__global__ void k_kavg_snap(const float* __restrict__ x, float* __restrict__ flat, float* __restrict__ snap,
                            long long n) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<float4*>(flat)[i] = v;
    reinterpret_cast<float4*>(snap)[i] = v;
  }
  for (long long i = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    flat[i] = x[i];
    snap[i] = x[i];
  }
}

// x + (flat / world - snap): a multiply by the fp32 reciprocal (computed once on the host), then
// the subtraction and the addition, each rounded on its own (no contraction into an FMA)
__device__ __forceinline__ float kavg_step(float x, float f, float sn, float inv) {
  // the build's -ffp-contract=fast ignores contract pragmas: an empty asm on the product keeps
  // it a rounded value of its own, so the subtraction is not fused into an FMA
  float q = f * inv;
  asm volatile("" : "+v"(q));
  return x + (q - sn);
}

__global__ void k_kavg_async_apply(float* __restrict__ x, const float* __restrict__ flat,
                                   const float* __restrict__ snap, bf16_t* __restrict__ shadow, float inv,
                                   long long n, long long n_params) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<float4*>(x)[i];
    const float4 f = reinterpret_cast<const float4*>(flat)[i], sn = reinterpret_cast<const float4*>(snap)[i];
    v.x = kavg_step(v.x, f.x, sn.x, inv); v.y = kavg_step(v.y, f.y, sn.y, inv);
    v.z = kavg_step(v.z, f.z, sn.z, inv); v.w = kavg_step(v.w, f.w, sn.w, inv);
    reinterpret_cast<float4*>(x)[i] = v;
    if (shadow && 4 * i + 3 < n_params) {
      uint2 sh;
      sh.x = pack_bf2(v.x, v.y);
      sh.y = pack_bf2(v.z, v.w);
      reinterpret_cast<uint2*>(shadow)[i] = sh;
    } else if (shadow) {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int k = 0; k < 4; ++k)
        if (4 * i + k < n_params) shadow[4 * i + k] = f2bf(vv[k]);
    }
  }
  for (long long i = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    x[i] = kavg_step(x[i], flat[i], snap[i], inv);
    if (shadow && i < n_params) shadow[i] = f2bf(x[i]);
  }
}

KML_API int kml_kavg_snap(const float* x, float* flat, float* snap, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_kavg_snap, dim3(kml_stream_grid((n + 3) / 4, 256)), dim3(256), 0, s, x, flat, snap, n);
  KML_LAUNCH_CHECK();
}

KML_API int kml_kavg_async_apply(float* x, const float* flat, const float* snap, bf16_t* shadow, float world,
                                 long long n, long long n_params, hipStream_t s) {
  hipLaunchKernelGGL(k_kavg_async_apply, dim3(kml_stream_grid((n + 3) / 4, 256)), dim3(256), 0, s, x, flat, snap,
                     shadow, 1.0f / world, n, n_params);
  KML_LAUNCH_CHECK();
}

KML_API int kml_kavg_pack(float* state, const long long* i64, long long i64_off, int n_i64, long long count_idx,
                          int participate, hipStream_t s) {
  const int n = n_i64 > 1 ? n_i64 : 1;
  hipLaunchKernelGGL(k_kavg_pack, dim3((n + 255) / 256), dim3(256), 0, s, state, i64, i64_off, n_i64, count_idx,
                     participate);
  KML_LAUNCH_CHECK();
}

KML_API int kml_kavg_finish(float* state, long long n_params, long long count_idx, bf16_t* shadow, long long* i64,
                            long long i64_off, int n_i64, hipStream_t s) {
  hipLaunchKernelGGL(k_kavg_finish, dim3(kml_stream_grid((count_idx + 3) / 4, 256)), dim3(256), 0, s, state,
                     n_params, count_idx, shadow, i64, i64_off, n_i64);
  KML_LAUNCH_CHECK();
}
