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

// one SGD range carried by extra blocks of another launch (blocks == 0: none)
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

// block `b` of the rider's `blocks` (256 threads each)
__device__ __forceinline__ void kml_sgd_rider_run(const KmlSgdRider& r, int b) {
  const float lr = *r.lr_ptr;
  const int first = r.first_ptr ? (*r.first_ptr != 0.f) : 0;
  kml_sgd_range(r.w, r.g, r.mom, r.shadow, lr, r.wd, r.momentum, r.dampening, r.nesterov, first, r.grad_scale, r.n,
                (long long)b * blockDim.x + threadIdx.x, (long long)r.blocks * blockDim.x);
}
