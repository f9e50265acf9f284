// pool.hip — pooling for NHWC bf16 on gfx950.
//
//   maxpool fwd : one thread per (output pixel, 8-channel chunk); writes the window
//                 argmax (uint8, row-major tap index) for backward.
//   maxpool bwd : gather formulation (each input element sums the output gradients of
//                 the windows that selected it) — no atomics, no zero-fill pass.
//   global avgpool fwd/bwd (AdaptiveAvgPool2d(1)).
//   option-A shortcut fwd/bwd (CIFAR ResNet, reference ml/experiments/kubeml/resnet32.py
//                 LambdaLayer): stride-2 subsample + zero channel padding, 16-byte chunks.
// Reference parity: nn.MaxPool2d(3,2,1) of the ResNet stem / nn.MaxPool2d(2) of LeNet
// (function_lenet.py:25-31), AdaptiveAvgPool2d((1,1)) of torchvision resnet.
#include "kml_common.h"

namespace {

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

struct PoolGeom { int B, H, W, C, OH, OW, k, s, p; };

__global__ void k_maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                              unsigned char* __restrict__ idx, PoolGeom g) {
  const int CH = g.C / 8;
  const long long total = (long long)g.B * g.OH * g.OW * CH;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(t % CH);
    long long pix = t / CH;
    const int ow = (int)(pix % g.OW); pix /= g.OW;
    const int oh = (int)(pix % g.OH); const int b = (int)(pix / g.OH);
    float best[8]; int bi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; bi[i] = 0; }
    for (int r = 0; r < g.k; ++r) {
      const int ih = oh * g.s - g.p + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int q = 0; q < g.k; ++q) {
        const int iw = ow * g.s - g.p + q;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + ((long long)(b * g.H + ih) * g.W + iw) * g.C + ch * 8), f);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (f[i] > best[i] || (f[i] != f[i])) { best[i] = f[i]; bi[i] = r * g.k + q; }
      }
    }
    reinterpret_cast<uint4*>(y)[t] = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    reinterpret_cast<uint2*>(idx)[t] = packed;
  }
}

// relu_out (optional): the pooled forward output of a fused BN -> ReLU -> max-pool; a window
// whose maximum is not > 0 passes no gradient (its argmax sat at ReLU's zero), so dx is
// already dz = d(BN output) and the BN backward needs no ReLU mask.
// Every thread owns one 16-byte chunk (b, ih, iw, 8 channels) of dx; blocks of RPB whole input rows
// (a row of R34's 16x16x64 stem map is 128 chunks: one row per block left half the threads idle on
// 4096 blocks).  Per-row window bounds, 32-bit indices (the flat 64-bit div / mod chain per element
// cost more than the memory traffic on ResNet-50's 112x112 stem pool: 164 us for 256 MB).
// MW: at most MW windows per dimension cover an input element ((k + s - 1) / s; 2 for the 3x3/s2
// and 2x2/s2 pools): the MW x MW candidate windows are unrolled and all their loads issued before
// any is used (the data-dependent loop waited on each window's loads in turn)
template <int MW>
__global__ __launch_bounds__(256) void k_maxpool_bwd(const bf16_t* __restrict__ dy, const unsigned char* __restrict__ idx,
                                                     const bf16_t* __restrict__ relu_out, bf16_t* __restrict__ dx,
                                                     PoolGeom g, int rpb) {
  const int CH = g.C / 8;
  const int per_row = g.W * CH;
  const int lr = (int)threadIdx.x / per_row;   // row within the block (rpb > 1: per_row <= 128)
  const int ustart = rpb > 1 ? (int)threadIdx.x - lr * per_row : (int)threadIdx.x;
  if (lr >= rpb) return;
  for (int row = blockIdx.y * rpb + lr; row < g.B * g.H; row += gridDim.y * rpb) {
    const int b = row / g.H, ih = row - b * g.H;
    // outputs whose window contains ih: oh*s - p <= ih <= oh*s - p + k - 1
    const int oh_lo = max(0, (ih + g.p - g.k + g.s) / g.s), oh_hi = min(g.OH - 1, (ih + g.p) / g.s);
    for (int u = blockIdx.x * 256 + ustart; u < per_row; u += gridDim.x * 256) {
      const int iw = u / CH, ch = u - iw * CH;
      const int ow_lo = max(0, (iw + g.p - g.k + g.s) / g.s), ow_hi = min(g.OW - 1, (iw + g.p) / g.s);
      uint2 pk[MW * MW];
      uint4 dv[MW * MW], mv[MW * MW];
      int tap[MW * MW];
#pragma unroll
      for (int a = 0; a < MW; ++a)
#pragma unroll
        for (int c = 0; c < MW; ++c) {
          const int oh = oh_lo + a, ow = ow_lo + c, w = a * MW + c;
          const int r = ih - (oh * g.s - g.p), q = iw - (ow * g.s - g.p);
          const bool ok = oh <= oh_hi && ow <= ow_hi && r >= 0 && r < g.k && q >= 0 && q < g.k;
          tap[w] = ok ? r * g.k + q : -1;
          const long long o = ok ? ((long long)(b * g.OH + oh) * g.OW + ow) * CH + ch : 0;
          pk[w] = reinterpret_cast<const uint2*>(idx)[o];
          dv[w] = reinterpret_cast<const uint4*>(dy)[o];
          if (relu_out) mv[w] = reinterpret_cast<const uint4*>(relu_out)[o];
        }
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int w = 0; w < MW * MW; ++w) {   // window order (oh, ow) ascending, as the loop summed
        float d[8];
        unpack8(dv[w], d);
        if (relu_out) {
          float m[8];
          unpack8(mv[w], m);
#pragma unroll
          for (int i = 0; i < 8; ++i) d[i] = m[i] > 0.f ? d[i] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned x = i < 4 ? pk[w].x : pk[w].y;
          if (tap[w] >= 0 && (int)((x >> (8 * (i & 3))) & 0xff) == tap[w]) acc[i] += d[i];
        }
      }
      reinterpret_cast<uint4*>(dx)[(long long)row * per_row + u] = pack8(acc);
    }
  }
}

// global average pool: x [B][HW][C] -> y [B][C]; one thread per (b, chunk)
__global__ void k_gavg_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B, int HW, int C) {
  const int CH = C / 8;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * CH) return;
  const int b = t / CH, ch = t % CH;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int p = 0; p < HW; ++p) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + ((long long)b * HW + p) * C + ch * 8), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += f[i];
  }
  const float inv = 1.f / HW;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] *= inv;
  reinterpret_cast<uint4*>(y)[t] = pack8(acc);
}

__global__ void k_gavg_bwd(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int B, int HW, int C) {
  const int CH = C / 8;
  const long long total = (long long)B * HW * CH;
  const float inv = 1.f / HW;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(t % CH);
    const long long b = t / CH / HW;
    float d[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[b * CH + ch], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] *= inv;
    reinterpret_cast<uint4*>(dx)[t] = pack8(d);
  }
}

// option-A shortcut forward: y[b,oh,ow,:] = [0]*pad ++ x[b,2oh,2ow,:] ++ [0]*pad; one thread per
// 8-channel output chunk (pad % 8 == 0 keeps every chunk wholly data or wholly zero)
__global__ void k_shortcut_a_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B, int H, int W, int C,
                                 int OH, int OW, int pad) {
  const int Co8 = (C + 2 * pad) / 8;
  const long long total = (long long)B * OH * OW * Co8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Co8) * 8 - pad;
    const long long pix = i / Co8;
    const int ow = (int)(pix % OW), oh = (int)((pix / OW) % OH), b = (int)(pix / ((long long)OW * OH));
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (c >= 0 && c < C) v = *reinterpret_cast<const uint4*>(x + (((long long)b * H + 2 * oh) * W + 2 * ow) * C + c);
    reinterpret_cast<uint4*>(y)[i] = v;
  }
}

// option-A shortcut backward: dx at even (h, w) takes the un-padded channels of dy, zero elsewhere
__global__ void k_shortcut_a_bwd(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int B, int H, int W, int C,
                                 int OH, int OW, int pad) {
  const int C8 = C / 8, Co = C + 2 * pad;
  const long long total = (long long)B * H * W * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const long long pix = i / C8;
    const int w = (int)(pix % W), h = (int)((pix / W) % H), b = (int)(pix / ((long long)W * H));
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (!(h & 1) && !(w & 1))
      v = *reinterpret_cast<const uint4*>(dy + (((long long)b * OH + (h >> 1)) * OW + (w >> 1)) * Co + pad + c);
    reinterpret_cast<uint4*>(dx)[i] = v;
  }
}

}  // namespace

KML_API int kml_maxpool_fwd(const bf16_t* x, bf16_t* y, unsigned char* idx, int B, int H, int W, int C, int k,
                            int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return (int)hipErrorInvalidValue;
  PoolGeom g{B, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  long long total = (long long)B * g.OH * g.OW * (C / 8);
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(kml_stream_grid(total, 256)), dim3(256), 0, st, x, y, idx, g);
  KML_LAUNCH_CHECK();
}

KML_API int kml_maxpool_bwd(const bf16_t* dy, const unsigned char* idx, const bf16_t* relu_out, bf16_t* dx, int B,
                            int H, int W, int C, int k, int s, int p, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolGeom g{B, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  const int per_row = W * (C / 8), rows = B * H;
  const int rpb = per_row <= 128 ? 256 / per_row : 1;   // whole rows per 256-thread block
  const int gy = (rows + rpb - 1) / rpb;
  const dim3 grid(rpb > 1 ? 1 : (per_row + 255) / 256, gy < 65535 ? gy : 65535);
  const int mw = (k + s - 1) / s;
  if (mw <= 1) hipLaunchKernelGGL(k_maxpool_bwd<1>, grid, dim3(256), 0, st, dy, idx, relu_out, dx, g, rpb);
  else if (mw == 2) hipLaunchKernelGGL(k_maxpool_bwd<2>, grid, dim3(256), 0, st, dy, idx, relu_out, dx, g, rpb);
  else if (mw == 3) hipLaunchKernelGGL(k_maxpool_bwd<3>, grid, dim3(256), 0, st, dy, idx, relu_out, dx, g, rpb);
  else return (int)hipErrorInvalidValue;
  KML_LAUNCH_CHECK();
}

KML_API int kml_gavgpool_fwd(const bf16_t* x, bf16_t* y, int B, int HW, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  int n = B * (C / 8);
  hipLaunchKernelGGL(k_gavg_fwd, dim3((n + 255) / 256), dim3(256), 0, st, x, y, B, HW, C);
  KML_LAUNCH_CHECK();
}

KML_API int kml_gavgpool_bwd(const bf16_t* dy, bf16_t* dx, int B, int HW, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  long long total = (long long)B * HW * (C / 8);
  hipLaunchKernelGGL(k_gavg_bwd, dim3(kml_stream_grid(total, 256)), dim3(256), 0, st, dy, dx, B, HW, C);
  KML_LAUNCH_CHECK();
}

KML_API int kml_shortcut_a_fwd(const bf16_t* x, bf16_t* y, int B, int H, int W, int C, int pad, hipStream_t st) {
  if (C % 8 || pad % 8 || pad < 0) return (int)hipErrorInvalidValue;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long long total = (long long)B * OH * OW * ((C + 2 * pad) / 8);
  hipLaunchKernelGGL(k_shortcut_a_fwd, dim3(kml_stream_grid(total, 256)), dim3(256), 0, st, x, y, B, H, W, C, OH, OW,
                     pad);
  KML_LAUNCH_CHECK();
}

KML_API int kml_shortcut_a_bwd(const bf16_t* dy, bf16_t* dx, int B, int H, int W, int C, int pad, hipStream_t st) {
  if (C % 8 || pad % 8 || pad < 0) return (int)hipErrorInvalidValue;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long long total = (long long)B * H * W * (C / 8);
  hipLaunchKernelGGL(k_shortcut_a_bwd, dim3(kml_stream_grid(total, 256)), dim3(256), 0, st, dy, dx, B, H, W, C, OH, OW,
                     pad);
  KML_LAUNCH_CHECK();
}
