// augment.hip — on-device image batch preparation (gfx950).
//
// The dataset stays resident in HBM as raw uint8 NHWC (CIFAR-10 is 150 MB; 288 GB of
// HBM holds any of the reference's datasets many times over).  One kernel turns a
// contiguous range of samples into the network input:
//   random crop with zero padding (RandomCrop(32, 4)), random horizontal flip,
//   ToTensor (/255) + Normalize(mean, std), cast to bf16, NHWC with channels padded
//   to a multiple of 8 (the conv kernels' 16-byte vector width).
// Randomness is a counter-based hash of (seed, step, sample) where seed/step are read
// from device memory, so a hipGraph replay draws fresh crops every step.
// Reference transform chain: function_resnet34.py:17-30 (train) / :27-30 (val).
#include "kml_common.h"

namespace {

__device__ __forceinline__ unsigned hash3(unsigned a, unsigned b, unsigned c) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

struct AugArgs {
  const unsigned char* src;  // [N][H][W][C] uint8
  const long long* labels_src;
  bf16_t* dst;               // [B][H][W][CP]
  long long* labels_dst;
  const float* ctr;          // device [seed, step, start]
  int N, H, W, C, CP, B;
  int pad, flip, train;
  float mean[4], inv_std[4];
};

// one thread per output pixel (all CP channels -> one 16-byte store when CP == 8)
__global__ void k_augment(AugArgs a) {
  const long long total = (long long)a.B * a.H * a.W;
  const unsigned seed = (unsigned)a.ctr[0], step = (unsigned)a.ctr[1];
  const long long start = (long long)a.ctr[2];
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(t % a.W);
    const int y = (int)((t / a.W) % a.H);
    const int b = (int)(t / ((long long)a.W * a.H));
    const long long sidx = (start + b) % a.N;
    int dx = 0, dy = 0, fl = 0;
    if (a.train) {
      const unsigned h = hash3(seed, step, (unsigned)sidx);
      const int span = 2 * a.pad + 1;
      dy = (int)(h % span) - a.pad;
      dx = (int)((h / span) % span) - a.pad;
      fl = a.flip ? (int)((h >> 24) & 1) : 0;
    }
    int sx = fl ? (a.W - 1 - x) : x;
    sx += dx;
    const int sy = y + dy;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if ((unsigned)sx < (unsigned)a.W && (unsigned)sy < (unsigned)a.H) {
      const unsigned char* p = a.src + ((sidx * a.H + sy) * a.W + sx) * a.C;
      for (int c = 0; c < a.C && c < 4; ++c) v[c] = ((float)p[c] * (1.f / 255.f) - a.mean[c]) * a.inv_std[c];
    } else {
      // zero padding happens BEFORE normalisation in the reference chain (pad on the uint8 image)
      for (int c = 0; c < a.C && c < 4; ++c) v[c] = (0.f - a.mean[c]) * a.inv_std[c];
    }
    bf16_t* o = a.dst + t * a.CP;
    if (a.CP == 8) {
      uint4 q;
      q.x = pack_bf2(v[0], v[1]); q.y = pack_bf2(v[2], v[3]); q.z = pack_bf2(v[4], v[5]); q.w = pack_bf2(v[6], v[7]);
      *reinterpret_cast<uint4*>(o) = q;
    } else {
      for (int c = 0; c < a.CP; ++c) o[c] = f2bf(c < 8 ? v[c] : 0.f);
    }
    if (x == 0 && y == 0 && a.labels_dst) a.labels_dst[b] = a.labels_src[sidx];
  }
}

}  // namespace

KML_API int kml_augment(const unsigned char* src, const long long* labels_src, bf16_t* dst, long long* labels_dst,
                        const float* ctr, int N, int H, int W, int C, int CP, int B, int pad, int flip, int train,
                        const float* mean, const float* std, hipStream_t s) {
  if (C > 4 || CP < C) return (int)hipErrorInvalidValue;
  AugArgs a;
  a.src = src; a.labels_src = labels_src; a.dst = dst; a.labels_dst = labels_dst; a.ctr = ctr;
  a.N = N; a.H = H; a.W = W; a.C = C; a.CP = CP; a.B = B; a.pad = pad; a.flip = flip; a.train = train;
  for (int i = 0; i < 4; ++i) {
    a.mean[i] = i < C ? mean[i] : 0.f;
    a.inv_std[i] = i < C ? 1.f / std[i] : 0.f;
  }
  long long total = (long long)B * H * W;
  hipLaunchKernelGGL(k_augment, dim3(kml_stream_grid(total, 256)), dim3(256), 0, s, a);
  KML_LAUNCH_CHECK();
}

// advance the data-pipeline counters in place: ctr = [seed, step, start]
__global__ void k_advance(float* ctr, float batch, float n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ctr[1] += 1.f;
    float s = ctr[2] + batch;
    if (s >= n) s -= n;
    ctr[2] = s;
  }
}

KML_API int kml_advance_counter(float* ctr, float batch, float n, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, ctr, batch, n);
  KML_LAUNCH_CHECK();
}
