// adam_probe.hip — access-pattern probe for the fused Adam step on a VGG-16-sized flat space
// (34.0 M parameters: 14.7 M conv + 19.3 M classifier).  Times variants of the same update
// with hipEvents and prints the achieved HBM rate, next to a v4f copy of the same bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/adam_probe tools/adam_probe.hip && /tmp/adam_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned short bf16_t;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{a, b}), bf16x2_hw));
}
template <typename T> __device__ __forceinline__ T ld(const T* p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T> __device__ __forceinline__ void st(T* p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
// stochastic rounding of a float to bf16 with 16 random bits
__device__ __forceinline__ unsigned sr_bf(float f, unsigned r16) { return (__float_as_uint(f) + r16) >> 16; }

struct P { float b1, b2, eps, wd, step_size, rbc2, lr; };

__device__ __forceinline__ void upd(float& w, float g, float& m, float& v, const P& p) {
  g += p.wd * w;
  m = p.b1 * m + (1.f - p.b1) * g;
  v = p.b2 * v + (1.f - p.b2) * g * g;
  w -= p.step_size * m / (sqrtf(v) * p.rbc2 + p.eps);
}

__device__ __forceinline__ void upd4(v4f& W, v4f G, v4f& M, v4f& V, const P& p) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float w = W[k], m = M[k], v = V[k];
    upd(w, G[k], m, v, p);
    W[k] = w; M[k] = m; V[k] = v;
  }
}

// grid-stride, U v4f groups per thread per iteration
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_gs(float* w, const float* g, float* m, float* v, bf16_t* sh, P p, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    v4f W[U], G[U], M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i < n4) {
        W[u] = ld((v4f*)w + i, NT); G[u] = ld((const v4f*)g + i, NT);
        M[u] = ld((v4f*)m + i, NT); V[u] = ld((v4f*)v + i, NT);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n4) break;
      upd4(W[u], G[u], M[u], V[u], p);
      st((v4f*)w + i, W[u], NT); st((v4f*)m + i, M[u], NT); st((v4f*)v + i, V[u], NT);
      v2u s; s.x = pack_bf2(W[u].x, W[u].y); s.y = pack_bf2(W[u].z, W[u].w);
      st((v2u*)sh + i, s, NT);
    }
  }
}

// contiguous chunk per block (each block streams its own span of every array)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_chunk(float* w, const float* g, float* m, float* v, bf16_t* sh, P p, long long n4) {
  const long long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long long lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  for (long long i0 = lo + threadIdx.x; i0 < hi; i0 += U * 256) {
    v4f W[U], G[U], M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * 256;
      if (i < hi) {
        W[u] = ld((v4f*)w + i, NT); G[u] = ld((const v4f*)g + i, NT);
        M[u] = ld((v4f*)m + i, NT); V[u] = ld((v4f*)v + i, NT);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * 256;
      if (i >= hi) break;
      upd4(W[u], G[u], M[u], V[u], p);
      st((v4f*)w + i, W[u], NT); st((v4f*)m + i, M[u], NT); st((v4f*)v + i, V[u], NT);
      v2u s; s.x = pack_bf2(W[u].x, W[u].y); s.y = pack_bf2(W[u].z, W[u].w);
      st((v2u*)sh + i, s, NT);
    }
  }
}

// bf16 moments with stochastic rounding (22 B / parameter instead of 30)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_bf16m(float* w, const float* g, bf16_t* m, bf16_t* v, bf16_t* sh, P p,
                                               long long n4, unsigned seed) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    v4f W[U], G[U];
    v2u M[U], V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i < n4) {
        W[u] = ld((v4f*)w + i, NT); G[u] = ld((const v4f*)g + i, NT);
        M[u] = ld((v2u*)m + i, NT); V[u] = ld((v2u*)v + i, NT);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n4) break;
      float wv[4] = {W[u].x, W[u].y, W[u].z, W[u].w}, gv[4] = {G[u].x, G[u].y, G[u].z, G[u].w};
      float mv[4] = {__uint_as_float(M[u].x << 16), __uint_as_float(M[u].x & 0xffff0000u),
                     __uint_as_float(M[u].y << 16), __uint_as_float(M[u].y & 0xffff0000u)};
      float vv[4] = {__uint_as_float(V[u].x << 16), __uint_as_float(V[u].x & 0xffff0000u),
                     __uint_as_float(V[u].y << 16), __uint_as_float(V[u].y & 0xffff0000u)};
      unsigned mo[4], vo[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        upd(wv[k], gv[k], mv[k], vv[k], p);
        const unsigned r = hash32((unsigned)(i * 4 + k) ^ seed);
        mo[k] = sr_bf(mv[k], r & 0xffffu);
        vo[k] = sr_bf(vv[k], r >> 16);
      }
      st((v4f*)w + i, v4f{wv[0], wv[1], wv[2], wv[3]}, NT);
      v2u a; a.x = mo[0] | (mo[1] << 16); a.y = mo[2] | (mo[3] << 16); st((v2u*)m + i, a, NT);
      v2u b; b.x = vo[0] | (vo[1] << 16); b.y = vo[2] | (vo[3] << 16); st((v2u*)v + i, b, NT);
      v2u s; s.x = pack_bf2(wv[0], wv[1]); s.y = pack_bf2(wv[2], wv[3]); st((v2u*)sh + i, s, NT);
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4f* a, v4f* b, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) st(b + i, ld(a + i, NT), NT);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const long long n = 34015396LL & ~3LL, n4 = n / 4;
  float *w, *g, *m, *v, *c0, *c1;
  bf16_t *sh, *mb, *vb;
  CK(hipMalloc(&w, n * 4)); CK(hipMalloc(&g, n * 4)); CK(hipMalloc(&m, n * 4)); CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&sh, n * 2)); CK(hipMalloc(&mb, n * 2)); CK(hipMalloc(&vb, n * 2));
  CK(hipMalloc(&c0, n * 4 * 4)); CK(hipMalloc(&c1, n * 4 * 4));
  CK(hipMemset(w, 0, n * 4)); CK(hipMemset(g, 0, n * 4)); CK(hipMemset(m, 0, n * 4)); CK(hipMemset(v, 0, n * 4));
  CK(hipMemset(mb, 0, n * 2)); CK(hipMemset(vb, 0, n * 2)); CK(hipMemset(c0, 0, n * 16));
  P p{0.9f, 0.999f, 1e-8f, 0.f, 1e-3f, 1.f, 1e-3f};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 20;
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / iters;
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  const double b30 = 30.0 * n, b22 = 22.0 * n;
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64];
    printf("-- grid %d\n", grid);
    snprintf(nm, 64, "copy 30B-eq");
    timeit(nm, 30.0 * n, [&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), 0, 0, (const v4f*)c0, (v4f*)c1, (long long)(n * 15 / 16)); });
    timeit("copy nt", 30.0 * n, [&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, 0, (const v4f*)c0, (v4f*)c1, (long long)(n * 15 / 16)); });
    timeit("gs U2", b30, [&] { hipLaunchKernelGGL((k_gs<2, false>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("gs U2 nt", b30, [&] { hipLaunchKernelGGL((k_gs<2, true>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("gs U1", b30, [&] { hipLaunchKernelGGL((k_gs<1, false>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("gs U4", b30, [&] { hipLaunchKernelGGL((k_gs<4, false>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("chunk U2", b30, [&] { hipLaunchKernelGGL((k_chunk<2, false>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("chunk U2 nt", b30, [&] { hipLaunchKernelGGL((k_chunk<2, true>), dim3(grid), dim3(256), 0, 0, w, g, m, v, sh, p, n4); });
    timeit("bf16m U2", b22, [&] { hipLaunchKernelGGL((k_bf16m<2, false>), dim3(grid), dim3(256), 0, 0, w, g, mb, vb, sh, p, n4, 77u); });
    timeit("bf16m U2 nt", b22, [&] { hipLaunchKernelGGL((k_bf16m<2, true>), dim3(grid), dim3(256), 0, 0, w, g, mb, vb, sh, p, n4, 77u); });
    timeit("bf16m U4", b22, [&] { hipLaunchKernelGGL((k_bf16m<4, false>), dim3(grid), dim3(256), 0, 0, w, g, mb, vb, sh, p, n4, 77u); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
