// transformer.hip — the non-GEMM ops of a BERT-style encoder for gfx950:
//   LayerNorm fwd (+ fused residual add) / bwd (dgamma, dbeta two-level deterministic),
//   GELU (erf) fwd/bwd, counter-based dropout fwd/bwd (mask regenerated, never stored),
//   fused embedding (word + position + token type) gather fwd / scatter-add bwd,
//   row gather / scatter (masked-LM positions).
// Rows are bf16 vectors of length N (N % 4 == 0); one wave per row, 8-byte lane loads;
// statistics in fp32.  Random numbers come from a hash of (seed, step, element) with
// seed/step in device memory, so hipGraph replays draw fresh masks.
#include "kml_common.h"

namespace {

__device__ __forceinline__ void ld4(const bf16_t* p, float* f) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
}
__device__ __forceinline__ void st4(bf16_t* p, const float* f) {
  uint2 v;
  v.x = pack_bf2(f[0], f[1]);
  v.y = pack_bf2(f[2], f[3]);
  *reinterpret_cast<uint2*>(p) = v;
}

constexpr int MAXV = 8;  // up to 8 x (64 lanes x 4) = 2048 columns held in registers

__device__ __forceinline__ unsigned hash3(unsigned a, unsigned b, unsigned c) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

// dropout of 4 consecutive elements starting at flat (even) index e, bit-identical to
// k_dropout: element pair j = e / 2 keeps its low / high element when the matching 16-bit
// half of hash(seed ^ salt, step, j) >= p * 2^16; kept values are bf16(x / (1 - p))
__device__ __forceinline__ void drop4(float* v, long long e, const float* ctr, unsigned salt, float p) {
  const unsigned seed = (unsigned)ctr[0], step = (unsigned)ctr[1];
  const unsigned thr = (unsigned)(p * 65536.0f);
  const float sc = 1.f / (1.f - p);
  const unsigned j = (unsigned)(e >> 1);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const unsigned h = hash3(seed ^ salt, step, j + q);
    const float a = (h & 0xFFFFu) >= thr ? v[2 * q] * sc : 0.f;
    const float b = (h >> 16) >= thr ? v[2 * q + 1] * sc : 0.f;
    const unsigned pk = pack_bf2(a, b);
    v[2 * q] = lo_bf(pk);
    v[2 * q + 1] = hi_bf(pk);
  }
}

// ------------------------------------------------------------------------------ LayerNorm fwd
// y = LN(x [+ res]) * g + b ; sum_out (optional) = x + res (the LN input, kept for backward)
// One wave per row; NV = ceil(N / 256) register vectors (compile time: 3 for a 768-wide row).
template <int NV>
__global__ __launch_bounds__(256) void k_ln_fwd(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                bf16_t* __restrict__ y, bf16_t* __restrict__ sum_out,
                                                float* __restrict__ mean, float* __restrict__ rstd, long long M,
                                                int N, float eps, const float* __restrict__ dctr, unsigned dsalt,
                                                float dp) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + row * N;
  float v[NV][4];
  uint2 rv[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {  // all loads first
    const int c = (u * 64 + lane) * 4;
    if (c < N) {
      const uint2 xv = *reinterpret_cast<const uint2*>(xr + c);
      v[u][0] = lo_bf(xv.x); v[u][1] = hi_bf(xv.x); v[u][2] = lo_bf(xv.y); v[u][3] = hi_bf(xv.y);
      if (res) rv[u] = *reinterpret_cast<const uint2*>(res + row * N + c);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c = (u * 64 + lane) * 4;
    if (c < N) {
      if (dctr) drop4(v[u], row * N + c, dctr, dsalt, dp);  // x = dropout(x), as k_dropout
      if (res) {
        v[u][0] += lo_bf(rv[u].x); v[u][1] += hi_bf(rv[u].x); v[u][2] += lo_bf(rv[u].y); v[u][3] += hi_bf(rv[u].y);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) s += v[u][k];
    }
  }
  s = wave_sum(s);
  const float mu = s / N;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c = (u * 64 + lane) * 4;
    if (c < N)
#pragma unroll
      for (int k = 0; k < 4; ++k) { const float d = v[u][k] - mu; q += d * d; }
  }
  q = wave_sum(q);
  const float rs = rsqrtf(q / N + eps);
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c = (u * 64 + lane) * 4;
    if (c < N) {
      if (sum_out) st4(sum_out + row * N + c, v[u]);
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (v[u][k] - mu) * rs * gamma[c + k] + beta[c + k];
      st4(y + row * N + c, o);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// ------------------------------------------------------------------------------ LayerNorm bwd
// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat));  dx (+)= into dx (accumulate flag)
// dgamma/dbeta: per-block partials [gridDim][2N], then k_colreduce sums them in block order.
// One wave per row, NV = ceil(N / 256) register vectors per operand (compile time: a 768-wide
// BERT row holds 3, not the 8 of the widest shape), and the wave's NEXT row (row + 4) is
// loaded while this one is reduced and stored — the per-row chain (loads -> two wave
// reductions -> stores) otherwise leaves one row in flight per wave.  Same per-element
// arithmetic and per-wave row order as the one-row version: bit-identical results.
template <int NV>
__global__ __launch_bounds__(256) void k_ln_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ xin,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                                const bf16_t* __restrict__ dx_add, float* __restrict__ part,
                                                long long M, int N, int rows_per_block, bf16_t* __restrict__ dx_drop,
                                                const float* __restrict__ dctr, unsigned dsalt, float dp,
                                                int with_in) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pg[NV][4], pb[NV][4], pi[NV][4];  // pi: column sums of the input gradient (part_in)
  float gm[NV][4];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c = (u * 64 + lane) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pg[u][k] = 0.f; pb[u][k] = 0.f; pi[u][k] = 0.f;
      gm[u][k] = c < N ? gamma[c + k] : 0.f;
    }
  }
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  uint2 dv[NV], xv[NV], av[NV];
  float mu = 0.f, rs = 0.f;
  auto load = [&](long long row) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = (u * 64 + lane) * 4;
      if (c < N) {
        dv[u] = *reinterpret_cast<const uint2*>(dy + row * N + c);
        xv[u] = *reinterpret_cast<const uint2*>(xin + row * N + c);
        if (dx_add) av[u] = *reinterpret_cast<const uint2*>(dx_add + row * N + c);
      }
    }
    mu = mean[row];
    rs = rstd[row];
  };
  long long row = r0 + wv;
  if (row < r1) load(row);
  for (; row < r1; row += 4) {
    uint2 d_cur[NV], x_cur[NV], a_cur[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) { d_cur[u] = dv[u]; x_cur[u] = xv[u]; a_cur[u] = av[u]; }
    const float mu_c = mu, rs_c = rs;
    if (row + 4 < r1) load(row + 4);  // next row of this wave, in flight during this one
    float xh[NV][4], gd[NV][4];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = (u * 64 + lane) * 4;
      if (c < N) {
        const float d[4] = {lo_bf(d_cur[u].x), hi_bf(d_cur[u].x), lo_bf(d_cur[u].y), hi_bf(d_cur[u].y)};
        const float xf[4] = {lo_bf(x_cur[u].x), hi_bf(x_cur[u].x), lo_bf(x_cur[u].y), hi_bf(x_cur[u].y)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xh[u][k] = (xf[k] - mu_c) * rs_c;
          gd[u][k] = d[k] * gm[u][k];
          a1 += gd[u][k];
          a2 += gd[u][k] * xh[u][k];
          pg[u][k] += d[k] * xh[u][k];
          pb[u][k] += d[k];
        }
      }
    }
    a1 = wave_sum(a1) / N;
    a2 = wave_sum(a2) / N;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = (u * 64 + lane) * 4;
      if (c < N) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rs_c * (gd[u][k] - a1 - xh[u][k] * a2);
        if (dx_add) {
          const float e[4] = {lo_bf(a_cur[u].x), hi_bf(a_cur[u].x), lo_bf(a_cur[u].y), hi_bf(a_cur[u].y)};
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] += e[k];
        }
        st4(dx + row * N + c, o);
        float od[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) od[k] = bf2f(f2bf(o[k]));
        if (dx_drop) {  // gradient through the fused forward dropout: dropout(bf16(dx)), as k_dropout
          drop4(od, row * N + c, dctr, dsalt, dp);
          st4(dx_drop + row * N + c, od);
        }
        if (with_in) {  // bias gradient of the Linear that produced the LN input
#pragma unroll
          for (int k = 0; k < 4; ++k) pi[u][k] += od[k];
        }
      }
    }
  }
  // block partials: reduce the 4 waves in LDS, then one row of 2N floats per block
  __shared__ float red[4][2 * 2048];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c = (u * 64 + lane) * 4;
    if (c < N)
#pragma unroll
      for (int k = 0; k < 4; ++k) { red[wv][c + k] = pg[u][k]; red[wv][N + c + k] = pb[u][k]; }
  }
  __syncthreads();
  // one partial row per block: [dgamma(N) | dbeta(N) (| input-gradient column sums(N))]
  float* mine = part + (long long)blockIdx.x * (with_in ? 3 : 2) * N;
  for (int c = threadIdx.x; c < 2 * N; c += 256) mine[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  if (with_in) {  // third segment, through the same LDS (uniform branch)
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = (u * 64 + lane) * 4;
      if (c < N)
#pragma unroll
        for (int k = 0; k < 4; ++k) red[wv][c + k] = pi[u][k];
    }
    __syncthreads();
    float* mi = mine + 2 * N;
    for (int c = threadIdx.x; c < N; c += 256) mi[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// column sums of part[G][W] in row order (deterministic): out_a[c] += sum (c < Na),
// out_b[c - Na] += sum (c < Na + Nb), out_c[c - Na - Nb] += sum (the rest)
__global__ __launch_bounds__(256) void k_colreduce(const float* __restrict__ part, int G, int W, int Na,
                                                   float* __restrict__ out_a, float* __restrict__ out_b,
                                                   int Nb = 0x7fffffff, float* __restrict__ out_c = nullptr) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + tx;
  float acc = 0.f;
  if (col < W) {
#pragma unroll 8
    for (int g = ty; g < G; g += 4) acc += part[(long long)g * W + col];
  }
  __shared__ float red[4][64];
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && col < W) {
    const float t = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
    if (col < Na) out_a[col] += t;
    else if (col - Na < Nb) out_b[col - Na] += t;
    else out_c[col - Na - Nb] += t;
  }
}

// ------------------------------------------------------------------------------ GELU (erf form)
__device__ __forceinline__ float gelu(float x) { return kml_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return kml_gelu_grad(x); }

__global__ void k_gelu_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float f[4];
    ld4(x + i * 4, f);
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = gelu(f[k]);
    st4(y + i * 4, f);
  }
}

// 16-byte rows of 8 elements, two independent loads in flight per thread (the GELU pass
// after a library GEMM writes the pre-activation: 2 x 100 MB for BERT-base's FFN1)
__global__ void k_gelu_fwd8(const uint4* __restrict__ x, uint4* __restrict__ y, long long n8) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += 2 * stride) {
    const bool two = i + stride < n8;
    const uint4 a = x[i];
    const uint4 b = two ? x[i + stride] : a;
    auto g = [](uint4 v) {
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
      unsigned o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack_bf2(gelu(lo_bf(w[k])), gelu(hi_bf(w[k])));
      return make_uint4(o[0], o[1], o[2], o[3]);
    };
    y[i] = g(a);
    if (two) y[i + stride] = g(b);
  }
}

__global__ void k_gelu_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, bf16_t* __restrict__ dx,
                           long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float d[4], f[4];
    ld4(dy + i * 4, d);
    ld4(x + i * 4, f);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] *= gelu_grad(f[k]);
    st4(dx + i * 4, d);
  }
}

// GELU backward of a [M][N] row-major map that also writes per-row-block column sums of dx
// (part[blockIdx.y][N]; k_colreduce adds them to the bias gradient of the Linear whose
// pre-activation x is): the FFN1 bias gradient without a second pass over dx.  A block covers
// rows [y * rpb, +rpb) x 1024 columns; each thread owns 4 columns (8-byte accesses, a block
// row is 2 KB contiguous) and sums the bf16-rounded dx it stores.
__global__ __launch_bounds__(256) void k_gelu_bwd_colsum(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                        bf16_t* __restrict__ dx, float* __restrict__ part,
                                                        long long M, int N, int rpb) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= N) return;
  const long long r0 = (long long)blockIdx.y * rpb;
  const long long r1 = min(M, r0 + rpb);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 8;  // rows in flight per thread (loads of U rows issued before any math)
  long long r = r0;
  for (; r + U <= r1; r += U) {
    float d[U][4], f[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ld4(dy + (r + u) * N + c, d[u]);
      ld4(x + (r + u) * N + c, f[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) d[u][k] = bf2f(f2bf(d[u][k] * gelu_grad(f[u][k])));
      st4(dx + (r + u) * N + c, d[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += d[u][k];
    }
  }
  for (; r < r1; ++r) {
    float d[4], f[4];
    ld4(dy + r * N + c, d);
    ld4(x + r * N + c, f);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = bf2f(f2bf(d[k] * gelu_grad(f[k])));
    st4(dx + r * N + c, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += d[k];
  }
  *reinterpret_cast<float4*>(part + (long long)blockIdx.y * N + c) = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

// ------------------------------------------------------------------------------ dropout
// y = x * keep / (1 - p); ctr = [seed, step].  One hash per element PAIR j (elements 2j,
// 2j+1): keep = 16-bit half of hash(seed ^ salt, step, j) >= p * 2^16.  8 elements (16 B)
// per thread per iteration, 4 hashes.
__global__ void k_dropout(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, const float* __restrict__ ctr,
                          unsigned salt, float p, long long n8) {
  const unsigned seed = (unsigned)ctr[0], step = (unsigned)ctr[1];
  const unsigned thr = (unsigned)(p * 65536.0f);
  const float sc = 1.f / (1.f - p);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const uint4 v = reinterpret_cast<const uint4*>(x)[i];
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
    unsigned o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned hsh = hash3(seed ^ salt, step, (unsigned)(i * 4 + k));
      const float a = (hsh & 0xFFFFu) >= thr ? lo_bf(w[k]) * sc : 0.f;
      const float b = (hsh >> 16) >= thr ? hi_bf(w[k]) * sc : 0.f;
      o[k] = pack_bf2(a, b);
    }
    reinterpret_cast<uint4*>(y)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ------------------------------------------------------------------------------ embeddings
// sum[t] = word[ids[t]] + pos[t % L] + type[tt[t]]   (tables fp32 master? no: bf16 shadows)
__global__ __launch_bounds__(256) void k_embed_fwd(const long long* __restrict__ ids, const long long* __restrict__ tt,
                                                   const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                   const bf16_t* __restrict__ type, bf16_t* __restrict__ out,
                                                   long long T, int L, int N) {
  const int lane = threadIdx.x & 63;
  const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const long long w = ids[t];
  const int p = (int)(t % L);
  const long long ty = tt ? tt[t] : 0;
  for (int c = lane * 4; c < N; c += 256) {
    float a[4], b[4], e[4];
    ld4(word + w * N + c, a);
    ld4(pos + (long long)p * N + c, b);
    ld4(type + ty * N + c, e);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += b[k] + e[k];
    st4(out + t * N + c, a);
  }
}

// word table: scatter-add (ids rarely repeat within a batch -> low contention atomics)
__global__ __launch_bounds__(256) void k_embed_bwd_word(const long long* __restrict__ ids,
                                                        const bf16_t* __restrict__ dsum, float* __restrict__ dword,
                                                        long long T, int N) {
  const int lane = threadIdx.x & 63;
  const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const long long w = ids[t];
  for (int c = lane * 4; c < N; c += 256) {
    float d[4];
    ld4(dsum + t * N + c, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(dword + w * N + c + k, d[k]);
  }
}

// position table: one block owns position p and sums its B tokens (no atomics)
__global__ __launch_bounds__(256) void k_embed_bwd_pos(const bf16_t* __restrict__ dsum, float* __restrict__ dpos,
                                                       long long T, int L, int N) {
  const int p = blockIdx.x;
  const long long B = T / L;
  for (int c = threadIdx.x; c < N; c += 256) {
    float acc = 0.f;
    for (long long b = 0; b < B; ++b) acc += bf2f(dsum[(b * L + p) * N + c]);
    dpos[(long long)p * N + c] += acc;
  }
}

// token-type table (few rows): per-block register sums over a token range, one atomic per block/column
__global__ __launch_bounds__(256) void k_embed_bwd_type(const long long* __restrict__ tt,
                                                        const bf16_t* __restrict__ dsum, float* __restrict__ dtype,
                                                        long long T, int N, int ntypes, int tokens_per_block) {
  const long long t0 = (long long)blockIdx.x * tokens_per_block;
  const long long t1 = min(T, t0 + tokens_per_block);
  for (int c = threadIdx.x; c < N; c += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (long long t = t0; t < t1; ++t) {
      const int ty = tt ? (int)tt[t] : 0;
      const float v = bf2f(dsum[t * N + c]);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += (ty == k) ? v : 0.f;
    }
    for (int k = 0; k < ntypes && k < 4; ++k)
      if (acc[k] != 0.f) atomicAdd(dtype + (long long)k * N + c, acc[k]);
  }
}

// All three tables in ONE pass over dsum: one block per position p walks its B tokens
// (t = b L + p) in batch order.  Word rows: one fp32 atomic per (token, column), consecutive lanes
// on consecutive columns (256 contiguous bytes per wave instruction: the full atomic rate; the
// per-token kernel above strided its lanes 16 bytes apart).  Position row: summed in registers in
// the same order as k_embed_bwd_pos and added once (no atomics).  Token-type rows (<= 2 types):
// per-block register sums, one atomic per block and column.
__global__ __launch_bounds__(256) void k_embed_bwd_fused(const long long* __restrict__ ids,
                                                         const long long* __restrict__ tt,
                                                         const bf16_t* __restrict__ dsum, float* __restrict__ dword,
                                                         float* __restrict__ dpos, float* __restrict__ dtype,
                                                         long long T, int L, int N) {
  const int p = blockIdx.x;
  const long long B = T / L;
  for (int c = threadIdx.x; c < N; c += 256) {
    float ps = 0.f, ty0 = 0.f, ty1 = 0.f;
    long long b = 0;
    for (; b + 4 <= B; b += 4) {     // four tokens' loads in flight before their atomics
      float v[4];
      long long w[4];
      int ty[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long t = (b + u) * L + p;
        v[u] = bf2f(dsum[t * N + c]);
        w[u] = ids[t];
        ty[u] = tt ? (int)tt[t] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        atomicAdd(dword + w[u] * N + c, v[u]);
        ps += v[u];
        ty0 += ty[u] == 0 ? v[u] : 0.f;
        ty1 += ty[u] == 1 ? v[u] : 0.f;
      }
    }
    for (; b < B; ++b) {
      const long long t = b * L + p;
      const float v = bf2f(dsum[t * N + c]);
      atomicAdd(dword + ids[t] * N + c, v);
      ps += v;
      const int ty = tt ? (int)tt[t] : 0;
      ty0 += ty == 0 ? v : 0.f;
      ty1 += ty == 1 ? v : 0.f;
    }
    dpos[(long long)p * N + c] += ps;
    if (ty0 != 0.f) atomicAdd(dtype + c, ty0);
    if (ty1 != 0.f) atomicAdd(dtype + N + c, ty1);
  }
}

// ------------------------------------------------------------------------------ row gather / scatter
__global__ void k_gather_rows(const bf16_t* __restrict__ src, const long long* __restrict__ idx,
                              bf16_t* __restrict__ dst, long long R, int N) {
  const long long n8 = R * (N / 8);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / (N / 8);
    const int c = (int)(i - r * (N / 8)) * 8;
    *reinterpret_cast<uint4*>(dst + r * N + c) = *reinterpret_cast<const uint4*>(src + idx[r] * N + c);
  }
}

// dst rows idx[r] (+)= src rows r  (indices unique within a call)
__global__ void k_scatter_rows(const bf16_t* __restrict__ src, const long long* __restrict__ idx,
                               bf16_t* __restrict__ dst, long long R, int N, int accumulate) {
  const long long n4 = R * (N / 4);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / (N / 4);
    const int c = (int)(i - r * (N / 4)) * 4;
    float a[4];
    ld4(src + r * N + c, a);
    if (accumulate) {
      float b[4];
      ld4(dst + idx[r] * N + c, b);
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += b[k];
    }
    st4(dst + idx[r] * N + c, a);
  }
}

int ln_bwd_blocks(long long M, int* rpb) {
  long long r = 16;
  long long g = (M + r - 1) / r;
  if (g > 512) { r = (M + 511) / 512; g = (M + r - 1) / r; }
  *rpb = (int)r;
  return (int)g;
}

}  // namespace

// dctr (optional): dropout (ctr = [seed, step], salt, p; k_dropout's mask) applied to x as it
// is loaded — LN(dropout(x) + res) in one pass; sum_out then holds dropout(x) + res
KML_API int kml_ln_fwd(const bf16_t* x, const bf16_t* res, const float* gamma, const float* beta, bf16_t* y,
                       bf16_t* sum_out, float* mean, float* rstd, long long M, int N, float eps, const float* dctr,
                       unsigned dsalt, float dp, hipStream_t s) {
  if (N % 4 || N > 64 * 4 * MAXV) return (int)hipErrorInvalidValue;
  if (dctr && (dp < 0.f || dp >= 1.f)) return (int)hipErrorInvalidValue;
  const int nv = (N + 255) / 256;
#define KML_LNF(NVv)                                                                                           \
  if (nv == NVv)                                                                                               \
    hipLaunchKernelGGL(k_ln_fwd<NVv>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, x, res, gamma, beta, y, \
                       sum_out, mean, rstd, M, N, eps, dctr, dsalt, dp);
  KML_LNF(1) KML_LNF(2) KML_LNF(3) KML_LNF(4) KML_LNF(5) KML_LNF(6) KML_LNF(7) KML_LNF(8)
#undef KML_LNF
  KML_LAUNCH_CHECK();
}

// workspace floats of kml_ln_bwd: [g][2N] gamma/beta partials (+ [g][N] with dbias_in)
KML_API long long kml_ln_bwd_ws_floats(long long M, int N) {
  int rpb;
  return (long long)ln_bwd_blocks(M, &rpb) * 3 * N;
}

// dx_drop (optional, with dctr/dsalt/dp of the fused forward dropout): also the gradient of
// the pre-dropout input, dropout(dx) — one pass instead of LN backward + dropout backward
KML_API int kml_ln_bwd(const bf16_t* dy, const bf16_t* xin, const float* mean, const float* rstd, const float* gamma,
                       bf16_t* dx, const bf16_t* dx_add, float* dgamma, float* dbeta, float* ws, unsigned* counter,
                       long long M, int N, bf16_t* dx_drop, const float* dctr, unsigned dsalt, float dp,
                       float* dbias_in, hipStream_t s) {
  if (N % 4 || N > 2048) return (int)hipErrorInvalidValue;
  if (dx_drop && (!dctr || dp < 0.f || dp >= 1.f)) return (int)hipErrorInvalidValue;
  int rpb;
  const int g = ln_bwd_blocks(M, &rpb);
  (void)counter;
  // dbias_in (optional): += column sums of the input gradient (dx_drop, else dx) — the bias
  // gradient of the Linear feeding this LayerNorm; partials in ws after the [g][2N] block
  const int with_in = dbias_in ? 1 : 0;
  const int nv = (N + 255) / 256;
#define KML_LNB(NVv)                                                                                              \
  if (nv == NVv)                                                                                                  \
    hipLaunchKernelGGL(k_ln_bwd<NVv>, dim3(g), dim3(256), 0, s, dy, xin, mean, rstd, gamma, dx, dx_add, ws, M, N, \
                       rpb, dx_drop, dctr, dsalt, dp, with_in);
  KML_LNB(1) KML_LNB(2) KML_LNB(3) KML_LNB(4) KML_LNB(5) KML_LNB(6) KML_LNB(7) KML_LNB(8)
#undef KML_LNB
  const int W = (2 + with_in) * N;
  hipLaunchKernelGGL(k_colreduce, dim3((W + 63) / 64), dim3(256), 0, s, ws, g, W, N, dgamma, dbeta, N, dbias_in);
  KML_LAUNCH_CHECK();
}

KML_API int kml_gelu_fwd(const bf16_t* x, bf16_t* y, long long n, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  if (n % 8 == 0 && (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 == 0)
    hipLaunchKernelGGL(k_gelu_fwd8, dim3(kml_stream_grid(n / 16, 256)), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(x), reinterpret_cast<uint4*>(y), n / 8);
  else
    hipLaunchKernelGGL(k_gelu_fwd, dim3(kml_stream_grid(n / 4, 256)), dim3(256), 0, s, x, y, n / 4);
  KML_LAUNCH_CHECK();
}

KML_API int kml_gelu_bwd(const bf16_t* dy, const bf16_t* x, bf16_t* dx, long long n, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gelu_bwd, dim3(kml_stream_grid(n / 4, 256)), dim3(256), 0, s, dy, x, dx, n / 4);
  KML_LAUNCH_CHECK();
}

// rows per block / row blocks of kml_gelu_bwd_colsum (its workspace is G x N floats)
static int gelu_cs_blocks(long long M, int* rpb) {
  long long r = 64;
  long long g = (M + r - 1) / r;
  if (g > 1024) { r = (M + 1023) / 1024; g = (M + r - 1) / r; }
  *rpb = (int)r;
  return (int)g;
}

KML_API long long kml_gelu_bwd_colsum_ws_floats(long long M, int N) {
  int rpb;
  return (long long)gelu_cs_blocks(M, &rpb) * N;
}

// dx = dy * gelu'(x) over [M][N] and dbias[c] += sum_r dx[r][c] (deterministic row-block order)
KML_API int kml_gelu_bwd_colsum(const bf16_t* dy, const bf16_t* x, bf16_t* dx, float* dbias, float* ws, long long M,
                                int N, hipStream_t s) {
  if (N % 4 || M <= 0) return (int)hipErrorInvalidValue;
  int rpb;
  const int g = gelu_cs_blocks(M, &rpb);
  hipLaunchKernelGGL(k_gelu_bwd_colsum, dim3((unsigned)((N / 4 + 255) / 256), (unsigned)g), dim3(256), 0, s, dy, x,
                     dx, ws, M, N, rpb);
  hipLaunchKernelGGL(k_colreduce, dim3((N + 63) / 64), dim3(256), 0, s, ws, g, N, N, dbias, (float*)nullptr, 0,
                     (float*)nullptr);
  KML_LAUNCH_CHECK();
}

// out[c] += sum_g part[g][c] for part [G][N] fp32 (fixed row order; k_colreduce: 64 columns x
// 4 row slices per block) — e.g. the per-M-tile column sums of a GEMM epilogue
KML_API int kml_colreduce_add(const float* part, int G, int N, float* out, hipStream_t s) {
  if (G < 1 || N < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_colreduce, dim3((N + 63) / 64), dim3(256), 0, s, part, G, N, N, out, (float*)nullptr, 0,
                     (float*)nullptr);
  KML_LAUNCH_CHECK();
}

KML_API int kml_dropout(const bf16_t* x, bf16_t* y, const float* ctr, unsigned salt, float p, long long n,
                        hipStream_t s) {
  if (n % 8 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_dropout, dim3(kml_stream_grid(n / 8, 256)), dim3(256), 0, s, x, y, ctr, salt, p, n / 8);
  KML_LAUNCH_CHECK();
}

KML_API int kml_embed_fwd(const long long* ids, const long long* tt, const bf16_t* word, const bf16_t* pos,
                          const bf16_t* type, bf16_t* out, long long T, int L, int N, hipStream_t s) {
  if (N % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_embed_fwd, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, ids, tt, word, pos, type, out, T,
                     L, N);
  KML_LAUNCH_CHECK();
}

KML_API int kml_embed_bwd(const long long* ids, const long long* tt, const bf16_t* dsum, float* dword, float* dpos,
                          float* dtype, long long T, int L, int N, hipStream_t s) {
  if (N % 4 || T % L) return (int)hipErrorInvalidValue;
  if (dword && dpos && dtype) {   // the training step's case: one pass (k_embed_bwd_fused)
    hipLaunchKernelGGL(k_embed_bwd_fused, dim3((unsigned)L), dim3(256), 0, s, ids, tt, dsum, dword, dpos, dtype, T,
                       L, N);
    KML_LAUNCH_CHECK();
  }
  if (dword)
    hipLaunchKernelGGL(k_embed_bwd_word, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, ids, dsum, dword, T, N);
  if (dpos) hipLaunchKernelGGL(k_embed_bwd_pos, dim3(L), dim3(256), 0, s, dsum, dpos, T, L, N);
  if (dtype) {
    const int tpb = 64;
    hipLaunchKernelGGL(k_embed_bwd_type, dim3((unsigned)((T + tpb - 1) / tpb)), dim3(256), 0, s, tt, dsum, dtype, T,
                       N, 2, tpb);
  }
  KML_LAUNCH_CHECK();
}

KML_API int kml_gather_rows(const bf16_t* src, const long long* idx, bf16_t* dst, long long R, int N, hipStream_t s) {
  if (N % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gather_rows, dim3(kml_stream_grid(R * (N / 8), 256)), dim3(256), 0, s, src, idx, dst, R, N);
  KML_LAUNCH_CHECK();
}

KML_API int kml_scatter_rows(const bf16_t* src, const long long* idx, bf16_t* dst, long long R, int N, int accumulate,
                             hipStream_t s) {
  if (N % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_scatter_rows, dim3(kml_stream_grid(R * (N / 4), 256)), dim3(256), 0, s, src, idx, dst, R, N,
                     accumulate);
  KML_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// BERT masked-LM batch preparation on the device (Google BERT's recipe): per sequence, P of
// the L positions are chosen uniformly without replacement (the P largest keys of a hash of
// (seed, step, token), ties broken by position), listed in increasing order; each chosen token
// becomes [MASK] with probability 0.8, a uniformly random token with 0.1, and stays with 0.1.
// One block per sequence: keys in LDS, rank = count of larger keys (O(L^2 / threads)), slot =
// count of chosen positions before it.  ctr = [seed, step] (fp32, the RNGState layout); with a
// ticket the last block to finish advances ctr[1] (every block read it first), so a captured
// step draws a fresh mask at every replay.  Replaces the eager topk / sort / rand / where /
// scatter chain of the reference-style function (examples/function_bert.py).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mlm_mask(const long long* __restrict__ ids, long long* __restrict__ xout,
                                                  long long* __restrict__ pos, long long* __restrict__ lab,
                                                  float* __restrict__ ctr, unsigned* __restrict__ ticket, int L, int P,
                                                  long long mask_id, long long vocab) {
  __shared__ unsigned key[2048];
  __shared__ unsigned char sel[2048];
  const int b = blockIdx.x, tid = threadIdx.x;
  const unsigned seed = (unsigned)ctr[0], step = (unsigned)ctr[1];
  const long long* row = ids + (long long)b * L;
  for (int l = tid; l < L; l += 256) key[l] = hash3(seed ^ 0x6D61736Bu, step, (unsigned)(b * L + l));
  __syncthreads();
  for (int l = tid; l < L; l += 256) {
    const unsigned k = key[l];
    int rank = 0;
    for (int j = 0; j < L; ++j) {
      const unsigned kj = key[j];
      rank += (kj > k) || (kj == k && j < l);
    }
    sel[l] = rank < P ? 1 : 0;
  }
  __syncthreads();
  for (int l = tid; l < L; l += 256) {
    const long long t = row[l];
    long long o = t;
    if (sel[l]) {
      int slot = 0;
      for (int j = 0; j < l; ++j) slot += sel[j];
      const unsigned r = hash3(seed ^ 0x72706C63u, step, (unsigned)(b * P + slot));
      const float u = (float)(r >> 8) * (1.0f / 16777216.0f);
      if (u < 0.8f) o = mask_id;
      else if (u < 0.9f) o = (long long)(hash3(seed ^ 0x746F6B6Eu, step, (unsigned)(b * P + slot)) % (unsigned)vocab);
      pos[(long long)b * P + slot] = l;
      lab[(long long)b * P + slot] = t;
    }
    xout[(long long)b * L + l] = o;
  }
  if (ticket) {
    __syncthreads();
    if (tid == 0) {
      __threadfence();
      const unsigned t = atomicAdd(ticket, 1u);
      if (t == gridDim.x - 1) {
        ctr[1] = (float)(step + 1u);
        atomicExch(ticket, 0u);
      }
    }
  }
}

// ids / xout [B][L], pos / lab [B][P] int64; L <= 2048, 1 <= P <= L.  ticket: null = the step
// counter is not advanced (a fixed evaluation mask)
KML_API int kml_mlm_mask(const long long* ids, long long* xout, long long* pos, long long* lab, float* ctr,
                         unsigned* ticket, int B, int L, int P, long long mask_id, long long vocab, hipStream_t s) {
  if (B < 1 || L < 1 || L > 2048 || P < 1 || P > L || vocab < 1 || !ids || !xout || !pos || !lab || !ctr)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_mlm_mask, dim3(B), dim3(256), 0, s, ids, xout, pos, lab, ctr, ticket, L, P, mask_id, vocab);
  KML_LAUNCH_CHECK();
}
