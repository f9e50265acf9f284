// util.hip — small utility kernels: version probe, fill, scale, cast, axpby.
#include "kml_common.h"
#include "kml_sgd.h"

KML_API int kml_abi_version() { return 1; }

__global__ void k_fill_f32(float* __restrict__ p, float v, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}

KML_API int kml_fill_f32(float* p, float v, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_f32, dim3(kml_stream_grid(n, 256)), dim3(256), 0, s, p, v, n);
  KML_LAUNCH_CHECK();
}

// x *= a  (fp32, vectorised by 4 when aligned)
__global__ void k_scale_f32(float* __restrict__ p, float a, long long n) {
  long long n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = p4[i];
    v.x *= a; v.y *= a; v.z *= a; v.w *= a;
    p4[i] = v;
  }
  for (long long i = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] *= a;
}

KML_API int kml_scale_f32(float* p, float a, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_scale_f32, dim3(kml_stream_grid((n + 3) / 4, 256)), dim3(256), 0, s, p, a, n);
  KML_LAUNCH_CHECK();
}

__global__ void k_f32_to_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = f2bf(x[i]);
}
__global__ void k_bf16_to_f32(const bf16_t* __restrict__ x, float* __restrict__ y, long long n) {
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = bf2f(x[i]);
}

KML_API int kml_f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(kml_stream_grid(n, 256)), dim3(256), 0, s, x, y, n);
  KML_LAUNCH_CHECK();
}
KML_API int kml_bf16_to_f32(const bf16_t* x, float* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_bf16_to_f32, dim3(kml_stream_grid(n, 256)), dim3(256), 0, s, x, y, n);
  KML_LAUNCH_CHECK();
}

// y = a*x + b*y over bf16 NHWC tensors (used for residual-gradient sums), vectorised x8
__global__ void k_add_bf16(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                           bf16_t* __restrict__ y, long long n8) {
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    uint4 va = reinterpret_cast<const uint4*>(a)[i];
    uint4 vb = reinterpret_cast<const uint4*>(b)[i];
    uint4 o;
    o.x = pack_bf2(lo_bf(va.x) + lo_bf(vb.x), hi_bf(va.x) + hi_bf(vb.x));
    o.y = pack_bf2(lo_bf(va.y) + lo_bf(vb.y), hi_bf(va.y) + hi_bf(vb.y));
    o.z = pack_bf2(lo_bf(va.z) + lo_bf(vb.z), hi_bf(va.z) + hi_bf(vb.z));
    o.w = pack_bf2(lo_bf(va.w) + lo_bf(vb.w), hi_bf(va.w) + hi_bf(vb.w));
    reinterpret_cast<uint4*>(y)[i] = o;
  }
}

KML_API int kml_add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long long n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  long long n8 = n / 8;
  hipLaunchKernelGGL(k_add_bf16, dim3(kml_stream_grid(n8, 256)), dim3(256), 0, s, a, b, y, n8);
  KML_LAUNCH_CHECK();
}

// out[c] += sum_m x[m][c]   (bf16 [M][C] -> fp32, any C; used for Linear / conv bias grads)
__global__ __launch_bounds__(256) void k_colsum_bf16(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                     long long M, int C, int rows_per_block) {
  const long long r0 = (long long)blockIdx.y * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float s = 0.f;
    for (long long r = r0; r < r1; ++r) s += bf2f(x[r * C + c]);
    atomicAdd(out + c, s);
  }
}

// Vectorised form for C % 8 == 0: 64 lanes x 8 columns (one 16-byte load each) per row,
// the block's 4 waves on interleaved rows of its row slab, 8 independent loads in flight per
// lane, waves combined in LDS, one atomic per column per block.  The scalar kernel above
// issued one 2-byte load per lane per row (33 us avg per BERT bias gradient).
__global__ __launch_bounds__(256) void k_colsum8_bf16(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                      long long M, int C, int rows_per_block) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * 8;
  const long long r0 = (long long)blockIdx.y * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    constexpr int U = 8;
    for (long long r = r0 + w; r < r1; r += 4 * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long rr = min(r + 4LL * u, r1 - 1);  // clamped re-read, selected out below
        v[u] = *reinterpret_cast<const uint4*>(x + rr * C + c0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + 4LL * u >= r1) break;
        const unsigned* q = reinterpret_cast<const unsigned*>(&v[u]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += __uint_as_float(q[k] << 16);
          acc[2 * k + 1] += __uint_as_float(q[k] & 0xffff0000u);
        }
      }
    }
  }
  __shared__ float red[4][64 * 8];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = acc[k];
  __syncthreads();
  // atomics on consecutive columns per lane (4 cache lines per wave instruction, not 32)
  const int cb = blockIdx.x * 512;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = h * 256 + threadIdx.x;
    if (cb + j < C) atomicAdd(out + cb + j, red[0][j] + red[1][j] + red[2][j] + red[3][j]);
  }
}

// dst[i] += sum_s part[s][i]  (fp32, n % 4 == 0): the split-K slabs of a weight-gradient GEMM
// folded into the gradient storage in one pass, slabs summed in order (deterministic).
__global__ __launch_bounds__(256) void k_slab_sum_add(const float4* __restrict__ part, float4* __restrict__ dst,
                                                      long long n4, int S) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 a = dst[i];
    for (int k = 0; k < S; ++k) {
      const float4 v = part[(long long)k * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    dst[i] = a;
  }
}

KML_API int kml_slab_sum_add(const float* part, float* dst, long long n, int S, hipStream_t s) {
  if (n % 4 || S < 1) return (int)hipErrorInvalidValue;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_slab_sum_add, dim3(kml_stream_grid(n4, 256)), dim3(256), 0, s, (const float4*)part,
                     (float4*)dst, n4, S);
  KML_LAUNCH_CHECK();
}

KML_API int kml_colsum_bf16(const bf16_t* x, float* out, long long M, int C, hipStream_t s) {
  if (C % 8 == 0 && M >= 256 && ((uintptr_t)x & 15) == 0) {
    const int rpb = 128;
    const long long gy = (M + rpb - 1) / rpb;
    if (gy <= 65535) {
      dim3 grid((C / 8 + 63) / 64, (unsigned)gy);
      hipLaunchKernelGGL(k_colsum8_bf16, grid, dim3(256), 0, s, x, out, M, C, rpb);
      KML_LAUNCH_CHECK();
    }
  }
  int rpb = 64;
  long long gy = (M + rpb - 1) / rpb;
  if (gy > 65535) { rpb = (int)((M + 65534) / 65535); gy = (M + rpb - 1) / rpb; }
  dim3 grid((C + 255) / 256, (unsigned)gy);
  hipLaunchKernelGGL(k_colsum_bf16, grid, dim3(256), 0, s, x, out, M, C, rpb);
  KML_LAUNCH_CHECK();
}

__global__ void k_add_i64(long long* __restrict__ p, long long v, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += v;
}

// flat row index of (batch b, position pos[b][j]) in a [B*L] token-major tensor: out = b*L + pos
__global__ void k_row_index(const long long* __restrict__ pos, long long* __restrict__ out, int P, long long L,
                            int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (long long)(i / P) * L + pos[i];
}

KML_API int kml_row_index(const long long* pos, long long* out, int B, int P, long long L, hipStream_t s) {
  const int n = B * P;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_row_index, dim3((n + 255) / 256), dim3(256), 0, s, pos, out, P, L, n);
  KML_LAUNCH_CHECK();
}

KML_API int kml_add_i64(long long* p, long long v, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_add_i64, dim3((n + 255) / 256), dim3(256), 0, s, p, v, n);
  KML_LAUNCH_CHECK();
}

// zero-pad the channel dim: x [P][C] -> y [P][CP] (bf16), CP >= C
__global__ void k_pad_channels(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long P, int C, int CP) {
  long long total = P * CP;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p = i / CP;
    int c = (int)(i - p * CP);
    y[i] = c < C ? x[p * C + c] : (bf16_t)0;
  }
}

KML_API int kml_pad_channels(const bf16_t* x, bf16_t* y, long long P, int C, int CP, hipStream_t s) {
  hipLaunchKernelGGL(k_pad_channels, dim3(kml_stream_grid(P * CP, 256)), dim3(256), 0, s, x, y, P, C, CP);
  KML_LAUNCH_CHECK();
}

// NCHW fp32 -> NHWC bf16 with channel padding (input adapter for user tensors)
__global__ void k_nchw_to_nhwc_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, int B, int C, int HW,
                                    int CP) {
  long long total = (long long)B * HW * CP;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % CP);
    long long t = i / CP;
    int p = (int)(t % HW);
    int b = (int)(t / HW);
    y[i] = c < C ? f2bf(x[((long long)b * C + c) * HW + p]) : (bf16_t)0;
  }
}

KML_API int kml_nchw_to_nhwc_bf16(const float* x, bf16_t* y, int B, int C, int HW, int CP, hipStream_t s) {
  long long total = (long long)B * HW * CP;
  hipLaunchKernelGGL(k_nchw_to_nhwc_bf16, dim3(kml_stream_grid(total, 256)), dim3(256), 0, s, x, y, B, C, HW, CP);
  KML_LAUNCH_CHECK();
}

// Zero a byte range with a kernel.  Used instead of hipMemsetAsync everywhere on the
// training path: a memset captured into a hipGraph (memset node) was observed on this
// ROCm build to race with the following kernel nodes (graph-replay corruption,
// tools/graph_stress.py), whereas a kernel node is ordered like every other kernel.
__global__ void k_zero_bytes(unsigned char* __restrict__ p, long long bytes, int aligned) {
  const long long n16 = aligned ? (bytes >> 4) : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  uint4 z = {0, 0, 0, 0};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<uint4*>(p)[i] = z;
  for (long long i = (n16 << 4) + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < bytes; i += stride)
    p[i] = 0;
}

KML_API int kml_zero(void* p, long long bytes, hipStream_t s) {
  // unaligned base (rare; framework buffers are 256-B aligned): byte loop only
  const int aligned = (((unsigned long long)p) & 15ull) == 0;
  const long long work = aligned ? (bytes + 15) / 16 : bytes;
  hipLaunchKernelGGL(k_zero_bytes, dim3(kml_stream_grid(work, 256)), dim3(256), 0, s, (unsigned char*)p, bytes,
                     aligned);
  KML_LAUNCH_CHECK();
}

// Zero up to ZR_MAX fp32 ranges of one buffer in ONE launch (the flat gradient buffer's
// accumulate-only parameters, nn/flat.py FlatParamSpace.zero_grad): ranges passed by value,
// so nothing is copied to the device and the launch captures into a graph as one node.
namespace {
constexpr int ZR_MAX = 96;
struct ZeroRanges {
  long long off[ZR_MAX];  // element offsets (multiples of 4: 16-byte aligned)
  int n[ZR_MAX];          // element counts
  int count;
};
__global__ __launch_bounds__(256) void k_zero_ranges(float* __restrict__ base, ZeroRanges zr) {
  // one block-row per range, grid-stride inside it
  for (int r = blockIdx.y; r < zr.count; r += gridDim.y) {
    float* p = base + zr.off[r];
    const int n = zr.n[r];
    const int n4 = n >> 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
      reinterpret_cast<float4*>(p)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = (n4 << 2) + blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0.f;
  }
}
}  // namespace

KML_API int kml_zero_ranges_max() { return ZR_MAX; }

// offs / ns: host arrays of `count` ranges (count <= kml_zero_ranges_max())
KML_API int kml_zero_ranges(float* base, const long long* offs, const int* ns, int count, hipStream_t s) {
  if (count < 0 || count > ZR_MAX || (((unsigned long long)base) & 15ull)) return (int)hipErrorInvalidValue;
  if (count == 0) return (int)hipSuccess;
  ZeroRanges zr = {};
  int widest = 1;
  for (int i = 0; i < count; ++i) {
    if (offs[i] % 4 || ns[i] < 0) return (int)hipErrorInvalidValue;
    zr.off[i] = offs[i];
    zr.n[i] = ns[i];
    if (ns[i] > widest) widest = ns[i];
  }
  zr.count = count;
  int gx = (widest / 4 + 255) / 256;
  if (gx > 64) gx = 64;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(k_zero_ranges, dim3(gx, count), dim3(256), 0, s, base, zr);
  KML_LAUNCH_CHECK();
}


// ---- optimizer-update riders (kml_sgd.h) ------------------------------------------------------
KmlSgdRider g_kml_rider = {};

namespace {
__global__ __launch_bounds__(256) void k_sgd_rider_alone(KmlSgdRider r) { kml_sgd_rider_run(r, blockIdx.x); }
}  // namespace

// Arm an SGD range rider for the NEXT rider-capable launch of this process (kml_conv_bwd_pair,
// kml_conv_bwd_pair_bnb, kml_bn_bwd / kml_bn_bwd_apply_partial): `blocks` extra 256-thread blocks
// apply the fused SGD to n flat elements (w / g / mom / shadow offset to the range; lr and the
// first-step flag read on the device).  blocks = 0 disarms.
KML_API int kml_rider_set(float* w, const float* g, float* mom, bf16_t* shadow, const float* lr_ptr,
                          const float* first_ptr, float wd, float momentum, float dampening, int nesterov,
                          float grad_scale, long long n, int blocks) {
  if (blocks < 0 || (blocks > 0 && (!w || !g || !lr_ptr || n <= 0 || (((uintptr_t)w | (uintptr_t)g) & 15) ||
                                    (mom && ((uintptr_t)mom & 15)) || (shadow && ((uintptr_t)shadow & 7)))))
    return (int)hipErrorInvalidValue;
  g_kml_rider = KmlSgdRider{w, g, mom, shadow, lr_ptr, first_ptr, wd, momentum, dampening, grad_scale, nesterov,
                            blocks, n};
  return (int)hipSuccess;
}

// Arm a peer-shard slice (kml_sgd.h KmlZsRider; parallel/peer.py ShardRider) for the next
// rider-capable launch: kind 1 = reduce-scatter + fused SGD of this rank's chunk vectors [v0, v1)
// (w / mom / shadow at the segment, flags / data = every rank's flags area and fp32 gradient at the
// segment), kind 2 = all-gather of the peers' bf16 shadow chunks (data = every rank's shadow at the
// segment, shadow = the own).  Offsets / counts as in KmlZsRider; timeout_s bounds every wait.
KML_API int kml_zs_rider_set(int kind, const void* const* flags, const void* const* data, void* own_flags, void* ctrl,
                             int rank, int world, long long a, long long b, long long v0, long long v1, int ready,
                             int wait, int done, int done_blocks, int done_word, int advance, double timeout_s,
                             float* w, float* mom, bf16_t* shadow, const float* lr_ptr, const float* first_ptr,
                             float wd, float momentum, float dampening, int nesterov, float grad_scale, int blocks) {
  if ((kind != KML_RIDER_ZS_RS && kind != KML_RIDER_ZS_AG) || world < 1 || world > KML_ZS_MAX || rank < 0 ||
      rank >= world || blocks <= 0 || !flags || !data || !own_flags || !ctrl || !shadow || v1 < v0 ||
      done_word < 5 || done_word > 15 || (kind == KML_RIDER_ZS_RS && (!w || !lr_ptr)))
    return (int)hipErrorInvalidValue;
  KmlSgdRider r = {};
  r.w = w;
  r.mom = mom;
  r.shadow = shadow;
  r.lr_ptr = lr_ptr;
  r.first_ptr = first_ptr;
  r.wd = wd;
  r.momentum = momentum;
  r.dampening = dampening;
  r.grad_scale = grad_scale;
  r.nesterov = nesterov;
  r.blocks = blocks;
  r.n = 0;
  r.kind = kind;
  for (int p = 0; p < world; ++p) {
    r.zs.flags[p] = static_cast<const char*>(flags[p]);
    r.zs.data[p] = static_cast<const char*>(data[p]);
  }
  r.zs.own_flags = static_cast<unsigned*>(own_flags);
  r.zs.ctrl = static_cast<unsigned*>(ctrl);
  r.zs.rank = rank;
  r.zs.world = world;
  r.zs.a = a;
  r.zs.b = b;
  r.zs.v0 = v0;
  r.zs.v1 = v1;
  r.zs.ready = ready;
  r.zs.wait = wait;
  r.zs.done = done;
  r.zs.done_blocks = done_blocks;
  r.zs.done_word = done_word;
  r.zs.advance = advance;
  r.zs.limit = (unsigned long long)(timeout_s * 1e8);   // s_memrealtime runs at 100 MHz
  g_kml_rider = r;
  return (int)hipSuccess;
}

// run an armed rider as its own launch (a rider-capable call that took another path)
KML_API int kml_rider_flush(hipStream_t s) {
  const KmlSgdRider r = kml_rider_take();
  if (r.blocks <= 0) return (int)hipSuccess;
  hipLaunchKernelGGL(k_sgd_rider_alone, dim3(r.blocks), dim3(256), 0, s, r);
  KML_LAUNCH_CHECK();
}
