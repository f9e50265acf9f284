// conv_igemm.hip — MFMA implicit-GEMM convolution for NHWC bf16 on gfx950.
//
// One kernel family covers the three convolution GEMMs of training (and Linear
// layers, which are 1x1 convolutions over a 1x1 image):
//
//   FWD   : Y[m=(b,oh,ow)][n=cout]    = sum_k  im2col(X)[m][k=(tap,cin)] * W[n][k]
//   DGRAD : dX[m=(b,ih,iw)][n=cin]    = sum_k  dY[(b,oh,ow)][cout] * W[cout][tap][cin]   k=(tap,cout)
//   WGRAD : dW[m=cout][n=(tap,cin)]  += sum_k  dY[k=pixel][cout]  * im2col(X)[k][n]      (split-K, fp32 atomics)
//
// Layouts: activations NHWC bf16 (C % 8 == 0), weights KRSC bf16 ([Cout][KH][KW][Cin]),
// weight gradients KRSC fp32 (written straight into the flat fp32 gradient buffer the
// all-reduce and the fused optimizer consume).
//
// Tiling (CDNA4): 256 threads = 4 wave64 in a 2x2 grid, each wave owns a
// (BM/2)x(BN/2) sub-tile built from v_mfma_f32_16x16x32_bf16 fragments; BK = 32.
// Operands are staged global->registers->LDS (16 B per lane) with a two-buffer LDS
// ring and one barrier per K-step.  An operand whose K axis is contiguous in memory
// lives in LDS as [row][k] and is read with ds_read_b128; an operand whose K axis is
// strided (dgrad weights, both wgrad operands) lives as [k][row] in its natural memory
// order and is read with the gfx950 transposing read ds_read_b64_tr_b16, so no
// transpose pass or transposed weight copy is ever materialised.
//
// Only the convolution taps that can touch the image for SOME output pixel
// ([r0,r1) x [s0,s1), computed on the host) are enumerated: on ResNet-34's layer4
// (1x1 spatial at 32x32 input) a 3x3 conv degenerates to its centre tap and the
// GEMM K shrinks 9x.
//
// Epilogue options (FWD): fp32 bias, ReLU, and per-channel BatchNorm statistics
// (sum, sum of squares) accumulated from the fp32 accumulators with wave
// reductions + one atomic per (wave, channel) — this removes BN's stats pass.
//
// Reference parity: the reference runs these convolutions through cuDNN inside the
// user's torch module (ml/experiments/kubeml/function_resnet34.py:72-76).
#include "kml_common.h"

namespace {

constexpr int BK = 32;
constexpr int PADK = 8;   // K-contiguous LDS rows: 40 bf16 = 80 B (conflict-free b128 reads)
constexpr int PADR = 8;   // K-strided LDS rows: R+8 bf16

enum { FWD = 0, DGRAD = 1, WGRAD = 2 };

struct ConvArgs {
  const bf16_t* x;    // input activations NHWC (FWD, WGRAD)
  const bf16_t* w;    // weights KRSC (FWD, DGRAD)
  const bf16_t* dy;   // output grads NHWC (DGRAD, WGRAD)
  bf16_t* out;        // Y (FWD) or dX (DGRAD)
  float* dw;          // fp32 weight grads KRSC (WGRAD)
  float* stats;       // [2][Cout] BN sum / sumsq (FWD, optional)
  const float* bias;  // [Cout] (FWD, optional)
  const bf16_t* addend; // [M][N] added to the DGRAD output (fused residual-gradient sum)
  int B, H, W, C;     // input geometry (C = Cin)
  int OH, OW, K;      // output geometry (K = Cout)
  int KH, KW, sh, sw, ph, pw;
  int r0, r1, s0, s1; // valid tap window
  int M, N, Kd;       // GEMM dims
  int Kp;             // DGRAD: Cout padded to a multiple of BK (K index = tap*Kp + cout)
  int kchunk;         // WGRAD split-K chunk (multiple of BK)
  int relu;           // FWD epilogue ReLU
  int accumulate;     // WGRAD: atomicAdd (1) or store (0)
};

template <int R, bool KCONTIG>
struct TileShape {
  static constexpr int ELEMS = KCONTIG ? R * (BK + PADK) : BK * (R + PADR);
  static constexpr int CHUNKS = R * BK / 8;  // 16-byte chunks per stage
  static constexpr int PER_THREAD = (CHUNKS + 255) / 256;
};

__device__ __forceinline__ uint4 ld16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// ---- operand loaders: return the 16-byte chunk q of K-tile kt (zeros when out of range) ----

// A of FWD: im2col(X), row = output pixel, K-contiguous (chunk = 8 input channels of one tap)
struct FwdA {
  int valid, b, ih0, iw0;
  __device__ void init(const ConvArgs& a, int m) {
    valid = m < a.M;
    int mm = valid ? m : 0;
    int ow = mm % a.OW; int t = mm / a.OW; int oh = t % a.OH; b = t / a.OH;
    ih0 = oh * a.sh - a.ph; iw0 = ow * a.sw - a.pw;
  }
  __device__ uint4 load(const ConvArgs& a, int k) const {
    uint4 z = {0, 0, 0, 0};
    if (!valid || k >= a.Kd) return z;
    int tap = k / a.C, c = k - tap * a.C;
    int nts = a.s1 - a.s0;
    int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
    int ih = ih0 + r, iw = iw0 + s;
    if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return z;
    return ld16(a.x + ((long long)(b * a.H + ih) * a.W + iw) * a.C + c);
  }
};

// B of FWD: W[n][tap][cin], K-contiguous
struct FwdB {
  int valid; long long base;
  __device__ void init(const ConvArgs& a, int n) {
    valid = n < a.N; base = (long long)(valid ? n : 0) * a.KH * a.KW * a.C;
  }
  __device__ uint4 load(const ConvArgs& a, int k) const {
    uint4 z = {0, 0, 0, 0};
    if (!valid || k >= a.Kd) return z;
    int tap = k / a.C, c = k - tap * a.C;
    int nts = a.s1 - a.s0;
    int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
    return ld16(a.w + base + (r * a.KW + s) * a.C + c);
  }
};

// A of DGRAD: dY gathered for input pixel m, K = (tap, cout), K-contiguous over cout
struct DgradA {
  int valid, b, ih, iw;
  __device__ void init(const ConvArgs& a, int m) {
    valid = m < a.M;
    int mm = valid ? m : 0;
    iw = mm % a.W; int t = mm / a.W; ih = t % a.H; b = t / a.H;
  }
  __device__ uint4 load(const ConvArgs& a, int k) const {
    uint4 z = {0, 0, 0, 0};
    if (!valid) return z;
    int tap = k / a.Kp, n = k - tap * a.Kp;
    if (n >= a.K) return z;
    int nts = a.s1 - a.s0;
    int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
    int th = ih + a.ph - r, tw = iw + a.pw - s;
    if (th < 0 || tw < 0) return z;
    int oh = th / a.sh, ow = tw / a.sw;
    if (oh * a.sh != th || ow * a.sw != tw || oh >= a.OH || ow >= a.OW) return z;
    return ld16(a.dy + ((long long)(b * a.OH + oh) * a.OW + ow) * a.K + n);
  }
};

// B of DGRAD (K-strided): LDS row = k = (tap, cout), columns = cin; chunk = W[cout][tap][c..c+7]
__device__ __forceinline__ uint4 dgrad_b_load(const ConvArgs& a, int k, int c) {
  uint4 z = {0, 0, 0, 0};
  if (c >= a.N) return z;
  int tap = k / a.Kp, n = k - tap * a.Kp;
  if (n >= a.K) return z;
  int nts = a.s1 - a.s0;
  int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
  return ld16(a.w + ((long long)(n * a.KH + r) * a.KW + s) * a.C + c);
}

// A of WGRAD (K-strided): LDS row = pixel k, columns = cout; chunk = dY[k][n..n+7]
__device__ __forceinline__ uint4 wgrad_a_load(const ConvArgs& a, int k, int kend, int n) {
  uint4 z = {0, 0, 0, 0};
  if (k >= kend || n >= a.M) return z;
  return ld16(a.dy + (long long)k * a.K + n);
}

// B of WGRAD (K-strided): LDS row = pixel k, columns j = (tap, cin); chunk = X[pix shifted][c..c+7]
__device__ __forceinline__ uint4 wgrad_b_load(const ConvArgs& a, int k, int kend, int j) {
  uint4 z = {0, 0, 0, 0};
  if (k >= kend || j >= a.N) return z;
  int tap = j / a.C, c = j - tap * a.C;
  int nts = a.s1 - a.s0;
  int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
  int ow = k % a.OW; int t = k / a.OW; int oh = t % a.OH; int b = t / a.OH;
  int ih = oh * a.sh - a.ph + r, iw = ow * a.sw - a.pw + s;
  if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return z;
  return ld16(a.x + ((long long)(b * a.H + ih) * a.W + iw) * a.C + c);
}

// ---- fragment readers ----
template <int R>
__device__ __forceinline__ bf16x8_t frag_kcontig(const bf16_t* lds, int row0, int lane) {
  const bf16_t* p = lds + (row0 + (lane & 15)) * (BK + PADK) + 8 * (lane >> 4);
  return *reinterpret_cast<const bf16x8_t*>(p);
}

typedef __attribute__((ext_vector_type(4))) short v4s_t;

template <int R>
__device__ __forceinline__ bf16x8_t frag_kstrided(const bf16_t* lds, int row0, int lane) {
  const int il = lane & 15, g = lane >> 4;
  const int col = row0 + 4 * (il & 3);
  const bf16_t* p0 = lds + (8 * g + (il >> 2)) * (R + PADR) + col;
  const bf16_t* p1 = p0 + 4 * (R + PADR);
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p0));
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p1));
  bf16x8_t f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256) void k_conv_igemm(ConvArgs a) {
  constexpr bool A_KC = (MODE != WGRAD);
  constexpr bool B_KC = (MODE == FWD);
  using TA = TileShape<BM, A_KC>;
  using TB = TileShape<BN, B_KC>;
  constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;

  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (TA::ELEMS + TB::ELEMS)];
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;
#define sA(buf) (smem + (buf) * STAGE)
#define sB(buf) (smem + (buf) * STAGE + TA::ELEMS)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  int kbeg = 0, kend = a.Kd;
  if (MODE == WGRAD) {
    kbeg = blockIdx.z * a.kchunk;
    kend = min(a.Kd, kbeg + a.kchunk);
  }
  const int nk = (kend - kbeg + BK - 1) / BK;

  // per-thread chunk bookkeeping (rows fixed across K-steps for K-contiguous operands)
  FwdA fa[TA::PER_THREAD];
  DgradA da[TA::PER_THREAD];
  FwdB fb[TB::PER_THREAD];
  if (MODE == FWD) {
#pragma unroll
    for (int i = 0; i < TA::PER_THREAD; ++i) fa[i].init(a, m0 + (tid + i * 256) / 4);
#pragma unroll
    for (int i = 0; i < TB::PER_THREAD; ++i) fb[i].init(a, n0 + (tid + i * 256) / 4);
  } else if (MODE == DGRAD) {
#pragma unroll
    for (int i = 0; i < TA::PER_THREAD; ++i) da[i].init(a, m0 + (tid + i * 256) / 4);
  }

  uint4 ra[TA::PER_THREAD], rb[TB::PER_THREAD];

  auto gload = [&](int kt) {
    const int kb = kbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < TA::PER_THREAD; ++i) {
      const int q = tid + i * 256;
      if (q < TA::CHUNKS) {
        if (MODE == FWD) ra[i] = fa[i].load(a, kb + (q & 3) * 8);
        else if (MODE == DGRAD) ra[i] = da[i].load(a, kb + (q & 3) * 8);
        else {
          constexpr int CPR = BM / 8;  // chunks per LDS row
          ra[i] = wgrad_a_load(a, kb + q / CPR, kend, m0 + (q % CPR) * 8);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TB::PER_THREAD; ++i) {
      const int q = tid + i * 256;
      if (q < TB::CHUNKS) {
        if (MODE == FWD) rb[i] = fb[i].load(a, kb + (q & 3) * 8);
        else {
          constexpr int CPR = BN / 8;
          if (MODE == DGRAD) rb[i] = dgrad_b_load(a, kb + q / CPR, n0 + (q % CPR) * 8);
          else rb[i] = wgrad_b_load(a, kb + q / CPR, kend, n0 + (q % CPR) * 8);
        }
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TA::PER_THREAD; ++i) {
      const int q = tid + i * 256;
      if (q < TA::CHUNKS) {
        int off;
        if (A_KC) off = (q >> 2) * (BK + PADK) + (q & 3) * 8;
        else { constexpr int CPR = BM / 8; off = (q / CPR) * (BM + PADR) + (q % CPR) * 8; }
        *reinterpret_cast<uint4*>(sA(buf) + off) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < TB::PER_THREAD; ++i) {
      const int q = tid + i * 256;
      if (q < TB::CHUNKS) {
        int off;
        if (B_KC) off = (q >> 2) * (BK + PADK) + (q & 3) * 8;
        else { constexpr int CPR = BN / 8; off = (q / CPR) * (BN + PADR) + (q % CPR) * 8; }
        *reinterpret_cast<uint4*>(sB(buf) + off) = rb[i];
      }
    }
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt + 1);
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i)
        af[i] = A_KC ? frag_kcontig<BM>(sA(cur), wm * WM + i * 16, lane)
                     : frag_kstrided<BM>(sA(cur), wm * WM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bfr[j] = B_KC ? frag_kcontig<BN>(sB(cur), wn * WN + j * 16, lane)
                      : frag_kstrided<BN>(sB(cur), wn * WN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }
  }

#undef sA
#undef sB
  // ---- epilogue ----
  const int fr = lane & 15, fq = lane >> 4;
  if (MODE == WGRAD) {
    const int nts = a.s1 - a.s0;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int col = n0 + wn * WN + j * 16 + fr;
      if (col >= a.N) continue;
      const int tap = col / a.C, c = col - tap * a.C;
      const int r = a.r0 + tap / nts, s = a.s0 + tap % nts;
      const long long coff = (long long)(r * a.KW + s) * a.C + c;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WM + i * 16 + fq * 4 + e;
          if (row < a.M) {
            float* p = a.dw + (long long)row * a.KH * a.KW * a.C + coff;
            if (a.accumulate) atomicAdd(p, acc[i][j][e]);
            else *p = acc[i][j][e];
          }
        }
    }
    return;
  }

  const int ldc = a.N;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int col = n0 + wn * WN + j * 16 + fr;
    const bool cok = col < a.N;
    float bv = 0.f;
    if (MODE == FWD && a.bias && cok) bv = a.bias[col];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * WM + i * 16 + fq * 4 + e;
        float v = acc[i][j][e] + bv;
        if (MODE == FWD && a.relu) v = fmaxf(v, 0.f);
        if (MODE == DGRAD && a.addend && row < a.M && cok) v += bf2f(a.addend[(long long)row * ldc + col]);
        if (row < a.M && cok) {
          a.out[(long long)row * ldc + col] = f2bf(v);
          s1 += v; s2 += v * v;
        }
      }
    if (MODE == FWD && a.stats) {
      s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0 && cok) {
        atomicAdd(a.stats + col, s1);
        atomicAdd(a.stats + a.N + col, s2);
      }
    }
  }
}

template <int MODE, int BM, int BN>
int launch(const ConvArgs& a, int splits, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((k_conv_igemm<MODE, BM, BN>), grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

template <int MODE>
int dispatch(const ConvArgs& a, int bm, int bn, int splits, hipStream_t s) {
#define KML_T(BMv, BNv) if (bm == BMv && bn == BNv) return launch<MODE, BMv, BNv>(a, splits, s);
  KML_T(32, 32) KML_T(32, 64) KML_T(64, 32) KML_T(64, 64)
  KML_T(64, 128) KML_T(128, 64) KML_T(128, 128) KML_T(32, 128) KML_T(128, 32)
#undef KML_T
  return (int)hipErrorInvalidValue;
}

// valid tap window along one axis: taps t where some output o in [0,O) reads 0<=o*st-p+t<I
void tap_window(int I, int O, int KS, int st, int p, int* t0, int* t1) {
  int lo = KS, hi = 0;
  for (int t = 0; t < KS; ++t) {
    // smallest/largest input coordinate read by tap t
    int first = -p + t, last = (O - 1) * st - p + t;
    bool ok = false;
    for (int o = 0; o < O && !ok; ++o) { int i = o * st - p + t; ok = (i >= 0 && i < I); }
    (void)first; (void)last;
    if (ok) { if (t < lo) lo = t; if (t + 1 > hi) hi = t + 1; }
  }
  if (lo >= hi) { lo = 0; hi = 0; }
  *t0 = lo; *t1 = hi;
}

ConvArgs make_args(int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw) {
  ConvArgs a = {};
  a.B = B; a.H = H; a.W = W; a.C = C; a.K = K; a.KH = KH; a.KW = KW;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.OH = (H + 2 * ph - KH) / sh + 1; a.OW = (W + 2 * pw - KW) / sw + 1;
  tap_window(H, a.OH, KH, sh, ph, &a.r0, &a.r1);
  tap_window(W, a.OW, KW, sw, pw, &a.s0, &a.s1);
  return a;
}

}  // namespace

// Host-side helper exposed for the Python planner / tests.
KML_API int kml_conv_tap_window(int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw,
                                int ph, int pw, int* out4) {
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  out4[0] = a.r0; out4[1] = a.r1; out4[2] = a.s0; out4[3] = a.s1;
  return 0;
}

KML_API int kml_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const float* bias, float* stats,
                         int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw,
                         int relu, int bm, int bn, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.relu = relu;
  a.M = B * a.OH * a.OW; a.N = K; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * C;
  return dispatch<FWD>(a, bm, bn, 1, s);
}

KML_API int kml_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const bf16_t* addend,
                           int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw,
                           int bm, int bn, hipStream_t s) {
  if (C % 8 || K % 8) return (int)hipErrorInvalidValue;
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  a.Kp = (K + BK - 1) / BK * BK;
  a.dy = dy; a.w = w; a.out = dx; a.addend = addend;
  a.M = B * H * W; a.N = C; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * a.Kp;
  return dispatch<DGRAD>(a, bm, bn, 1, s);
}

KML_API int kml_conv_wgrad(const bf16_t* x, const bf16_t* dy, float* dw,
                           int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw,
                           int bm, int bn, int splits, int accumulate, hipStream_t s) {
  if (C % 8 || K % 8) return (int)hipErrorInvalidValue;
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  a.x = x; a.dy = dy; a.dw = dw;
  a.M = K; a.N = (a.r1 - a.r0) * (a.s1 - a.s0) * C; a.Kd = B * a.OH * a.OW;
  if (splits < 1) splits = 1;
  int chunk = (a.Kd + splits - 1) / splits;
  chunk = (chunk + BK - 1) / BK * BK;
  splits = (a.Kd + chunk - 1) / chunk;
  a.kchunk = chunk;
  a.accumulate = (splits > 1) ? 1 : accumulate;
  return dispatch<WGRAD>(a, bm, bn, splits, s);
}
