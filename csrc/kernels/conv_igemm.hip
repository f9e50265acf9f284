// conv_igemm.hip — MFMA implicit-GEMM convolution for NHWC bf16 on gfx950.
//
// One kernel family covers the three convolution GEMMs of training (and Linear
// layers, which are 1x1 convolutions over a 1x1 image):
//
//   FWD   : Y[m=(b,oh,ow)][n=cout]   = sum_k im2col(X)[m][k=(tap,cin)] * W[n][k]
//   DGRAD : dX[m=(b,ih,iw)][n=cin]   = sum_k dY[(b,oh,ow)][cout] * W[cout][tap][cin],  k=(tap,cout)
//   WGRAD : dW[m=cout][n=(tap,cin)] (=|+=) sum_k dY[k=pixel][cout] * im2col(X)[k][n]
//
// Layouts: activations NHWC bf16 (C % 8 == 0), weights KRSC bf16 ([Cout][KH][KW][Cin]),
// weight gradients KRSC fp32 — written straight into the flat fp32 gradient buffer that
// RCCL all-reduces and the fused optimizer consumes.
//
// CDNA4 mapping
// -------------
// * 256 threads = 4 wave64 in a 2x2 grid; each wave owns a (BM/2)x(BN/2) sub-tile of
//   v_mfma_f32_16x16x32_bf16 fragments; BK = 32 or 64 (1 or 2 MFMA k-substeps).
// * Software pipeline, prefetch distance 2: two register stages hold K-tiles t+1 and
//   t+2 in flight while the MFMAs consume tile t from a two-buffer LDS ring (one
//   barrier per K-step).  Every global load is unconditional — out-of-range chunks
//   (conv padding, ragged edges, split-K tails) are redirected to a zero page instead
//   of being branched around — so hipcc emits counted vmcnt waits rather than the
//   vmcnt(0)-per-load it generates for branch-guarded loads (CDNA guide §5, trap (c)),
//   and the loop body is a straight line.
// * Index math is hoisted: per-thread pixel/row state is computed once; when a K-tile
//   stays inside one filter tap (Cin % BK == 0, every ResNet layer but the stem) the tap
//   is block-uniform scalar math; remaining divisions use host-precomputed
//   multiply-shift magic numbers.
// * An operand whose K axis is contiguous in memory lives in LDS as [row][k] (+16 B pad,
//   conflict-free ds_read_b128); an operand whose K axis is strided (dgrad weights, both
//   wgrad operands) lives as [k][row] in its natural order and is read with the gfx950
//   transposing ds_read_b64_tr_b16 — no transpose pass, no transposed weight copy.
// * Only taps touching the image for SOME output pixel are enumerated ([r0,r1)x[s0,s1),
//   host-computed): ResNet-34's layer4 (1x1 spatial at 32x32 input) runs its 3x3
//   convolutions as centre-tap GEMMs, 9x less K.
// * Split-K for latency-bound small-M layers.  FWD/DGRAD: each split writes its fp32
//   partial tile to a slab (fragment order, coalesced float4), releases at agent scope,
//   takes a ticket; the last arriver acquires, sums the slabs in split order
//   (deterministic) and runs the epilogue; tickets are reset by the last arriver
//   (graph-replay safe, no memset per call).  WGRAD uses the same slabs: one writer per
//   weight-gradient element, stored (or added) without atomics.
// * Epilogues: FWD bias / ReLU / per-channel BatchNorm sum+sumsq from the fp32 values
//   (BN needs no statistics pass); DGRAD adds an optional bf16 addend (the other
//   branch of a residual block) so gradient merges need no add kernel.
//
// Reference parity: the reference runs these convolutions through cuDNN inside the
// user's torch module (ml/experiments/kubeml/function_resnet34.py:72-76).
#include "kml_common.h"
#include "kml_sgd.h"

#include <type_traits>

namespace {

constexpr int PADK = 16;  // K-contiguous LDS rows: BK+16 bf16 (fragment reads conflict-free; +8 was 2-way)
constexpr int PADR = 8;  // K-strided LDS rows: R+8 bf16

enum { FWD = 0, DGRAD = 1, WGRAD = 2 };

// n / d for 0 <= n < 2^31 via multiply-shift (host computes m, s)
struct FastDiv {
  unsigned m;
  int s;
  int d;
};
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)(((unsigned long long)(unsigned)n * f.m) >> f.s);
}

struct ConvArgs {
  const bf16_t* x;       // input activations NHWC (FWD, WGRAD)
  const bf16_t* w;       // weights KRSC (FWD, DGRAD)
  const bf16_t* dy;      // output grads NHWC (DGRAD, WGRAD)
  const bf16_t* zp;      // 16-byte zero page (target of out-of-range loads)
  bf16_t* out;           // Y (FWD) or dX (DGRAD)
  float* dw;             // fp32 weight grads KRSC (WGRAD)
  float* stats;          // [2][Cout] BN sum / sumsq (FWD, optional)
  const float* bias;     // [Cout] (FWD, optional)
  const bf16_t* addend;  // [M][N] added to the DGRAD output
  float* slab;           // split-K partial tiles (FWD/DGRAD, splits > 1)
  unsigned* counters;    // split-K tickets, one per output tile
  const bf16_t* wt;      // transposed weights for the direct dgrad variant
  // DGRAD -> consumer-BN backward fusion: partial [sum dz | sum dz*xhat] rows of the BN that
  // consumes this dX (dz = dX * [y > 0], xhat = (c - mean) * rstd), same row layout as stats_part
  const bf16_t* bnf_y; const bf16_t* bnf_c; const float* bnf_mean; const float* bnf_rstd; float* bnf_part;
  // bnf_mask_out: store dz = dX * [y > 0] (the consumer BN's ReLU mask applied) instead of dX,
  // so that BN's backward needs no mask and never reads y
  int bnf_mask_out;
  // Group reduction of the per-wave partial rows (FWD stats_part / DGRAD bnf_part): every
  // grp_tiles consecutive M-tiles form a group; the last-arriving block of a group (agent-scope
  // ticket per (group, n-tile)) sums the group's rows in a fixed order into grp_out[g][2N], so
  // the consumer BN kernel reads ceil(tiles/grp_tiles) rows instead of one per wave.
  float* grp_out;        // [NG][2N] or null (consumer sums the per-wave rows itself)
  unsigned* grp_cnt;     // NG * n-tiles tickets (zero on entry; the last arriver resets)
  int grp_tiles;
  int stats_part;        // FWD stats: 0 = atomics into stats[2N]; 1 = plain stores of per-wave
                         //   partial rows stats[(m0/WM + wm)][2N] (summed by bn_apply)
  int B, H, W, C;        // input geometry (C = Cin)
  int OH, OW, K;         // output geometry (K = Cout)
  int KH, KW, sh, sw, ph, pw;
  int r0, r1, s0, s1;    // valid tap window
  int M, N, Kd;          // GEMM dims
  int Kp;                // DGRAD: Cout padded to a multiple of BK (k = tap*Kp + cout)
  int kchunk;            // split-K chunk (multiple of BK)
  int splits;
  int relu;
  int accumulate;        // WGRAD: add (1) or store (0)
  // WGRAD of a 1x1/s1/p0 conv (a Linear): the bias gradient sum_k dY[k][m] comes out of the
  // same GEMM as one extra column n = C whose B operand is all ones (the ones page), so no
  // separate column-sum pass and no cross-block reduction.  N then counts that column.
  float* dbias;          // [Cout] fp32 or null
  int bias_acc;          // dbias: add (1) or store (0)
  const bf16_t* op;      // 16-byte ones page: bf16 {1, 0, 0, 0, 0, 0, 0, 0}
  // Unrolled small-map convs (ops.kernels.unrolled): a 3x3/s1/p1 conv on a 2x2 map runs as a
  // 1x1 conv of 4C -> 4K channels on a 1x1 map (only the taps that touch the image; the
  // im2col of the 3x3 form is 5/9 zero padding).  fold_c: the FWD/DGRAD output channel col =
  // (pos, c) belongs to BN channel c = col % fold_c, so a partial row is written as fold
  // rows of [sum(fold_c) | sumsq(fold_c)] (BN kernels see ordinary rows of the real
  // channels).  The WGRAD of an unrolled conv runs in the plain 3x3 form (prep_wgrad).
  int fold_c;
  // g22: an unrolled conv whose 1x1-form weight W'[(p, n)][(q, c)] = w[n][tap(p, q)][c] is
  // gathered by the FWD / DGRAD weight loaders straight from the 3x3 weight w (no unrolled
  // copy per step): K = 4 Kq, C = 4 Cq in the 1x1 form, fd_gK / fd_gC divide by Kq / Cq.
  int g22;
  FastDiv fd_gK, fd_gC;
  // FWD halo with the INPUT's BatchNorm + ReLU applied while the patch is staged (ibn_rows set):
  // the producer conv's partial statistics rows [ibn_G][2C] are summed in the prologue (same order
  // as the BN apply kernel), the interior patch chunks are normalised in registers, and the blocks
  // of N-tile 0 write the normalised map to ibn_y (the activation the backward keeps)
  const float* ibn_rows; int ibn_G; long long ibn_M;
  const float* ibn_gamma; const float* ibn_beta;
  float* ibn_mean; float* ibn_rstd; float* ibn_rmean; float* ibn_rvar;
  float ibn_eps, ibn_mom;
  bf16_t* ibn_y;
  FastDiv fd_C, fd_nts, fd_OW, fd_OH, fd_W, fd_H, fd_Kp, fd_sh, fd_sw;
  // Stride-2 DGRAD by parity class (kml_conv_dgrad_s2): this launch computes the input pixels
  // (ih, iw) = (2i + pa, 2j + pe) only — GEMM row m = (b, i, j) over an Hc x Wc grid — with
  // only the taps of matching parity (r = r0 + 2 tr, tap_rs2), so none of the 3/4 of
  // (pixel, tap) pairs a stride-2 dgrad gathers from the zero page is computed.
  // par: bit 0 = parity class, bit 1 = pa, bit 2 = pe (fd_W / fd_H then divide by the class
  // grid Wc / Hc; bnf_part points at the class's first partial row).
  int par;
};

// Block coordinates of one conv tile: kernels pass blockIdx; the grouped backward kernel
// (k_conv_pair) passes coordinates decoded from its flat block index.
struct Blk {
  int x, y, z, gx;
};
__device__ __forceinline__ Blk hw_blk() {
  return Blk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x};
}

// Forward pairs (kml_conv_fwd_pair): while g_fwd_rec is set, a forward launch of the register /
// LDS-DMA / direct kernels records its body, arguments and grid instead of launching.
struct FwdRec {
  int body = -1;        // index in the paired-body list (fwd_body_id), -1: not pairable
  ConvArgs a;
  int gx = 0, gy = 0;
  bool set = false;
};
FwdRec* g_fwd_rec = nullptr;
template <class B>
constexpr int fwd_body_id();

// K-strided [BK][R] tiles of R = 32/64/128 columns use the XOR chunk swizzle of the glds
// kernels (swz_ks, conflict-free reads and writes per tools/lds_banks.py); other widths keep
// the +PADR row padding (2-3-way conflicts).
template <int R>
struct KsSwz {
  static constexpr bool ON = (R == 32 || R == 64 || R == 128);
  static constexpr int LD = ON ? R : R + PADR;  // row length in bf16
};

template <int R, bool KCONTIG, int BK>
struct TileShape {
  static constexpr int ELEMS = KCONTIG ? R * (BK + PADK) : BK * KsSwz<R>::LD;
  static constexpr int CHUNKS = R * BK / 8;  // 16-byte chunks per stage
  static constexpr int PER_THREAD = (CHUNKS + 255) / 256;
};

__device__ __forceinline__ uint4 ld16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ void tap_rs(const ConvArgs& a, int tap, int& r, int& s) {
  const int tr = fdiv(tap, a.fd_nts);
  r = a.r0 + tr;
  s = a.s0 + (tap - tr * a.fd_nts.d);
}
// taps of one stride-2 parity class: every second row / column of the filter
__device__ __forceinline__ void tap_rs2(const ConvArgs& a, int tap, int& r, int& s) {
  const int tr = fdiv(tap, a.fd_nts);
  r = a.r0 + 2 * tr;
  s = a.s0 + 2 * (tap - tr * a.fd_nts.d);
}

// ---------------------------------------------------------------------------------
// Chunk address generators.  Each thread owns PER_THREAD 16-byte chunks of a stage;
// init() runs once, ptr(kb) returns the global address for K-tile base kb (or the
// zero page).  TAPU: the whole K-tile lies in one filter tap (block-uniform tap).
// ---------------------------------------------------------------------------------

template <int BK, bool TAPU>
struct FwdA {  // im2col(X): LDS row = output pixel, K-contiguous over cin
  int ih0, iw0, koff;
  int base;    // element offset of (b, ih0, iw0, 0)
  bool valid;
  __device__ void init(const ConvArgs& a, int m, int q) {
    valid = m < a.M;
    const int mm = valid ? m : 0;
    const int t = fdiv(mm, a.fd_OW), ow = mm - t * a.OW;
    const int b = fdiv(t, a.fd_OH), oh = t - b * a.OH;
    ih0 = oh * a.sh - a.ph;
    iw0 = ow * a.sw - a.pw;
    base = ((b * a.H + ih0) * a.W + iw0) * a.C;
    koff = (q % (BK / 8)) * 8;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int k = kb + koff;
    int r, s, c;
    if constexpr (TAPU) {
      const int tap = fdiv(kb, a.fd_C);  // uniform
      c = k - tap * a.C;
      tap_rs(a, tap, r, s);
    } else {
      const int tap = fdiv(k, a.fd_C);
      c = k - tap * a.C;
      tap_rs(a, tap, r, s);
    }
    const int ih = ih0 + r, iw = iw0 + s;
    const bool ok = valid && k < kend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    return ok ? a.x + base + (r * a.W + s) * a.C + c : a.zp;
  }
};

// 3x3 tap of the unrolled pair (output position p, input position q) on a 2x2 map
__device__ __forceinline__ int tap22(int p, int q) { return ((q >> 1) - (p >> 1) + 1) * 3 + ((q & 1) - (p & 1) + 1); }

template <int BK, bool TAPU>
struct FwdB {  // W[n][tap][cin], K-contiguous
  int base, koff, p22;
  bool valid;
  __device__ void init(const ConvArgs& a, int n, int q) {
    valid = n < a.N;
    const int nn = valid ? n : 0;
    if (a.g22) {  // row n = (p, n') of the unrolled weight
      p22 = fdiv(nn, a.fd_gK);
      base = (nn - p22 * a.fd_gK.d) * 9 * a.fd_gC.d;
    } else {
      p22 = 0;
      base = nn * a.KH * a.KW * a.C;
    }
    koff = (q % (BK / 8)) * 8;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int k = kb + koff;
    if (a.g22) {  // column k = (q, c): w[n'][tap(p, q)][c]
      const int q = fdiv(k, a.fd_gC), c = k - q * a.fd_gC.d;
      return (valid && k < kend) ? a.w + base + tap22(p22, q) * a.fd_gC.d + c : a.zp;
    }
    const int tap = TAPU ? fdiv(kb, a.fd_C) : fdiv(k, a.fd_C);
    const int c = k - tap * a.C;
    int r, s;
    tap_rs(a, tap, r, s);
    return (valid && k < kend) ? a.w + base + (r * a.KW + s) * a.C + c : a.zp;
  }
};

template <int BK>
struct DgradA {  // dY gathered for input pixel m; K = (tap, cout); Kp % BK == 0 -> tap uniform
  int b, ih, iw, koff;
  bool valid;
  __device__ void init(const ConvArgs& a, int m, int q) {
    valid = m < a.M;
    const int mm = valid ? m : 0;
    const int t = fdiv(mm, a.fd_W);
    iw = mm - t * a.W;
    b = fdiv(t, a.fd_H);
    ih = t - b * a.H;
    koff = (q % (BK / 8)) * 8;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int tap = fdiv(kb, a.fd_Kp);  // uniform
    const int n = kb - tap * a.Kp + koff;
    int r, s;
    tap_rs(a, tap, r, s);
    const int th = ih + a.ph - r, tw = iw + a.pw - s;
    const int oh = fdiv(th < 0 ? 0 : th, a.fd_sh), ow = fdiv(tw < 0 ? 0 : tw, a.fd_sw);
    const bool ok = valid && kb + koff < kend && n < a.K && th >= 0 && tw >= 0 && oh * a.sh == th &&
                    ow * a.sw == tw && oh < a.OH && ow < a.OW;
    return ok ? a.dy + ((b * a.OH + oh) * a.OW + ow) * a.K + n : a.zp;
  }
};

template <int BK>
// Stride-2 parity-class dgrad operands (kml_conv_dgrad_s2): GEMM row m = (b, i, j) is the input
// pixel (2i + pa, 2j + pe) and the taps are those of matching parity (tap_rs2).  Selected by
// the DGRAD bodies' TAPU = false instantiation (a plain DGRAD K-tile always sits in one tap,
// so TAPU = false is otherwise never launched for DGRAD): the plain kernels keep their code.
struct DgradAP {  // dY gathered for parity-class pixel m
  int b, ih, iw, koff;
  bool valid;
  __device__ void init(const ConvArgs& a, int m, int q) {
    valid = m < a.M;
    const int mm = valid ? m : 0;
    const int t = fdiv(mm, a.fd_W);  // fd_W / fd_H hold the class grid Wc / Hc here
    iw = 2 * (mm - t * a.fd_W.d) + ((a.par >> 2) & 1);
    b = fdiv(t, a.fd_H);
    ih = 2 * (t - b * a.fd_H.d) + ((a.par >> 1) & 1);
    koff = (q % (BK / 8)) * 8;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int tap = fdiv(kb, a.fd_Kp);  // uniform
    const int n = kb - tap * a.Kp + koff;
    int r, s;
    tap_rs2(a, tap, r, s);
    const int th = ih + a.ph - r, tw = iw + a.pw - s;
    const int oh = fdiv(th < 0 ? 0 : th, a.fd_sh), ow = fdiv(tw < 0 ? 0 : tw, a.fd_sw);
    const bool ok = valid && kb + koff < kend && n < a.K && th >= 0 && tw >= 0 && oh * a.sh == th &&
                    ow * a.sw == tw && oh < a.OH && ow < a.OW;
    return ok ? a.dy + ((b * a.OH + oh) * a.OW + ow) * a.K + n : a.zp;
  }
};

template <int BK, int BN>
struct DgradB {  // LDS row = k = (tap, cout), cols = cin; chunk = W[cout][tap][c..c+7]
  int krow, c, q22, c22;
  bool valid;
  __device__ void init(const ConvArgs& a, int n0, int q) {
    constexpr int CPR = BN / 8;
    krow = q / CPR;
    c = n0 + (q % CPR) * 8;
    valid = c < a.N;
    if (a.g22) {  // column c = (q, c') of the unrolled weight
      const int cc = valid ? c : 0;
      q22 = fdiv(cc, a.fd_gC);
      c22 = cc - q22 * a.fd_gC.d;
    } else {
      q22 = c22 = 0;
    }
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int tap = fdiv(kb, a.fd_Kp);  // uniform
    const int n = kb - tap * a.Kp + krow;
    if (a.g22) {  // 1x1 form (tap 0), row n = (p, n'): w[n'][tap(p, q)][c']
      const bool ok = valid && kb + krow < kend && n < a.K;
      const int nn = ok ? n : 0;
      const int p = fdiv(nn, a.fd_gK);
      return ok ? a.w + ((long long)(nn - p * a.fd_gK.d) * 9 + tap22(p, q22)) * a.fd_gC.d + c22 : a.zp;
    }
    int r, s;
    tap_rs(a, tap, r, s);
    const bool ok = valid && kb + krow < kend && n < a.K;
    return ok ? a.w + ((n * a.KH + r) * a.KW + s) * a.C + c : a.zp;
  }
};

template <int BK, int BN>
struct DgradBP {  // DgradB over one parity class's taps (tap_rs2; no unrolled-weight gather)  // LDS row = k = (tap, cout), cols = cin; chunk = W[cout][tap][c..c+7]
  int krow, c, q22, c22;
  bool valid;
  __device__ void init(const ConvArgs& a, int n0, int q) {
    constexpr int CPR = BN / 8;
    krow = q / CPR;
    c = n0 + (q % CPR) * 8;
    valid = c < a.N;
    if (a.g22) {  // column c = (q, c') of the unrolled weight
      const int cc = valid ? c : 0;
      q22 = fdiv(cc, a.fd_gC);
      c22 = cc - q22 * a.fd_gC.d;
    } else {
      q22 = c22 = 0;
    }
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int tap = fdiv(kb, a.fd_Kp);  // uniform
    const int n = kb - tap * a.Kp + krow;
    if (a.g22) {  // 1x1 form (tap 0), row n = (p, n'): w[n'][tap(p, q)][c']
      const bool ok = valid && kb + krow < kend && n < a.K;
      const int nn = ok ? n : 0;
      const int p = fdiv(nn, a.fd_gK);
      return ok ? a.w + ((long long)(nn - p * a.fd_gK.d) * 9 + tap22(p, q22)) * a.fd_gC.d + c22 : a.zp;
    }
    int r, s;
    tap_rs2(a, tap, r, s);
    const bool ok = valid && kb + krow < kend && n < a.K;
    return ok ? a.w + ((n * a.KH + r) * a.KW + s) * a.C + c : a.zp;
  }
};

template <int BK, int BM>
struct WgradA {  // LDS row = pixel k, cols = cout; chunk = dY[k][n..n+7]
  int krow, n;
  bool valid;
  __device__ void init(const ConvArgs& a, int m0, int q) {
    constexpr int CPR = BM / 8;
    krow = q / CPR;
    n = m0 + (q % CPR) * 8;
    valid = n < a.M;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int k = kb + krow;
    return (valid && k < kend) ? a.dy + (long long)k * a.K + n : a.zp;
  }
};

template <int BK, int BN>
struct WgradB {  // LDS row = pixel k, cols j = (tap, cin); chunk = X[pixel shifted by tap][c..c+7]
  int krow, r, s, c;
  bool valid, ones;
  __device__ void init(const ConvArgs& a, int n0, int q) {
    constexpr int CPR = BN / 8;
    krow = q / CPR;
    const int j = n0 + (q % CPR) * 8;
    const int nreal = a.dbias ? a.N - 1 : a.N;  // the bias column (if any) is n = nreal
    valid = j < nreal;
    ones = a.dbias && j == nreal;
    const int jj = valid ? j : 0;
    const int tap = fdiv(jj, a.fd_C);
    c = jj - tap * a.C;
    tap_rs(a, tap, r, s);
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int k = kb + krow;
    const int kk = k < kend ? k : 0;
    const int t = fdiv(kk, a.fd_OW), ow = kk - t * a.OW;
    const int b = fdiv(t, a.fd_OH), oh = t - b * a.OH;
    const int ih = oh * a.sh - a.ph + r, iw = ow * a.sw - a.pw + s;
    const bool ok = valid && k < kend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    if (ones) return k < kend ? a.op : a.zp;
    return ok ? a.x + ((b * a.H + ih) * a.W + iw) * a.C + c : a.zp;
  }
};

// ---- fragment readers (k-substep ks covers k = 32*ks .. 32*ks+31 of the LDS tile) ----
template <int BK>
__device__ __forceinline__ bf16x8_t frag_kcontig(const bf16_t* lds, int row0, int ks, int lane) {
  const bf16_t* p = lds + (row0 + (lane & 15)) * (BK + PADK) + 32 * ks + 8 * (lane >> 4);
  return *reinterpret_cast<const bf16x8_t*>(p);
}

typedef __attribute__((ext_vector_type(4))) short v4s_t;

template <int R>
__device__ __forceinline__ int swz_ks(int r);

template <int R>
__device__ __forceinline__ bf16x8_t frag_kstrided(const bf16_t* lds, int row0, int ks, int lane) {
  const int il = lane & 15, g = lane >> 4;
  const int col = row0 + 4 * (il & 3);
  const int k0 = 32 * ks + 8 * g + (il >> 2);
  const bf16_t* p0;
  const bf16_t* p1;
  if constexpr (KsSwz<R>::ON) {  // swizzled 16-byte chunk (col / 8) of rows k0, k0 + 4
    const int ch = col >> 3, within = col & 7;
    p0 = lds + k0 * R + ((ch ^ swz_ks<R>(k0)) << 3) + within;
    p1 = lds + (k0 + 4) * R + ((ch ^ swz_ks<R>(k0 + 4)) << 3) + within;
  } else {
    p0 = lds + k0 * (R + PADR) + col;
    p1 = p0 + 4 * (R + PADR);
  }
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p0));
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p1));
  bf16x8_t f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

// Last arriver of an M-tile group sums the group's per-wave partial rows (ConvArgs::grp_*).
// BMT/BNT: block tile, RPT: partial rows per M-tile, SINGLE: one live wave (direct variant).
// Hand-off without fences (CDNA guide §6 G16, R1 fan-in): the rows were stored write-through
// (sc1, store_row), every wave drains its stores before the barrier, one lane takes a relaxed
// agent-scope ticket, and the last arriver reads the rows with sc1 loads (past its L1).  A
// release fence here would write back the block's whole dirty L2 share (the conv output).
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// partial-row store: write-through (sc1) when a group reduction reads it in this launch
__device__ __forceinline__ void store_row(float* p, float v, bool sc1) {
  if (sc1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

template <int BMT, int BNT, int RPT, bool SINGLE>
__device__ __forceinline__ void group_reduce_rows(const ConvArgs& a, const float* rows, int m0, int n0, int tid,
                                                  unsigned* flag) {
  const int tile_m = m0 / BMT, tile_n = n0 / BNT;
  const int ntn = (a.N + BNT - 1) / BNT, ntm = (a.M + BMT - 1) / BMT;
  const int g = tile_m / a.grp_tiles;
  const int t0 = g * a.grp_tiles, t1 = min(ntm, t0 + a.grp_tiles);
  unsigned* cnt = a.grp_cnt + g * ntn + tile_n;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 rows
  unsigned last = 0;
  if constexpr (!SINGLE) __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == (unsigned)(t1 - t0 - 1)) ? 1u : 0u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (!SINGLE) flag[0] = last;
  }
  if constexpr (SINGLE) {
    last = (unsigned)__shfl((int)last, 0, 64);
  } else {
    __syncthreads();
    last = flag[0];
  }
  if (!last) return;
  constexpr int NT = SINGLE ? 64 : 256;
  const int r0 = t0 * RPT, r1 = t1 * RPT;
  for (int q = tid; q < 2 * BNT; q += NT) {
    const int half = q / BNT, col = n0 + (q - half * BNT);
    if (col >= a.N) continue;
    const float* src = rows + (long long)half * a.N + col;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    int r = r0;
    for (; r + 4 <= r1; r += 4) {  // 4 independent sc1 loads in flight, fixed summation order
      acc0 += ld_sc1(src + (long long)r * 2 * a.N);
      acc1 += ld_sc1(src + (long long)(r + 1) * 2 * a.N);
      acc2 += ld_sc1(src + (long long)(r + 2) * 2 * a.N);
      acc3 += ld_sc1(src + (long long)(r + 3) * 2 * a.N);
    }
    for (; r < r1; ++r) acc0 += ld_sc1(src + (long long)r * 2 * a.N);
    a.grp_out[(long long)g * 2 * a.N + (long long)half * a.N + col] = (acc0 + acc1) + (acc2 + acc3);
  }
}

// Offset of column col's sum inside a partial row (sumsq at + sq_off): [sum(N) | sumsq(N)],
// or with fold_c the row holds N / fold_c sub-rows [sum(fold_c) | sumsq(fold_c)].
__device__ __forceinline__ int row_off(const ConvArgs& a, int col) {
  if (!a.fold_c) return col;
  const int p = col / a.fold_c;
  return col + p * a.fold_c;
}
__device__ __forceinline__ int sq_off(const ConvArgs& a) { return a.fold_c ? a.fold_c : a.N; }

// Output pixel row of GEMM row `row` (identity except in a stride-2 parity-class DGRAD, which
// always runs the row-pass epilogue below: the per-element epilogue stays free of the remap).
__device__ __forceinline__ long long prow(const ConvArgs& a, int row) {
  if (!a.par) return row;
  const int t = fdiv(row, a.fd_W), j = row - t * a.fd_W.d;
  const int b = fdiv(t, a.fd_H), i = t - b * a.fd_H.d;
  return ((long long)b * a.H + 2 * i + ((a.par >> 1) & 1)) * a.W + 2 * j + ((a.par >> 2) & 1);
}

// DGRAD epilogue through LDS rows, for tiles whose output merges an addend and/or feeds the
// consumer BN's partial sums.  The per-element path gathers addend / y / c with 2-byte
// loads (one wave instruction = 4 rows x 32 B, address-unit bound): on ResNet-50's 56x56
// 1x1 dgrads that epilogue took ~5x the GEMM.  Here the fp32 tile is staged in LDS (column
// chunk XOR-swizzled by (row >> 2) & 3 so a fragment store's 4 rows x 16 columns hit 64
// distinct banks), then each thread owns one 8-channel chunk column and walks the tile's
// rows with 16-byte loads and stores: v = acc + addend, bf16 round, the consumer BN's
// masked dz and dz * xhat sums.  Partial rows: a shuffle butterfly over the lanes of a
// chunk column, then a fixed-order sum of the 4 waves — deterministic, one row per M-tile
// as in the per-element path.
template <int BMT, int BNT, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void dgrad_rowpass(const ConvArgs& a, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                              int wn, int lane, int tid, unsigned* flag) {
  constexpr int CPR = BNT / 8, RSTEP = 256 / CPR;
  static_assert(BNT % 64 == 0 && 64 % CPR == 0, "row pass: 64-column multiples");
  float* sF = reinterpret_cast<float*>(reinterpret_cast<char*>(flag) + 16);
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = wm * WM + i * 16 + fq * 4 + e, c = wn * WN + j * 16 + fr;
        sF[r * BNT + (c ^ (((r >> 2) & 3) << 4))] = acc[i][j][e];
      }
  __syncthreads();
  const int cc = tid % CPR, r0 = tid / CPR;
  const int col0 = n0 + cc * 8;
  const bool cok = col0 < a.N;
  const bool bnf = a.bnf_part != nullptr;
  float mean[8], rstd[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { mean[k] = 0.f; rstd[k] = 0.f; s1[k] = 0.f; s2[k] = 0.f; }
  if (bnf && cok) {
    const int bc0 = a.fold_c ? col0 % a.fold_c : col0;  // 8 channels never straddle a fold group
#pragma unroll
    for (int k = 0; k < 8; ++k) { mean[k] = a.bnf_mean[bc0 + k]; rstd[k] = a.bnf_rstd[bc0 + k]; }
  }
  for (int r = r0; r < BMT; r += RSTEP) {
    const int row = m0 + r;
    if (row >= a.M || !cok) continue;
    const float* src = sF + r * BNT + ((cc * 8) ^ (((r >> 2) & 3) << 4));
    const float4 p0 = *reinterpret_cast<const float4*>(src), p1 = *reinterpret_cast<const float4*>(src + 4);
    float v[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    const long long idx = prow(a, row) * a.N + col0;
    if (a.addend) {
      const uint4 ad = ld16(a.addend + idx);
      const unsigned aw[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[2 * k] += lo_bf(aw[k]); v[2 * k + 1] += hi_bf(aw[k]); }
    }
    unsigned ow[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ow[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
    if (bnf) {
      const uint4 cv = ld16(a.bnf_c + idx);
      const uint4 yv = a.bnf_y ? ld16(a.bnf_y + idx) : make_uint4(0, 0, 0, 0);
      const unsigned cw[4] = {cv.x, cv.y, cv.z, cv.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float dz0 = lo_bf(ow[k]), dz1 = hi_bf(ow[k]);
        if (a.bnf_y) {
          const bool k0 = lo_bf(yw[k]) > 0.f, k1 = hi_bf(yw[k]) > 0.f;
          if (!k0) dz0 = 0.f;
          if (!k1) dz1 = 0.f;
          if (a.bnf_mask_out) ow[k] &= (k0 ? 0x0000ffffu : 0u) | (k1 ? 0xffff0000u : 0u);
        }
        const float x0 = (lo_bf(cw[k]) - mean[2 * k]) * rstd[2 * k];
        const float x1 = (hi_bf(cw[k]) - mean[2 * k + 1]) * rstd[2 * k + 1];
        s1[2 * k] += dz0; s2[2 * k] += dz0 * x0;
        s1[2 * k + 1] += dz1; s2[2 * k + 1] += dz1 * x1;
      }
    }
    *reinterpret_cast<uint4*>(a.out + idx) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
  if (!bnf) return;
#pragma unroll
  for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s1[k] += __shfl_xor(s1[k], off, 64);
      s2[k] += __shfl_xor(s2[k], off, 64);
    }
  __syncthreads();  // staging reads done: the tile area is reused as [4 waves][CPR][17]
  const int wave = tid >> 6;
  if (lane < CPR) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sF[(wave * CPR + lane) * 17 + k] = s1[k];   // odd row stride: the active lanes' stores hit distinct banks
      sF[(wave * CPR + lane) * 17 + 8 + k] = s2[k];
    }
  }
  __syncthreads();
  float* rows = a.bnf_part;
  const bool sc1_rows = a.grp_out != nullptr;
  const long long rrow = (long long)(m0 / BMT) * 2 * a.N;
  for (int q = tid; q < 2 * BNT; q += 256) {
    const int half = q / BNT, cl = q - half * BNT, col = n0 + cl;
    if (col >= a.N) continue;
    const int c8 = cl >> 3, k = (cl & 7) + 8 * half;
    const float sum = ((sF[(0 * CPR + c8) * 17 + k] + sF[(1 * CPR + c8) * 17 + k]) +
                       sF[(2 * CPR + c8) * 17 + k]) + sF[(3 * CPR + c8) * 17 + k];
    store_row(rows + rrow + row_off(a, col) + (half ? sq_off(a) : 0), sum, sc1_rows);
  }
  if (a.grp_out) group_reduce_rows<BMT, BNT, 1, false>(a, rows, m0, n0, tid, flag);
}

template <int MODE, int MR, int NR, int WM, int WN, bool SINGLE = false, bool STAGE_ALL = false, int LDSB = 0>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                              int wn, int lane, int tid, int tile, int bz, unsigned* flag) {
  const int fr = lane & 15, fq = lane >> 4;

  // -------------------------------------------------------- split-K: last arriver reduces
  // (every mode: the fp32 partial tiles are summed in split order by the last block of a
  // tile, so FWD/DGRAD outputs and WGRAD weight gradients are bitwise reproducible).
  // Publish without a release fence (CDNA guide §6 G16 R1): the partial tile is stored
  // write-through (16-byte sc1 stores), every storing wave drains, one lane takes the
  // relaxed agent-scope ticket; only the last arriver pays one agent acquire before its
  // plain loads.  A release fence would write back each split block's whole dirty XCD L2.
  if (a.splits > 1) {
    constexpr int NACC = MR * NR * 4;
    float* slab = a.slab + ((long long)tile * a.splits) * (256 * NACC);
    {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab + (long long)bz * 256 * NACC, (short)0,
                                                        256 * NACC * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          __attribute__((ext_vector_type(4))) float v = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                 rs, (tid * (NACC / 4) + i * NR + j) * 16, 0, 16 /* sc1 */);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add(a.counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned lastp = (t == (unsigned)a.splits - 1) ? 1u : 0u;
      if (lastp) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.counters + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      flag[0] = lastp;
    }
    __syncthreads();
    if (flag[0] == 0) return;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // Batches of U slabs are loaded before any of them is added: the reduce costs
    // ceil(splits / U) memory round trips instead of one per split (the additions stay in
    // split order, so the sum is unchanged bit for bit).  U keeps the batch at 8 float4.
    constexpr int NV = MR * NR;
    constexpr int U = NV >= 8 ? 1 : 8 / NV;
    int sp = 0;
    for (; sp + U <= a.splits; sp += U) {
      float4 v[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float4* src = reinterpret_cast<const float4*>(slab + (long long)(sp + u) * 256 * NACC) + tid * (NACC / 4);
#pragma unroll
        for (int k = 0; k < NV; ++k) v[u][k] = src[k];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j) {
            const float4 w = v[u][i * NR + j];
            acc[i][j][0] += w.x; acc[i][j][1] += w.y; acc[i][j][2] += w.z; acc[i][j][3] += w.w;
          }
    }
    for (; sp < a.splits; ++sp) {
      const float4* src = reinterpret_cast<const float4*>(slab + (long long)sp * 256 * NACC) + tid * (NACC / 4);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const float4 v = src[i * NR + j];
          acc[i][j][0] += v.x; acc[i][j][1] += v.y; acc[i][j][2] += v.z; acc[i][j][3] += v.w;
        }
    }
  }

  // ---------------------------------------------------------------- WGRAD epilogue
  if constexpr (MODE == WGRAD) {
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int col = n0 + wn * WN + j * 16 + fr;
      if (col >= a.N) continue;
      if (a.dbias && col == a.N - 1) {  // the ones column: bias gradient of output channel row
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * WM + i * 16 + fq * 4 + e;
            if (row < a.M) a.dbias[row] = a.bias_acc ? a.dbias[row] + acc[i][j][e] : acc[i][j][e];
          }
        continue;
      }
      const int tap = fdiv(col, a.fd_C), c = col - tap * a.C;
      int r, s;
      tap_rs(a, tap, r, s);
      const long long coff = (long long)(r * a.KW + s) * a.C + c;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WM + i * 16 + fq * 4 + e;
          if (row < a.M) {
            // one writer per element (split-K partials were summed above): no atomics
            float* p = a.dw + (long long)row * a.KH * a.KW * a.C + coff;
            if (a.accumulate) *p += acc[i][j][e];
            else *p = acc[i][j][e];
          }
        }
    }
    return;
  } else {
    // ---------------------------------------------------------- FWD / DGRAD epilogue
    // (entered after a block barrier: the main loops end with one, so LDS is free here)
    // tile geometry: 2x2 waves (SINGLE: one live wave owns the whole tile)
    constexpr int BMT = SINGLE ? WM : 2 * WM, BNT = SINGLE ? WN : 2 * WN;
    constexpr bool ROWPASS = MODE == DGRAD && !SINGLE && BNT % 64 == 0 && BMT * BNT >= 4096 &&
                             LDSB >= 16 + BMT * BNT * 4;
    if constexpr (ROWPASS) {
      if (a.addend || a.bnf_part) {
        dgrad_rowpass<BMT, BNT, MR, NR, WM, WN>(a, acc, m0, n0, wm, wn, lane, tid, flag);
        return;
      }
    }
    // Large tiles stage the bf16 output through LDS (past the 16-byte split-K flag word) and
    // write it back as 16-byte row chunks instead of one 2-byte store per element.
    constexpr bool STAGE_OK = !SINGLE && (STAGE_ALL || BMT * BNT >= 8192);
    constexpr int LDO = BNT + 8;  // padded LDS row (bf16 elements)
    constexpr int RED_OFF = 16 + (STAGE_OK ? BMT * LDO * 2 : 0);
    const bool stage = STAGE_OK && flag != nullptr && (a.N % 8) == 0;
    bf16_t* sout = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(flag) + 16);
    float* red = reinterpret_cast<float*>(reinterpret_cast<char*>(flag) + RED_OFF);  // [2][BNT]
    // Per-channel partial rows for the BN kernel (FWD statistics / consumer-BN partials of a
    // DGRAD), ONE row per M-tile: the two wave row-bands of a tile are summed through LDS, so
    // the BN kernel (every block of which reads all rows) reads half as many.
    float* rows = (MODE == DGRAD) ? a.bnf_part : ((a.stats && a.stats_part) ? a.stats : nullptr);
    const bool sc1_rows = a.grp_out != nullptr;
    const long long rrow = (long long)(m0 / BMT) * 2 * a.N;
    const int ldc = a.N;
    float k1[NR], k2[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int col = n0 + wn * WN + j * 16 + fr;
      const bool cok = col < a.N;
      float bv = 0.f;
      const int bc = a.fold_c ? col % a.fold_c : col;  // BN / bias channel of this column
      if (MODE == FWD && a.bias && cok) bv = a.bias[bc];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WM + i * 16 + fq * 4 + e;
          if (row < a.M && cok) {
            float v = acc[i][j][e] + bv;
            if (MODE == FWD && a.relu) v = fmaxf(v, 0.f);
            if (MODE == DGRAD && a.addend) v += bf2f(a.addend[(long long)row * ldc + col]);
            bf16_t vb = f2bf(v);
            if (MODE == DGRAD && a.bnf_part) {  // consumer BN's dbeta / dgamma partials
              const long long idx = (long long)row * ldc + col;
              float dz = bf2f(vb);
              if (a.bnf_y && !(bf2f(a.bnf_y[idx]) > 0.f)) {
                dz = 0.f;
                if (a.bnf_mask_out) vb = 0;
              }
              const float xh = (bf2f(a.bnf_c[idx]) - a.bnf_mean[bc]) * a.bnf_rstd[bc];
              s1 += dz;
              s2 += dz * xh;
            } else {
              s1 += v;
              s2 += v * v;
            }
            if (stage) sout[(row - m0) * LDO + (col - n0)] = vb;
            else a.out[(long long)row * ldc + col] = vb;
          }
        }
      if ((MODE == DGRAD && a.bnf_part) || (MODE == FWD && a.stats)) {
        s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      }
      k1[j] = s1;
      k2[j] = s2;
      if (MODE == FWD && a.stats && !a.stats_part) {
        if (fq == 0 && cok) {
          atomicAdd(a.stats + col, s1);
          atomicAdd(a.stats + a.N + col, s2);
        }
      } else if (rows != nullptr && fq == 0 && cok) {
        if (SINGLE) {
          store_row(rows + rrow + row_off(a, col), s1, sc1_rows);
          store_row(rows + rrow + row_off(a, col) + sq_off(a), s2, sc1_rows);
        } else if (wm == 1) {
          red[col - n0] = s1;
          red[BNT + col - n0] = s2;
        }
      }
    }
    if constexpr (!SINGLE) {
      if (stage || rows != nullptr) __syncthreads();
      if (rows != nullptr && wm == 0 && fq == 0) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int col = n0 + wn * WN + j * 16 + fr;
          if (col < a.N) {
            store_row(rows + rrow + row_off(a, col), k1[j] + red[col - n0], sc1_rows);
            store_row(rows + rrow + row_off(a, col) + sq_off(a), k2[j] + red[BNT + col - n0], sc1_rows);
          }
        }
      }
      if (stage) {
        constexpr int CPR = BNT / 8;  // 16-byte chunks per tile row
        for (int q = tid; q < BMT * CPR; q += 256) {
          const int r = q / CPR, c8 = (q - r * CPR) * 8;
          const int row = m0 + r, col = n0 + c8;
          if (row < a.M && col < a.N)
            *reinterpret_cast<uint4*>(a.out + (long long)row * ldc + col) =
                *reinterpret_cast<const uint4*>(sout + r * LDO + c8);
        }
      }
    }
    if (a.grp_out && rows != nullptr) group_reduce_rows<BMT, BNT, 1, SINGLE>(a, rows, m0, n0, tid, flag);
  }
}

template <int MODE, int BM, int BN, int BK, bool TAPU>
struct IgemmBody {
  static constexpr bool A_KC = (MODE != WGRAD);
  static constexpr bool B_KC = (MODE == FWD);
  using TA = TileShape<BM, A_KC, BK>;
  using TB = TileShape<BN, B_KC, BK>;
  static constexpr int STAGE = TA::ELEMS + TB::ELEMS;
  static constexpr int THREADS = 256;
  static constexpr int SMEM_PIPE = 2 * STAGE * (int)sizeof(bf16_t);
  static constexpr int SMEM = SMEM_PIPE;
  static_assert(MODE == WGRAD || SMEM >= 16 + 8 * BN, "epilogue BN-row scratch must fit the LDS");
  static_assert(MODE == WGRAD || BM * BN < 8192 || SMEM >= 16 + BM * (BN + 8) * 2 + 8 * BN,
                "epilogue output staging must fit the LDS");
  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem_raw);
};

template <int MODE, int BM, int BN, int BK, bool TAPU>
__device__ __forceinline__ void IgemmBody<MODE, BM, BN, BK, TAPU>::run(const ConvArgs& a, const Blk& bk,
                                                                           char* smem_raw) {
  constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  constexpr int KC = BK / 8;  // 16-byte chunks per K-contiguous row
  constexpr int PA = TA::PER_THREAD, PB = TB::PER_THREAD;
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile_m = bk.y, tile_n = bk.x;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const int kbeg = bk.z * a.kchunk;
  const int kend = min(a.Kd, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // ---- per-thread chunk generators ----
  using GA = typename std::conditional<MODE == FWD, FwdA<BK, TAPU>,
             typename std::conditional<MODE == DGRAD, typename std::conditional<TAPU, DgradA<BK>, DgradAP<BK>>::type,
                                       WgradA<BK, BM>>::type>::type;
  using GB = typename std::conditional<MODE == FWD, FwdB<BK, TAPU>,
             typename std::conditional<MODE == DGRAD, typename std::conditional<TAPU, DgradB<BK, BN>, DgradBP<BK, BN>>::type,
                                       WgradB<BK, BN>>::type>::type;
  GA ga[PA];
  GB gb[PB];
  int offA[PA], offB[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    int q = tid + i * 256;
    if (q >= TA::CHUNKS) q = TA::CHUNKS - 1;  // surplus threads duplicate the last chunk
    if constexpr (A_KC) { ga[i].init(a, m0 + q / KC, q); offA[i] = (q / KC) * (BK + PADK) + (q % KC) * 8; }
    else {
      ga[i].init(a, m0, q);
      constexpr int CPR = BM / 8;
      const int r = q / CPR, c = q % CPR;
      offA[i] = KsSwz<BM>::ON ? r * BM + ((c ^ swz_ks<BM>(r)) << 3) : r * (BM + PADR) + c * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    int q = tid + i * 256;
    if (q >= TB::CHUNKS) q = TB::CHUNKS - 1;
    if constexpr (B_KC) { gb[i].init(a, n0 + q / KC, q); offB[i] = (q / KC) * (BK + PADK) + (q % KC) * 8; }
    else {
      gb[i].init(a, n0, q);
      constexpr int CPR = BN / 8;
      const int r = q / CPR, c = q % CPR;
      offB[i] = KsSwz<BN>::ON ? r * BN + ((c ^ swz_ks<BN>(r)) << 3) : r * (BN + PADR) + c * 8;
    }
  }

  uint4 ra0[PA], rb0[PB], ra1[PA], rb1[PB];
  auto issue = [&](uint4* ra, uint4* rb, int kt) {
    const int kb = kbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < PA; ++i) ra[i] = ld16(ga[i].ptr(a, kb, kend));
#pragma unroll
    for (int i = 0; i < PB; ++i) rb[i] = ld16(gb[i].ptr(a, kb, kend));
  };
  auto stash = [&](const uint4* ra, const uint4* rb, int buf) {
    bf16_t* sA = smem + buf * STAGE;
    bf16_t* sB = sA + TA::ELEMS;
#pragma unroll
    for (int i = 0; i < PA; ++i) *reinterpret_cast<uint4*>(sA + offA[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < PB; ++i) *reinterpret_cast<uint4*>(sB + offB[i]) = rb[i];
  };
  // register stage 0 / 1 (no runtime choice between register arrays: they must stay in VGPRs)
  auto issue0 = [&](int kt) { issue(ra0, rb0, kt); };
  auto issue1 = [&](int kt) { issue(ra1, rb1, kt); };
  auto stash0 = [&](int buf) { stash(ra0, rb0, buf); };
  auto stash1 = [&](int buf) { stash(ra1, rb1, buf); };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16_t* sA = smem + buf * STAGE;
    const bf16_t* sB = sA + TA::ELEMS;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i)
        af[i] = A_KC ? frag_kcontig<BK>(sA, wm * WM + i * 16, ks, lane)
                     : frag_kstrided<BM>(sA, wm * WM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bfr[j] = B_KC ? frag_kcontig<BK>(sB, wn * WN + j * 16, ks, lane)
                      : frag_kstrided<BN>(sB, wn * WN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  if (nk > 0) {
    const int last = nk - 1;
    issue0(0);
    issue1(1);  // past-the-end K-tiles load the zero page (ptr() redirects k >= kend)
    stash0(0);
    __syncthreads();
    for (int kt = 0;; kt += 2) {
      // even half: LDS[0] holds tile kt, stage 1 holds kt+1 (in flight), stage 0 is free
      issue0(kt + 2);
      compute(0);
      stash1(1);
      __syncthreads();
      if (kt + 1 > last) break;
      // odd half: LDS[1] holds kt+1, stage 0 holds kt+2 (in flight), stage 1 is free
      issue1(kt + 3);
      compute(1);
      stash0(0);
      __syncthreads();
      if (kt + 2 > last) break;
    }
  }

  conv_epilogue<MODE, MR, NR, WM, WN, false, false, SMEM_PIPE>(a, acc, m0, n0, wm, wn, lane, tid,
                                                          tile_m * bk.gx + tile_n, bk.z,
                                                          reinterpret_cast<unsigned*>(smem));
}

// rider: an SGD range (kml_sgd.h) carried by the z-slices past the split-K slices of a WGRAD
// launch (ResNet's stem weight gradient: 416 latency-bound tiles on 256 CUs, the last kernel of
// the backward, carries the update of layers 2-3 — engine/dp.py ``ride``)
template <int MODE, int BM, int BN, int BK, bool TAPU>
__global__ __launch_bounds__(256) void k_conv_igemm(ConvArgs a, KmlSgdRider rider) {
  if (MODE == WGRAD && rider.blocks > 0 && (int)blockIdx.z >= a.splits) {
    kml_sgd_rider_run(rider, (((int)blockIdx.z - a.splits) * (int)gridDim.y + (int)blockIdx.y) * (int)gridDim.x +
                                 (int)blockIdx.x);
    return;
  }
  using Body = IgemmBody<MODE, BM, BN, BK, TAPU>;
  __shared__ __attribute__((aligned(16))) char smem[Body::SMEM];
  Body::run(a, hw_blk(), smem);
}

// =====================================================================================
// Variant 1/2: LDS-DMA pipeline (global_load_lds_dwordx4), BK = 64, S-stage LDS ring.
//
// Operands go global -> LDS directly (no VGPR staging, no compiler-inserted register
// waits); each wave issues NI = (BM+BN)/32 one-KiB DMA instructions per stage and the
// loop keeps S-2 stages in flight across raw s_barriers with a counted vmcnt.  The LDS
// image is lane-linear (the DMA writes base + 16*lane), so bank-conflict swizzles are
// applied on the per-lane SOURCE address and undone on the read (CDNA guide §5.4 rule
// 21): K-contiguous [row][64] tiles use chunk ^= row&7, K-strided [64][R] tiles a
// row-bit permutation chosen per R — all verified conflict-free by tools/lds_banks.py.
// =====================================================================================

template <int R>
__device__ __forceinline__ int swz_ks(int r) {  // K-strided [64][R] chunk swizzle
  if constexpr (R == 32) return (r >> 2) & 3;
  else if constexpr (R == 64) return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
  else return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
}

// glds fragment readers
__device__ __forceinline__ bf16x8_t gfrag_kcontig(const char* lds, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  const int c = 4 * ks + (lane >> 4);
  return *reinterpret_cast<const bf16x8_t*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
}

template <int R>
__device__ __forceinline__ bf16x8_t gfrag_kstrided(const char* lds, int row0, int ks, int lane) {
  const int il = lane & 15, g = lane >> 4;
  const int col = row0 + 4 * (il & 3);
  const int k0 = 32 * ks + 8 * g + (il >> 2);
  const int k1 = k0 + 4;
  const int ch = col >> 3, within = (col & 7) * 2;
  const char* p0 = lds + k0 * (2 * R) + ((ch ^ swz_ks<R>(k0)) << 4) + within;
  const char* p1 = lds + k1 * (2 * R) + ((ch ^ swz_ks<R>(k1)) << 4) + within;
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p0));
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p1));
  bf16x8_t f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

// Which tile row / logical chunk a lane's DMA covers in instruction u of an operand.
template <int R, bool KC>
__device__ __forceinline__ void glds_slot(int u, int lane, int& row, int& chunk) {
  if constexpr (KC) {  // [R rows][64 k] 128-byte rows, 8 rows per KiB
    row = 8 * u + (lane >> 3);
    chunk = (lane & 7) ^ (row & 7);
  } else {             // [64 k][R cols], 2R-byte rows
    constexpr int CPR = R / 8;          // 16-byte chunks per row
    constexpr int RPI = 64 / CPR;       // rows per KiB instruction
    row = RPI * u + lane / CPR;
    chunk = (lane % CPR) ^ swz_ks<R>(row);
  }
}

template <int MODE, int BM, int BN, int S, bool TAPU>
struct GldsBody {
  static constexpr int BK = 64;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int THREADS = 256;
  static constexpr int SMEM = S * STAGE;
  static_assert(MODE == WGRAD || BM * BN < 8192 || SMEM >= 16 + BM * (BN + 8) * 2 + 8 * BN,
                "epilogue output staging must fit the LDS");
  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem);
};

template <int MODE, int BM, int BN, int S, bool TAPU>
__device__ __forceinline__ void GldsBody<MODE, BM, BN, S, TAPU>::run(const ConvArgs& a, const Blk& bk, char* smem) {
  constexpr bool A_KC = (MODE != WGRAD);
  constexpr bool B_KC = (MODE == FWD);
  constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  constexpr int NA = BM / 32, NB = BN / 32;  // DMA instructions per wave per stage
  constexpr int NI = NA + NB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile_m = bk.y, tile_n = bk.x;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = bk.z * a.kchunk;
  const int kend = min(a.Kd, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  using GA = typename std::conditional<MODE == FWD, FwdA<BK, TAPU>,
             typename std::conditional<MODE == DGRAD, typename std::conditional<TAPU, DgradA<BK>, DgradAP<BK>>::type,
                                       WgradA<BK, BM>>::type>::type;
  using GB = typename std::conditional<MODE == FWD, FwdB<BK, TAPU>,
             typename std::conditional<MODE == DGRAD, typename std::conditional<TAPU, DgradB<BK, BN>, DgradBP<BK, BN>>::type,
                                       WgradB<BK, BN>>::type>::type;
  GA ga[NA];
  GB gb[NB];
  // Generators are addressed like the register-staged kernel: K-contiguous ones take
  // (row, q) with q % 8 = logical chunk; K-strided ones take q = row*CPR + chunk.
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    int row, ch;
    glds_slot<BM, A_KC>(wave * NA + j, lane, row, ch);
    if constexpr (A_KC) ga[j].init(a, m0 + row, ch);
    else ga[j].init(a, m0, row * (BM / 8) + ch);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    int row, ch;
    glds_slot<BN, B_KC>(wave * NB + j, lane, row, ch);
    if constexpr (B_KC) gb[j].init(a, n0 + row, ch);
    else gb[j].init(a, n0, row * (BN / 8) + ch);
  }

  auto issue = [&](int kt, int buf) {
    const int kb = kbeg + kt * BK;
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)ga[j].ptr(a, kb, kend),
                                       (__attribute__((address_space(3))) void*)(base + (wave * NA + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)gb[j].ptr(a, kb, kend),
                                       (__attribute__((address_space(3))) void*)(base + A_BYTES + (wave * NB + j) * 1024),
                                       16, 0, 0);
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < S - 1; ++s) issue(s, s);  // tiles past the end DMA the zero page
    int cur = 0;
    for (int t = 0; t < nk; ++t) {
      // tile t landed for this wave; S-2 younger stages may stay in flight
      if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      int nb = cur + S - 1;
      if (nb >= S) nb -= S;
      issue(t + S - 1, nb);
      const char* sA = smem + cur * STAGE;
      const char* sB = sA + A_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t af[MR], bfr[NR];
#pragma unroll
        for (int i = 0; i < MR; ++i)
          af[i] = A_KC ? gfrag_kcontig(sA, wm * WM + i * 16, ks, lane)
                       : gfrag_kstrided<BM>(sA, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          bfr[j] = B_KC ? gfrag_kcontig(sB, wn * WN + j * 16, ks, lane)
                        : gfrag_kstrided<BN>(sB, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      cur = (cur + 1 == S) ? 0 : cur + 1;
    }
  }
  // drain the (zero-page) tail DMAs before LDS is reused by the epilogue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  conv_epilogue<MODE, MR, NR, WM, WN, false, false, SMEM>(a, acc, m0, n0, wm, wn, lane, tid,
                                                          tile_m * bk.gx + tile_n, bk.z,
                                                          reinterpret_cast<unsigned*>(smem));
}

// XCD-aware tile order (CDNA guide T1): blocks b and b+8 share an XCD (round-robin
// dispatch), so hand each XCD a contiguous run of tiles, N-tiles fastest: neighbouring
// tiles share their A panel (and the B panels of a row of tiles) in that XCD's L2.
// Bijective for any grid (nwg % 8 != 0 included).
__device__ __forceinline__ Blk xcd_blk() {
  const int gx = (int)gridDim.x, gy = (int)gridDim.y;
  const int nwg = gx * gy * (int)gridDim.z;
  const int lin = ((int)blockIdx.z * gy + (int)blockIdx.y) * gx + (int)blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, x = lin & 7, k = lin >> 3;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  Blk b;
  b.gx = gx;
  b.x = id % gx;
  const int t = id / gx;
  b.y = t % gy;
  b.z = t / gy;
  return b;
}

template <int MODE, int BM, int BN, int S, bool TAPU>
__global__ __launch_bounds__(256) void k_conv_glds(ConvArgs a) {
  using Body = GldsBody<MODE, BM, BN, S, TAPU>;
  __shared__ __attribute__((aligned(1024))) char smem[Body::SMEM];
  Body::run(a, xcd_blk(), smem);
}

template <int MODE, int BM, int BN, int S>
int launch_glds(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, a.splits);
  const bool tapu = (MODE != FWD) || (a.C % 64 == 0);
  if constexpr (MODE == FWD) {
    if (g_fwd_rec) {
      *g_fwd_rec = FwdRec{tapu && a.splits == 1 ? fwd_body_id<GldsBody<FWD, BM, BN, S, true>>() : -1, a,
                          (int)grid.x, (int)grid.y, true};
      return 0;
    }
  }
  if (tapu) hipLaunchKernelGGL((k_conv_glds<MODE, BM, BN, S, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_conv_glds<MODE, BM, BN, S, false>), grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

template <int MODE, int BM, int BN, int BK>
int launch(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, a.splits);
  // a WGRAD launch takes an armed SGD-range rider (whole extra z-slices of gx * gy blocks; a
  // peer-shard slice, whose phase counts its blocks exactly, stays armed and runs alone)
  KmlSgdRider rider{};
  if constexpr (MODE == WGRAD) {
    if (g_kml_rider.blocks > 0 && g_kml_rider.kind == KML_RIDER_SGD) rider = kml_rider_take();
    if (rider.blocks > 0) {
      const int per = (int)(grid.x * grid.y);
      const int ez = (rider.blocks + per - 1) / per;
      rider.blocks = ez * per;
      grid.z += ez;
    }
  }
  // K-tile inside one tap: FWD needs Cin % BK == 0; DGRAD/WGRAD tap math is already per-tile/per-column
  const bool tapu = (MODE != FWD) || (a.C % BK == 0);
  if constexpr (MODE == FWD) {
    if (g_fwd_rec) {
      *g_fwd_rec = FwdRec{tapu && a.splits == 1 ? fwd_body_id<IgemmBody<FWD, BM, BN, BK, true>>() : -1, a,
                          (int)grid.x, (int)grid.y, true};
      return 0;
    }
  }
  if (tapu) hipLaunchKernelGGL((k_conv_igemm<MODE, BM, BN, BK, true>), grid, dim3(256), 0, s, a, rider);
  else hipLaunchKernelGGL((k_conv_igemm<MODE, BM, BN, BK, false>), grid, dim3(256), 0, s, a, rider);
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------------
// Direct (LDS-free) variant for small-M/N, deep-K layers (ResNet layer2-4 at 32x32
// input: M = 256..4096 pixels, K = 1152..4608).  Both operands of FWD and DGRAD (with
// a k-contiguous transposed weight copy) are K-contiguous, so every lane loads its MFMA
// fragments straight from global memory (16 B = 8 bf16 of one row) — no LDS staging,
// no barriers in the k-loop.  The W waves of a block split K and keep a D-deep register
// ring of in-flight fragments; partial tiles are summed through LDS once at the end and
// wave 0 runs the shared epilogue.  Replaces cross-block split-K (whose agent-scope
// release/acquire costs microseconds) with an intra-block one.
// ---------------------------------------------------------------------------------
template <int BK>
struct DgradBT {  // transposed weights wT[cin][KH*KW][Kp] (k-contiguous over cout)
  int base, koff;
  bool valid;
  __device__ void init(const ConvArgs& a, int n, int q) {
    valid = n < a.N;
    base = (valid ? n : 0) * a.KH * a.KW * a.Kp;
    koff = (q % (BK / 8)) * 8;
  }
  __device__ const bf16_t* ptr(const ConvArgs& a, int kb, int kend) const {
    const int tap = fdiv(kb, a.fd_Kp);  // uniform
    const int kk = kb - tap * a.Kp + koff;
    int r, s;
    tap_rs(a, tap, r, s);
    const bool ok = valid && kb + koff < kend && kk < a.K;
    return ok ? a.wt + base + (r * a.KW + s) * a.Kp + kk : a.zp;
  }
};

template <int MODE, int MR, int NR, int NW, int D>
struct DirectBody {
  static_assert(MODE != WGRAD, "direct variant: fwd/dgrad only");
  static constexpr int NA = MR * NR * 4;
  static constexpr int THREADS = 64 * NW;
  static constexpr int SMEM = (NW > 1 ? NW - 1 : 1) * NA * 64 * (int)sizeof(float);
  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem);
};

template <int MODE, int MR, int NR, int NW, int D>
__device__ __forceinline__ void DirectBody<MODE, MR, NR, NW, D>::run(const ConvArgs& a, const Blk& bk, char* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int m0 = bk.y * 16 * MR, n0 = bk.x * 16 * NR;
  using GA = typename std::conditional<MODE == FWD, FwdA<32, true>, DgradA<32>>::type;
  using GB = typename std::conditional<MODE == FWD, FwdB<32, true>, DgradBT<32>>::type;
  GA ga[MR];
  GB gb[NR];
#pragma unroll
  for (int i = 0; i < MR; ++i) ga[i].init(a, m0 + 16 * i + (lane & 15), g);
#pragma unroll
  for (int j = 0; j < NR; ++j) gb[j].init(a, n0 + 16 * j + (lane & 15), g);

  // each wave owns k-steps [s0, s1); its loop runs a multiple of D steps without any
  // branch (steps past s1 read the zero page via kend), so the compiler can keep the
  // D-deep ring of loads in flight with counted vmcnt waits across iterations
  const int nst = (a.Kd + 31) / 32;
  const int per = (nst + NW - 1) / NW;
  const int s0 = wave * per, s1 = min(nst, s0 + per);
  const int kend = max(0, min(a.Kd, s1 * 32));
  const int nloop = (max(s1 - s0, 0) + D - 1) / D;
  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t ra[D][MR], rb[D][NR];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int kb = (s0 + d) * 32;
#pragma unroll
    for (int i = 0; i < MR; ++i) ra[d][i] = *reinterpret_cast<const bf16x8_t*>(ga[i].ptr(a, kb, kend));
#pragma unroll
    for (int j = 0; j < NR; ++j) rb[d][j] = *reinterpret_cast<const bf16x8_t*>(gb[j].ptr(a, kb, kend));
  }
  int kb_next = (s0 + D) * 32;
  for (int it = 0; it < nloop; ++it) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[d][i], rb[d][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < MR; ++i) ra[d][i] = *reinterpret_cast<const bf16x8_t*>(ga[i].ptr(a, kb_next, kend));
#pragma unroll
      for (int j = 0; j < NR; ++j) rb[d][j] = *reinterpret_cast<const bf16x8_t*>(gb[j].ptr(a, kb_next, kend));
      kb_next += 32;
    }
  }
  // intra-block reduction of the NW partial tiles
  float* red = reinterpret_cast<float*>(smem);
  if (NW > 1) {
    if (wave > 0) {
      float4* dst = reinterpret_cast<float4*>(red + (wave - 1) * NA * 64) + lane;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          dst[(i * NR + j) * 64] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    __syncthreads();
    if (wave > 0) return;
    for (int w = 1; w < NW; ++w) {
      const float4* src = reinterpret_cast<const float4*>(red + (w - 1) * NA * 64) + lane;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const float4 v = src[(i * NR + j) * 64];
          acc[i][j][0] += v.x; acc[i][j][1] += v.y; acc[i][j][2] += v.z; acc[i][j][3] += v.w;
        }
    }
  }
  conv_epilogue<MODE, MR, NR, 16 * MR, 16 * NR, true>(a, acc, m0, n0, 0, 0, lane, lane, 0, 0, nullptr);
}

template <int MODE, int MR, int NR, int NW, int D>
__global__ __launch_bounds__(64 * NW) void k_conv_direct(ConvArgs a) {
  using Body = DirectBody<MODE, MR, NR, NW, D>;
  __shared__ __attribute__((aligned(16))) char smem[Body::SMEM];
  Body::run(a, hw_blk(), smem);
}

template <int MODE, int MR, int NR, int NW>
int launch_direct(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.N + 16 * NR - 1) / (16 * NR), (a.M + 16 * MR - 1) / (16 * MR), 1);
  // ring depth: keep ~16 fragment loads per lane in flight
  constexpr int D = (MR + NR) <= 2 ? 8 : ((MR + NR) <= 4 ? 4 : 2);
  if constexpr (MODE == FWD) {
    if (g_fwd_rec) {
      *g_fwd_rec = FwdRec{NW == 4 ? fwd_body_id<DirectBody<FWD, MR, NR, NW, D>>() : -1, a, (int)grid.x, (int)grid.y,
                          true};
      return 0;
    }
  }
  hipLaunchKernelGGL((k_conv_direct<MODE, MR, NR, NW, D>), grid, dim3(64 * NW), 0, s, a);
  KML_LAUNCH_CHECK();
}

template <int MODE>
int dispatch_direct(const ConvArgs& a, int bm, int bn, int nw, hipStream_t s) {
#define KML_D(BMv, BNv)                                                                   \
  if (bm == BMv && bn == BNv) {                                                           \
    if (nw == 8) return launch_direct<MODE, BMv / 16, BNv / 16, 8>(a, s);               \
    return launch_direct<MODE, BMv / 16, BNv / 16, 4>(a, s);                            \
  }
  KML_D(16, 16) KML_D(16, 32) KML_D(32, 16) KML_D(32, 32) KML_D(32, 64) KML_D(64, 32) KML_D(64, 64)
#undef KML_D
  return (int)hipErrorInvalidValue;
}

// wT[c][t][k] = w[k][t][c] (k < K), 0 for K <= k < Kp   (t = tap index r*KW + s)
__global__ void k_weight_transpose(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, int K, int T, int C,
                                   int Kp) {
  const long long total = (long long)C * T * Kp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % Kp);
    const long long ct = i / Kp;
    const int t = (int)(ct % T), c = (int)(ct / T);
    wt[i] = k < K ? w[((long long)k * T + t) * C + c] : (bf16_t)0;
  }
}

// =====================================================================================
// Variant 4: halo-patch forward for 3x3 / stride 1 / pad 1 convolutions on small maps.
//
// The implicit-GEMM kernels above stage im2col(X) tiles: every input pixel passes through
// LDS once per filter tap (9x the activation bytes), plus a weight panel per M-tile.  On
// ResNet-34's 8x8 / 4x4 layers that traffic, not the MFMA, bounds them (47-55 MB through
// the CU's L2->LDS path per call, profiles/resnet34_bench_r3.md).  Here a block owns IMG
// whole images: their zero-padded (HW+2)^2 x C patches are staged into LDS ONCE and the 9
// taps are LDS address offsets; the weights never touch LDS — each lane streams its MFMA B
// fragments (16 B = 8 consecutive k of one output channel, K-contiguous KRSC) straight from
// L2 into registers, D K-steps ahead.  Per block: IMG*(HW)^2*C*2 activation bytes + a BN x 9C
// weight slice (shared by the two waves of a column through L1), instead of
// 9*BM*C*2 + BN*9C*2 through LDS.
//
// Waves: 2x2, each (BM/2) x (BN/2) of v_mfma_f32_16x16x32_bf16 fragments.  Patch pixels are
// C*2-byte rows of 16-byte chunks, chunk XOR (pixel & SWZ): a fragment read (16 rows x 4
// chunks) touches every bank group once for consecutive pixels.  The epilogue is the shared
// conv_epilogue (BN statistics partial rows per M-tile, bias/ReLU, bf16 store).
// =====================================================================================
// MODE = FWD : A = patch of x (C = Cin channels), B[n = cout][k = (tap, cin)] = w rows.
// MODE = DGRAD: A = patch of dy (C = Cout channels), B[n = cin][k = (tap', cout)] =
//               w[cout][8 - tap'][cin] (stride 1 / pad 1: dX is the correlation of the padded dY
//               with the flipped filter).  Its weight slice is staged K-strided ([k][BN], one
//               16-byte chunk = 8 cin of one (cout, tap)) and read with ds_read_b64_tr_b16.
template <int MODE, int C, int HW, int IMG, int BN, int D>
struct HaloBody {
  static constexpr int HP = HW + 2;              // padded patch side
  static constexpr int CH = C / 8;               // 16-byte chunks per patch pixel
  // patch row pitch (pixels) and chunk swizzle, chosen with tools/lds_banks.py's model of
  // ds_read_b128 lane groups over every (tap, fragment, k-chunk) read of the main loop:
  // pitch 16 on 8x8 maps is conflict-free at C = 64; pixel*13 on 4x4 maps (pitch 8) leaves
  // 1/3 of the reads 2-way instead of all of them with the natural pitch.
  static constexpr int PITCH0 = HW == 8 ? 16 : 8;
  static constexpr int PITCH = IMG * HP * PITCH0 * C * 2 <= 96 * 1024 ? PITCH0 : HP;
  static constexpr int IMGPIX = HP * PITCH;      // patch pixels per image (incl. unused pitch)
  static constexpr int PIX = IMG * IMGPIX;
  static constexpr int SWZ = CH >= 16 ? 15 : 7;  // chunk swizzle mask
  static constexpr int BM = IMG * HW * HW;
  static constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  static constexpr int KS = 9 * C / 32;          // 32-deep K-steps (tap-major, channel-minor)
  static constexpr int WCH = 9 * CH;             // FWD: 16-byte chunks per weight row
  static constexpr int SMEM_PATCH = PIX * C * 2;
  static constexpr int SMEM_W = BN * 9 * C * 2;  // the block's whole weight slice
  // weights staged in LDS with the patch when both fit (coalesced loads, 4x fewer L2 requests
  // than per-fragment row segments); otherwise (FWD only) streamed into registers
  static constexpr bool WLDS = MODE == DGRAD || SMEM_PATCH + SMEM_W <= 128 * 1024;
  static constexpr int SMEM_EPI = 16 + BM * (BN + 8) * 2 + 2 * BN * 4;
  static constexpr int SMEM_BN = MODE == FWD ? (4 * C + 4 * 256) * 4 : 0;  // scale, shift, sums, scratch
  static constexpr int SMEM_MAIN = SMEM_PATCH + (WLDS ? SMEM_W : 0) + SMEM_BN;
  static constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __device__ __forceinline__ static int swz(int pix) {
    // 4x4 maps at pitch 8 (pixel = 8 y + x inside an image of 48 patch pixels): 2x + 8y spreads
    // every read group over 16 distinct chunks (tools/lds_banks.py model: 1.33 -> 1.0 cycles per
    // ds_read_b128; measured 14 % conflicts in profiles/r6/final/r34_pmc.md); pixel * 13 for
    // the pitch-6 layouts
    if constexpr (HW == 4 && PITCH == 8) return (2 * (pix & 7) + (pix & 8)) & SWZ;
    const int h = (HW == 8) ? (C == 64 ? pix : pix * 9) : pix * 13;
    return h & SWZ;
  }
  static_assert(MODE == FWD || MODE == DGRAD, "halo: fwd / dgrad");
  static_assert(BM % 32 == 0 && BN % 32 == 0 && C % 32 == 0, "halo tile shape");
  static_assert(MODE == FWD || BN == 32 || BN == 64, "dgrad halo: K-strided tile of 32 or 64 columns");
  static_assert(SMEM <= 160 * 1024, "halo working set exceeds LDS");
  static constexpr int THREADS = 256;
  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem);
};

template <int MODE, int C, int HW, int IMG, int BN, int D>
__device__ __forceinline__ void HaloBody<MODE, C, HW, IMG, BN, D>::run(const ConvArgs& a, const Blk& bk, char* smem) {
  using P = HaloBody<MODE, C, HW, IMG, BN, D>;
  constexpr int MR = P::MR, NR = P::NR, KS = P::KS, CH = P::CH, HP = P::HP, PITCH = P::PITCH;
  constexpr bool WL = P::WLDS;
  char* const swt = smem + P::SMEM_PATCH;  // weight slice (WLDS)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int m0 = bk.y * P::BM, n0 = bk.x * BN, img0 = bk.y * IMG;
  const bf16_t* const src = (MODE == FWD) ? a.x : a.dy;   // patch source, C channels

  // folded input BN: the first 16 statistics rows of this thread's slice are requested before
  // anything else, so their round trip overlaps the weight / patch loads (vmcnt retires in
  // issue order: rows issued after the patch would wait for it)
  constexpr int BQ = 2 * C / 4, BS = 256 / BQ;   // float4 columns of a statistics row, row slices
  float4 brow_early[16];
  const bool bnin = MODE == FWD && a.ibn_rows != nullptr;
  if constexpr (MODE == FWD) {
    if (bnin && tid / BQ < BS) {
      const float4* p4 = reinterpret_cast<const float4*>(a.ibn_rows) + tid % BQ;
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) brow_early[uu] = p4[(long long)min(tid / BQ + uu * BS, a.ibn_G - 1) * BQ];
    }
  }

  // weights first (FWD register stream: D K-steps of B fragments; otherwise the block's whole
  // slice), in flight while the patch loads are issued
  const bf16_t* wp[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j)
    wp[j] = a.w + (long long)(n0 + wn * P::WN + j * 16 + (lane & 15)) * (9 * C) + 8 * (lane >> 4);
  constexpr int DD = WL ? 1 : D;
  bf16x8_t bq[DD][NR];
  constexpr int WCHUNKS = BN * 9 * C / 8;
  constexpr int WPER = WL ? (WCHUNKS + 255) / 256 : 1;
  uint4 wv[WPER];
  if constexpr (WL) {
#pragma unroll
    for (int u = 0; u < WPER; ++u) {
      const int q = tid + u * 256;
      const int qq = q < WCHUNKS ? q : 0;
      const bf16_t* p;
      if constexpr (MODE == FWD) {  // contiguous [n0, n0+BN) x 9C slice
        p = a.w + (long long)n0 * (9 * C) + qq * 8;
      } else {                      // chunk q = (row (cout, tap), cin chunk): w[cout][tap][n0 + 8c ..]
        const int row = qq / (BN / 8), c = qq - row * (BN / 8);
        p = a.w + (long long)row * a.C + n0 + c * 8;
      }
      wv[u] = ld16(q < WCHUNKS ? p : a.zp);
    }
  } else {
#pragma unroll
    for (int d = 0; d < DD; ++d)
#pragma unroll
      for (int j = 0; j < NR; ++j) bq[d][j] = *reinterpret_cast<const bf16x8_t*>(wp[j] + d * 32);
  }

  // zero-padded patches of images img0 .. img0+IMG-1 (images past B read the zero page)
  constexpr int CHUNKS = IMG * HP * HP * CH;
  constexpr int PER = (CHUNKS + 255) / 256;
  uint4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + u * 256;
    const int qq = q < CHUNKS ? q : 0;
    const int pix = qq / CH, ch = qq - pix * CH;
    const int im = pix / (HP * HP), rem = pix - im * (HP * HP);
    const int ih = rem / HP - 1, iw = rem - (rem / HP) * HP - 1;
    const bool in = q < CHUNKS && (unsigned)ih < (unsigned)HW && (unsigned)iw < (unsigned)HW && img0 + im < a.B;
    v[u] = ld16(in ? src + (((long long)(img0 + im) * HW + ih) * HW + iw) * C + ch * 8 : a.zp);
  }
  // folded BN with a residual (addend in FWD): y = relu(bn(c) + res), res chunks beside the patch's
  uint4 rv[MODE == FWD ? PER : 1];
  const bool bres = MODE == FWD && bnin && a.addend != nullptr;
  if constexpr (MODE == FWD) {
    if (bres) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int q = tid + u * 256;
        const int qq = q < CHUNKS ? q : 0;
        const int pix = qq / CH, ch = qq - pix * CH;
        const int im = pix / (HP * HP), rem = pix - im * (HP * HP);
        const int ih = rem / HP - 1, iw = rem - (rem / HP) * HP - 1;
        const bool in = q < CHUNKS && (unsigned)ih < (unsigned)HW && (unsigned)iw < (unsigned)HW && img0 + im < a.B;
        rv[u] = ld16(in ? a.addend + (((long long)(img0 + im) * HW + ih) * HW + iw) * C + ch * 8 : a.zp);
      }
    }
  }
  if constexpr (WL) {
#pragma unroll
    for (int u = 0; u < WPER; ++u) {
      const int q = tid + u * 256;
      if (q < WCHUNKS) {
        if constexpr (MODE == FWD) {
          const int n = q / P::WCH, c = q - n * P::WCH;
          *reinterpret_cast<uint4*>(swt + (n * P::WCH + (c ^ (n & P::SWZ))) * 16) = wv[u];
        } else {  // LDS row k = (8 - tap) * C + cout, K-strided swizzled chunk
          const int row = q / (BN / 8), c = q - row * (BN / 8);
          const int cout = row / 9, tap = row - cout * 9;
          const int k = (8 - tap) * C + cout;
          *reinterpret_cast<uint4*>(swt + (k * BN + ((c ^ swz_ks<BN>(k)) << 3)) * 2) = wv[u];
        }
      }
    }
  }
  if constexpr (MODE == FWD) {
    if (a.ibn_rows) {  // the input's BatchNorm (training statistics) + ReLU, applied here
      float* bsc = reinterpret_cast<float*>(smem + P::SMEM_MAIN - P::SMEM_BN);
      float* bsf = bsc + C;
      float* sums = bsf + C;
      float4* scratch = reinterpret_cast<float4*>(sums + 2 * C);
      constexpr int Q = BQ, S = BS;
      const int q = tid % Q, sl = tid / Q;
      float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (sl < S) {  // rows sl, sl + S, ... in order (the BN apply kernel's summation order)
        const float4* p4 = reinterpret_cast<const float4*>(a.ibn_rows) + q;
#pragma unroll
        for (int uu = 0; uu < 16; ++uu) {
          const bool in = sl + uu * S < a.ibn_G;
          acc4.x += in ? brow_early[uu].x : 0.f; acc4.y += in ? brow_early[uu].y : 0.f;
          acc4.z += in ? brow_early[uu].z : 0.f; acc4.w += in ? brow_early[uu].w : 0.f;
        }
        for (int g = sl + 16 * S; g < a.ibn_G; g += 16 * S) {
          float4 rv[16];
#pragma unroll
          for (int uu = 0; uu < 16; ++uu) rv[uu] = p4[(long long)min(g + uu * S, a.ibn_G - 1) * Q];
#pragma unroll
          for (int uu = 0; uu < 16; ++uu) {
            const bool in = g + uu * S < a.ibn_G;
            acc4.x += in ? rv[uu].x : 0.f; acc4.y += in ? rv[uu].y : 0.f;
            acc4.z += in ? rv[uu].z : 0.f; acc4.w += in ? rv[uu].w : 0.f;
          }
        }
      }
      scratch[tid] = acc4;
      __syncthreads();
      if (tid < Q) {
        float4 t4 = scratch[tid];
        for (int k = 1; k < S; ++k) {
          const float4 w4 = scratch[k * Q + tid];
          t4.x += w4.x; t4.y += w4.y; t4.z += w4.z; t4.w += w4.w;
        }
        reinterpret_cast<float4*>(sums)[tid] = t4;
      }
      __syncthreads();
      for (int c = tid; c < C; c += 256) {
        const float mean = sums[c] / (float)a.ibn_M;
        const float var = fmaxf(sums[C + c] / (float)a.ibn_M - mean * mean, 0.f);
        const float rstd = rsqrtf(var + a.ibn_eps);
        const float g = a.ibn_gamma ? a.ibn_gamma[c] : 1.f, bb = a.ibn_beta ? a.ibn_beta[c] : 0.f;
        bsc[c] = g * rstd;
        bsf[c] = bb - mean * g * rstd;
        if (bk.x == 0 && bk.y == 0) {
          if (a.ibn_mean) { a.ibn_mean[c] = mean; a.ibn_rstd[c] = rstd; }
          if (a.ibn_rmean) {
            const float unb = a.ibn_M > 1 ? var * (float)a.ibn_M / (float)(a.ibn_M - 1) : var;
            a.ibn_rmean[c] = (1.f - a.ibn_mom) * a.ibn_rmean[c] + a.ibn_mom * mean;
            a.ibn_rvar[c] = (1.f - a.ibn_mom) * a.ibn_rvar[c] + a.ibn_mom * unb;
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int q2 = tid + u * 256;
        if (q2 < CHUNKS) {
          const int pix = q2 / CH, ch = q2 - pix * CH;
          const int im = pix / (HP * HP), rem = pix - im * (HP * HP);
          const int ih = rem / HP - 1, iw = rem - (rem / HP) * HP - 1;
          if ((unsigned)ih < (unsigned)HW && (unsigned)iw < (unsigned)HW && img0 + im < a.B) {
            float f[8];
            const unsigned* wv32 = reinterpret_cast<const unsigned*>(&v[u]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              f[2 * k] = bf2f((bf16_t)(wv32[k] & 0xffffu));
              f[2 * k + 1] = bf2f((bf16_t)(wv32[k] >> 16));
            }
            unsigned o32[4];
            const unsigned r32[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int c0 = ch * 8 + 2 * k;
              float lo = f[2 * k] * bsc[c0] + bsf[c0];      // the BN apply kernel's order:
              float hi = f[2 * k + 1] * bsc[c0 + 1] + bsf[c0 + 1];   // scale-shift, + res, ReLU
              if (bres) { lo += lo_bf(r32[k]); hi += hi_bf(r32[k]); }
              o32[k] = pack_bf2(fmaxf(lo, 0.f), fmaxf(hi, 0.f));
            }
            v[u] = make_uint4(o32[0], o32[1], o32[2], o32[3]);
            if (bk.x == 0)
              *reinterpret_cast<uint4*>(a.ibn_y + (((long long)(img0 + im) * HW + ih) * HW + iw) * C + ch * 8) = v[u];
          }
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + u * 256;
    if (q < CHUNKS) {
      const int pix = q / CH, ch = q - pix * CH;
      const int im = pix / (HP * HP), rem = pix - im * (HP * HP);
      const int lp = im * P::IMGPIX + (rem / HP) * PITCH + (rem - (rem / HP) * HP);
      *reinterpret_cast<uint4*>(smem + (lp * CH + (ch ^ P::swz(lp))) * 16) = v[u];
    }
  }
  __syncthreads();

  // patch pixel of tap (0,0) for each A row this lane feeds
  int abase[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int r = wm * P::WM + i * 16 + (lane & 15);
    const int im = r / (HW * HW), p = r - im * (HW * HW);
    abase[i] = im * P::IMGPIX + (p / HW) * PITCH + (p % HW);
  }
  // FWD weight-slice row of each B fragment this lane feeds (WLDS)
  int brow[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) brow[j] = wn * P::WN + j * 16 + (lane & 15);
  auto read_ab = [&](int ks, bf16x8_t (&af)[MR], bf16x8_t (&bf)[NR]) {
    const int tap = ks / (C / 32);
    const int toff = (tap / 3) * PITCH + (tap % 3);
    const int chunk = (ks % (C / 32)) * 4 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int pix = abase[i] + toff;
      af[i] = *reinterpret_cast<const bf16x8_t*>(smem + (pix * CH + (chunk ^ P::swz(pix))) * 16);
    }
    if constexpr (WL && MODE == FWD) {
      const int wc = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bf[j] = *reinterpret_cast<const bf16x8_t*>(swt + (brow[j] * P::WCH + (wc ^ (brow[j] & P::SWZ))) * 16);
    } else if constexpr (MODE == DGRAD) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bf[j] = frag_kstrided<BN>(reinterpret_cast<const bf16_t*>(swt), wn * P::WN + j * 16, ks, lane);
    }
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // LDS fragments one K-step ahead (the MFMAs of step ks never wait on its LDS reads)
  bf16x8_t af[2][MR], bl[2][NR];
  read_ab(0, af[0], bl[0]);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 1 < KS) read_ab(ks + 1, af[(ks + 1) & 1], bl[(ks + 1) & 1]);
    bf16x8_t bf[NR];
    if constexpr (WL) {
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[j] = bl[ks & 1][j];
    } else {
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[j] = bq[ks % DD][j];
      if (ks + DD < KS) {
#pragma unroll
        for (int j = 0; j < NR; ++j) bq[ks % DD][j] = *reinterpret_cast<const bf16x8_t*>(wp[j] + (ks + DD) * 32);
      }
    }
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bf[j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // LDS is reused by the epilogue
  conv_epilogue<MODE, MR, NR, P::WM, P::WN, false, true>(a, acc, m0, n0, wm, wn, lane, tid, 0, 0,
                                                         reinterpret_cast<unsigned*>(smem));
}

template <int MODE, int C, int HW, int IMG, int BN, int D>
__global__ __launch_bounds__(256) void k_conv_halo(ConvArgs a) {
  using Body = HaloBody<MODE, C, HW, IMG, BN, D>;
  __shared__ __attribute__((aligned(16))) char smem[Body::SMEM];
  Body::run(a, xcd_blk(), smem);
}

template <int MODE, int C, int HW, int IMG, int BN>
int launch_halo(const ConvArgs& a, hipStream_t s) {
  using P = HaloBody<MODE, C, HW, IMG, BN, 1>;
  constexpr int D = P::NR >= 4 ? 4 : (P::NR == 2 ? 8 : 12);
  dim3 grid(a.N / BN, (a.M + P::BM - 1) / P::BM, 1);
  hipLaunchKernelGGL((k_conv_halo<MODE, C, HW, IMG, BN, D>), grid, dim3(256), 0, s, a);
  KML_LAUNCH_CHECK();
}

// bm = pixels per block (IMG whole images), bn = output channels per block
bool halo_shape_ok(int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, int bm, int bn) {
  return KH == 3 && KW == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && H == W && bn > 0 && K % bn == 0 &&
         bm % (H * W) == 0;
}

// FWD: a.C = patch channels (Cin), N = Cout.  DGRAD: a.K = patch channels (Cout), N = Cin.
template <int MODE>
int dispatch_halo(const ConvArgs& a, int bm, int bn, hipStream_t s) {
  const int cp = MODE == FWD ? a.C : a.K;
#define KML_H(Cv, HWv, BMv, BNv)                                                   \
  if (cp == Cv && a.H == HWv && bm == BMv && bn == BNv)                            \
    return launch_halo<MODE, Cv, HWv, BMv / (HWv * HWv), BNv>(a, s);
  if constexpr (MODE == FWD) {
    KML_H(64, 8, 64, 64) KML_H(64, 8, 128, 64) KML_H(64, 8, 64, 32)
    KML_H(128, 4, 64, 32) KML_H(128, 4, 64, 64) KML_H(128, 4, 128, 32) KML_H(128, 4, 64, 128) KML_H(128, 4, 128, 64)
    KML_H(256, 4, 64, 32) KML_H(256, 4, 64, 64) KML_H(256, 8, 64, 32) KML_H(256, 8, 64, 64)
    KML_H(512, 4, 64, 32) KML_H(512, 4, 64, 64)
  } else {
    KML_H(64, 8, 64, 32) KML_H(64, 8, 64, 64) KML_H(64, 8, 128, 64)
    KML_H(128, 4, 64, 32)
  }
#undef KML_H
  return (int)hipErrorInvalidValue;
}

// =====================================================================================
// Variant 5: one-shot panels for single-tap forward GEMMs with a short K (1x1-form convs:
// ResNet-34's unrolled 2x2-map layer3 convs, K = 4C = 1024, and layer4's centre-tap convs
// on 1x1 maps, K = 512).  The implicit-GEMM pipelines keep 2-3 BK=64 stages in flight per
// block, so a K = 1024 panel pair is 16 dependent round trips; here every byte of the block's
// A (BM x K) and B (BN x K) panels is requested at once by LDS-DMA (global_load_lds, no VGPR
// staging; the chunk swizzle is applied on the per-lane SOURCE address because the DMA image
// is lane-linear), one wait, one barrier, then the MFMA loop runs out of LDS.  Rows are
// 2K-byte pitched, so the swizzle is chunk ^ (row & 15) (conflict-free ds_read_b128 over a
// fragment's 16 rows x 4 chunks).  The unrolled convs' B rows are gathered from the 3x3
// weight (g22) per 16-byte chunk.
// =====================================================================================
template <int BM, int BN, int KD>
struct OneShotBody {
  static constexpr int CPR = KD / 8;                    // 16-byte chunks per panel row
  static constexpr int A_BYTES = BM * KD * 2, B_BYTES = BN * KD * 2;
  static constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  static constexpr int NIA = BM * CPR / 64, NIB = BN * CPR / 64;  // 1 KiB DMA instructions per panel
  static constexpr int SMEM_EPI = 16 + BM * (BN + 8) * 2 + 2 * BN * 4;
  static constexpr int SMEM_PANELS = A_BYTES + B_BYTES > SMEM_EPI ? A_BYTES + B_BYTES : SMEM_EPI;
  static constexpr int SMEM = SMEM_PANELS;
  static constexpr int THREADS = 256;
  static_assert(CPR % 16 == 0 && NIA % 4 == 0 && NIB % 4 == 0, "one-shot panel shape");
  static_assert(SMEM <= 160 * 1024, "one-shot panels exceed LDS");
  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int m0 = bk.y * BM, n0 = bk.x * BN;
    const int tapoff = (a.r0 * a.KW + a.s0) * a.C;
#pragma unroll
    for (int j = 0; j < NIA / 4; ++j) {
      const int u = j * 4 + wave;
      const int L = u * 64 + lane, row = L / CPR, lc = (L % CPR) ^ (row & 15);
      const int m = m0 + row;
      const bf16_t* src = m < a.M ? a.x + (long long)m * a.C + lc * 8 : a.zp;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(smem + u * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NIB / 4; ++j) {
      const int u = j * 4 + wave;
      const int L = u * 64 + lane, row = L / CPR, lc = (L % CPR) ^ (row & 15);
      const int n = n0 + row, k = lc * 8;
      const bf16_t* src = a.zp;
      if (n < a.N) {
        if (a.g22) {  // W'[(p, n')][(q, c)] = w[n'][tap(p, q)][c]
          const int p = fdiv(n, a.fd_gK), q = fdiv(k, a.fd_gC);
          src = a.w + ((long long)(n - p * a.fd_gK.d) * 9 + tap22(p, q)) * a.fd_gC.d + (k - q * a.fd_gC.d);
        } else {
          src = a.w + (long long)n * a.KH * a.KW * a.C + tapoff + k;
        }
      }
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + A_BYTES + u * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* sA = smem;
    const char* sB = smem + A_BYTES;
    auto rd = [&](const char* base, int row, int ks) {
      const int c = 4 * ks + (lane >> 4);
      return *reinterpret_cast<const bf16x8_t*>(base + (row * CPR + (c ^ (row & 15))) * 16);
    };
    f32x4_t acc[MR][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int KS = KD / 32;
    bf16x8_t af[2][MR], bf[2][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i) af[0][i] = rd(sA, wm * WM + i * 16 + (lane & 15), 0);
#pragma unroll
    for (int j = 0; j < NR; ++j) bf[0][j] = rd(sB, wn * WN + j * 16 + (lane & 15), 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int i = 0; i < MR; ++i) af[(ks + 1) & 1][i] = rd(sA, wm * WM + i * 16 + (lane & 15), ks + 1);
#pragma unroll
        for (int j = 0; j < NR; ++j) bf[(ks + 1) & 1][j] = rd(sB, wn * WN + j * 16 + (lane & 15), ks + 1);
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bf[ks & 1][j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // LDS is reused by the epilogue
    conv_epilogue<FWD, MR, NR, WM, WN, false, true>(a, acc, m0, n0, wm, wn, lane, tid, 0, 0,
                                                    reinterpret_cast<unsigned*>(smem));
  }
};

// One-shot backward bodies for the same single-tap convs.  K-strided operands (the dgrad
// weight W'[k][c] read along k for a fixed c; both wgrad operands, read along the pixel axis)
// are staged as [K rows][R cols] tiles with the K-strided XOR swizzle (swz_ks, applied on the
// DMA source address) and read with ds_read_b64_tr_b16 (frag_kstrided).
//   DGRAD: dX[m][c] = sum_k dY[m][k] W'[k][c]   (A = dY rows, K = Cout)
//   WGRAD: dW'[k][c] = sum_m dY[m][k] X[m][c]   (K = pixels; both panels K-strided)
template <int MODE, int BM, int BN, int KD>
struct OneShotBwdBody {
  static_assert(MODE == DGRAD || MODE == WGRAD, "one-shot backward: dgrad / wgrad");
  static constexpr bool A_KC = MODE == DGRAD;             // A K-contiguous (dY rows) or K-strided
  static constexpr int A_BYTES = BM * KD * 2, B_BYTES = BN * KD * 2;
  static constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  static constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024;
  static constexpr int SMEM_EPI = 16 + BM * (BN + 8) * 2 + 2 * BN * 4;
  static constexpr int SMEM = A_BYTES + B_BYTES > SMEM_EPI ? A_BYTES + B_BYTES : SMEM_EPI;
  static constexpr int THREADS = 256;
  static_assert(NIA % 4 == 0 && NIB % 4 == 0 && (KD / 8) % 16 == 0, "one-shot panel shape");
  static_assert((BM == 32 || BM == 64) && (BN == 32 || BN == 64), "K-strided tiles of 32 / 64 columns");
  static_assert(SMEM <= 160 * 1024, "one-shot panels exceed LDS");

  // one 16-byte chunk of a K-strided [KD][R] tile: DMA slot L -> (k row, logical chunk)
  template <int R>
  __device__ __forceinline__ static void ks_slot(int L, int& k, int& lc) {
    k = L / (R / 8);
    lc = (L % (R / 8)) ^ swz_ks<R>(k);
  }

  __device__ __forceinline__ static void run(const ConvArgs& a, const Blk& bk, char* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int m0 = bk.y * BM, n0 = bk.x * BN;
    const int tapoff = (a.r0 * a.KW + a.s0) * a.C;
    char* const sA = smem;
    char* const sB = smem + A_BYTES;
#pragma unroll
    for (int j = 0; j < NIA / 4; ++j) {
      const int u = j * 4 + wave, L = u * 64 + lane;
      const bf16_t* src;
      if constexpr (MODE == DGRAD) {  // dY rows [BM][KD], chunk ^ (row & 15)
        const int row = L / (KD / 8), lc = (L % (KD / 8)) ^ (row & 15), m = m0 + row;
        src = m < a.M ? a.dy + (long long)m * a.K + lc * 8 : a.zp;
      } else {                        // dY as [KD pixels][BM out-channels]
        int k, lc;
        ks_slot<BM>(L, k, lc);
        const int col = m0 + lc * 8;
        src = (k < a.Kd && col < a.M) ? a.dy + (long long)k * a.K + col : a.zp;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(sA + u * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NIB / 4; ++j) {
      const int u = j * 4 + wave, L = u * 64 + lane;
      int k, lc;
      ks_slot<BN>(L, k, lc);
      const int col = n0 + lc * 8;
      const bf16_t* src = a.zp;
      if constexpr (MODE == DGRAD) {  // W'[k][col]: k = output channel, col = input channel
        if (k < a.K && col < a.N) {
          if (a.g22) {
            const int p = fdiv(k, a.fd_gK), q = fdiv(col, a.fd_gC);
            src = a.w + ((long long)(k - p * a.fd_gK.d) * 9 + tap22(p, q)) * a.fd_gC.d + (col - q * a.fd_gC.d);
          } else {
            src = a.w + (long long)k * a.KH * a.KW * a.C + tapoff + col;
          }
        }
      } else {                        // X as [KD pixels][BN in-channels]
        if (k < a.Kd && col < a.N) src = a.x + (long long)k * a.C + col;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(sB + u * 1024),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    auto rdA = [&](int i, int ks) -> bf16x8_t {
      if constexpr (A_KC) {
        const int row = wm * WM + i * 16 + (lane & 15), c = 4 * ks + (lane >> 4);
        return *reinterpret_cast<const bf16x8_t*>(sA + (row * (KD / 8) + (c ^ (row & 15))) * 16);
      } else {
        return frag_kstrided<BM>(reinterpret_cast<const bf16_t*>(sA), wm * WM + i * 16, ks, lane);
      }
    };
    auto rdB = [&](int j, int ks) -> bf16x8_t {
      return frag_kstrided<BN>(reinterpret_cast<const bf16_t*>(sB), wn * WN + j * 16, ks, lane);
    };
    f32x4_t acc[MR][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int KS = KD / 32;
    bf16x8_t af[2][MR], bf[2][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i) af[0][i] = rdA(i, 0);
#pragma unroll
    for (int j = 0; j < NR; ++j) bf[0][j] = rdB(j, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int i = 0; i < MR; ++i) af[(ks + 1) & 1][i] = rdA(i, ks + 1);
#pragma unroll
        for (int j = 0; j < NR; ++j) bf[(ks + 1) & 1][j] = rdB(j, ks + 1);
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bf[ks & 1][j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // LDS is reused by the epilogue
    conv_epilogue<MODE, MR, NR, WM, WN, false, true>(a, acc, m0, n0, wm, wn, lane, tid, 0, 0,
                                                     reinterpret_cast<unsigned*>(smem));
  }
};

template <int MODE, int BM, int BN, int KD>
__global__ __launch_bounds__(256) void k_conv_oneshot_bwd(ConvArgs a) {
  using Body = OneShotBwdBody<MODE, BM, BN, KD>;
  __shared__ __attribute__((aligned(1024))) char smem[Body::SMEM];
  Body::run(a, xcd_blk(), smem);
}

template <int MODE>
int dispatch_oneshot_bwd(const ConvArgs& a, int bm, int bn, hipStream_t s) {
  dim3 grid((a.N + bn - 1) / bn, (a.M + bm - 1) / bm, 1);
#define KML_OB(BMv, BNv, KDv)                                                              \
  if (bm == BMv && bn == BNv && a.Kd == KDv) {                                             \
    hipLaunchKernelGGL((k_conv_oneshot_bwd<MODE, BMv, BNv, KDv>), grid, dim3(256), 0, s, a); \
    KML_LAUNCH_CHECK();                                                                    \
  }
  if constexpr (MODE == DGRAD) {
    KML_OB(32, 32, 1024) KML_OB(32, 32, 512) KML_OB(32, 64, 512)
  } else {
    KML_OB(32, 32, 256) KML_OB(64, 32, 256) KML_OB(32, 64, 256) KML_OB(64, 64, 256)
  }
#undef KML_OB
  return (int)hipErrorInvalidValue;
}

template <int BM, int BN, int KD>
__global__ __launch_bounds__(256) void k_conv_oneshot(ConvArgs a) {
  using Body = OneShotBody<BM, BN, KD>;
  __shared__ __attribute__((aligned(1024))) char smem[Body::SMEM];
  Body::run(a, xcd_blk(), smem);
}

// single-tap forward whose A rows are contiguous C-element rows: 1x1 maps (centre tap) or
// a 1x1 / stride-1 / pad-0 conv
bool oneshot_shape_ok(const ConvArgs& a) {
  const bool one_tap = (a.r1 - a.r0) == 1 && (a.s1 - a.s0) == 1;
  const bool rows = (a.H * a.W == 1 && a.OH * a.OW == 1) ||
                    (a.KH == 1 && a.KW == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0);
  return one_tap && rows && a.Kd == a.C;
}

int dispatch_oneshot(const ConvArgs& a, int bm, int bn, hipStream_t s) {
  dim3 grid((a.N + bn - 1) / bn, (a.M + bm - 1) / bm, 1);
#define KML_O(BMv, BNv, KDv)                                                          \
  if (bm == BMv && bn == BNv && a.Kd == KDv) {                                        \
    hipLaunchKernelGGL((k_conv_oneshot<BMv, BNv, KDv>), grid, dim3(256), 0, s, a);     \
    KML_LAUNCH_CHECK();                                                               \
  }
  KML_O(32, 32, 512) KML_O(32, 32, 1024) KML_O(32, 64, 512) KML_O(64, 32, 512) KML_O(32, 32, 256)
  KML_O(32, 64, 256) KML_O(64, 64, 256)
#undef KML_O
  return (int)hipErrorInvalidValue;
}

// =====================================================================================
// Variant 6: the ImageNet stem (7x7 / stride 2 / pad 3, Cin padded to 8) as a halo-patch
// kernel: one block per image stages the zero-padded (HW+6)^2 x 8 patch (one 16-byte chunk per
// pixel) and the whole 64 x 392 weight (K padded to 416 = 13 K-steps with zero rows) in LDS
// once; a 32-deep K-step is 4 taps x 8 channels, so each lane's A fragment is ONE patch pixel
// (tap 4 ks + lane/16 of its output pixel).  The implicit-GEMM pipeline re-read every input
// pixel once per tap (49x) through LDS.
// =====================================================================================
template <int HW>
struct StemBody {
  static constexpr int HP = HW + 6, OHW = HW / 2, BM = OHW * OHW, BN = 64;
  // K padded to 416 (13 K-steps); weight rows pitched at 56 chunks so the chunk ^ (n & 7)
  // swizzle stays inside the row (chunks 49..55 hold zeros / are never read)
  static constexpr int KP = 416, KSTEPS = KP / 32, WCH = 56;
  static constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  static constexpr int SMEM_PATCH = HP * HP * 16, SMEM_W = BN * WCH * 16;
  static constexpr int SMEM_EPI = 16 + 2 * BN * 4;
  static constexpr int SMEM = SMEM_PATCH + SMEM_W > SMEM_EPI ? SMEM_PATCH + SMEM_W : SMEM_EPI;
  static_assert(SMEM <= 160 * 1024, "stem patch exceeds LDS");
};

template <int HW>
__global__ __launch_bounds__(256) void k_conv_stem(ConvArgs a) {
  using P = StemBody<HW>;
  constexpr int HP = P::HP, OHW = P::OHW, MR = P::MR, NR = P::NR;
  __shared__ __attribute__((aligned(16))) char smem[P::SMEM];
  char* const swt = smem + P::SMEM_PATCH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int img = (int)blockIdx.x, m0 = img * P::BM;
  // weights [64][392] -> LDS rows of 56 chunks (chunks 49..55 zero), chunk ^ (n & 7)
  constexpr int WCHUNKS = P::BN * P::WCH;
  constexpr int WPER = (WCHUNKS + 255) / 256;
  uint4 wv[WPER];
#pragma unroll
  for (int u = 0; u < WPER; ++u) {
    const int q = tid + u * 256, n = q / P::WCH, c = q - n * P::WCH;
    wv[u] = ld16(q < WCHUNKS && c < 49 ? a.w + (long long)n * 392 + c * 8 : a.zp);
  }
  constexpr int PCH = HP * HP;
  constexpr int PER = (PCH + 255) / 256;
  uint4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + u * 256;
    const int ih = q / HP - 3, iw = q - (q / HP) * HP - 3;
    const bool in = q < PCH && (unsigned)ih < (unsigned)HW && (unsigned)iw < (unsigned)HW && img < a.B;
    v[u] = ld16(in ? a.x + (((long long)img * HW + ih) * HW + iw) * 8 : a.zp);
  }
#pragma unroll
  for (int u = 0; u < WPER; ++u) {
    const int q = tid + u * 256, n = q / P::WCH, c = q - n * P::WCH;
    if (q < WCHUNKS) *reinterpret_cast<uint4*>(swt + (n * P::WCH + (c ^ (n & 7))) * 16) = wv[u];
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + u * 256;
    if (q < PCH) *reinterpret_cast<uint4*>(smem + q * 16) = v[u];
  }
  __syncthreads();
  int pbase[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int r = wm * P::WM + i * 16 + (lane & 15);
    pbase[i] = (2 * (r / OHW)) * HP + 2 * (r % OHW);
  }
  int brow[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) brow[j] = wn * P::WN + j * 16 + (lane & 15);
  auto rd = [&](int ks, bf16x8_t (&af)[MR], bf16x8_t (&bf)[NR]) {
    const int tap = min(4 * ks + (lane >> 4), 48);  // taps 49..51 meet zero weights
    const int toff = (tap / 7) * HP + (tap % 7);
#pragma unroll
    for (int i = 0; i < MR; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(smem + (pbase[i] + toff) * 16);
    const int wc = 4 * ks + (lane >> 4);
#pragma unroll
    for (int j = 0; j < NR; ++j)
      bf[j] = *reinterpret_cast<const bf16x8_t*>(swt + (brow[j] * P::WCH + (wc ^ (brow[j] & 7))) * 16);
  };
  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t af[2][MR], bf[2][NR];
  rd(0, af[0], bf[0]);
#pragma unroll
  for (int ks = 0; ks < P::KSTEPS; ++ks) {
    if (ks + 1 < P::KSTEPS) rd(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bf[ks & 1][j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();
  conv_epilogue<FWD, MR, NR, P::WM, P::WN>(a, acc, m0, 0, wm, wn, lane, tid, 0, 0, reinterpret_cast<unsigned*>(smem));
}

// Variant 6 on ImageNet-size images: the same patch-in-LDS im2col, tiled by PAIRS OF OUTPUT
// ROWS (GEMM rows m0 = tile * 2 * OW.., contiguous, so the FWD epilogue and its BN partial
// rows are unchanged).  A tile reads a 9 x (2 * OW + 6) input patch (the 7 tap rows of two
// stride-2 output rows); every A fragment is one 16-byte LDS read at (patch pixel, tap) —
// no im2col staging — and the 64 x 392 weight matrix stays in LDS for the whole launch:
// persistent blocks (one per CU) walk tiles b, b + grid, ..., the next tile's patch loaded
// into registers while this tile's MFMAs run.  (The general implicit GEMM gathers 392 K per
// row through 16-byte chunks that are 5/8 zero channels and re-stages the weights per tile.)
template <int OW>
struct StemRowsBody {
  static constexpr int WIN = 2 * OW, PW = WIN + 6, PH = 9, BM = 2 * OW, BN = 64;
  static constexpr int KP = 416, KSTEPS = KP / 32, WCH = 56;
  static constexpr int WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  static constexpr int PCH = PH * PW;
  static constexpr int SMEM_EPI = 16 + BM * (BN + 8) * 2 + 2 * BN * 4;
  static constexpr int SMEM_PATCH0 = PCH * 16;
  static constexpr int SMEM_PATCH = ((SMEM_PATCH0 > SMEM_EPI ? SMEM_PATCH0 : SMEM_EPI) + 1023) / 1024 * 1024;
  static constexpr int SMEM_W = BN * WCH * 16;
  static constexpr int SMEM = SMEM_PATCH + SMEM_W;
  static_assert(WM % 16 == 0, "two output rows must split into 16-row wave fragments");
  static_assert(SMEM <= 160 * 1024, "stem row-pair patch exceeds LDS");
};

template <int OW>
__global__ __launch_bounds__(256) void k_conv_stem_rows(ConvArgs a) {
  using P = StemRowsBody<OW>;
  constexpr int PW = P::PW, MR = P::MR, NR = P::NR, PER = (P::PCH + 255) / 256;
  __shared__ __attribute__((aligned(1024))) char smem[P::SMEM];
  char* const swt = smem + P::SMEM_PATCH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int tiles_per_img = a.OH / 2, T = a.B * tiles_per_img;
  {  // weights [64][392] -> LDS rows of 56 chunks (49..55 zero), chunk ^ (n & 7)
    constexpr int WCHUNKS = P::BN * P::WCH;
    for (int q = tid; q < WCHUNKS; q += 256) {
      const int n = q / P::WCH, c = q - n * P::WCH;
      *reinterpret_cast<uint4*>(swt + (n * P::WCH + (c ^ (n & 7))) * 16) =
          ld16(c < 49 ? a.w + (long long)n * 392 + c * 8 : a.zp);
    }
  }
  uint4 v[PER];
  auto load_patch = [&](int tile) {
    const int img = tile / tiles_per_img, ih0 = 2 * 2 * (tile - img * tiles_per_img) - 3;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int q = tid + u * 256;
      const int pr = q / PW, ih = ih0 + pr, iw = q - pr * PW - 3;
      const bool in = q < P::PCH && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      v[u] = ld16(in ? a.x + (((long long)img * a.H + ih) * a.W + iw) * 8 : a.zp);
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int q = tid + u * 256;
      if (q < P::PCH) *reinterpret_cast<uint4*>(smem + q * 16) = v[u];
    }
  };
  int tile = (int)blockIdx.x;
  if (tile >= T) return;
  load_patch(tile);
  store_patch();
  int pbase[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int r = wm * P::WM + i * 16 + (lane & 15);
    pbase[i] = (2 * (r / OW)) * PW + 2 * (r % OW);
  }
  int brow[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) brow[j] = wn * P::WN + j * 16 + (lane & 15);
  auto rd = [&](int ks, bf16x8_t (&af)[MR], bf16x8_t (&bf)[NR]) {
    const int tap = min(4 * ks + (lane >> 4), 48);  // taps 49..51 meet zero weights
    const int toff = (tap / 7) * PW + (tap % 7);
#pragma unroll
    for (int i = 0; i < MR; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(smem + (pbase[i] + toff) * 16);
    const int wc = 4 * ks + (lane >> 4);
#pragma unroll
    for (int j = 0; j < NR; ++j)
      bf[j] = *reinterpret_cast<const bf16x8_t*>(swt + (brow[j] * P::WCH + (wc ^ (brow[j] & 7))) * 16);
  };
  __syncthreads();
  for (;;) {
    const int next = tile + (int)gridDim.x;
    if (next < T) load_patch(next);  // in flight during this tile's MFMAs
    f32x4_t acc[MR][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t af[2][MR], bf[2][NR];
    rd(0, af[0], bf[0]);
#pragma unroll
    for (int ks = 0; ks < P::KSTEPS; ++ks) {
      if (ks + 1 < P::KSTEPS) rd(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bf[ks & 1][j], acc[i][j], 0, 0, 0);
    }
    // raw barriers (LDS ordering only): __syncthreads would also drain the vector-memory
    // counter, i.e. wait for this tile's output stores before the next tile may start
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // patch reads done: the epilogue stages its output over the patch
    conv_epilogue<FWD, MR, NR, P::WM, P::WN>(a, acc, tile * P::BM, 0, wm, wn, lane, tid, 0, 0,
                                             reinterpret_cast<unsigned*>(smem));
    if (next >= T) break;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // epilogue LDS reads done
    store_patch();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    tile = next;
  }
}

template <int MODE>
int dispatch(const ConvArgs& a, int bm, int bn, int bk, int variant, hipStream_t s) {
#define KML_T(BMv, BNv)                                                  \
  if (bm == BMv && bn == BNv) {                                          \
    if (variant == 1) return launch_glds<MODE, BMv, BNv, 3>(a, s);       \
    if (variant == 2) return launch_glds<MODE, BMv, BNv, 4>(a, s);       \
    if (bk == 64) return launch<MODE, BMv, BNv, 64>(a, s);               \
    return launch<MODE, BMv, BNv, 32>(a, s);                             \
  }
  KML_T(32, 32) KML_T(32, 64) KML_T(64, 32) KML_T(64, 64)
  KML_T(64, 128) KML_T(128, 64) KML_T(128, 128) KML_T(32, 128) KML_T(128, 32)
#undef KML_T
  // 256-wide tiles: LDS-DMA pipeline only (3 stages x 48 KB; each of the 4 waves owns 128x64
  // or 64x128, 96 B/clk of fragment reads per CU instead of the 64x64 waves' 128)
  if (variant == 1 && bm == 256 && bn == 128) return launch_glds<MODE, 256, 128, 3>(a, s);
  if (variant == 1 && bm == 128 && bn == 256) return launch_glds<MODE, 128, 256, 3>(a, s);
  return (int)hipErrorInvalidValue;
}

// Parity-class DGRAD launches (kml_conv_dgrad_s2): the TAPU = false DGRAD bodies (DgradAP /
// DgradBP), for the tiles whose epilogue is the row pass (kml_conv_dgrad_s2_ok).
int dispatch_par(const ConvArgs& a, int bm, int bn, int bk, int variant, hipStream_t s) {
  dim3 grid((a.N + bn - 1) / bn, (a.M + bm - 1) / bm, 1);
#define KML_P(BMv, BNv, BKv)                                                                             \
  if (variant == 0 && bm == BMv && bn == BNv && bk == BKv) {                                             \
    hipLaunchKernelGGL((k_conv_igemm<DGRAD, BMv, BNv, BKv, false>), grid, dim3(256), 0, s, a, KmlSgdRider{}); \
    return (int)hipGetLastError();                                                                       \
  }
#define KML_PG(BMv, BNv, Sv, Vv)                                                                         \
  if (variant == Vv && bm == BMv && bn == BNv) {                                                         \
    hipLaunchKernelGGL((k_conv_glds<DGRAD, BMv, BNv, Sv, false>), grid, dim3(256), 0, s, a);             \
    return (int)hipGetLastError();                                                                       \
  }
  KML_P(64, 64, 32) KML_P(64, 64, 64) KML_P(64, 128, 64) KML_P(128, 64, 64) KML_P(128, 128, 64)
  KML_PG(64, 64, 3, 1) KML_PG(64, 128, 3, 1) KML_PG(128, 64, 3, 1) KML_PG(128, 128, 3, 1)
  KML_PG(64, 64, 4, 2) KML_PG(64, 128, 4, 2) KML_PG(128, 64, 4, 2)
#undef KML_P
#undef KML_PG
  return (int)hipErrorInvalidValue;
}

FastDiv make_fd(int d) {
  FastDiv f;
  f.d = d < 1 ? 1 : d;
  int p = 0;
  while ((1ll << p) < f.d) ++p;
  f.s = 31 + p;
  f.m = (unsigned)(((1ull << (31 + p)) + f.d - 1) / f.d);
  if (f.d == 1) { f.m = 1u << 31; f.s = 31; }
  return f;
}

void tap_window(int I, int O, int KS, int st, int p, int* t0, int* t1) {
  int lo = KS, hi = 0;
  for (int t = 0; t < KS; ++t) {
    bool ok = false;
    for (int o = 0; o < O && !ok; ++o) { const int i = o * st - p + t; ok = (i >= 0 && i < I); }
    if (ok) { if (t < lo) lo = t; if (t + 1 > hi) hi = t + 1; }
  }
  if (lo >= hi) { lo = 0; hi = 0; }
  *t0 = lo; *t1 = hi;
}

ConvArgs make_args(int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw) {
  ConvArgs a = {};
  a.B = B; a.H = H; a.W = W; a.C = C; a.K = K; a.KH = KH; a.KW = KW;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.OH = (H + 2 * ph - KH) / sh + 1;
  a.OW = (W + 2 * pw - KW) / sw + 1;
  tap_window(H, a.OH, KH, sh, ph, &a.r0, &a.r1);
  tap_window(W, a.OW, KW, sw, pw, &a.s0, &a.s1);
  a.fd_C = make_fd(C);
  a.fd_nts = make_fd(a.s1 - a.s0);
  a.fd_OW = make_fd(a.OW);
  a.fd_OH = make_fd(a.OH);
  a.fd_W = make_fd(W);
  a.fd_H = make_fd(H);
  a.fd_sh = make_fd(sh);
  a.fd_sw = make_fd(sw);
  a.fd_Kp = make_fd(1);
  return a;
}

int set_splits(ConvArgs& a, int bk, int splits) {
  if (splits < 1) splits = 1;
  int chunk = (a.Kd + splits - 1) / splits;
  chunk = (chunk + bk - 1) / bk * bk;
  if (chunk < bk) chunk = bk;
  a.kchunk = chunk;
  a.splits = (a.Kd + chunk - 1) / chunk;
  if (a.splits < 1) a.splits = 1;
  return a.splits;
}

// ---------------------------------------------------------------------------------
// Grouped backward: the dgrad and the wgrad of one conv layer in ONE launch.
//
// Both GEMMs read the same upstream gradient and are independent of each other, so a
// flat grid runs the dgrad tiles (blocks [0, nd), dispatched first: dgrad is the
// critical path of backward) next to the wgrad tiles (blocks [nd, nd + nw)).  At
// ResNet-34/CIFAR sizes each GEMM alone fills 8-72 of the 256 CUs and every dependent
// launch costs ~4-5 us on the MI355X queue, so pairing halves the conv-backward launch
// count and lets the two small GEMMs share the chip.
// ---------------------------------------------------------------------------------
// Optional third role: an SGD range "rider" (kml_sgd.h) in blocks [nd + nw, nd + nw + rider.blocks):
// the update of parameters whose gradients are already final (ResNet's layer4 + fc while layer3
// runs backward) streams through HBM beside the latency-bound conv tiles of the same launch —
// no second queue, no extra launch (engine/dp.py ``ride``).
template <class DB, class WB>
__global__ __launch_bounds__(256) void k_conv_pair(ConvArgs ad, ConvArgs aw, int dgx, int dgy, int wgx, int wgy,
                                                   int nd, int nw, KmlSgdRider rider) {
  static_assert(DB::THREADS == 256 && WB::THREADS == 256, "paired bodies run 256-thread blocks");
  constexpr int SM = DB::SMEM > WB::SMEM ? DB::SMEM : WB::SMEM;
  __shared__ __attribute__((aligned(1024))) char smem[SM];
  int id = (int)blockIdx.x;
  if (id >= nd + nw) {
    kml_sgd_rider_run(rider, id - nd - nw);
    return;
  }
  if (id < nd) {
    Blk b;
    b.gx = dgx;
    b.x = id % dgx;
    const int t = id / dgx;
    b.y = t % dgy;
    b.z = t / dgy;
    DB::run(ad, b, smem);
  } else {
    id -= nd;
    Blk b;
    b.gx = wgx;
    b.x = id % wgx;
    const int t = id / wgx;
    b.y = t % wgy;
    b.z = t / wgy;
    WB::run(aw, b, smem);
  }
}

// Instantiated pairs: X(dgrad variant, dgrad cfg bm, bn, bk, dgrad body, dgrad tile M, N,
// wgrad body, wgrad tile M, N).  Variant codes as in plan_conv (0 = register-staged,
// 3 = direct with bk = waves); the wgrad side is always the register-staged BK=64 kernel.
// Any other combination runs as two launches (kml_conv_pair_supported).
using DgIg3264 = IgemmBody<DGRAD, 32, 64, 64, true>;
using DgIg3232 = IgemmBody<DGRAD, 32, 32, 64, true>;
using DgDi3232 = DirectBody<DGRAD, 2, 2, 4, 4>;
using DgDi3216 = DirectBody<DGRAD, 2, 1, 4, 4>;
using DgDi6432 = DirectBody<DGRAD, 4, 2, 4, 2>;
using WgIg3232 = IgemmBody<WGRAD, 32, 32, 64, true>;
using WgIg6432 = IgemmBody<WGRAD, 64, 32, 64, true>;
// halo dgrad bodies (variant 4): the plan's bk slot carries Cout * 16 + H (the body's geometry)
using DgHa64x8 = HaloBody<DGRAD, 64, 8, 1, 32, 1>;
using DgHa128x4 = HaloBody<DGRAD, 128, 4, 4, 32, 1>;
#define KML_PAIR_LIST(X)                                   \
  X(4, 64, 32, 1032, DgHa64x8, 64, 32, WgIg3232, 32, 32)   \
  X(4, 64, 32, 1032, DgHa64x8, 64, 32, WgIg6432, 64, 32)   \
  X(4, 64, 32, 2052, DgHa128x4, 64, 32, WgIg3232, 32, 32)  \
  X(4, 64, 32, 2052, DgHa128x4, 64, 32, WgIg6432, 64, 32)  \
  X(0, 32, 64, 64, DgIg3264, 32, 64, WgIg3232, 32, 32)     \
  X(0, 32, 64, 64, DgIg3264, 32, 64, WgIg6432, 64, 32)     \
  X(0, 32, 32, 64, DgIg3232, 32, 32, WgIg3232, 32, 32)     \
  X(0, 32, 32, 64, DgIg3232, 32, 32, WgIg6432, 64, 32)     \
  X(3, 32, 32, 4, DgDi3232, 32, 32, WgIg3232, 32, 32)      \
  X(3, 32, 32, 4, DgDi3232, 32, 32, WgIg6432, 64, 32)      \
  X(3, 32, 16, 4, DgDi3216, 32, 16, WgIg3232, 32, 32)      \
  X(3, 32, 16, 4, DgDi3216, 32, 16, WgIg6432, 64, 32)      \
  X(3, 64, 32, 4, DgDi6432, 64, 32, WgIg3232, 32, 32)      \
  X(3, 64, 32, 4, DgDi6432, 64, 32, WgIg6432, 64, 32)

template <class DB, class WB>
int launch_pair(const ConvArgs& ad, int dbm, int dbn, const ConvArgs& aw, int wbm, int wbn, hipStream_t s) {
  const int dgx = (ad.N + dbn - 1) / dbn, dgy = (ad.M + dbm - 1) / dbm;
  const int wgx = (aw.N + wbn - 1) / wbn, wgy = (aw.M + wbm - 1) / wbm;
  const long long nd = (long long)dgx * dgy * ad.splits, nw = (long long)wgx * wgy * aw.splits;
  const KmlSgdRider rider = kml_rider_take();
  if (nd + nw + rider.blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((k_conv_pair<DB, WB>), dim3((unsigned)(nd + nw + rider.blocks)), dim3(256), 0, s, ad, aw, dgx,
                     dgy, wgx, wgy, (int)nd, (int)nw, rider);
  KML_LAUNCH_CHECK();
}

// 1 + index of the instantiated pair, 0 if none
int pair_index(int dv, int dbm, int dbn, int dbk, int wv, int wbm, int wbn, int wbk) {
  int idx = 0;
#define KML_PAIR_FIND(DV, DBM, DBN, DBK, DB, DTM, DTN, WB, WBM, WBN)                                   \
  ++idx;                                                                                             \
  if (dv == DV && dbm == DBM && dbn == DBN && dbk == DBK && wv == 0 && wbm == WBM && wbn == WBN && wbk == 64) \
    return idx;
  KML_PAIR_LIST(KML_PAIR_FIND)
#undef KML_PAIR_FIND
  return 0;
}

int dispatch_pair(int which, const ConvArgs& ad, const ConvArgs& aw, hipStream_t s) {
  int idx = 0;
#define KML_PAIR_RUN(DV, DBM, DBN, DBK, DB, DTM, DTN, WB, WBM, WBN) \
  if (++idx == which) return launch_pair<DB, WB>(ad, DTM, DTN, aw, WBM, WBN, s);
  KML_PAIR_LIST(KML_PAIR_RUN)
#undef KML_PAIR_RUN
  return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------
// Forward pairs: the two independent convolutions of a downsampling residual block (the strided
// 3x3 main conv and the strided 1x1 projection, both reading the block input) in ONE launch —
// the forward twin of k_conv_pair.  On ResNet-34/CIFAR each fills 128-256 of the 256 CUs and
// costs a ~4-5 us dependent launch; pairing lets them share the chip.  The flat grid takes the
// XCD-aware order of xcd_blk over both bodies' tiles.
// ---------------------------------------------------------------------------------
template <class B1, class B2>
__global__ __launch_bounds__(256) void k_conv_fwd_pair(ConvArgs a1, ConvArgs a2, int g1x, int g1y, int g2x, int n1,
                                                       int n2) {
  static_assert(B1::THREADS == 256 && B2::THREADS == 256, "paired bodies run 256-thread blocks");
  constexpr int SM = B1::SMEM > B2::SMEM ? B1::SMEM : B2::SMEM;
  __shared__ __attribute__((aligned(1024))) char smem[SM];
  const int nwg = n1 + n2, lin = (int)blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, x = lin & 7, k = lin >> 3;
  int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  Blk b;
  if (id < n1) {
    b.gx = g1x;
    b.x = id % g1x;
    b.y = id / g1x;
    b.z = 0;
    (void)g1y;
    B1::run(a1, b, smem);
  } else {
    id -= n1;
    b.gx = g2x;
    b.x = id % g2x;
    b.y = id / g2x;
    b.z = 0;
    B2::run(a2, b, smem);
  }
}

using FwGl6432 = GldsBody<FWD, 64, 32, 3, true>;
using FwIg6432 = IgemmBody<FWD, 64, 32, 32, true>;
using FwIg3232 = IgemmBody<FWD, 32, 32, 64, true>;
using FwGl3232 = GldsBody<FWD, 32, 32, 3, true>;
using FwDi3216 = DirectBody<FWD, 2, 1, 4, 4>;
// ResNet-34/CIFAR's downsampling blocks: layer2 (3x3 on the LDS-DMA kernel + 1x1 register-staged),
// layer3 (register-staged + LDS-DMA), layer4 (direct + register-staged)
#define KML_FWD_PAIR_LIST(X) \
  X(0, 1, FwGl6432, FwIg6432) \
  X(2, 3, FwIg3232, FwGl3232) \
  X(4, 2, FwDi3216, FwIg3232)

template <class B>
constexpr int fwd_body_id() {
  if constexpr (std::is_same<B, FwGl6432>::value) return 0;
  else if constexpr (std::is_same<B, FwIg6432>::value) return 1;
  else if constexpr (std::is_same<B, FwIg3232>::value) return 2;
  else if constexpr (std::is_same<B, FwGl3232>::value) return 3;
  else if constexpr (std::is_same<B, FwDi3216>::value) return 4;
  else return -1;
}

int launch_fwd_pair(const FwdRec& r1, const FwdRec& r2, hipStream_t s) {
#define KML_FWD_PAIR_RUN(I1, I2, B1, B2)                                                                   \
  if (r1.body == I1 && r2.body == I2) {                                                                     \
    hipLaunchKernelGGL((k_conv_fwd_pair<B1, B2>), dim3((unsigned)(r1.gx * r1.gy + r2.gx * r2.gy)), dim3(256), 0, s, \
                       r1.a, r2.a, r1.gx, r1.gy, r2.gx, r1.gx * r1.gy, r2.gx * r2.gy);                        \
    KML_LAUNCH_CHECK();                                                                                     \
  }                                                                                                         \
  if (r1.body == I2 && r2.body == I1) {                                                                     \
    hipLaunchKernelGGL((k_conv_fwd_pair<B1, B2>), dim3((unsigned)(r1.gx * r1.gy + r2.gx * r2.gy)), dim3(256), 0, s, \
                       r2.a, r1.a, r2.gx, r2.gy, r1.gx, r2.gx * r2.gy, r1.gx * r1.gy);                        \
    KML_LAUNCH_CHECK();                                                                                     \
  }
  KML_FWD_PAIR_LIST(KML_FWD_PAIR_RUN)
#undef KML_FWD_PAIR_RUN
  return -1;
}

// wT[c][t][k] = w[k][t][c] for up to 16 weights in one launch (kml_weight_transpose_multi).
// One block per 64(k) x 64(c) tile of one tap: 16-byte loads along c into an LDS tile,
// 16-byte stores along k out of it (k >= K zero-filled up to Kp).
struct TransposeJob {
  const bf16_t* w;
  bf16_t* wt;
  int tile_begin;  // first block of this job
  int K, T, C, Kp, tk, tc;  // tk / tc: 64-wide tiles along Kp / C
};
struct TransposeBatch {
  TransposeJob j[16];
  int n;
};

__global__ __launch_bounds__(256) void k_weight_transpose_multi(TransposeBatch tb) {
  __shared__ bf16_t tile[64][64 + 8];
  int q = 0;
  while (q + 1 < tb.n && (int)blockIdx.x >= tb.j[q + 1].tile_begin) ++q;  // block-uniform
  const TransposeJob& jb = tb.j[q];
  int id = (int)blockIdx.x - jb.tile_begin;
  const int ic = id % jb.tc;
  id /= jb.tc;
  const int ik = id % jb.tk;
  const int t = id / jb.tk;
  const int k0 = ik * 64, c0 = ic * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // 64 k-rows x 8 chunks of 8 c
    const int q2 = tid + 256 * u, r = q2 >> 3, ch = q2 & 7;
    const int k = k0 + r, c = c0 + ch * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k < jb.K && c < jb.C) v = *reinterpret_cast<const uint4*>(jb.w + ((long long)k * jb.T + t) * jb.C + c);
    *reinterpret_cast<uint4*>(&tile[r][ch * 8]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // 64 c-rows x 8 chunks of 8 k
    const int q2 = tid + 256 * u, r = q2 >> 3, ch = q2 & 7;
    const int c = c0 + r, k = k0 + ch * 8;
    if (c >= jb.C || k >= jb.Kp) continue;
    bf16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = tile[ch * 8 + e][r];
    *reinterpret_cast<uint4*>(jb.wt + ((long long)c * jb.T + t) * jb.Kp + k) = *reinterpret_cast<const uint4*>(o);
  }
}

// Unrolled-conv weights (ConvArgs::fold_c): wu[(p, n)][(q, c)] = w[n][tap(p, q)][c] for a
// 3x3 / stride 1 / pad 1 conv on a 2x2 map (p, q = output / input position, tap =
// (qh - ph + 1, qw - pw + 1)), up to 16 convs per launch, one 16-byte chunk per thread.
struct UnrollJob {
  const bf16_t* w;
  bf16_t* wu;
  int block_begin;
  int K, C;
};
struct UnrollBatch {
  UnrollJob j[16];
  int n;
};

constexpr int UNROLL_V = 8;  // 16-byte chunks per thread (all loads issued before the stores)

__global__ __launch_bounds__(256) void k_unroll22_multi(UnrollBatch ub) {
  int q = 0;
  while (q + 1 < ub.n && (int)blockIdx.x >= ub.j[q + 1].block_begin) ++q;  // block-uniform
  const UnrollJob& jb = ub.j[q];
  const int cpr = jb.C / 2;  // 16-byte chunks per wu row (4C / 8)
  const int total = 4 * jb.K * cpr;
  const int base = ((int)blockIdx.x - jb.block_begin) * 256 * UNROLL_V + (int)threadIdx.x;
  uint4 v[UNROLL_V];
  long long dst[UNROLL_V];
#pragma unroll
  for (int u = 0; u < UNROLL_V; ++u) {
    const int idx = min(base + u * 256, total - 1);  // clamped: tail lanes reload / rewrite the last chunk
    const int row = idx / cpr, col = (idx - row * cpr) * 8;
    const int p = row / jb.K, n = row - p * jb.K;
    const int qq = col / jb.C, c = col - qq * jb.C;
    const int tap = ((qq >> 1) - (p >> 1) + 1) * 3 + ((qq & 1) - (p & 1) + 1);
    v[u] = *reinterpret_cast<const uint4*>(jb.w + ((long long)n * 9 + tap) * jb.C + c);
    dst[u] = (long long)row * 4 * jb.C + col;
  }
#pragma unroll
  for (int u = 0; u < UNROLL_V; ++u)
    if (base + u * 256 < total) *reinterpret_cast<uint4*>(jb.wu + dst[u]) = v[u];
}

__device__ __attribute__((aligned(64))) bf16_t g_zero_page[32];  // zero-initialised device global
__device__ __attribute__((aligned(64))) bf16_t g_one_page[8] = {0x3F80, 0, 0, 0, 0, 0, 0, 0};  // bf16 1.0, 0 x 7

const bf16_t* zero_page() {
  static const bf16_t* p = nullptr;
  if (!p) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_zero_page)) == hipSuccess) p = (const bf16_t*)d;
  }
  return p;
}

const bf16_t* one_page() {
  static const bf16_t* p = nullptr;
  if (!p) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_one_page)) == hipSuccess) p = (const bf16_t*)d;
  }
  return p;
}

}  // namespace

namespace {
// g22 needs the 1x1 form of an unrolled 3x3 conv: Cq = C / 4 a multiple of 8 (a 16-byte chunk
// never straddles two input positions), Kq = K / 4
bool g22_ok(int C, int K, int KH, int KW) { return KH == 1 && KW == 1 && C % 32 == 0 && K % 4 == 0; }
void set_g22(ConvArgs& a, int g22, int C, int K) {
  a.g22 = g22 ? 1 : 0;
  if (a.g22) { a.fd_gK = make_fd(K / 4); a.fd_gC = make_fd(C / 4); }
}
}  // namespace

KML_API int kml_conv_tap_window(int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw,
                                int* out4) {
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  out4[0] = a.r0; out4[1] = a.r1; out4[2] = a.s0; out4[3] = a.s1;
  return 0;
}

KML_API int kml_conv_effective_splits(int Kd, int bk, int splits) {
  ConvArgs a = {};
  a.Kd = Kd;
  return set_splits(a, bk, splits);
}

// stats_part = 1: stats is [G][2K] with G = ceil(M / bm), one row per M-tile;
// every row is written (no zeroing needed) and bn_apply sums the rows.
// grp_out / grp_cnt / grp_tiles: optional group reduction of the stats_part rows (ConvArgs).
KML_API int kml_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const float* bias, float* stats, int stats_part,
                         int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, int relu,
                         int bm, int bn, int bk, int splits, int variant, float* slab, unsigned* counters,
                         float* grp_out, unsigned* grp_cnt, int grp_tiles, int fold_c, int g22, hipStream_t s) {
  if (grp_out && (!stats || !stats_part || !grp_cnt || grp_tiles < 1)) return (int)hipErrorInvalidValue;
  if (g22 && !g22_ok(C, K, KH, KW)) return (int)hipErrorInvalidValue;
  if (fold_c && (grp_out || K % fold_c || (stats && !stats_part))) return (int)hipErrorInvalidValue;
  if (C % 8) return (int)hipErrorInvalidValue;
  if (variant == 3) {  // direct: bk carries the wave count; needs 32-aligned taps
    if (C % 32) return (int)hipErrorInvalidValue;
    ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
    a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
    a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles; a.fold_c = fold_c;
    set_g22(a, g22, C, K);
    a.zp = zero_page();
    a.M = B * a.OH * a.OW; a.N = K; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * C;
    a.splits = 1; a.kchunk = a.Kd;
    if (!a.zp) return (int)hipErrorInvalidSymbol;
    return dispatch_direct<FWD>(a, bm, bn, bk, s);
  }
  if (variant == 6) {  // stem halo: 7x7 / s2 / p3, Cin 8, Cout 64; 32x32: one image per block,
                       // 224x224: persistent blocks over output row pairs
    if (g22 || fold_c || C != 8 || K != 64 || KH != 7 || KW != 7 || sh != 2 || sw != 2 || ph != 3 || pw != 3 ||
        H != W || (H != 32 && H != 224))
      return (int)hipErrorInvalidValue;
    if (H == 224) {
      if (bm != 224) return (int)hipErrorInvalidValue;
      ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
      a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
      a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles;
      a.zp = zero_page();
      a.M = B * a.OH * a.OW; a.N = K; a.Kd = 392;
      a.splits = 1; a.kchunk = a.Kd;
      if (!a.zp) return (int)hipErrorInvalidSymbol;
      const int T = B * (a.OH / 2);
      hipLaunchKernelGGL((k_conv_stem_rows<112>), dim3(T < 256 ? T : 256), dim3(256), 0, s, a);
      KML_LAUNCH_CHECK();
    }
    ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
    a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
    a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles;
    a.zp = zero_page();
    a.M = B * a.OH * a.OW; a.N = K; a.Kd = 392;
    a.splits = 1; a.kchunk = a.Kd;
    if (!a.zp) return (int)hipErrorInvalidSymbol;
    hipLaunchKernelGGL((k_conv_stem<32>), dim3(B), dim3(256), 0, s, a);
    KML_LAUNCH_CHECK();
  }
  if (variant == 5) {  // one-shot panels: single-tap, contiguous A rows, short K
    ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
    a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
    a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles; a.fold_c = fold_c;
    set_g22(a, g22, C, K);
    a.zp = zero_page();
    a.M = B * a.OH * a.OW; a.N = K; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * C;
    a.splits = 1; a.kchunk = a.Kd;
    if (!a.zp) return (int)hipErrorInvalidSymbol;
    if (!oneshot_shape_ok(a)) return (int)hipErrorInvalidValue;
    return dispatch_oneshot(a, bm, bn, s);
  }
  if (variant == 4) {  // halo patch: bm = pixels per block (whole images), bn = channels per block
    if (g22 || fold_c || !halo_shape_ok(H, W, C, K, KH, KW, sh, sw, ph, pw, bm, bn)) return (int)hipErrorInvalidValue;
    ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
    a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
    a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles;
    a.zp = zero_page();
    a.M = B * a.OH * a.OW; a.N = K; a.Kd = 9 * C;
    a.splits = 1; a.kchunk = a.Kd;
    if (!a.zp) return (int)hipErrorInvalidSymbol;
    return dispatch_halo<FWD>(a, bm, bn, s);
  }
  if (variant) bk = 64;
  ConvArgs a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  a.x = x; a.w = w; a.out = y; a.bias = bias; a.stats = stats; a.stats_part = stats_part; a.relu = relu;
  a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles; a.fold_c = fold_c;
  set_g22(a, g22, C, K);
  a.zp = zero_page();
  a.M = B * a.OH * a.OW; a.N = K; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * C;
  if (!a.zp) return (int)hipErrorInvalidSymbol;
  set_splits(a, bk, splits);
  if (a.splits > 1 && (!slab || !counters)) return (int)hipErrorInvalidValue;
  a.slab = slab; a.counters = counters;
  return dispatch<FWD>(a, bm, bn, bk, variant, s);
}

// Two independent forward convolutions in one launch (k_conv_fwd_pair).  q1 / q2: the 30
// arguments of kml_conv_fwd (stream excluded) as 64-bit values, in its order.  Returns 0 when
// launched as a pair, 1 when the two plans are not an instantiated pair (nothing launched: the
// caller launches them with kml_conv_fwd), or an error code.
KML_API int kml_conv_fwd_pair(const long long* q1, const long long* q2, hipStream_t s) {
  FwdRec r[2];
  const long long* q[2] = {q1, q2};
  for (int i = 0; i < 2; ++i) {
    const long long* v = q[i];
    const int variant = (int)v[22];
    if (variant != 0 && variant != 1 && variant != 2 && variant != 3) return 1;
    g_fwd_rec = &r[i];
    const int rc = kml_conv_fwd((const bf16_t*)v[0], (const bf16_t*)v[1], (bf16_t*)v[2], (const float*)v[3],
                                (float*)v[4], (int)v[5], (int)v[6], (int)v[7], (int)v[8], (int)v[9], (int)v[10],
                                (int)v[11], (int)v[12], (int)v[13], (int)v[14], (int)v[15], (int)v[16], (int)v[17],
                                (int)v[18], (int)v[19], (int)v[20], (int)v[21], variant, (float*)v[23],
                                (unsigned*)v[24], (float*)v[25], (unsigned*)v[26], (int)v[27], (int)v[28], (int)v[29],
                                s);
    g_fwd_rec = nullptr;
    if (rc) return rc;
    if (!r[i].set || r[i].body < 0) return 1;
  }
  const long long n = (long long)r[0].gx * r[0].gy + (long long)r[1].gx * r[1].gy;
  if (n <= 0 || n > 0x7fffffffLL) return 1;
  const int rc = launch_fwd_pair(r[0], r[1], s);
  return rc < 0 ? 1 : rc;
}

// Halo forward (variant 4) of a conv whose INPUT is the raw output of another conv: that
// conv's BatchNorm (training statistics from its partial rows) + ReLU is applied while the
// patch is staged; the normalised input is written to ibn_y, the statistics to mean / rstd and
// the running buffers updated — the BN apply launch between the two convs disappears.
KML_API int kml_conv_fwd_bnin(const bf16_t* x, const bf16_t* w, bf16_t* y, float* stats, int stats_part, int B,
                              int H, int W, int C, int K, int bm, int bn, float* grp_out, unsigned* grp_cnt,
                              int grp_tiles, const float* ibn_rows, int ibn_G, const float* gamma, const float* beta,
                              float* mean, float* rstd, float* rmean, float* rvar, float eps, float momentum,
                              bf16_t* ibn_y, const bf16_t* res, hipStream_t s) {
  if (!ibn_rows || ibn_G < 1 || !ibn_y || !halo_shape_ok(H, W, C, K, 3, 3, 1, 1, 1, 1, bm, bn) || 2 * C > 1024 ||
      (256 % (2 * C / 4)) != 0)
    return (int)hipErrorInvalidValue;
  ConvArgs a = make_args(B, H, W, C, K, 3, 3, 1, 1, 1, 1);
  a.x = x; a.w = w; a.out = y; a.stats = stats; a.stats_part = stats_part;
  a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles;
  a.zp = zero_page();
  a.M = B * H * W; a.N = K; a.Kd = 9 * C;
  a.splits = 1; a.kchunk = a.Kd;
  a.ibn_rows = ibn_rows; a.ibn_G = ibn_G; a.ibn_M = (long long)B * H * W;
  a.ibn_gamma = gamma; a.ibn_beta = beta; a.ibn_mean = mean; a.ibn_rstd = rstd; a.ibn_rmean = rmean;
  a.ibn_rvar = rvar; a.ibn_eps = eps; a.ibn_mom = momentum; a.ibn_y = ibn_y;
  a.addend = res;   // FWD: the folded BN's residual (y = relu(bn(x) + res))
  if (!a.zp) return (int)hipErrorInvalidSymbol;
  return dispatch_halo<FWD>(a, bm, bn, s);
}

namespace {
int prep_dgrad(ConvArgs& a, const bf16_t* dy, const bf16_t* w, const bf16_t* wt, bf16_t* dx, const bf16_t* addend,
               const bf16_t* bnf_y, const bf16_t* bnf_c, const float* bnf_mean, const float* bnf_rstd,
               float* bnf_part, float* grp_out, unsigned* grp_cnt, int grp_tiles, int B, int H, int W, int C, int K,
               int KH, int KW, int sh, int sw, int ph, int pw, int bk, int splits, int variant, float* slab,
               unsigned* counters, int fold_c, int bnf_mask_out, int g22) {
  if (C % 8 || K % 8) return (int)hipErrorInvalidValue;
  if (g22 && (variant == 3 || !g22_ok(C, K, KH, KW))) return (int)hipErrorInvalidValue;
  if (grp_out && (!bnf_part || !grp_cnt || grp_tiles < 1)) return (int)hipErrorInvalidValue;
  if (bnf_mask_out && !bnf_part) return (int)hipErrorInvalidValue;
  if (fold_c && (grp_out || C % fold_c)) return (int)hipErrorInvalidValue;
  const bool direct = (variant == 3);
  if (!direct && variant) bk = 64;
  a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  const int kq = direct ? 32 : bk;
  a.Kp = (K + kq - 1) / kq * kq;
  a.fd_Kp = make_fd(a.Kp);
  a.dy = dy; a.w = w; a.wt = wt; a.out = dx; a.addend = addend; a.zp = zero_page();
  a.bnf_y = bnf_y; a.bnf_c = bnf_c; a.bnf_mean = bnf_mean; a.bnf_rstd = bnf_rstd; a.bnf_part = bnf_part;
  a.bnf_mask_out = bnf_mask_out;
  a.grp_out = grp_out; a.grp_cnt = grp_cnt; a.grp_tiles = grp_tiles; a.fold_c = fold_c;
  set_g22(a, g22, C, K);
  a.M = B * H * W; a.N = C; a.Kd = (a.r1 - a.r0) * (a.s1 - a.s0) * a.Kp;
  if (!a.zp) return (int)hipErrorInvalidSymbol;
  if (direct) {
    if (!wt) return (int)hipErrorInvalidValue;
    a.splits = 1; a.kchunk = a.Kd;
    return 0;
  }
  set_splits(a, bk, splits);
  if (a.splits > 1 && (!slab || !counters)) return (int)hipErrorInvalidValue;
  a.slab = slab; a.counters = counters;
  return 0;
}

// WGRAD overwrites dw (accumulate = 0) or adds to it (1); either way every element has ONE
// writer — split-K partial tiles go through the slab and are summed in split order by the
// last block of the tile — so weight gradients are bitwise reproducible and need no zeroed
// buffer.  (An unrolled conv's dense 1x1-form gradient goes to a scratch that
// kml_conv_fold22_multi folds onto the 3x3 taps in a fixed order.)
int prep_wgrad(ConvArgs& a, const bf16_t* x, const bf16_t* dy, float* dw, int B, int H, int W, int C, int K, int KH,
               int KW, int sh, int sw, int ph, int pw, int bk, int splits, int variant, int accumulate, float* slab,
               unsigned* counters, float* dbias, int bias_acc) {
  if (variant) bk = 64;
  if (C % 8 || K % 8) return (int)hipErrorInvalidValue;
  // the ones column needs every pixel to see every input channel once: 1x1, stride 1, no pad
  if (dbias && (KH != 1 || KW != 1 || sh != 1 || sw != 1 || ph || pw)) return (int)hipErrorInvalidValue;
  a = make_args(B, H, W, C, K, KH, KW, sh, sw, ph, pw);
  a.x = x; a.dy = dy; a.dw = dw; a.zp = zero_page();
  a.dbias = dbias; a.bias_acc = bias_acc ? 1 : 0; a.op = one_page();
  a.M = K; a.N = (a.r1 - a.r0) * (a.s1 - a.s0) * C + (dbias ? 1 : 0); a.Kd = B * a.OH * a.OW;
  if (!a.zp || !a.op) return (int)hipErrorInvalidSymbol;
  set_splits(a, bk, splits);
  if (a.splits > 1 && (!slab || !counters)) return (int)hipErrorInvalidValue;
  a.slab = slab; a.counters = counters;
  a.accumulate = accumulate ? 1 : 0;
  return 0;
}
}  // namespace

KML_API int kml_conv_pair_supported(int dvariant, int dbm, int dbn, int dbk, int wvariant, int wbm, int wbn, int wbk) {
  return pair_index(dvariant, dbm, dbn, dbk, wvariant, wbm, wbn, wbk) > 0 ? 1 : 0;
}

// dX (dgrad, + addend, + consumer-BN partials) and dW (wgrad, fp32 +=) of one conv in one
// launch.  wt: transposed weights for the direct dgrad variant (else null).
KML_API int kml_conv_bwd_pair(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, bf16_t* dx, const bf16_t* addend,
                              const bf16_t* bnf_y, const bf16_t* bnf_c, const float* bnf_mean, const float* bnf_rstd,
                              float* bnf_part, float* grp_out, unsigned* grp_cnt, int grp_tiles, const bf16_t* x,
                              float* dw, int B, int H, int W, int C, int K, int KH,
                              int KW, int sh, int sw, int ph, int pw, int dbm, int dbn, int dbk, int dsplits,
                              int dvariant, float* slab, unsigned* counters, int wbm, int wbn, int wbk, int wsplits,
                              int wvariant, int fold_c, int bnf_mask_out, float* wslab, unsigned* wcounters,
                              int waccumulate, float* wbias, int wbias_acc, int g22, hipStream_t s) {
  const int which = pair_index(dvariant, dbm, dbn, dbk, wvariant, wbm, wbn, wbk);
  if (!which) return (int)hipErrorInvalidValue;
  if (dvariant == 4 && (g22 || fold_c || dsplits != 1 || dbk != K * 16 + H ||
                        !halo_shape_ok(H, W, K, C, KH, KW, sh, sw, ph, pw, dbm, dbn)))
    return (int)hipErrorInvalidValue;
  ConvArgs ad, aw;
  int e = prep_dgrad(ad, dy, w, wt, dx, addend, bnf_y, bnf_c, bnf_mean, bnf_rstd, bnf_part, grp_out, grp_cnt,
                     grp_tiles, B, H, W, C, K, KH, KW, sh, sw, ph, pw, dbk, dsplits, dvariant, slab, counters,
                     fold_c, bnf_mask_out, g22);
  if (e) return e;
  e = prep_wgrad(aw, x, dy, dw, B, H, W, C, K, KH, KW, sh, sw, ph, pw, wbk, wsplits, wvariant, waccumulate, wslab,
                 wcounters, wbias, wbias_acc);
  if (e) return e;
  return dispatch_pair(which, ad, aw, s);
}

// Up to 16 transposes wT = [C][KH*KW][Kp] (Kp = roundup(K, 32)) in one launch.
// dims: n x 4 ints (K, KH*KW, C, unused).
KML_API int kml_weight_transpose_multi(const bf16_t* const* ws, bf16_t* const* wts, const int* dims, int n,
                                       hipStream_t s) {
  if (n < 1 || n > 16) return (int)hipErrorInvalidValue;
  TransposeBatch tb = {};
  tb.n = n;
  long long tiles = 0;
  for (int i = 0; i < n; ++i) {
    TransposeJob& j = tb.j[i];
    j.w = ws[i]; j.wt = wts[i];
    j.K = dims[4 * i]; j.T = dims[4 * i + 1]; j.C = dims[4 * i + 2];
    if (j.C % 8) return (int)hipErrorInvalidValue;  // 16-byte rows along c
    j.Kp = (j.K + 31) / 32 * 32;
    j.tk = (j.Kp + 63) / 64;
    j.tc = (j.C + 63) / 64;
    j.tile_begin = (int)tiles;
    tiles += (long long)j.T * j.tk * j.tc;
  }
  if (tiles <= 0 || tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_weight_transpose_multi, dim3((unsigned)tiles), dim3(256), 0, s, tb);
  KML_LAUNCH_CHECK();
}

// wus[i][4K][4C] = unrolled 2x2-map form of ws[i][K][3][3][C] (k_unroll22_multi), up to 16
// convs in one launch.  dims: n x 2 ints (K, C).
KML_API int kml_conv_unroll22_multi(const bf16_t* const* ws, bf16_t* const* wus, const int* dims, int n,
                                    hipStream_t s) {
  if (n < 1 || n > 16) return (int)hipErrorInvalidValue;
  UnrollBatch ub = {};
  ub.n = n;
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    UnrollJob& j = ub.j[i];
    j.w = ws[i]; j.wu = wus[i];
    j.K = dims[2 * i]; j.C = dims[2 * i + 1];
    if (j.C % 8 || j.K < 1 || !j.w || !j.wu) return (int)hipErrorInvalidValue;
    j.block_begin = (int)blocks;
    blocks += ((long long)4 * j.K * (j.C / 2) + 256 * UNROLL_V - 1) / (256 * UNROLL_V);
  }
  if (blocks <= 0 || blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_unroll22_multi, dim3((unsigned)blocks), dim3(256), 0, s, ub);
  KML_LAUNCH_CHECK();
}

// bnf_*: optional consumer-BN backward partials (see ConvArgs); bnf_part = null disables.
// grp_*: optional group reduction of those partial rows.  variant 3 (direct): wt is the
// transposed weight copy (kml_weight_transpose, Kp = roundup(K, 32)) and bk the wave count.
KML_API int kml_conv_dgrad(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, bf16_t* dx, const bf16_t* addend,
                           const bf16_t* bnf_y, const bf16_t* bnf_c, const float* bnf_mean, const float* bnf_rstd,
                           float* bnf_part, float* grp_out, unsigned* grp_cnt, int grp_tiles, int B, int H, int W,
                           int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, int bm, int bn, int bk,
                           int splits, int variant, float* slab, unsigned* counters, int fold_c, int bnf_mask_out,
                           int g22, hipStream_t s) {
  ConvArgs a;
  const int e = prep_dgrad(a, dy, w, wt, dx, addend, bnf_y, bnf_c, bnf_mean, bnf_rstd, bnf_part, grp_out, grp_cnt,
                           grp_tiles, B, H, W, C, K, KH, KW, sh, sw, ph, pw, bk, splits, variant, slab, counters,
                           fold_c, bnf_mask_out, g22);
  if (e) return e;
  if (variant == 3) return dispatch_direct<DGRAD>(a, bm, bn, bk, s);
  if (variant == 5) {  // one-shot panels (single tap, contiguous dY rows, K = Cout)
    const bool one_tap = (a.r1 - a.r0) == 1 && (a.s1 - a.s0) == 1;
    const bool rows = (H * W == 1 && a.OH * a.OW == 1) || (KH == 1 && KW == 1 && sh == 1 && sw == 1 && !ph && !pw);
    if (!one_tap || !rows || a.splits != 1) return (int)hipErrorInvalidValue;
    a.Kd = K;
    return dispatch_oneshot_bwd<DGRAD>(a, bm, bn, s);
  }
  if (variant == 4) {  // halo patch of dy (Cout channels), flipped-filter slice of Cin columns
    if (g22 || fold_c || a.splits != 1 || !halo_shape_ok(H, W, K, C, KH, KW, sh, sw, ph, pw, bm, bn))
      return (int)hipErrorInvalidValue;
    return dispatch_halo<DGRAD>(a, bm, bn, s);
  }
  if (variant) bk = 64;
  return dispatch<DGRAD>(a, bm, bn, bk, variant, s);
}

// Stride-2 DGRAD as four parity classes (ConvArgs::par): class (pa, pe) computes the input
// pixels (2i + pa, 2j + pe) from the taps of matching parity only — 1/4 of the gathered
// (pixel, tap) pairs of the plain stride-2 dgrad are non-zero, and a class with no taps
// (1x1/s2: three of four) runs the epilogue alone (addend / zeros, consumer-BN partials).
// Plain igemm / glds variants, no split-K, no group reduction; bnf_part holds the classes'
// partial rows back to back (kml_conv_dgrad_s2_rows).
// Host mirror of conv_epilogue's ROWPASS condition for a DGRAD plan (Body::SMEM formulas of
// IgemmBody / GldsBody): the parity-class launches need the row-pass epilogue.
static bool s2_rowpass_ok(int bm, int bn, int bk, int variant) {
  if (bn % 64 || bm * bn < 4096) return false;
  long long smem;
  if (variant == 1 || variant == 2) {
    smem = (long long)(variant == 1 ? 3 : 4) * (bm + bn) * 64 * 2;
  } else {
    const long long ta = (long long)bm * (bk + PADK);
    const long long tb = (bn == 32 || bn == 64 || bn == 128) ? (long long)bk * bn : (long long)bk * (bn + PADR);
    smem = 2 * (ta + tb) * 2;
  }
  return smem >= 16 + (long long)bm * bn * 4;
}

KML_API int kml_conv_dgrad_s2_ok(int bm, int bn, int bk, int variant) {
  // the instantiations of dispatch_par (all of which take the row pass)
  bool listed = false;
  if (variant == 0)
    listed = (bm == 64 && bn == 64 && (bk == 32 || bk == 64)) ||
             (bk == 64 && ((bm == 64 && bn == 128) || (bm == 128 && bn == 64) || (bm == 128 && bn == 128)));
  else if (variant == 1)
    listed = (bm == 64 || bm == 128) && (bn == 64 || bn == 128);
  else if (variant == 2)
    listed = (bm == 64 && (bn == 64 || bn == 128)) || (bm == 128 && bn == 64);
  return listed && s2_rowpass_ok(bm, bn, variant ? 64 : bk, variant) ? 1 : 0;
}

KML_API int kml_conv_dgrad_s2_rows(int B, int H, int W, int bm) {
  int rows = 0;
  for (int c = 0; c < 4; ++c) {
    const int pa = c >> 1, pe = c & 1;
    const long long Mc = (long long)B * ((H - pa + 1) / 2) * ((W - pe + 1) / 2);
    rows += (int)((Mc + bm - 1) / bm);
  }
  return rows;
}

KML_API int kml_conv_dgrad_s2(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const bf16_t* addend,
                              const bf16_t* bnf_y, const bf16_t* bnf_c, const float* bnf_mean, const float* bnf_rstd,
                              float* bnf_part, int B, int H, int W, int C, int K, int KH, int KW, int ph, int pw,
                              int bm, int bn, int bk, int variant, int bnf_mask_out, hipStream_t s) {
  if (!kml_conv_dgrad_s2_ok(bm, bn, bk, variant) || (!addend && !bnf_part)) return (int)hipErrorInvalidValue;
  ConvArgs a0;
  int e = prep_dgrad(a0, dy, w, nullptr, dx, addend, bnf_y, bnf_c, bnf_mean, bnf_rstd, bnf_part, nullptr, nullptr, 0,
                     B, H, W, C, K, KH, KW, 2, 2, ph, pw, bk, 1, variant, nullptr, nullptr, 0, bnf_mask_out, 0);
  if (e) return e;
  if (variant) bk = 64;
  int rowbase = 0;
  for (int c = 0; c < 4; ++c) {
    ConvArgs a = a0;
    const int pa = c >> 1, pe = c & 1;
    a.par = 1 | (pa << 1) | (pe << 2);
    const int Hc = (H - pa + 1) / 2, Wc = (W - pe + 1) / 2;
    a.fd_H = make_fd(Hc > 0 ? Hc : 1); a.fd_W = make_fd(Wc > 0 ? Wc : 1);
    a.M = B * Hc * Wc;
    if (a.M <= 0) continue;
    a.r0 = (pa + ph) & 1; a.s0 = (pe + pw) & 1;
    const int nr = a.r0 < KH ? (KH - a.r0 + 1) / 2 : 0, ns = a.s0 < KW ? (KW - a.s0 + 1) / 2 : 0;
    a.r1 = a.r0 + 2 * nr; a.s1 = a.s0 + 2 * ns;
    a.fd_nts = make_fd(ns > 0 ? ns : 1);
    a.Kd = nr * ns * a.Kp;
    a.kchunk = a.Kd > 0 ? (a.Kd + bk - 1) / bk * bk : bk;
    a.splits = 1;
    if (bnf_part) a.bnf_part = bnf_part + (long long)rowbase * 2 * C;
    rowbase += (a.M + bm - 1) / bm;
    e = dispatch_par(a, bm, bn, bk, variant, s);
    if (e) return e;
  }
  return 0;
}

KML_API int kml_weight_transpose(const bf16_t* w, bf16_t* wt, int K, int KH, int KW, int C, hipStream_t s) {
  const int Kp = (K + 31) / 32 * 32, T = KH * KW;
  hipLaunchKernelGGL(k_weight_transpose, dim3(kml_stream_grid((long long)C * T * Kp, 256)), dim3(256), 0, s, w, wt,
                     K, T, C, Kp);
  KML_LAUNCH_CHECK();
}

KML_API int kml_conv_wgrad(const bf16_t* x, const bf16_t* dy, float* dw, int B, int H, int W, int C, int K, int KH,
                           int KW, int sh, int sw, int ph, int pw, int bm, int bn, int bk, int splits, int variant,
                           int accumulate, float* slab, unsigned* counters, float* dbias, int bias_acc,
                           hipStream_t s) {
  ConvArgs a;
  const int e = prep_wgrad(a, x, dy, dw, B, H, W, C, K, KH, KW, sh, sw, ph, pw, bk, splits, variant, accumulate,
                           slab, counters, dbias, bias_acc);
  if (e) return e;
  if (variant == 5) {  // one-shot panels: single tap, K = pixels, no split-K, no bias column
    const bool one_tap = (a.r1 - a.r0) == 1 && (a.s1 - a.s0) == 1;
    const bool rows = (H * W == 1 && a.OH * a.OW == 1) || (KH == 1 && KW == 1 && sh == 1 && sw == 1 && !ph && !pw);
    if (!one_tap || !rows || dbias || a.splits != 1) return (int)hipErrorInvalidValue;
    return dispatch_oneshot_bwd<WGRAD>(a, bm, bn, s);
  }
  if (variant) bk = 64;
  return dispatch<WGRAD>(a, bm, bn, bk, variant, s);
}

// ---------------------------------------------------------------------------------
// Weight gradient of an unrolled conv (3x3/s1/p1 on a 2x2 map, run as its dense 1x1 form):
// the 1x1-form GEMM leaves G[(p, n)][(q, c)] (p, q = output / input position 0..3) in a
// scratch, and dW[n][tap][c] = sum over the (p, q) with tap(p, q) = tap of G — 4 pairs on the
// centre tap, 2 on an edge, 1 on a corner, 9 taps — summed here in a fixed pair order and
// stored (acc = 0) or added (acc = 1): deterministic, no atomics.  Up to 16 convs per launch
// (all the unrolled convs of one backward stage); one thread per (n, c4) of one job.
// ---------------------------------------------------------------------------------
struct Fold22Job {
  const float* g;  // [4K][4C]
  float* dw;       // [K][3][3][C]
  int K, C, acc, block_begin;
};
struct Fold22Batch {
  Fold22Job j[16];
  int n;
};

__global__ __launch_bounds__(256) void k_fold22_multi(Fold22Batch fb) {
  int q = 0;
  while (q + 1 < fb.n && (int)blockIdx.x >= fb.j[q + 1].block_begin) ++q;  // block-uniform
  const Fold22Job& jb = fb.j[q];
  const long long idx = (long long)((int)blockIdx.x - jb.block_begin) * 256 + threadIdx.x;
  const int C4 = jb.C / 4;
  if (idx >= (long long)jb.K * C4) return;
  const int n = (int)(idx / C4), c = (int)(idx - (long long)n * C4) * 4;
  const long long ldg = 4LL * jb.C;  // G row length
  float4 t[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) t[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {  // fixed (p, q) order: bitwise reproducible
      const int tap = ((qq >> 1) - (p >> 1) + 1) * 3 + ((qq & 1) - (p & 1) + 1);
      const float4 v = *reinterpret_cast<const float4*>(jb.g + ((long long)p * jb.K + n) * ldg + (long long)qq * jb.C + c);
      t[tap].x += v.x; t[tap].y += v.y; t[tap].z += v.z; t[tap].w += v.w;
    }
  float* base = jb.dw + (long long)n * 9 * jb.C + c;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    float4* d = reinterpret_cast<float4*>(base + (long long)k * jb.C);
    if (jb.acc) {
      const float4 o = *d;
      *d = make_float4(o.x + t[k].x, o.y + t[k].y, o.z + t[k].z, o.w + t[k].w);
    } else {
      *d = t[k];
    }
  }
}

// gs[i] = [4K][4C] fp32 1x1-form gradient, dws[i] = [K][3][3][C] fp32; dims: n x 3 ints (K, C, acc)
KML_API int kml_conv_fold22_multi(const float* const* gs, float* const* dws, const int* dims, int n, hipStream_t s) {
  if (n < 1 || n > 16) return (int)hipErrorInvalidValue;
  Fold22Batch fb = {};
  fb.n = n;
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    Fold22Job& j = fb.j[i];
    j.g = gs[i]; j.dw = dws[i];
    j.K = dims[3 * i]; j.C = dims[3 * i + 1]; j.acc = dims[3 * i + 2];
    if (!j.g || !j.dw || j.K < 1 || j.C % 4 || (((uintptr_t)j.g | (uintptr_t)j.dw) & 15)) return (int)hipErrorInvalidValue;
    j.block_begin = (int)blocks;
    blocks += ((long long)j.K * (j.C / 4) + 255) / 256;
  }
  if (blocks <= 0 || blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fold22_multi, dim3((unsigned)blocks), dim3(256), 0, s, fb);
  KML_LAUNCH_CHECK();
}
