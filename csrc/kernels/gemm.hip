// gemm.hip — large bf16 GEMMs (BERT-size linears) on gfx950 MFMA, fp32 accumulate.
//
//   C[m][n] = act( sum_k A[m][k] * B[n][k] + bias[n] )        (bf16 out, optional pre-act copy)
//   C[m][n] = beta * C[m][n] + sum_k A[m][k] * B[n][k]         (fp32 out: weight gradients)
//   C[m][n] += sum_{k in slice z} A[m][k] * B[n][k]            (fp32 split-K, agent atomics)
//
// Operand layouts (row = m for A, n for B):  KC: X[row][k] (k contiguous), KS: X[k][row].
// The three GEMMs of a linear layer y = x W^T + b (x [T][in], W [out][in]):
//   forward  y[T][out]   A = x   (KC)  B = W   (KC)
//   dgrad    dx[T][in]   A = dy  (KC)  B = W   (KS: reduction over out, rows of W)
//   wgrad    dW[out][in] A = dy  (KS)  B = x   (KS: reduction over tokens)
//
// CDNA4 mapping (CDNA guide §5):
// * 512 threads = 8 wave64 as 2 (M) x 4 (N); a BM x BN block tile (256 or 128 per side),
//   wave tile (BM/2) x (BN/4) of v_mfma_f32_16x16x32_bf16 fragments, BK = 64.
// * Operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//   instruction), two LDS stages: the DMA of K-tile t+1 is issued right after the barrier
//   that publishes tile t and overlaps tile t's MFMAs; one barrier per K-step.  The LDS
//   image is lane-linear, so bank swizzles go on the per-lane SOURCE address and are undone
//   on the fragment read (guide §5.4 rule 21): KC tiles [rows][64] (128 B rows) use
//   chunk ^= row & 7 (ds_read_b128), KS tiles [64][R] a row-bit permutation read with the
//   transposing ds_read_b64_tr_b16 — both conflict-free (tools/lds_banks.py).
// * The MFMA is issued with the B fragment as its first operand, so a lane's accumulator
//   holds 4 consecutive OUTPUT COLUMNS of one output row: the epilogue (bias, erf-GELU,
//   bf16 pack, or fp32 beta / atomic accumulate) stores 8 or 16 contiguous bytes per lane
//   straight from registers — no LDS staging pass.
// * Out-of-range rows / K columns read a zero page instead of branching (counted vmcnt
//   stays straight-line); stores are masked.  XCD-aware block order (guide T1).
//
// Replaces hipBLASLt/Tensile on the BERT hot path (the reference has no BERT; SURVEY §2.8
// north-star config 5).
#include "kml_common.h"

#include <type_traits>

namespace {

typedef __attribute__((ext_vector_type(4))) short v4s_t;

constexpr int GEMM_ADD_C2 = 3;  // act code: C = bf16(bf16(A B) + c2)
// act code (k_gemm8 dgrad only): C = bf16(bf16(A B) * gelu'(c2)) — the FFN's GELU backward in
// the epilogue of the dgrad that produced d(activation), c2 = the saved pre-activation; the
// column sums of C (the FFN1 bias gradient) go to colpart[M / 256][N] (one row per M-tile)
constexpr int GEMM_GELU_BWD = 4;
// act code (layout 0, bf16 out): BatchNorm statistics of the output in the epilogue — a 1x1
// stride-1 convolution run as this GEMM (ops.kernels.conv_fwd's GEMM route) writes one partial
// row [sum(N) | sumsq(N)] per M-tile to colpart[M / BM][2 N], the layout of the implicit-GEMM
// conv's stats_part rows that the BN apply kernel folds.  Sums are over the bf16-rounded outputs
// (the values BN normalises) in a fixed order, so the rows are deterministic.
constexpr int GEMM_STATS = 5;
// act code (layout 1, bf16 out, tiles 0-4): the epilogue of a 1x1 stride-1 conv's input gradient
// (ops.kernels.conv_dgrad's GEMM route), as the implicit-GEMM dgrad's: v = A B (+ the bf16 addend
// c2, the residual branch's gradient) rounded once; with bc (the consumer BN's input) the masked
// dz = v * [by > 0] (by optional) gives colpart[M / BM][2 N] = per-M-tile [sum dz | sum dz * xhat],
// xhat = (bc - bmean[n]) * brstd[n]; mask_out stores dz instead of v.
constexpr int GEMM_BNF = 6;

struct GemmArgs {
  const bf16_t* a;
  const bf16_t* b;
  void* c;
  bf16_t* c2;          // optional pre-activation copy (bf16 out only); with act == GEMM_ADD_C2 a
                       // bf16 addend summed into the output (fused residual-gradient sum)
  const float* bias;   // [N] fp32 or null
  const bf16_t* zp;    // >= 16 zero bytes
  long long lda, ldb, ldc;
  int M, N, K;
  int act;             // 0 none, 1 erf-GELU
  float beta;
  int kchunk;          // split-K slice length (multiple of 64)
  float* colpart;      // GEMM_GELU_BWD: per-M-tile column sums of the output; GEMM_STATS / BNF: [M/BM][2N]
  const bf16_t* by;    // GEMM_BNF: consumer BN's ReLU output (mask) or null
  const bf16_t* bc;    // GEMM_BNF: consumer BN's input or null (no partial rows)
  const float* bmean;  // GEMM_BNF: [N]
  const float* brstd;  // GEMM_BNF: [N]
  int mask_out;        // GEMM_BNF: store dz = v * [by > 0]
  // implicit-GEMM forward (k_gemm AG = 1): A = im2col(x) gathered by ConvStagerA; x NHWC [B][H][W][C],
  // output pixel m = (b, oh, ow), K index k = tap * C + c (C % 64 == 0: a K-tile sits in one tap)
  int cH, cW, cC, cOH, cOW, cKW, csh, csw, cph, cpw;
  int cK;              // implicit-GEMM dgrad (AG = 2): output channels of dy (K % 64 == 0)
  int rowpass;         // bf16 output of a 128 x 128 tile through LDS rows (gemm_out_rowpass)
  // group reduction of the row-pass partial rows (GEMM_STATS / GEMM_BNF): every grp_tiles consecutive
  // M-tiles form a group whose last-arriving block (agent-scope ticket per (group, n-tile)) sums the
  // group's rows in order into grp_out[g][2N] — the BN kernel then reads <= 16 rows, no fold launch
  float* grp_out;
  unsigned* grp_cnt;
  int grp_tiles;
};

// the conv routes' forward GEMMs store through LDS rows (ResNet-50 15.82 -> 15.63 ms/step,
// profiles/r5/r50/r50_ab_out_rowpass.txt)
static int out_rowpass_default() { return 1; }

constexpr int BK = 64;
constexpr int NT = 512;

template <int R>
__device__ __forceinline__ int swz_ks(int r) {  // K-strided [64][R] chunk swizzle (R >= 128)
  if constexpr (R == 192)  // 384-byte rows: flips inside aligned groups of 8 chunks (24 per row)
    return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
  else
    return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
}

__device__ __forceinline__ bf16x8_t frag_kc(const char* lds, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  const int c = 4 * ks + (lane >> 4);
  return *reinterpret_cast<const bf16x8_t*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
}

template <int R>
__device__ __forceinline__ bf16x8_t frag_ks(const char* lds, int row0, int ks, int lane) {
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

// One operand's DMA plan: NI instructions per wave per stage.  KC: tile [R][64], 8 rows
// per 1 KiB instruction; KS: tile [64][R], 512/R k-rows per instruction.
template <int R, bool KC>
struct Stager {
  static constexpr int NI = R / 64;   // (R * 64 * 2 bytes) / 1 KiB / 8 waves
  const bf16_t* base[NI];              // source of K-tile 0 (before the kb offset)
  int lim[NI];                         // KC: k offset of the lane's chunk; KS: k-row in tile
  bool ok[NI];                         // row (KC) / column chunk (KS) in range
  long long kstep;                     // address delta per K element
  __device__ void init(const bf16_t* p, long long ld, int r0, int rows, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int u = wave * NI + j;
      if constexpr (KC) {
        const int row = 8 * u + (lane >> 3);
        const int chunk = (lane & 7) ^ (row & 7);
        ok[j] = r0 + row < rows;
        base[j] = p + (long long)(ok[j] ? r0 + row : 0) * ld + chunk * 8;
        lim[j] = chunk * 8;
      } else {
        constexpr int CPR = R / 8, RPI = 64 / CPR;
        const int krow = RPI * u + lane / CPR;
        const int chunk = (lane % CPR) ^ swz_ks<R>(krow);
        ok[j] = r0 + chunk * 8 < rows;
        base[j] = p + (long long)krow * ld + (ok[j] ? r0 + chunk * 8 : 0);
        lim[j] = krow;
      }
    }
    kstep = KC ? 1 : ld;
  }
  __device__ __forceinline__ void issue(char* lds, int kb, int kend, const bf16_t* zp, int wave) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const bool in = ok[j] && kb + lim[j] < kend;
      const bf16_t* src = in ? base[j] + (long long)kb * kstep : zp;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + (wave * NI + j) * 1024), 16, 0,
                                       0);
    }
  }
};

// A operand of the implicit-GEMM forward: the KC [R][64] tile of im2col(x) for R output pixels.
// Same lane -> (row, chunk) mapping and LDS image as Stager<R, true>; per K-tile the tap is uniform
// (k = tap * C + c, C % 64 == 0), so a lane's source is its pixel's input row shifted by the tap,
// or the zero page where the tap falls in the padding.
template <int R, bool DG = false>
struct ConvStagerA {
  // DG = false (forward): row = output pixel (b, oh, ow), source x [B][H][W][C], tap (r, s) reads
  //   (oh sh - ph + r, ow sw - pw + s).
  // DG = true (stride-1 input gradient): row = input pixel (b, ih, iw), source dy [B][OH][OW][K],
  //   tap (r, s) reads (ih + ph - r, iw + pw - s); k = tap * K + cout.
  static constexpr int NI = R / 64;
  const bf16_t* base[NI];   // source + ((b SH + p0) SW + q0) SC + chunk * 8 (may point outside the source)
  int p0[NI], q0[NI];
  bool ok[NI];
  __device__ void init(const GemmArgs& g, int r0, int wave, int lane) {
    const int GW = DG ? g.cW : g.cOW, GH = DG ? g.cH : g.cOH;
    const int SH = DG ? g.cOH : g.cH, SW = DG ? g.cOW : g.cW, SC = DG ? g.cK : g.cC;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int u = wave * NI + j;
      const int row = 8 * u + (lane >> 3);
      const int chunk = (lane & 7) ^ (row & 7);
      const int m = r0 + row;
      ok[j] = m < g.M;
      const int mm = ok[j] ? m : 0;
      const int t = mm / GW, x = mm - t * GW;
      const int b = t / GH, y = t - b * GH;
      p0[j] = DG ? y + g.cph : y * g.csh - g.cph;
      q0[j] = DG ? x + g.cpw : x * g.csw - g.cpw;
      base[j] = g.a + ((long long)(b * SH + p0[j]) * SW + q0[j]) * SC + chunk * 8;
    }
  }
  __device__ __forceinline__ void issue(char* lds, const GemmArgs& g, int kb, int kend, int wave) const {
    const int SH = DG ? g.cOH : g.cH, SW = DG ? g.cOW : g.cW, SC = DG ? g.cK : g.cC;
    const int tap = kb / SC, c0 = kb - tap * SC;
    const int r = tap / g.cKW, sx = tap - r * g.cKW;
    const long long shift = (DG ? -((long long)r * SW + sx) : ((long long)r * SW + sx)) * SC + c0;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int ih = DG ? p0[j] - r : p0[j] + r, iw = DG ? q0[j] - sx : q0[j] + sx;
      const bool in = ok[j] && kb < kend && (unsigned)ih < (unsigned)SH && (unsigned)iw < (unsigned)SW;
      const bf16_t* src = in ? base[j] + shift : g.zp;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + (wave * NI + j) * 1024), 16, 0,
                                       0);
    }
  }
};

// B operand of the implicit-GEMM input gradient: the KS [64][R] tile of W^T with k = tap * K + cout
// and n = cin — W [K][KH][KW][C] read as rows cout (stride KH KW C) shifted by the K-tile's tap.
// Same lane mapping / LDS image as Stager<R, false>.
// B operand of the implicit-GEMM weight gradient: the KS [64][R] tile of im2col(x), k = output pixel,
// n = tap * C + cin.  A lane's 8-channel column chunk stays in one tap (C % 8 == 0), so (r, s, c) are
// fixed at init; its k-row's pixel (b, oh, ow) is decoded per K-tile.
template <int R>
struct ConvStagerBW {
  static constexpr int NI = R / 64;
  int krow[NI], r[NI], sx[NI], c[NI];
  bool ok[NI];
  __device__ void init(const GemmArgs& g, int n0, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int u = wave * NI + j;
      constexpr int CPR = R / 8, RPI = 64 / CPR;
      krow[j] = RPI * u + lane / CPR;
      const int chunk = (lane % CPR) ^ swz_ks<R>(krow[j]);
      const int col = n0 + chunk * 8;
      ok[j] = col < g.N;
      const int cc = ok[j] ? col : 0;
      const int tap = cc / g.cC;
      c[j] = cc - tap * g.cC;
      r[j] = tap / g.cKW;
      sx[j] = tap - r[j] * g.cKW;
    }
  }
  __device__ __forceinline__ void issue(char* lds, const GemmArgs& g, int kb, int kend, int wave) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int p = kb + krow[j];
      bool in = ok[j] && p < kend;
      const int pp = in ? p : 0;
      const int t = pp / g.cOW, ow = pp - t * g.cOW;
      const int b = t / g.cOH, oh = t - b * g.cOH;
      const int ih = oh * g.csh - g.cph + r[j], iw = ow * g.csw - g.cpw + sx[j];
      in = in && (unsigned)ih < (unsigned)g.cH && (unsigned)iw < (unsigned)g.cW;
      const bf16_t* src = in ? g.b + ((long long)(b * g.cH + ih) * g.cW + iw) * g.cC + c[j] : g.zp;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + (wave * NI + j) * 1024), 16, 0,
                                       0);
    }
  }
};

template <int R>
struct ConvStagerB {
  static constexpr int NI = R / 64;
  const bf16_t* base[NI];
  int lim[NI];
  bool ok[NI];
  __device__ void init(const GemmArgs& g, int r0, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int u = wave * NI + j;
      constexpr int CPR = R / 8, RPI = 64 / CPR;
      const int krow = RPI * u + lane / CPR;
      const int chunk = (lane % CPR) ^ swz_ks<R>(krow);
      ok[j] = r0 + chunk * 8 < g.N;
      base[j] = g.b + (long long)krow * g.ldb + (ok[j] ? r0 + chunk * 8 : 0);
      lim[j] = krow;
    }
  }
  __device__ __forceinline__ void issue(char* lds, const GemmArgs& g, int kb, int kend, int wave) const {
    const int tap = kb / g.cK, k0 = kb - tap * g.cK;
    const long long shift = (long long)k0 * g.ldb + (long long)tap * g.cC;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const bool in = ok[j] && kb + lim[j] < kend;
      const bf16_t* src = in ? base[j] + shift : g.zp;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + (wave * NI + j) * 1024), 16, 0,
                                       0);
    }
  }
};

__device__ __forceinline__ float gelu_erf(float x) { return kml_gelu(x); }

// XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a contiguous run of
// tiles (bijective remap, CDNA guide T1), and walk that run in GROUPS of up to 8 tile rows
// (column-major inside a group), so the ~32 tiles an XCD's CUs hold at once form a block
// of 8 rows x 4 columns: 12 operand panels through its 4 MB L2 instead of 33 for a
// row-major run (1 A panel + 32 B panels) — an operand panel of a 256-wide tile is
// re-fetched past L2 by a quarter / an eighth of the CUs instead of by every one.
__device__ __forceinline__ void xcd_tile(int& tx, int& ty, int& tz) {
  const int gx = (int)gridDim.x, gy = (int)gridDim.y;
  const int nwg = gx * gy * (int)gridDim.z;
  const int lin = ((int)blockIdx.z * gy + (int)blockIdx.y) * gx + (int)blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, x = lin & 7, k = lin >> 3;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  const int per = gx * gy;
  tz = id / per;
  const int t = id - tz * per;
  constexpr int G = 8;
  const int grp = t / (G * gx);
  const int row0 = grp * G;
  const int rows = min(G, gy - row0);
  const int w = t - grp * G * gx;
  ty = row0 + w % rows;
  tx = w / rows;
}

// epilogue: lane holds C[m][n .. n+3], m = .. + (lane & 15), n = .. + 4 * (lane >> 4)
template <int OUT, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                              int wn, int lane, int tz) {
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = m0 + wm * WM + i * 16 + (lane & 15);
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (OUT == 0) {
        if (g.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(g.bias + n);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        }
        const long long off = (long long)m * g.ldc + n;
        if (g.act == GEMM_ADD_C2) {  // + bf16 addend: round, add, round (= a separate bf16 add)
          const uint2 ad = *reinterpret_cast<const uint2*>(g.c2 + off);
          const uint2 q = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
          v[0] = lo_bf(q.x) + lo_bf(ad.x); v[1] = hi_bf(q.x) + hi_bf(ad.x);
          v[2] = lo_bf(q.y) + lo_bf(ad.y); v[3] = hi_bf(q.y) + hi_bf(ad.y);
        } else if (g.c2) {
          uint2 p;
          p.x = pack_bf2(v[0], v[1]);
          p.y = pack_bf2(v[2], v[3]);
          *reinterpret_cast<uint2*>(g.c2 + off) = p;
        }
        if (g.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
        }
        uint2 p;
        p.x = pack_bf2(v[0], v[1]);
        p.y = pack_bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.c) + off) = p;
      } else if constexpr (OUT == 1) {
        float4* p = reinterpret_cast<float4*>(static_cast<float*>(g.c) + (long long)m * g.ldc + n);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g.beta != 0.f) {
          o = *p;
          o.x *= g.beta; o.y *= g.beta; o.z *= g.beta; o.w *= g.beta;
        }
        o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
        *p = o;
      } else if constexpr (OUT == 2) {
        float* p = static_cast<float*>(g.c) + (long long)m * g.ldc + n;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __hip_atomic_fetch_add(p + r, v[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {   // OUT 3: this K-slice's partial tile into slab tz (plain 16-byte stores)
        float* p = static_cast<float*>(g.c) + (long long)tz * g.M * g.ldc + (long long)m * g.ldc + n;
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// 32x32x16 variant (k_gemm MF = 32): the A / B fragment of lane l is row (l & 31), k = 8 (l >> 5) .. +7
// of a KC [rows][64] tile (same chunk swizzle as frag_kc); with B as the MFMA's first operand a lane's
// accumulator registers 4g .. 4g+3 hold output row m = .. + (l & 31), columns n = .. + 8g + 4 (l >> 5) .. +3
__device__ __forceinline__ bf16x8_t frag_kc32(const char* lds, int row0, int ks, int lane) {
  const int r = row0 + (lane & 31);
  const int c = 2 * ks + (lane >> 5);
  return *reinterpret_cast<const bf16x8_t*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
}

// the 4 consecutive output columns n .. n+3 of row m (OUT 0: bias, GELU, pre-activation copy; OUT 1)
template <int OUT>
__device__ __forceinline__ void gemm_store4(const GemmArgs& g, int m, int n, float (&v)[4]) {
  if constexpr (OUT == 0) {
    if (g.bias) {
      const float4 bb = *reinterpret_cast<const float4*>(g.bias + n);
      v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
    }
    const long long off = (long long)m * g.ldc + n;
    if (g.act == GEMM_ADD_C2) {
      const uint2 ad = *reinterpret_cast<const uint2*>(g.c2 + off);
      const uint2 q = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      v[0] = lo_bf(q.x) + lo_bf(ad.x); v[1] = hi_bf(q.x) + hi_bf(ad.x);
      v[2] = lo_bf(q.y) + lo_bf(ad.y); v[3] = hi_bf(q.y) + hi_bf(ad.y);
    } else if (g.c2) {
      *reinterpret_cast<uint2*>(g.c2 + off) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
    if (g.act == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
    }
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.c) + off) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
  } else {
    float4* p = reinterpret_cast<float4*>(static_cast<float*>(g.c) + (long long)m * g.ldc + n);
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.beta != 0.f) {
      o = *p;
      o.x *= g.beta; o.y *= g.beta; o.z *= g.beta; o.w *= g.beta;
    }
    o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
    *p = o;
  }
}

template <int OUT, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_epilogue32(const GemmArgs& g, f32x16_t (&acc)[MR][NR], int m0, int n0, int wm,
                                                int wn, int lane) {
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = m0 + wm * WM + i * 32 + (lane & 31);
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * WN + j * 32 + 8 * q + 4 * (lane >> 5);
        if (n >= g.N) continue;
        float v[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        gemm_store4<OUT>(g, m, n, v);
      }
  }
}

// GEMM_STATS rows of a k_gemm tile (bf16 out): per-lane sums of the bf16-rounded outputs over the
// lane's rows, a butterfly over the 16 lanes of a column group, then the two wave rows summed
// through LDS (wave row 0 + wave row 1, fixed order).  Entered by every thread of the block.
template <int BM, int BN, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_stats_rows(const GemmArgs& g, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                                int wn, int lane, char* smem) {
  float s1[NR][4], s2[NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
    const float4 bb = (g.bias && n < g.N) ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      if (m < g.M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = lo_bf(pack_bf2(acc[i][j][r] + bv[r], 0.f));
          s1[j][r] += x;
          s2[j][r] += x * x;
        }
      }
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] += __shfl_xor(s1[j][r], off, 64);
        s2[j][r] += __shfl_xor(s2[j][r], off, 64);
      }
  }
  __syncthreads();  // every wave is done with the operand stages
  float* red = reinterpret_cast<float*>(smem);  // [sum | sumsq][BN] of wave row 1
  if (wm == 1 && (lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * WN + j * 16 + 4 * (lane >> 4) + r;
        red[col] = s1[j][r];
        red[BN + col] = s2[j][r];
      }
  }
  __syncthreads();
  if (wm == 0 && (lane & 15) == 0) {
    float* row = g.colpart + (long long)(m0 / BM) * 2 * g.N;
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * WN + j * 16 + 4 * (lane >> 4) + r, n = n0 + col;
        if (n < g.N) {
          row[n] = s1[j][r] + red[col];
          row[g.N + n] = s2[j][r] + red[BN + col];
        }
      }
  }
}

// GEMM_BNF epilogue of a k_gemm tile (layout 1, bf16 out): lane holds C[m][n .. n+3]; the addend,
// mask and BN input are read as 8-byte chunks beside the 8-byte output store; the per-lane partial
// sums are reduced as in gemm_stats_rows (16-lane butterfly, wave rows 0 + 1 through LDS).
template <int BM, int BN, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_bnf_epilogue(const GemmArgs& g, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                                  int wn, int lane, char* smem) {
  const bool bnf = g.bc != nullptr;
  float s1[NR][4], s2[NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
    const bool nok = n < g.N;
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, rs[4] = {0.f, 0.f, 0.f, 0.f};
    if (bnf && nok) {
      const float4 a4 = *reinterpret_cast<const float4*>(g.bmean + n);
      const float4 b4 = *reinterpret_cast<const float4*>(g.brstd + n);
      mu[0] = a4.x; mu[1] = a4.y; mu[2] = a4.z; mu[3] = a4.w;
      rs[0] = b4.x; rs[1] = b4.y; rs[2] = b4.z; rs[3] = b4.w;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      if (m >= g.M || !nok) continue;
      const long long off = (long long)m * g.ldc + n;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (g.c2) {
        const uint2 ad = *reinterpret_cast<const uint2*>(g.c2 + off);
        v[0] += lo_bf(ad.x); v[1] += hi_bf(ad.x); v[2] += lo_bf(ad.y); v[3] += hi_bf(ad.y);
      }
      unsigned w0 = pack_bf2(v[0], v[1]), w1 = pack_bf2(v[2], v[3]);
      if (bnf) {
        const uint2 cv = *reinterpret_cast<const uint2*>(g.bc + off);
        float dz[4] = {lo_bf(w0), hi_bf(w0), lo_bf(w1), hi_bf(w1)};
        if (g.by) {
          const uint2 yv = *reinterpret_cast<const uint2*>(g.by + off);
          const bool k0 = lo_bf(yv.x) > 0.f, k1 = hi_bf(yv.x) > 0.f, k2 = lo_bf(yv.y) > 0.f, k3 = hi_bf(yv.y) > 0.f;
          if (!k0) dz[0] = 0.f;
          if (!k1) dz[1] = 0.f;
          if (!k2) dz[2] = 0.f;
          if (!k3) dz[3] = 0.f;
          if (g.mask_out) {
            w0 &= (k0 ? 0x0000ffffu : 0u) | (k1 ? 0xffff0000u : 0u);
            w1 &= (k2 ? 0x0000ffffu : 0u) | (k3 ? 0xffff0000u : 0u);
          }
        }
        const float c[4] = {lo_bf(cv.x), hi_bf(cv.x), lo_bf(cv.y), hi_bf(cv.y)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] += dz[r];
          s2[j][r] += dz[r] * ((c[r] - mu[r]) * rs[r]);
        }
      }
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.c) + off) = make_uint2(w0, w1);
    }
    if (bnf) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] += __shfl_xor(s1[j][r], off, 64);
          s2[j][r] += __shfl_xor(s2[j][r], off, 64);
        }
    }
  }
  if (!bnf) return;
  __syncthreads();  // every wave is done with the operand stages
  float* red = reinterpret_cast<float*>(smem);
  if (wm == 1 && (lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * WN + j * 16 + 4 * (lane >> 4) + r;
        red[col] = s1[j][r];
        red[BN + col] = s2[j][r];
      }
  }
  __syncthreads();
  if (wm == 0 && (lane & 15) == 0) {
    float* row = g.colpart + (long long)(m0 / BM) * 2 * g.N;
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * WN + j * 16 + 4 * (lane >> 4) + r, n = n0 + col;
        if (n < g.N) {
          row[n] = s1[j][r] + red[col];
          row[g.N + n] = s2[j][r] + red[BN + col];
        }
      }
  }
}

// Partial-row store of a row-pass epilogue: write-through at agent scope when a group reduction in
// this launch reads it (the conv kernels' store_row / group_reduce_rows protocol: no fences; every
// storing wave drains before the ticket; the last arriver reads past its L1 with agent-scope loads).
__device__ __forceinline__ void gemm_store_row(float* p, float v, bool grp) {
  if (grp) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

template <int BM, int BN>
__device__ __forceinline__ void gemm_group_rows(const GemmArgs& g, int m0, int n0, int tid, unsigned* flag) {
  const int tile_m = m0 / BM, tile_n = n0 / BN;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int grp = tile_m / g.grp_tiles;
  const int t0 = grp * g.grp_tiles, t1 = min(ntm, t0 + g.grp_tiles);
  unsigned* cnt = g.grp_cnt + grp * ntn + tile_n;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its rows
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = (t == (unsigned)(t1 - t0 - 1)) ? 1u : 0u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  for (int q = tid; q < 2 * BN; q += NT) {
    const int half = q / BN, col = n0 + (q - half * BN);
    if (col >= g.N) continue;
    const float* src = g.colpart + (long long)half * g.N + col;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int r = t0;
    for (; r + 4 <= t1; r += 4) {  // 4 loads in flight, fixed summation order
      a0 += __hip_atomic_load(const_cast<float*>(src + (long long)r * 2 * g.N), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a1 += __hip_atomic_load(const_cast<float*>(src + (long long)(r + 1) * 2 * g.N), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a2 += __hip_atomic_load(const_cast<float*>(src + (long long)(r + 2) * 2 * g.N), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a3 += __hip_atomic_load(const_cast<float*>(src + (long long)(r + 3) * 2 * g.N), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (; r < t1; ++r)
      a0 += __hip_atomic_load(const_cast<float*>(src + (long long)r * 2 * g.N), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g.grp_out[(long long)grp * 2 * g.N + (long long)half * g.N + col] = (a0 + a1) + (a2 + a3);
  }
}

// Per-thread rows of the epilogue column-sum partials: 16 (or 8) floats padded to an odd stride,
// so the per-k stores of a 32-lane half hit 32 distinct banks (a 16-float stride put every other
// lane on one bank: a 16-way ds_write_b32 conflict) and the fixed-order column reads at most 2-way.
constexpr int RED_STR = 17, RED_STR8 = 9;

// GEMM_BNF epilogue through LDS rows (128 x 128 tiles): the fp32 tile is staged in LDS (16-byte
// chunks XOR-swizzled by row), then every thread owns one 8-column chunk and walks rows with 16-byte
// loads of the addend / mask / BN input and 16-byte stores — full cache lines instead of the register
// epilogue's 16 rows x 32 B per wave instruction.  v = acc + addend is rounded once, as in the
// register path; the partial rows are summed in a fixed order (deterministic).
template <int BM, int BN, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_bnf_rowpass(const GemmArgs& g, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                                 int wn, int lane, int tid, char* smem) {
  constexpr int CPR = BN / 8, RSTEP = NT / CPR;
  float* sF = reinterpret_cast<float*>(smem);
  __syncthreads();  // every wave is done with the operand stages
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int row = wm * WM + i * 16 + (lane & 15), ch = (wn * WN + j * 16) / 4 + (lane >> 4);
      const f32x4_t a = acc[i][j];
      *reinterpret_cast<float4*>(sF + row * BN + ((ch ^ (row & 15)) << 2)) = make_float4(a[0], a[1], a[2], a[3]);
    }
  __syncthreads();
  const int q = tid % CPR, r0 = tid / CPR;
  const int n = n0 + q * 8;
  const bool nok = n < g.N, bnf = g.bc != nullptr;
  float mu[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { mu[k] = 0.f; rs[k] = 0.f; s1[k] = 0.f; s2[k] = 0.f; }
  if (bnf && nok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { mu[k] = g.bmean[n + k]; rs[k] = g.brstd[n + k]; }
  }
  for (int r = r0; r < BM; r += RSTEP) {
    const int m = m0 + r;
    if (m >= g.M || !nok) continue;
    // (reading the odd chunk first on lanes q >= 8, conflict-free 16-lane phases, measured neutral:
    // profiles/r5/r50/ab12_rowpass_swz_run{1,2}.txt)
    const float4 p0 = *reinterpret_cast<const float4*>(sF + r * BN + (((2 * q) ^ (r & 15)) << 2));
    const float4 p1 = *reinterpret_cast<const float4*>(sF + r * BN + (((2 * q + 1) ^ (r & 15)) << 2));
    float v[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    const long long off = (long long)m * g.ldc + n;
    if (g.c2) {
      const uint4 ad = *reinterpret_cast<const uint4*>(g.c2 + off);
      const unsigned aw[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[2 * k] += lo_bf(aw[k]); v[2 * k + 1] += hi_bf(aw[k]); }
    }
    unsigned ow[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ow[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
    if (bnf) {
      const uint4 cv = *reinterpret_cast<const uint4*>(g.bc + off);
      const uint4 yv = g.by ? *reinterpret_cast<const uint4*>(g.by + off) : make_uint4(0, 0, 0, 0);
      const unsigned cw[4] = {cv.x, cv.y, cv.z, cv.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float dz0 = lo_bf(ow[k]), dz1 = hi_bf(ow[k]);
        if (g.by) {
          const bool k0 = lo_bf(yw[k]) > 0.f, k1 = hi_bf(yw[k]) > 0.f;
          if (!k0) dz0 = 0.f;
          if (!k1) dz1 = 0.f;
          if (g.mask_out) ow[k] &= (k0 ? 0x0000ffffu : 0u) | (k1 ? 0xffff0000u : 0u);
        }
        s1[2 * k] += dz0; s2[2 * k] += dz0 * ((lo_bf(cw[k]) - mu[2 * k]) * rs[2 * k]);
        s1[2 * k + 1] += dz1; s2[2 * k + 1] += dz1 * ((hi_bf(cw[k]) - mu[2 * k + 1]) * rs[2 * k + 1]);
      }
    }
    *reinterpret_cast<uint4*>(static_cast<bf16_t*>(g.c) + off) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
  if (!bnf) return;
  __syncthreads();  // staging reads done: the area is reused as [NT][16] partial sums
  float* red = sF;
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[tid * RED_STR + k] = s1[k]; red[tid * RED_STR + 8 + k] = s2[k]; }
  __syncthreads();
  for (int t = tid; t < 2 * BN; t += NT) {
    const int half = t / BN, cl = t - half * BN, nn = n0 + cl;
    if (nn >= g.N) continue;
    const int qq = cl >> 3, k = (cl & 7) + 8 * half;
    float sum = 0.f;
    for (int rr = 0; rr < RSTEP; ++rr) sum += red[(rr * CPR + qq) * RED_STR + k];
    gemm_store_row(g.colpart + (long long)(m0 / BM) * 2 * g.N + (half ? g.N : 0) + nn, sum, g.grp_out != nullptr);
  }
  if (g.grp_out) {
    __syncthreads();  // red reads done: smem word 0 becomes the ticket flag
    gemm_group_rows<BM, BN>(g, m0, n0, tid, reinterpret_cast<unsigned*>(smem));
  }
}

// bf16 output of a 128 x 128 k_gemm tile through LDS rows (act 0 or GEMM_STATS, no c2): fp32 tile
// (+ bias) staged as in gemm_bnf_rowpass, then 16-byte row-contiguous stores; with GEMM_STATS every
// thread sums its 8 columns' bf16 outputs over its rows and the 32 partials per chunk are added in a
// fixed order into the tile's [sum | sumsq] row.
template <int BM, int BN, int MR, int NR, int WM, int WN>
__device__ __forceinline__ void gemm_out_rowpass(const GemmArgs& g, f32x4_t (&acc)[MR][NR], int m0, int n0, int wm,
                                                 int wn, int lane, int tid, char* smem) {
  constexpr int CPR = BN / 8, RSTEP = NT / CPR;
  float* sF = reinterpret_cast<float*>(smem);
  __syncthreads();  // every wave is done with the operand stages
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int col = wn * WN + j * 16 + 4 * (lane >> 4), n = n0 + col;
    const float4 bb = (g.bias && n < g.N) ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int row = wm * WM + i * 16 + (lane & 15), ch = col / 4;
      const f32x4_t a = acc[i][j];
      *reinterpret_cast<float4*>(sF + row * BN + ((ch ^ (row & 15)) << 2)) =
          make_float4(a[0] + bb.x, a[1] + bb.y, a[2] + bb.z, a[3] + bb.w);
    }
  }
  __syncthreads();
  const int q = tid % CPR, r0 = tid / CPR;
  const int n = n0 + q * 8;
  const bool nok = n < g.N, st = g.act == GEMM_STATS;
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  for (int r = r0; r < BM; r += RSTEP) {
    const int m = m0 + r;
    if (m >= g.M || !nok) continue;
    const float4 p0 = *reinterpret_cast<const float4*>(sF + r * BN + (((2 * q) ^ (r & 15)) << 2));
    const float4 p1 = *reinterpret_cast<const float4*>(sF + r * BN + (((2 * q + 1) ^ (r & 15)) << 2));
    const unsigned ow[4] = {pack_bf2(p0.x, p0.y), pack_bf2(p0.z, p0.w), pack_bf2(p1.x, p1.y), pack_bf2(p1.z, p1.w)};
    if (st) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x0 = lo_bf(ow[k]), x1 = hi_bf(ow[k]);
        s1[2 * k] += x0; s2[2 * k] += x0 * x0;
        s1[2 * k + 1] += x1; s2[2 * k + 1] += x1 * x1;
      }
    }
    *reinterpret_cast<uint4*>(static_cast<bf16_t*>(g.c) + (long long)m * g.ldc + n) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
  if (!st) return;
  __syncthreads();
  float* red = sF;
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[tid * RED_STR + k] = s1[k]; red[tid * RED_STR + 8 + k] = s2[k]; }
  __syncthreads();
  for (int t = tid; t < 2 * BN; t += NT) {
    const int half = t / BN, cl = t - half * BN, nn = n0 + cl;
    if (nn >= g.N) continue;
    const int qq = cl >> 3, k = (cl & 7) + 8 * half;
    float sum = 0.f;
    for (int rr = 0; rr < RSTEP; ++rr) sum += red[(rr * CPR + qq) * RED_STR + k];
    gemm_store_row(g.colpart + (long long)(m0 / BM) * 2 * g.N + (half ? g.N : 0) + nn, sum, g.grp_out != nullptr);
  }
  if (g.grp_out) {
    __syncthreads();  // red reads done: smem word 0 becomes the ticket flag
    gemm_group_rows<BM, BN>(g, m0, n0, tid, reinterpret_cast<unsigned*>(smem));
  }
}

// OUT: 0 bf16 (bias, act, optional pre-act copy), 1 fp32 beta, 2 fp32 atomic add (split-K)
// S: LDS stages.  S = 2: the DMA of tile t+1 overlaps tile t's MFMAs, vmcnt(0) per step.
// S = 3: tiles t+1 and t+2 in flight; each step waits with a COUNTED vmcnt for tile t only,
// so one tile's DMA stays in flight across the raw s_barrier (CDNA guide §5 "Pipelining
// across barriers"; trailing steps re-issue the last tile into a stage nobody reads, so
// the count never changes).
template <int BM, int BN, bool A_KC, bool B_KC, int OUT, int S, int AG = 0, int MF = 16>
__global__ __launch_bounds__(NT) void k_gemm(GemmArgs g) {
  static_assert(AG == 0 || (AG == 1 && A_KC && B_KC && OUT == 0) || (AG == 2 && A_KC && !B_KC && OUT == 0) ||
                    (AG == 3 && !A_KC && !B_KC && OUT == 3),
                "implicit-GEMM gather: forward (AG 1) / input-gradient (AG 2) bf16 out, weight gradient (AG 3) slabs");
  static_assert(MF == 16 || (MF == 32 && A_KC && B_KC && AG == 0 && OUT <= 1),
                "the 32x32x16 form: K-contiguous operands, register epilogue (bf16 / fp32 out)");
  constexpr int WM = BM / 2, WN = BN / 4, MR = WM / MF, NR = WN / MF;
  using acc_t = typename std::conditional<MF == 32, f32x16_t, f32x4_t>::type;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int NI = BM / 64 + BN / 64;   // DMA instructions per wave per stage
  static_assert(S * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];

  int tx, ty, tz;
  xcd_tile(tx, ty, tz);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = ty * BM, n0 = tx * BN;
  const int kbeg = tz * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  constexpr bool AGA = AG == 1 || AG == 2;   // gathered A (forward / input gradient)
  typename std::conditional<AGA, ConvStagerA<BM, AG == 2>, Stager<BM, A_KC>>::type sa;
  typename std::conditional<AG == 2, ConvStagerB<BN>,
                            typename std::conditional<AG == 3, ConvStagerBW<BN>, Stager<BN, B_KC>>::type>::type sb;
  if constexpr (AGA) sa.init(g, m0, wave, lane);
  else sa.init(g.a, g.lda, m0, g.M, wave, lane);
  if constexpr (AG >= 2) sb.init(g, n0, wave, lane);
  else sb.init(g.b, g.ldb, n0, g.N, wave, lane);

  acc_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = acc_t{};

  auto issue = [&](int kt, int st) {
    char* dst = smem + st * STAGE;
    if constexpr (AGA) sa.issue(dst, g, kbeg + kt * BK, kend, wave);
    else sa.issue(dst, kbeg + kt * BK, kend, g.zp, wave);
    if constexpr (AG >= 2) sb.issue(dst + A_BYTES, g, kbeg + kt * BK, kend, wave);
    else sb.issue(dst + A_BYTES, kbeg + kt * BK, kend, g.zp, wave);
  };
  auto compute = [&](int st) {
    const char* sA = smem + st * STAGE;
    const char* sB = sA + A_BYTES;
    if constexpr (MF == 32) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8_t af[MR], bfr[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) bfr[j] = frag_kc32(sB, wn * WN + j * 32, ks, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i) af[i] = frag_kc32(sA, wm * WM + i * 32, ks, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t af[MR], bfr[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j)
          bfr[j] = B_KC ? frag_kc(sB, wn * WN + j * 16, ks, lane) : frag_ks<BN>(sB, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i)
          af[i] = A_KC ? frag_kc(sA, wm * WM + i * 16, ks, lane) : frag_ks<BM>(sA, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  };

  if (nk > 0) {
    if constexpr (S == 2) {
      issue(0, 0);
      for (int t = 0; t < nk; ++t) {
        // stage t landed for this wave's DMAs; after the barrier, for every wave's; and every
        // wave finished reading the other stage (its fragment reads were waited for by the MFMAs)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
        compute(t & 1);
      }
    } else {
      const int last = nk - 1;
      issue(0, 0);
      issue(min(1, last), 1);
      int cur = 0;
      for (int t = 0; t < nk; ++t) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");   // tile t done, t+1 may fly
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int nx = cur == 0 ? 2 : cur - 1;                       // (t + 2) % 3
        issue(min(t + 2, last), nx);
        compute(cur);
        cur = cur == 2 ? 0 : cur + 1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");               // drain redundant tail DMAs
    }
  }

  if constexpr (MF == 32) {
    gemm_epilogue32<OUT, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane);
    return;
  } else {
  if constexpr (OUT == 0) {
    if (g.act == GEMM_BNF) {
      if constexpr (BM == 128 && BN == 128 && S * STAGE >= BM * BN * 4) {
        gemm_bnf_rowpass<BM, BN, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, tid, smem);
      } else {
        gemm_bnf_epilogue<BM, BN, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, smem);
      }
      return;
    }
  }
  if constexpr (OUT == 0 && BM == 128 && BN == 128 && S * STAGE >= BM * BN * 4) {
    if (g.rowpass && (g.act == 0 || g.act == GEMM_STATS) && !g.c2 && g.N % 8 == 0 && g.ldc % 8 == 0) {
      gemm_out_rowpass<BM, BN, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, tid, smem);
      return;
    }
  }
  gemm_epilogue<OUT, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, tz);
  if constexpr (OUT == 0) {
    if (g.act == GEMM_STATS) gemm_stats_rows<BM, BN, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, smem);
  }
  }
}

// ---------------------------------------------------------------------------------------
// 256 x 256 tile, BK = 32 slots in a 4-deep LDS ring (4 x 32 KB): TWO K-tiles stay in
// flight behind the one being consumed, and the fragments of tile t+1 are read from LDS
// while tile t's MFMAs run (register double buffer), so neither the DMA latency nor the
// LDS read latency sits on the MFMA path.  Per step: counted vmcnt for tile t+1, one
// raw barrier, DMA of tile t+3 into the slot tile t-1 vacated, ds_reads of t+1, MFMAs of
// t.  (The CDNA guide's half-tile 8-phase idea at the granularity this code can express.)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bf16x8_t frag_kc64(const char* lds, int row0, int lane) {  // [R][32] tiles
  const int r = row0 + (lane & 15);
  const int c = lane >> 4;
  return *reinterpret_cast<const bf16x8_t*>(lds + r * 64 + ((c ^ ((r >> 1) & 3)) << 4));
}

// Fragment reads as inline asm (k_gemm8): hipcc's waitcnt pass cannot count LDS reads
// across the loop back-edge and would put lgkmcnt(0) in front of every MFMA cluster; with
// the reads hidden from it, each C segment waits with its own counted lgkmcnt (CDNA guide
// §5.4 rule 18: a sched_barrier(0) follows every such wait).
__device__ __forceinline__ unsigned lds_off(const char* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ bf16x8_t ds_rd128(const char* p) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_off(p)));
  return v;
}
__device__ __forceinline__ v4s_t ds_rd_tr(const char* p) {
  v4s_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_off(p)));
  return v;
}
__device__ __forceinline__ bf16x8_t frag_kc64_asm(const char* lds, int row0, int lane) {
  const int r = row0 + (lane & 15);
  const int c = lane >> 4;
  return ds_rd128(lds + r * 64 + ((c ^ ((r >> 1) & 3)) << 4));
}
template <int R>
__device__ __forceinline__ bf16x8_t frag_ks_asm(const char* lds, int row0, int lane) {  // k rows 0-31
  const int il = lane & 15, g = lane >> 4;
  const int col = row0 + 4 * (il & 3);
  const int k0 = 8 * g + (il >> 2);
  const int k1 = k0 + 4;
  const int ch = col >> 3, within = (col & 7) * 2;
  v4s_t lo = ds_rd_tr(lds + k0 * (2 * R) + ((ch ^ swz_ks<R>(k0)) << 4) + within);
  v4s_t hi = ds_rd_tr(lds + k1 * (2 * R) + ((ch ^ swz_ks<R>(k1)) << 4) + within);
  bf16x8_t f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

// R = 192 (the 256x192 phase tile's B operand): 12 instructions per slot, two on waves 0-5 and
// none on waves 6-7 — see k_gemm8 for why the counted waits stay exact.
template <int R, bool KC>
struct Stager32 {  // BK = 32 slots: KC [R][32] (16 rows / KiB), KS [32][R] (R / 8 16-byte chunks per k-row)
  static constexpr int NTOT = R / 16;          // 1 KiB instructions per slot
  static constexpr int NI = (NTOT + 7) / 8;    // per wave (the last waves may issue fewer)
  const bf16_t* base[NI];
  int lim[NI];
  bool ok[NI];
  long long kstep;
  __device__ void init(const bf16_t* p, long long ld, int r0, int rows, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int u = min(wave * NI + j, NTOT - 1);   // clamped: unused slots are never issued
      if constexpr (KC) {
        const int row = 16 * u + (lane >> 2);
        const int chunk = (lane & 3) ^ ((row >> 1) & 3);
        ok[j] = r0 + row < rows;
        base[j] = p + (long long)(ok[j] ? r0 + row : 0) * ld + chunk * 8;
        lim[j] = chunk * 8;
      } else {
        constexpr int CPR = R / 8;
        const int idx = 64 * u + lane;           // lane-linear 16-byte position in the slot
        const int krow = idx / CPR;
        const int chunk = (idx % CPR) ^ swz_ks<R>(krow);
        ok[j] = r0 + chunk * 8 < rows;
        base[j] = p + (long long)krow * ld + (ok[j] ? r0 + chunk * 8 : 0);
        lim[j] = krow;
      }
    }
    kstep = KC ? 1 : ld;
  }
  __device__ __forceinline__ void issue(char* lds, int kb, int kend, const bf16_t* zp, int wave) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      if (NTOT % 8 != 0 && wave * NI + j >= NTOT) break;   // wave-uniform
      const bool in = ok[j] && kb + lim[j] < kend;
      const bf16_t* src = in ? base[j] + (long long)kb * kstep : zp;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds + (wave * NI + j) * 1024), 16, 0,
                                       0);
    }
  }
};

template <bool A_KC, bool B_KC, int OUT>
__global__ __launch_bounds__(NT) void k_gemm4(GemmArgs g) {
  constexpr int BM = 256, BN = 256, BK32 = 32;
  constexpr int WM = BM / 2, WN = BN / 4, MR = WM / 16, NR = WN / 16;
  constexpr int A_BYTES = BM * BK32 * 2, B_BYTES = BN * BK32 * 2, SLOT = A_BYTES + B_BYTES;
  constexpr int NI = BM / 128 + BN / 128;
  __shared__ __attribute__((aligned(1024))) char smem[4 * SLOT];

  int tx, ty, tz;
  xcd_tile(tx, ty, tz);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = ty * BM, n0 = tx * BN;
  const int kbeg = tz * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK32 - 1) / BK32 : 0;

  Stager32<BM, A_KC> sa;
  Stager32<BN, B_KC> sb;
  sa.init(g.a, g.lda, m0, g.M, wave, lane);
  sb.init(g.b, g.ldb, n0, g.N, wave, lane);

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int slot) {
    char* dst = smem + slot * SLOT;
    sa.issue(dst, kbeg + kt * BK32, kend, g.zp, wave);
    sb.issue(dst + A_BYTES, kbeg + kt * BK32, kend, g.zp, wave);
  };
  auto read = [&](int slot, bf16x8_t* af, bf16x8_t* bfr) {
    const char* sA = smem + slot * SLOT;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int j = 0; j < NR; ++j)
      bfr[j] = B_KC ? frag_kc64(sB, wn * WN + j * 16, lane) : frag_ks<BN>(sB, wn * WN + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < MR; ++i)
      af[i] = A_KC ? frag_kc64(sA, wm * WM + i * 16, lane) : frag_ks<BM>(sA, wm * WM + i * 16, 0, lane);
  };
  auto mma = [&](const bf16x8_t* af, const bf16x8_t* bfr) {
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

  if (nk > 0) {
    const int last = nk - 1;
    bf16x8_t a0[MR], b0[NR], a1[MR], b1[NR];
    issue(0, 0);
    issue(min(1, last), 1);
    issue(min(2, last), 2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");   // tile 0 landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read(0, a0, b0);
    // two K-tiles per trip so the fragment double buffer has static register names
    for (int t = 0; t < nk; t += 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");       // tile t+1 landed, t+2 flies
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");              // reads of tile t done
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue(min(t + 3, last), (t + 3) & 3);                           // into tile t-1's slot
      read((t + 1) & 3, a1, b1);
      mma(a0, b0);
      if (t + 1 >= nk) break;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue(min(t + 4, last), (t + 4) & 3);
      read((t + 2) & 3, a0, b0);
      mma(a1, b1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gemm_epilogue<OUT, MR, NR, WM, WN>(g, acc, m0, n0, wm, wn, lane, tz);
}

// ---------------------------------------------------------------------------------------
// 256 x 256 tile, two-group phase schedule (CDNA guide §5 "256² 8-phase template", T3-T5).
//
// K-tiles of 64 are split into four 16 KB half-tiles {A k0-31, B k0-31, A k32-63, B
// k32-63}; LDS holds two K-tiles (8 half-tile slots, 128 KB).  A K-tile is four PHASES:
//   q = 0: k 0-31,  wave rows 0-63   (reads 4 A + 4 B fragments)
//   q = 1: k 0-31,  wave rows 64-127 (reads 4 A; B fragments kept)
//   q = 2 / 3: the same on k 32-63
// and every phase is an L segment (fragment ds_reads + this thread's two LDS-DMAs of one
// half-tile) and a C segment (lgkmcnt(0), 16 MFMAs under s_setprio 1), separated by raw
// s_barriers.  Waves 4-7 (group 1, the M rows 128-255) run one barrier behind waves 0-3,
// so on every SIMD one wave is in its MFMA segment while its partner reads / issues DMAs:
// the matrix pipe never waits for the LDS.
//
// Half-tile h (= 4 * tile + q) is issued in phase h - 5, i.e. five half-tiles ahead; its
// slot was last read >= 2 phases earlier (WAR safe for both groups).  The L segment of
// phase P reads phase P+1's fragments (register double buffer), so the MFMAs never wait
// for a just-issued ds_read.  Each group retires DMAs with ONE counted vmcnt per two
// phases — group 0 vmcnt(4) after even phases, group 1 vmcnt(2) after odd phases — which
// lands every half-tile before the barrier that precedes its first read by either group
// (derivation in the comment of k_gemm8 below).
//
// Epilogue (bf16 out): bias / erf-GELU in registers, the tile staged through the (now
// idle) LDS with a row-XOR swizzle, then 16-byte row-contiguous global stores (512 B per
// half-wave): full cache lines instead of 16 rows x 32 B per store instruction.
// ---------------------------------------------------------------------------------------
template <bool A_KC, bool B_KC, int OUT, int BN = 256>
__global__ __launch_bounds__(NT) void k_gemm8(GemmArgs g) {
  static_assert(BN == 256 || BN == 192, "k_gemm8: BN is 256 or 192");
  constexpr int HT = 256 * 32 * 2;  // half-tile slot bytes (a 192-row B half-tile uses 12 of 16 KB)
  constexpr int MR = 8, NR = BN / 64;  // wave tile 128 x (BN / 4)
  constexpr int WN = BN / 4;
  __shared__ __attribute__((aligned(1024))) char smem[8 * HT];

  int tx, ty, tz;
  xcd_tile(tx, ty, tz);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = ty * 256, n0 = tx * BN;
  const int kbeg = tz * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + 63) / 64 : 0;

  Stager32<256, A_KC> sa;
  Stager32<BN, B_KC> sb;
  sa.init(g.a, g.lda, m0, g.M, wave, lane);
  sb.init(g.b, g.ldb, n0, g.N, wave, lane);

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // half-tile h -> slot (h/4 & 1)*4 + h%4; past the last K-tile the stager reads the zero
  // page (kb >= kend), so the DMA count per phase never changes
  auto issue_h = [&](int h) {
    const int u = h >> 2, q = h & 3;
    char* dst = smem + ((u & 1) * 4 + q) * HT;
    const int kb = kbeg + u * 64 + ((q & 2) ? 32 : 0);
    if (q & 1) sb.issue(dst, kb, kend, g.zp, wave);
    else sa.issue(dst, kb, kend, g.zp, wave);
  };

  if (nk > 0) {
    // fragment double buffer: the L segment of phase P reads phase P+1's fragments, so the
    // C segment's counted lgkmcnt only waits for reads issued a whole phase earlier
    bf16x8_t af0[4], af1[4], bf0[NR], bf1[NR];
    auto read_frags = [&](auto qc, int u, bf16x8_t(&af)[4], bf16x8_t(&bfr)[NR]) {
      constexpr int q = decltype(qc)::value;
      const char* sA = smem + ((u & 1) * 4 + ((q & 2) ? 2 : 0)) * HT;
      const char* sB = smem + ((u & 1) * 4 + ((q & 2) ? 3 : 1)) * HT;
      if constexpr ((q & 1) == 0) {
#pragma unroll
        for (int j = 0; j < NR; ++j)
          bfr[j] = B_KC ? frag_kc64_asm(sB, wn * WN + j * 16, lane) : frag_ks_asm<BN>(sB, wn * WN + j * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 128 + (q & 1) * 64 + i * 16;
        af[i] = A_KC ? frag_kc64_asm(sA, r, lane) : frag_ks_asm<256>(sA, r, lane);
      }
    };
    // LDS read instructions one L segment issues for phase q (B fragments on even q only)
    constexpr int RA = A_KC ? 4 : 8, RB = B_KC ? NR : 2 * NR;
    // Phase P = 4u + q.  Group 0: L_P between barriers 2P and 2P+1, C_P between 2P+1 and
    // 2P+2; group 1 one barrier later.  L_P reads phase P+1's fragments; C_P's lgkmcnt
    // retires phase P's reads (issued in L_{P-1}) before barrier 2P+2 (group 0) / 2P+3
    // (group 1).  WAR: a slot holding phase-R data is refilled by the DMA of L_{R+2}, past
    // barrier 2R+4 for both groups.  RAW: the lo half-tiles of tile u+1 (issued in phases
    // 4u-1, 4u) are first read in L_{4u+3} (group 0 after barrier 8u+6): group 0's vmcnt(4)
    // after C_{4u+2} and group 1's vmcnt(2) after C_{4u+1} retire them before barriers
    // 8u+6 / 8u+5.  The hi half-tiles (issued 4u+1, 4u+2) are first read in L_{4u+5} (after
    // barrier 8u+10): group 0's wait after C_{4u+4}, group 1's after C_{4u+3}.
    auto phase = [&](auto qc, int u, bf16x8_t(&afc)[4], bf16x8_t(&bfc)[NR], bf16x8_t(&afn)[4],
                     bf16x8_t(&bfn)[NR]) {
      constexpr int q = decltype(qc)::value;
      constexpr int qn = (q + 1) & 3;
      const int P = 4 * u + q;
      // ---- L segment: next phase's fragments + one half-tile of DMA
      read_frags(std::integral_constant<int, qn>{}, qn == 0 ? u + 1 : u, afn, bfn);
      issue_h(P + 5);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- C segment: retire phase P's fragment reads (issued in L_{P-1}); L_P's stay in flight
      constexpr int NREAD = RA + ((qn & 1) == 0 ? RB : 0);
      static_assert(NREAD == 4 || NREAD == 7 || NREAD == 8 || NREAD == 10 || NREAD == 11 || NREAD == 12 ||
                    NREAD >= 14, "k_gemm8: add the lgkmcnt for this read count");
      if constexpr (NREAD >= 15) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
      else if constexpr (NREAD == 14) asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
      else if constexpr (NREAD == 12) asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
      else if constexpr (NREAD == 11) asm volatile("s_waitcnt lgkmcnt(11)" ::: "memory");
      else if constexpr (NREAD == 10) asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
      else if constexpr (NREAD == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else if constexpr (NREAD == 7) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[(q & 1) * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfc[j], afc[i], acc[(q & 1) * 4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (q & 1) {
        if (wm == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        if (wm == 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int h = 0; h < 5; ++h) issue_h(h);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // tile 0 landed (half-tile 4 may fly)
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();           // group 1 starts one barrier behind
    __builtin_amdgcn_sched_barrier(0);
    read_frags(std::integral_constant<int, 0>{}, 0, af0, bf0);
    __builtin_amdgcn_sched_barrier(0);
    for (int u = 0; u < nk; ++u) {
      phase(std::integral_constant<int, 0>{}, u, af0, bf0, af1, bf0);   // reads phase 1 (A only)
      phase(std::integral_constant<int, 1>{}, u, af1, bf0, af0, bf1);   // reads phase 2 (A + B)
      phase(std::integral_constant<int, 2>{}, u, af0, bf1, af1, bf1);   // reads phase 3 (A only)
      phase(std::integral_constant<int, 3>{}, u, af1, bf1, af0, bf0);   // reads phase 4 = next tile q 0
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // trailing DMAs / reads touch LDS
  }

  if constexpr (OUT != 0) {
    gemm_epilogue<OUT, MR, NR, 128, WN>(g, acc, m0, n0, wm, wn, lane, tz);
  } else {
    // staged tile [256][BN] bf16: row stride 2 BN bytes, 16-byte chunk ch of row r at ch ^ swz(r)
    // (BN = 192: 24 chunks per row, the XOR stays inside aligned groups of 8)
    constexpr int CPR = BN / 8;
    auto stg = [](int row, int ch) { return row * (2 * BN) + ((ch ^ (BN == 256 ? (row & 15) : (row & 7))) << 4); };
    __syncthreads();
    float4 bias4[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
      bias4[j] = (g.bias && n < g.N) ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // fp32 accumulators -> (+bias, act) bf16 -> swizzled LDS tile [256][256]
    auto stage = [&](bool act) {
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const int row = wm * 128 + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int col = wn * WN + j * 16 + 4 * (lane >> 4);
          float v0 = acc[i][j][0] + bias4[j].x, v1 = acc[i][j][1] + bias4[j].y;
          float v2 = acc[i][j][2] + bias4[j].z, v3 = acc[i][j][3] + bias4[j].w;
          if (act) { v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3); }
          uint2 p;
          p.x = pack_bf2(v0, v1);
          p.y = pack_bf2(v2, v3);
          const int off = stg(row, col >> 3) + ((col >> 2) & 1) * 8;
          *reinterpret_cast<uint2*>(smem + off) = p;
        }
        __builtin_amdgcn_sched_barrier(0);   // one fragment row at a time: bounds the temporaries
      }
      __syncthreads();
    };
    // LDS tile -> 16-byte row-contiguous global stores (512 B per half-wave)
    const bool gbwd = g.act == GEMM_GELU_BWD, gst = BN == 256 && g.act == GEMM_STATS;
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // GELU_BWD / STATS: this thread's 8 columns
    float csq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // STATS: sums of squares
    auto store = [&](bf16_t* dst) {
#pragma unroll 2
      for (int it = 0; it < 256 * CPR / NT; ++it) {
        const int idx = it * NT + tid;
        const int row = idx / CPR, ch = idx % CPR;
        uint4 v = *reinterpret_cast<const uint4*>(smem + stg(row, ch));
        const int m = m0 + row, n = n0 + ch * 8;
        if (m < g.M && n < g.N) {
          if (BN == 256 && gbwd) {  // d(pre) = bf16(bf16(d act) * gelu'(pre)), as k_gelu_bwd_colsum
            const uint4 pv = *reinterpret_cast<const uint4*>(g.c2 + (long long)m * g.ldc + n);
            const unsigned dw[4] = {v.x, v.y, v.z, v.w}, pw[4] = {pv.x, pv.y, pv.z, pv.w};
            unsigned ow[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              ow[k] = pack_bf2(lo_bf(dw[k]) * kml_gelu_grad(lo_bf(pw[k])), hi_bf(dw[k]) * kml_gelu_grad(hi_bf(pw[k])));
              csum[2 * k] += lo_bf(ow[k]);
              csum[2 * k + 1] += hi_bf(ow[k]);
            }
            v = make_uint4(ow[0], ow[1], ow[2], ow[3]);
          }
          if (gst) {  // BN statistics of the bf16 output (BN = 256: a thread's 8 columns are fixed)
            const unsigned ow[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float x0 = lo_bf(ow[k]), x1 = hi_bf(ow[k]);
              csum[2 * k] += x0; csq[2 * k] += x0 * x0;
              csum[2 * k + 1] += x1; csq[2 * k + 1] += x1 * x1;
            }
          }
          if (g.act == GEMM_ADD_C2) {  // + bf16 addend (the staged tile is already bf16-rounded)
            const uint4 ad = *reinterpret_cast<const uint4*>(g.c2 + (long long)m * g.ldc + n);
            v.x = pack_bf2(lo_bf(v.x) + lo_bf(ad.x), hi_bf(v.x) + hi_bf(ad.x));
            v.y = pack_bf2(lo_bf(v.y) + lo_bf(ad.y), hi_bf(v.y) + hi_bf(ad.y));
            v.z = pack_bf2(lo_bf(v.z) + lo_bf(ad.z), hi_bf(v.z) + hi_bf(ad.z));
            v.w = pack_bf2(lo_bf(v.w) + lo_bf(ad.w), hi_bf(v.w) + hi_bf(ad.w));
          }
          *reinterpret_cast<uint4*>(dst + (long long)m * g.ldc + n) = v;
        }
      }
      __syncthreads();
    };
    if (g.c2 && g.act != GEMM_ADD_C2 && !gbwd) {   // pre-activation copy first: the accumulators stay live across it
      stage(false);
      store(g.c2);
    }
    stage(g.act == 1);
    store(static_cast<bf16_t*>(g.c));
    if (BN == 256 && gbwd) {  // column sums: 16 threads (tid >> 5) share each 8-column chunk; fixed order
      float* red = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int k = 0; k < 8; ++k) red[tid * RED_STR8 + k] = csum[k];
      __syncthreads();
      if (tid < 256) {
        const int ch = tid >> 3, k = tid & 7, n = n0 + tid;
        float sum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += red[((r << 5) + ch) * RED_STR8 + k];
        if (n < g.N) g.colpart[(long long)(m0 / 256) * g.N + n] = sum;
      }
    }
    if (gst) {  // [sum | sumsq] row of this M-tile: 16 threads share each 8-column chunk, fixed order
      float* red = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int k = 0; k < 8; ++k) { red[tid * RED_STR + k] = csum[k]; red[tid * RED_STR + 8 + k] = csq[k]; }
      __syncthreads();
      if (tid < 256) {
        const int ch = tid >> 3, k = tid & 7, n = n0 + tid;
        float sum = 0.f, sq = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sum += red[((r << 5) + ch) * RED_STR + k];
          sq += red[((r << 5) + ch) * RED_STR + 8 + k];
        }
        if (n < g.N) {
          float* row = g.colpart + (long long)(m0 / 256) * 2 * g.N;
          row[n] = sum;
          row[g.N + n] = sq;
        }
      }
    }
  }
}

template <bool A_KC, bool B_KC, int OUT, int BN = 256>
int launch8(GemmArgs g, int splits, hipStream_t s) {
  if (BN != 256 && g.act == GEMM_GELU_BWD) return (int)hipErrorInvalidValue;
  splits = splits < 1 ? 1 : splits;
  int chunk = (g.K + splits - 1) / splits;
  chunk = ((chunk + 63) / 64) * 64;
  g.kchunk = chunk > 0 ? chunk : 64;
  const int z = g.K > 0 ? (g.K + g.kchunk - 1) / g.kchunk : 1;
  dim3 grid((g.N + BN - 1) / BN, (g.M + 255) / 256, z);
  hipLaunchKernelGGL((k_gemm8<A_KC, B_KC, OUT, BN>), grid, dim3(NT), 0, s, g);
  KML_LAUNCH_CHECK();
}

template <int BM, int BN, bool A_KC, bool B_KC, int OUT, int S = (3 * (BM + BN) * BK * 2 <= 160 * 1024) ? 3 : 2,
          int AG = 0, int MF = 16>
int launch(GemmArgs g, int splits, hipStream_t s) {
  splits = splits < 1 ? 1 : splits;
  int chunk = (g.K + splits - 1) / splits;
  chunk = ((chunk + BK - 1) / BK) * BK;
  g.kchunk = chunk > 0 ? chunk : BK;
  const int z = g.K > 0 ? (g.K + g.kchunk - 1) / g.kchunk : 1;
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, z);
  hipLaunchKernelGGL((k_gemm<BM, BN, A_KC, B_KC, OUT, S, AG, MF>), grid, dim3(NT), 0, s, g);
  KML_LAUNCH_CHECK();
}

template <bool A_KC, bool B_KC, int OUT>
int launch4(GemmArgs g, int splits, hipStream_t s) {
  splits = splits < 1 ? 1 : splits;
  int chunk = (g.K + splits - 1) / splits;
  chunk = ((chunk + 63) / 64) * 64;
  g.kchunk = chunk > 0 ? chunk : 64;
  const int z = g.K > 0 ? (g.K + g.kchunk - 1) / g.kchunk : 1;
  dim3 grid((g.N + 255) / 256, (g.M + 255) / 256, z);
  hipLaunchKernelGGL((k_gemm4<A_KC, B_KC, OUT>), grid, dim3(NT), 0, s, g);
  KML_LAUNCH_CHECK();
}

template <bool A_KC, bool B_KC, int OUT>
int by_tile(const GemmArgs& g, int tile, int splits, hipStream_t s) {
  switch (tile) {
    case 0: return launch<256, 256, A_KC, B_KC, OUT>(g, splits, s);
    case 1: return launch<256, 128, A_KC, B_KC, OUT>(g, splits, s);
    case 2: return launch<128, 256, A_KC, B_KC, OUT>(g, splits, s);
    case 3: return launch<128, 128, A_KC, B_KC, OUT>(g, splits, s);
    case 4: return launch<128, 128, A_KC, B_KC, OUT, 2>(g, splits, s);   // 2 stages: 2 blocks per CU
    case 5: return launch4<A_KC, B_KC, OUT>(g, splits, s);
    case 6: return launch8<A_KC, B_KC, OUT>(g, splits, s);
    case 7: return launch8<A_KC, B_KC, OUT, 192>(g, splits, s);
    case 8:   // tiles 3 / 4 on v_mfma_f32_32x32x16_bf16 (forward layout, bf16 / fp32 out)
      if constexpr (A_KC && B_KC && OUT <= 1) return launch<128, 128, A_KC, B_KC, OUT, 3, 0, 32>(g, splits, s);
      break;
    case 9:
      if constexpr (A_KC && B_KC && OUT <= 1) return launch<128, 128, A_KC, B_KC, OUT, 2, 0, 32>(g, splits, s);
      break;
  }
  return (int)hipErrorInvalidValue;
}

// dw[i] = beta * dw[i] + sum_z slab[z][i] over float4 columns, in slab order (deterministic).
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ slab, float* __restrict__ dw,
                                                       long long n4, int S, float beta) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 acc = beta != 0.f ? reinterpret_cast<const float4*>(dw)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (beta != 0.f && beta != 1.f) { acc.x *= beta; acc.y *= beta; acc.z *= beta; acc.w *= beta; }
    int z = 0;
    for (; z + 4 <= S; z += 4) {   // four slabs in flight per thread
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = reinterpret_cast<const float4*>(slab)[(long long)(z + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; z < S; ++z) {
      const float4 v = reinterpret_cast<const float4*>(slab)[(long long)z * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(dw)[i] = acc;
  }
}

}  // namespace

// layout: 0 = forward (A KC, B KC), 1 = dgrad (A KC, B KS), 2 = wgrad (A KS, B KS)
// out:    0 = bf16 (+bias, act, pre-act copy), 1 = fp32 beta, 2 = fp32 atomic (split-K)
// tile:   0 = 256x256, 1 = 256x128, 2 = 128x256, 3 = 128x128 (BM x BN; 3-stage where LDS allows),
//         4 = 128x128 with 2 stages (64 KB: two blocks per CU), 5 = 256x256 BK=32 4-slot ring,
//         6 = 256x256 two-group phase schedule (k_gemm8), 7 = the same schedule on 256x192 tiles
//         (BERT's N = 768 / 2304 / 3072 outputs split into 4 / 12 / 16 column tiles: with T = 16384
//         tokens every launch is a whole number of waves over 256 CUs), 8 / 9 = tiles 3 / 4 with
//         v_mfma_f32_32x32x16_bf16 fragments (layout 0, out 0 / 1; measured against 3 / 4 in
//         profiles/r6/gemm/mfma_32x32.md)
// Host contract (checked by ops/gemm.py): N % 4 == 0, ldc % 4 == 0, K-contiguous leading
// dimensions % 8 == 0, 16-byte aligned pointers; a zero page of >= 16 bytes.  Tile 6 with
// bf16 output also needs N % 8 == 0 and ldc % 8 == 0 (16-byte staged stores).
KML_API int kml_gemm(const bf16_t* a, long long lda, const bf16_t* b, long long ldb, void* c, long long ldc,
                     bf16_t* c2, const float* bias, const bf16_t* zp, int M, int N, int K, int layout, int out,
                     int act, float beta, int tile, int splits, hipStream_t s) {
  GemmArgs g;
  g.a = a; g.b = b; g.c = c; g.c2 = c2; g.bias = bias; g.zp = zp;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.act = act; g.beta = beta; g.kchunk = K; g.colpart = nullptr;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0;
  // the linear-layer GEMMs keep the register epilogue: BERT's QKV forward on the 128 x 128 row-pass
  // tile beat hipBLASLt alone (71 vs 88 us) but not inside the step (profiles/r5/bert_qkv_rowpass.md)
  g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  if (M <= 0 || N <= 0) return 0;
  if (act == GEMM_GELU_BWD) return (int)hipErrorInvalidValue;  // kml_gemm_dgrad_gelu
  if (layout == 0 && out == 0) return by_tile<true, true, 0>(g, tile, 1, s);
  if (layout == 0 && out == 1) return by_tile<true, true, 1>(g, tile, 1, s);
  if (layout == 0 && out == 2) return by_tile<true, true, 2>(g, tile, splits, s);
  if (layout == 1 && out == 2) return by_tile<true, false, 2>(g, tile, splits, s);
  if (layout == 1 && out == 0) return by_tile<true, false, 0>(g, tile, 1, s);
  if (layout == 2 && out == 1) return by_tile<false, false, 1>(g, tile, 1, s);
  if (layout == 2 && out == 2) return by_tile<false, false, 2>(g, tile, splits, s);
  return (int)hipErrorInvalidValue;
}

// Implicit-GEMM convolution forward on the k_gemm tiles (0-4): y[M = B OH OW][N = K] = im2col(x) W^T
// with W [K][KH][KW][C] as the KC B operand (ldb = KH KW C) and A gathered per K-tile by ConvStagerA
// (C % 64 == 0).  rows: the GEMM_STATS partial rows [M / BM][2 N] or null (plain bf16 output + bias).
KML_API int kml_gemm_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const float* bias, float* rows,
                              const bf16_t* zp, int B, int H, int W, int C, int K, int KH, int KW, int sh, int sw,
                              int ph, int pw, int tile, float* grp_out, unsigned* grp_cnt, int grp_tiles,
                              hipStream_t s) {
  if (C % 64 || K % 8 || tile < 0 || tile > 4 || KH < 1 || KW < 1 || sh < 1 || sw < 1) return (int)hipErrorInvalidValue;
  const int OH = (H + 2 * ph - KH) / sh + 1, OW = (W + 2 * pw - KW) / sw + 1;
  if (OH <= 0 || OW <= 0) return 0;
  GemmArgs g;
  g.a = x; g.b = w; g.c = y; g.c2 = nullptr; g.bias = bias; g.zp = zp;
  g.lda = C; g.ldb = (long long)KH * KW * C; g.ldc = K;
  g.M = B * OH * OW; g.N = K; g.K = KH * KW * C; g.act = rows ? GEMM_STATS : 0; g.beta = 0.f; g.kchunk = g.K;
  g.colpart = rows;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cOH = OH; g.cOW = OW; g.cKW = KW; g.csh = sh; g.csw = sw; g.cph = ph; g.cpw = pw;
  g.rowpass = out_rowpass_default(); g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  if (grp_out) {
    if (!rows || !grp_cnt || grp_tiles < 1 || !g.rowpass || (tile != 3 && tile != 4)) return (int)hipErrorInvalidValue;
    g.grp_out = grp_out; g.grp_cnt = grp_cnt; g.grp_tiles = grp_tiles;
  }
  switch (tile) {
    case 0: return launch<256, 256, true, true, 0, 2, 1>(g, 1, s);
    case 1: return launch<256, 128, true, true, 0, 3, 1>(g, 1, s);
    case 2: return launch<128, 256, true, true, 0, 3, 1>(g, 1, s);
    case 3: return launch<128, 128, true, true, 0, 3, 1>(g, 1, s);
    case 4: return launch<128, 128, true, true, 0, 2, 1>(g, 1, s);
  }
  return (int)hipErrorInvalidValue;
}

// Implicit-GEMM input gradient of a stride-1 conv on the k_gemm tiles (0-4): dx[M = B H W][N = C] =
// sum over (tap, cout) of dy[pixel shifted by the tap][cout] W[cout][tap][cin]; A gathered from dy by
// ConvStagerA<DG>, B = W read per tap by ConvStagerB (K % 64 == 0), the dgrad epilogue of
// kml_gemm_dgrad_bnf (addend, consumer-BN rows, ReLU mask).
KML_API int kml_gemm_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const bf16_t* addend, const bf16_t* y,
                                const bf16_t* cin, const float* mean, const float* rstd, float* rows, int mask_out,
                                const bf16_t* zp, int B, int H, int W, int C, int K, int KH, int KW, int ph, int pw,
                                int tile, float* grp_out, unsigned* grp_cnt, int grp_tiles, hipStream_t s) {
  if (K % 64 || C % 8 || tile < 0 || tile > 4 || KH < 1 || KW < 1) return (int)hipErrorInvalidValue;
  if (cin && (!mean || !rstd || !rows)) return (int)hipErrorInvalidValue;
  const int OH = H + 2 * ph - KH + 1, OW = W + 2 * pw - KW + 1;
  if (OH <= 0 || OW <= 0 || B * H * W <= 0) return 0;
  GemmArgs g;
  g.a = dy; g.b = w; g.c = dx; g.c2 = const_cast<bf16_t*>(addend); g.bias = nullptr; g.zp = zp;
  g.lda = K; g.ldb = (long long)KH * KW * C; g.ldc = C;
  g.M = B * H * W; g.N = C; g.K = KH * KW * K; g.act = GEMM_BNF; g.beta = 0.f; g.kchunk = g.K;
  g.colpart = rows;
  g.by = y; g.bc = cin; g.bmean = mean; g.brstd = rstd; g.mask_out = mask_out; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cOH = OH; g.cOW = OW; g.cKW = KW; g.csh = 1; g.csw = 1; g.cph = ph; g.cpw = pw;
  g.cK = K;
  if (grp_out) {
    if (!cin || !grp_cnt || grp_tiles < 1 || (tile != 3 && tile != 4)) return (int)hipErrorInvalidValue;
    g.grp_out = grp_out; g.grp_cnt = grp_cnt; g.grp_tiles = grp_tiles;
  }
  switch (tile) {
    case 0: return launch<256, 256, true, false, 0, 2, 2>(g, 1, s);
    case 1: return launch<256, 128, true, false, 0, 3, 2>(g, 1, s);
    case 2: return launch<128, 256, true, false, 0, 3, 2>(g, 1, s);
    case 3: return launch<128, 128, true, false, 0, 3, 2>(g, 1, s);
    case 4: return launch<128, 128, true, false, 0, 2, 2>(g, 1, s);
  }
  return (int)hipErrorInvalidValue;
}

// Implicit-GEMM weight gradient on the k_gemm tiles (0-4): dw[M = K][N = KH KW C] = beta dw + sum over the
// output pixels of dy[p][k] im2col(x)[p][(tap, c)] (dy the KS A operand, ld K; im2col(x) gathered by
// ConvStagerBW), each K-slice's fp32 tile to slab[z] and one ordered pass summing the slabs into dw
// (deterministic, as kml_gemm_wgrad_splitk).  slab holds ceil(P / chunk) * M * N floats.
KML_API int kml_gemm_conv_wgrad(const bf16_t* x, const bf16_t* dy, float* dw, float* slab, const bf16_t* zp, int B,
                                int H, int W, int C, int K, int KH, int KW, int sh, int sw, int ph, int pw, float beta,
                                int tile, int splits, hipStream_t s) {
  if (C % 8 || K % 4 || tile < 0 || tile > 4 || KH < 1 || KW < 1 || sh < 1 || sw < 1) return (int)hipErrorInvalidValue;
  const int OH = (H + 2 * ph - KH) / sh + 1, OW = (W + 2 * pw - KW) / sw + 1;
  if (OH <= 0 || OW <= 0) return 0;
  GemmArgs g;
  g.a = dy; g.b = x; g.c = slab; g.c2 = nullptr; g.bias = nullptr; g.zp = zp;
  g.lda = K; g.ldb = 0; g.ldc = (long long)KH * KW * C;
  g.M = K; g.N = KH * KW * C; g.K = B * OH * OW; g.act = 0; g.beta = 0.f; g.kchunk = g.K; g.colpart = nullptr;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cOH = OH; g.cOW = OW; g.cKW = KW; g.csh = sh; g.csw = sw; g.cph = ph; g.cpw = pw;
  g.cK = K;
  splits = splits < 1 ? 1 : splits;
  int rc = (int)hipErrorInvalidValue;
  switch (tile) {
    case 0: rc = launch<256, 256, false, false, 3, 2, 3>(g, splits, s); break;
    case 1: rc = launch<256, 128, false, false, 3, 3, 3>(g, splits, s); break;
    case 2: rc = launch<128, 256, false, false, 3, 3, 3>(g, splits, s); break;
    case 3: rc = launch<128, 128, false, false, 3, 3, 3>(g, splits, s); break;
    case 4: rc = launch<128, 128, false, false, 3, 2, 3>(g, splits, s); break;
  }
  if (rc) return rc;
  const int chunk = ((g.K + splits - 1) / splits + BK - 1) / BK * BK;
  const int z = (g.K + chunk - 1) / chunk;
  const long long n4 = (long long)g.M * g.N / 4;
  hipLaunchKernelGGL(k_splitk_reduce, dim3(kml_stream_grid(n4, 256)), dim3(256), 0, s, slab, dw, n4, z, beta);
  KML_LAUNCH_CHECK();
}

// Forward GEMM (layout 0, bf16 out, optional fp32 bias) with BatchNorm partial statistics in the
// epilogue (GEMM_STATS): rows[M / BM][2 N] = per-M-tile [sum | sumsq] of the bf16 outputs, BM = 256
// (tiles 0, 1, 6) or 128 (tiles 2, 3, 4).  The GEMM route of a 1x1 / stride-1 convolution.
KML_API int kml_gemm_stats(const bf16_t* a, long long lda, const bf16_t* b, long long ldb, bf16_t* c, long long ldc,
                           const float* bias, float* rows, const bf16_t* zp, int M, int N, int K, int tile,
                           float* grp_out, unsigned* grp_cnt, int grp_tiles, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (!rows || N % 8 || ldc % 8 || lda % 8 || ldb % 8 || K % 8) return (int)hipErrorInvalidValue;
  if (tile == 5 || tile == 7 || tile < 0 || tile > 7) return (int)hipErrorInvalidValue;
  GemmArgs g;
  g.a = a; g.b = b; g.c = c; g.c2 = nullptr; g.bias = bias; g.zp = zp;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.act = GEMM_STATS; g.beta = 0.f; g.kchunk = K; g.colpart = rows;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0;
  g.rowpass = out_rowpass_default(); g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  if (grp_out) {  // group reduction: row-pass tiles only
    if (!grp_cnt || grp_tiles < 1 || !g.rowpass || (tile != 3 && tile != 4)) return (int)hipErrorInvalidValue;
    g.grp_out = grp_out; g.grp_cnt = grp_cnt; g.grp_tiles = grp_tiles;
  }
  return by_tile<true, true, 0>(g, tile, 1, s);
}

// Input gradient of a 1x1 / stride-1 conv as a GEMM (layout 1: dx[M][N] = dy[M][K] W[K][N]) with the
// implicit-GEMM dgrad's epilogue (GEMM_BNF): optional residual addend, consumer-BN partial rows
// rows[M / BM][2 N] and ReLU-masked output.  Tiles 0-4 (register epilogue; BM = 256 for 0 / 1).
KML_API int kml_gemm_dgrad_bnf(const bf16_t* a, long long lda, const bf16_t* b, long long ldb, bf16_t* c,
                               long long ldc, const bf16_t* addend, const bf16_t* y, const bf16_t* cin,
                               const float* mean, const float* rstd, float* rows, int mask_out, const bf16_t* zp,
                               int M, int N, int K, int tile, float* grp_out, unsigned* grp_cnt, int grp_tiles,
                               hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (N % 8 || ldc % 8 || lda % 8 || ldb % 8 || K % 8 || tile < 0 || tile > 4) return (int)hipErrorInvalidValue;
  if (cin && (!mean || !rstd || !rows)) return (int)hipErrorInvalidValue;
  GemmArgs g;
  g.a = a; g.b = b; g.c = c; g.c2 = const_cast<bf16_t*>(addend); g.bias = nullptr; g.zp = zp;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.act = GEMM_BNF; g.beta = 0.f; g.kchunk = K; g.colpart = rows;
  g.by = y; g.bc = cin; g.bmean = mean; g.brstd = rstd; g.mask_out = mask_out; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  if (grp_out) {  // the BNF row pass runs on the 128 x 128 tiles
    if (!cin || !grp_cnt || grp_tiles < 1 || (tile != 3 && tile != 4)) return (int)hipErrorInvalidValue;
    g.grp_out = grp_out; g.grp_cnt = grp_cnt; g.grp_tiles = grp_tiles;
  }
  return by_tile<true, false, 0>(g, tile, 1, s);
}

// dgrad (layout 1, 256x256 phase tile) with the GELU backward of the layer that produced its
// operand's forward input in the epilogue: c = bf16(bf16(dy W) * gelu'(pre)), colpart[M/256][N]
// = per-M-tile column sums of c (summed in order by the caller: the FFN1 bias gradient).
KML_API int kml_gemm_dgrad_gelu(const bf16_t* a, long long lda, const bf16_t* b, long long ldb, bf16_t* c,
                                long long ldc, const bf16_t* pre, float* colpart, const bf16_t* zp, int M, int N,
                                int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (N % 8 || ldc % 8 || !pre || !colpart) return (int)hipErrorInvalidValue;
  GemmArgs g;
  g.a = a; g.b = b; g.c = c; g.c2 = const_cast<bf16_t*>(pre); g.bias = nullptr; g.zp = zp;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.act = GEMM_GELU_BWD; g.beta = 0.f; g.kchunk = K; g.colpart = colpart;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  return launch8<true, false, 0>(g, 1, s);
}

// Deterministic split-K weight gradient: dw[M][N] = beta * dw + sum_k A^T B (layout 2), each
// K-slice's fp32 partial tile stored to slab[z] (plain coalesced stores, no atomics), then one
// bandwidth-bound pass sums the slabs in order into dw.  dw and slab are contiguous (ldc == N);
// slab holds splits * M * N floats.
KML_API int kml_gemm_wgrad_splitk(const bf16_t* a, long long lda, const bf16_t* b, long long ldb, float* dw,
                                  float* slab, const bf16_t* zp, int M, int N, int K, float beta, int tile, int splits,
                                  hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  GemmArgs g;
  g.a = a; g.b = b; g.c = slab; g.c2 = nullptr; g.bias = nullptr; g.zp = zp;
  g.lda = lda; g.ldb = ldb; g.ldc = N;
  g.M = M; g.N = N; g.K = K; g.act = 0; g.beta = 0.f; g.kchunk = K; g.colpart = nullptr;
  g.by = nullptr; g.bc = nullptr; g.bmean = nullptr; g.brstd = nullptr; g.mask_out = 0; g.rowpass = 0; g.grp_out = nullptr; g.grp_cnt = nullptr; g.grp_tiles = 0;
  splits = splits < 1 ? 1 : splits;
  int rc = by_tile<false, false, 3>(g, tile, splits, s);
  if (rc) return rc;
  // the launcher rounds the K chunk up to the tile's K step: count the slices it produced
  int step = (tile == 5 || tile == 6 || tile == 7) ? 64 : BK;
  int chunk = ((K + splits - 1) / splits + step - 1) / step * step;
  const int z = K > 0 ? (K + chunk - 1) / chunk : 1;
  const long long n4 = (long long)M * N / 4;
  hipLaunchKernelGGL(k_splitk_reduce, dim3(kml_stream_grid(n4, 256)), dim3(256), 0, s, slab, dw, n4, z, beta);
  KML_LAUNCH_CHECK();
}
