// attention.hip — fused multi-head attention (flash-attention style) for gfx950.
//
// BERT-base MLM (north-star config 5; the reference has no attention model, SURVEY
// §2.8/§5.7): head_dim 64, non-causal, optional additive key bias (padding mask),
// sequence length L <= any (tiles of 64, tails masked).  Scores never touch HBM:
//
//   fwd   : per (64 queries, b, h) block; loop over 64-key tiles: S^T = K Q^T (MFMA),
//           online softmax in registers (exp2 domain), O^T += V^T P^T (MFMA);
//           writes O and the per-row log-sum-exp (base 2) for backward.
//   bwd   : dq-kernel per query tile (also computes D = rowsum(dO * O)), dkv-kernel per
//           key tile; both recompute P from the saved LSE — no atomics, deterministic.
//
// Attention-probability dropout (HF BERT attention_probs_dropout_prob): keep mask
// Z[b,h,q,key] = half16(word(seed ^ salt, step, b, h, q, key / 2), key & 1) >= p * 2^16
// (word: Drop below), hashed once by the forward, which stores the decisions as a bit mask
// (1 bit per probability, AttnArgs::keep) that both backward kernels read.  Forward: O = softmax(S) (.) Z/(1-p) @ V, the row normaliser from
// the undropped probabilities; backward: dV = (P (.) Z/(1-p))^T dO, dP = (dO V^T) (.) Z/(1-p),
// dS = P (.) (dP - D) with D = rowsum(dO (.) O) (unchanged by the mask).
//
// MFMA v_mfma_f32_16x16x32_bf16, wave64: lane l holds A[l&15][8(l>>4)+j],
// B[8(l>>4)+j][l&15], C[4(l>>4)+i][l&15].  Each wave owns 16 queries (or keys) so the
// softmax statistics of a row live in one lane column (l&15) and the 4 lanes sharing it
// (l>>4 = 0..3) combine with two xor-shuffles.  The probability tile produced in C layout
// is reused as the next MFMA's operand without data movement by permuting the k index
// of that MFMA: k-slot 8g+j <-> key 32ks + 4g + j (j<4) / 32ks + 16 + 4g + (j-4); the other
// operand is read with the matching rows through ds_read_b64_tr_b16 (transpose read).
//
// LDS tiles are 64 rows x 128 B with a 16-byte-chunk XOR swizzle (chunk ^ (row & 7)),
// conflict-free for both the row-fragment (ds_read_b128) and transpose reads.
// Layout: token-major activations [B*L, ld] with head h at column offset 64 h, so the
// fused QKV projection output / dQKV gradient buffers are used in place.
#include "kml_common.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace {

typedef __attribute__((ext_vector_type(4))) short v4s_t;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o; const bf16_t* dout;
  bf16_t* out; bf16_t* dq; bf16_t* dk; bf16_t* dv;
  float* lse;          // [B*H][L] base-2 log-sum-exp of scaled scores
  float* dsum;         // [B*H][L] D = rowsum(dO * O)
  const float* bias;   // [B][L] additive key bias (natural-log units) or null
  int ldq, ldk, ldv, ldo, lddo, ldout, lddq, lddk, lddv;
  int B, H, L;
  float scale;         // softmax scale (1/sqrt(64))
  const float* ctr;    // [seed, step] (device) for attention dropout, or null
  unsigned salt;
  float pdrop;         // dropout probability (0: off)
  int xcd;             // XCD-aware block order (attn_blk); 0: plain grid order (A/B switch)
  unsigned char* keep; // dropout keep bits written by the forward, read by the backward (Drop), or null
};

__device__ __forceinline__ unsigned ahash(unsigned a, unsigned b, unsigned c) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

// per-kernel dropout state.  One 32-bit word per (q, key pair): its low 16 bits decide the
// even key, the high 16 bits the odd one (threshold p * 2^16).  The words of the 16 keys a
// forward lane holds (query q, keys kbase + 16t + i, kbase = kb*64 + 4g) come from ONE full
// hash of (q, kbase) followed by a one-multiply finaliser per pair: word(off) =
// fmix1(ahash(q*LP + kbase/2) + off * golden), off = 8t + i/2 — 11 multiplies per lane per
// key tile instead of 24 (the hash was a quarter of the forward's vector-ALU work).
//
// The forward also stores the decisions as a bit mask (AttnArgs::keep), so the backward
// kernels read 1 bit per probability instead of re-hashing (the hash is most of their
// vector-ALU work): u64 word (bh, key tile kb, query q) at byte ((bh*nkb + kb)*Lp + q)*8,
// Lp = 64*nkb; bit 16g + 4t + i = key kb*64 + 16t + 4g + i — the 16 keys a forward lane
// holds (lane group g, S-tile t, element i) are one u16 at byte 2g.
__device__ __forceinline__ unsigned fmix1(unsigned x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15;
  return x;
}

struct Drop {
  unsigned k0, k1, thr;
  float sc;
  unsigned LP;   // key pairs per query row
  bool on;
  __device__ void init(const AttnArgs& a, int bh) {
    on = a.ctr != nullptr && a.pdrop > 0.f;
    LP = (unsigned)(a.L + 1) >> 1;
    sc = 1.f;
    if (on) {
      k0 = (unsigned)a.ctr[0] ^ a.salt;
      k1 = (unsigned)a.ctr[1] * 0x632BE5ABu ^ (unsigned)bh * 0x5851F42Du;
      thr = (unsigned)(a.pdrop * 65536.0f);
      sc = 1.f / (1.f - a.pdrop);
    }
  }
  // keep bits of keys kbase + 16t + i (bit 4t + i), kbase = kb*64 + 4g
  __device__ __forceinline__ unsigned bits16(int q, int kbase) const {
    const unsigned h0 = ahash(k0, k1, (unsigned)q * LP + ((unsigned)kbase >> 1));
    unsigned bits = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const unsigned h = fmix1(h0 + (unsigned)(8 * t + i / 2) * 0x9E3779B9u);
        bits |= ((h & 0xFFFFu) >= thr ? 1u : 0u) << (4 * t + i);
        bits |= (h >= (thr << 16) ? 1u : 0u) << (4 * t + i + 1);
      }
    return bits;
  }
  // all-ones / zero mask of one (q, key)
  __device__ __forceinline__ int keep1(int q, int key) const {
    const int kbase = (key & ~63) + 4 * ((key & 15) >> 2);
    const unsigned h0 = ahash(k0, k1, (unsigned)q * LP + ((unsigned)kbase >> 1));
    const unsigned h = fmix1(h0 + (unsigned)((key >> 1) - (kbase >> 1)) * 0x9E3779B9u);
    return ((key & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thr ? -1 : 0;
  }
};

// bit j of w as an all-ones / zero mask (v_bfe_i32)
__device__ __forceinline__ int bitmask(unsigned w, int j) { return __builtin_amdgcn_sbfe((int)w, j, 1); }
__device__ __forceinline__ float fmask(float x, int m) { return __int_as_float(__float_as_int(x) & m); }

__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

// XCD-aware block order.  Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
// one), so with the plain (tile, b*h) grid the 8 tiles of one head land on 8 different L2s
// and each XCD fetches that head's K/V (or Q/dO) again.  Renumbered so each XCD runs a
// contiguous range of ids, tile fastest: the tiles of one head share one L2.
__device__ __forceinline__ void attn_blk(const AttnArgs& a, int& xt, int& bh) {
  const int gx = (int)gridDim.x, nwg = gx * (int)gridDim.y;
  const int lin = (int)blockIdx.y * gx + (int)blockIdx.x;
  if (!a.xcd) { xt = (int)blockIdx.x; bh = (int)blockIdx.y; return; }
  const int q = nwg >> 3, r = nwg & 7, x = lin & 7, k = lin >> 3;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  bh = id / gx;
  xt = id - bh * gx;
}

struct TileRegs { uint4 v[2]; };

__device__ __forceinline__ void tile_load(TileRegs& R, const bf16_t* base, int ld, int row0, int L, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (tid >> 3) + 32 * u, c = tid & 7, row = row0 + r;
    R.v[u] = row < L ? *reinterpret_cast<const uint4*>(base + (long long)row * ld + c * 8) : make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void tile_store(char* lds, const TileRegs& R, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (tid >> 3) + 32 * u, c = tid & 7;
    *reinterpret_cast<uint4*>(lds + swz(r, c)) = R.v[u];
  }
}

// rows row0 + (lane & 15), k = 32 ks + 8 (lane >> 4) + j
__device__ __forceinline__ bf16x8_t frag_rows(const char* lds, int row0, int ks, int lane) {
  return *reinterpret_cast<const bf16x8_t*>(lds + swz(row0 + (lane & 15), 4 * ks + (lane >> 4)));
}

// f[j] = T[key(j)][col0 + (lane & 15)], key(j) = 32ks + 4g + j (j<4), 32ks + 16 + 4g + j-4 (j>=4)
__device__ __forceinline__ bf16x8_t frag_tr(const char* lds, int col0, int ks, int lane) {
  const int il = lane & 15, g = lane >> 4;
  const int col = col0 + 4 * (il & 3);
  const int r0 = 32 * ks + 4 * g + (il >> 2), r1 = r0 + 16;
  const char* p0 = lds + swz(r0, col >> 3) + (col & 7) * 2;
  const char* p1 = lds + swz(r1, col >> 3) + (col & 7) * 2;
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p0));
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p1));
  bf16x8_t f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

// bf16 operand from 8 accumulator values of tiles 2ks, 2ks+1 (the permuted k order)
// (v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN — one instruction per pair)
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t{a, b}), bf16x2_hw));
}
__device__ __forceinline__ bf16x8_t pack_p(const f32x4_t& t0, const f32x4_t& t1) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  const u32x4_t u = {cvt2(t0[0], t0[1]), cvt2(t0[2], t0[3]), cvt2(t1[0], t1[1]), cvt2(t1[2], t1[3])};
  return __builtin_bit_cast(bf16x8_t, u);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }  // v_exp_f32

__device__ __forceinline__ bf16x8_t load_frag_g(const bf16_t* row_ptr, int ks, int g, bool ok) {
  if (!ok) { bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0}; return z; }
  return *reinterpret_cast<const bf16x8_t*>(row_ptr + 32 * ks + 8 * g);
}

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ void store4(bf16_t* p, const f32x4_t& v, float s) {
  uint2 w;
  w.x = pack_bf2(v[0] * s, v[1] * s);
  w.y = pack_bf2(v[2] * s, v[3] * s);
  *reinterpret_cast<uint2*>(p) = w;
}

// ------------------------------------------------------------------------------ forward
// OCC: waves per SIMD the register budget is sized for (launch bounds; the occupancy /
// register trade of each kernel was measured, profiles/bert_base_r3.md)
// DM: dropout mode (0 none, 1 hashed keep decisions, stored as bits when a.keep is set), BIAS:
// additive key bias — compile-time like the backward kernels
template <int OCC, int DM, bool BIAS>
__global__ __launch_bounds__(256, OCC) void k_attn_fwd(AttnArgs a) {
  // K/V double-buffered (40 KB: 4 blocks per CU, the VGPR occupancy): one barrier per key
  // tile, and the register-staged next tile is stored after this tile's MFMAs, a whole tile
  // after its global loads were issued
  __shared__ __attribute__((aligned(16))) char sQ[8192];
  __shared__ __attribute__((aligned(16))) char sK2[2][8192];
  __shared__ __attribute__((aligned(16))) char sV2[2][8192];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  int xt, bh;
  attn_blk(a, xt, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int L = a.L, q0 = xt * 64;
  const bf16_t* Qb = a.q + (long long)b * L * a.ldq + h * 64;
  const bf16_t* Kb = a.k + (long long)b * L * a.ldk + h * 64;
  const bf16_t* Vb = a.v + (long long)b * L * a.ldv + h * 64;
  const float sl2 = a.scale * LOG2E;
  const float* bias = BIAS ? a.bias + (long long)b * L : nullptr;
  Drop drop;
  drop.init(a, bh);

  TileRegs rq, rk, rv;
  tile_load(rq, Qb, a.ldq, q0, L, tid);
  tile_load(rk, Kb, a.ldk, 0, L, tid);
  tile_load(rv, Vb, a.ldv, 0, L, tid);
  tile_store(sQ, rq, tid);
  tile_store(sK2[0], rk, tid);
  tile_store(sV2[0], rv, tid);
  const int nkb = (L + 63) / 64;
  if (nkb > 1) {
    tile_load(rk, Kb, a.ldk, 64, L, tid);
    tile_load(rv, Vb, a.ldv, 64, L, tid);
  }
  __syncthreads();
  const bf16x8_t qf0 = frag_rows(sQ, 16 * w, 0, lane), qf1 = frag_rows(sQ, 16 * w, 1, lane);

  float m2 = -INFINITY, lsum = 0.f;
  f32x4_t acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkb; ++kb) {
    const char* sK = sK2[kb & 1];
    const char* sV = sV2[kb & 1];
    f32x4_t s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      s[t] = MFMA16(frag_rows(sK, 16 * t, 0, lane), qf0, s[t]);
      s[t] = MFMA16(frag_rows(sK, 16 * t, 1, lane), qf1, s[t]);
    }
    // bias or key tail: scale + bias + mask every score; otherwise the max of the raw scores
    // (scale > 0) and one fma per probability below
    const bool gen = BIAS || kb * 64 + 64 > L;
    float mx = -INFINITY;
    if (gen) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = kb * 64 + 16 * t + 4 * g + i;
          float v = s[t][i] * sl2;
          if (BIAS && key < L) v += bias[key] * LOG2E;
          if (key >= L) v = -INFINITY;
          s[t][i] = v;
          mx = fmaxf(mx, v);
        }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) mx = fmaxf(mx, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
      mx *= sl2;
    }
    // lazy rescale: the running max m2 moves only when a score exceeds it by 8 (P <= 2^8,
    // exact in fp32, the same relative precision in bf16) — most tiles skip the shuffles and
    // the accumulator scaling.  The four lanes of a query column always agree on m2.
    if (__any(mx > m2 + 8.f)) {
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m2, mx);
      const float alpha = mn == -INFINITY ? 1.f : fexp2(m2 - mn);
      lsum *= alpha;
#pragma unroll
      for (int d = 0; d < 4; ++d) acc[d] *= alpha;
      m2 = mn;
    }
    const float off = m2 == -INFINITY ? 0.f : m2;
    if (gen) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[t][i] = fexp2(s[t][i] - off);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[t][i] = fexp2(fmaf(s[t][i], sl2, -off));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) lsum += (s[t][0] + s[t][1]) + (s[t][2] + s[t][3]);
    if constexpr (DM != 0) {   // zero the dropped probabilities (1/(1-p) is applied to O at the end)
      const int qq = q0 + 16 * w + (lane & 15);
      const unsigned bits = drop.bits16(qq, kb * 64 + 4 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[t][i] = fmask(s[t][i], bitmask(bits, 4 * t + i));
      if (a.keep && qq < L)
        *reinterpret_cast<unsigned short*>(a.keep + (((long long)bh * nkb + kb) * (nkb * 64) + qq) * 8 + 2 * g) =
            (unsigned short)bits;
    }
    const bf16x8_t p0 = pack_p(s[0], s[1]), p1 = pack_p(s[2], s[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      acc[d] = MFMA16(frag_tr(sV, 16 * d, 0, lane), p0, acc[d]);
      acc[d] = MFMA16(frag_tr(sV, 16 * d, 1, lane), p1, acc[d]);
    }
    if (kb + 1 < nkb) {   // buffer (kb+1)&1 last held tile kb-1: every wave left it at the last barrier
      tile_store(sK2[(kb + 1) & 1], rk, tid);
      tile_store(sV2[(kb + 1) & 1], rv, tid);
      if (kb + 2 < nkb) {
        tile_load(rk, Kb, a.ldk, (kb + 2) * 64, L, tid);
        tile_load(rv, Vb, a.ldv, (kb + 2) * 64, L, tid);
      }
      __syncthreads();
    }
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const int q = q0 + 16 * w + (lane & 15);
  if (q < L) {
    const float inv = lsum > 0.f ? drop.sc / lsum : 0.f;
    bf16_t* op = a.out + (long long)(b * L + q) * a.ldout + h * 64;
#pragma unroll
    for (int d = 0; d < 4; ++d) store4(op + 16 * d + 4 * g, acc[d], inv);
    if (g == 0) a.lse[(long long)bh * L + q] = lsum > 0.f ? m2 + log2f(lsum) : INFINITY;
  }
}

// ------------------------------------------------------------------------------ backward: dQ (+D)
// DM: dropout mode (0 none, 1 the forward's keep bits, 2 re-hashed), BIAS: additive key bias —
// compile-time, so the per-probability code carries no uniform branches (a branch per element
// was a scheduling barrier between the VALU work and the MFMAs around it)
template <int OCC, int DM, bool BIAS>
__global__ __launch_bounds__(256, OCC) void k_attn_bwd_dq(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char sK2[2][8192];   // K/V double-buffered (k_attn_fwd)
  __shared__ __attribute__((aligned(16))) char sV2[2][8192];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  int xt, bh;
  attn_blk(a, xt, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int L = a.L;
  const int q = xt * 64 + 16 * w + (lane & 15);
  const bool qok = q < L;
  const bf16_t* Kb = a.k + (long long)b * L * a.ldk + h * 64;
  const bf16_t* Vb = a.v + (long long)b * L * a.ldv + h * 64;
  const float sl2 = a.scale * LOG2E;
  const float* bias = BIAS ? a.bias + (long long)b * L : nullptr;

  Drop drop;
  drop.init(a, bh);
  const bf16_t* qrow = a.q + (long long)(b * L + (qok ? q : 0)) * a.ldq + h * 64;
  const bf16_t* dorow = a.dout + (long long)(b * L + (qok ? q : 0)) * a.lddo + h * 64;
  const bf16_t* orow = a.o + (long long)(b * L + (qok ? q : 0)) * a.ldo + h * 64;
  const bf16x8_t qf0 = load_frag_g(qrow, 0, g, qok), qf1 = load_frag_g(qrow, 1, g, qok);
  const bf16x8_t df0 = load_frag_g(dorow, 0, g, qok), df1 = load_frag_g(dorow, 1, g, qok);
  // D = rowsum(dO * O): lane covers d = 16g .. 16g+15
  float D = 0.f;
  if (qok) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint4 x = *reinterpret_cast<const uint4*>(dorow + 16 * g + 8 * u);
      const uint4 y = *reinterpret_cast<const uint4*>(orow + 16 * g + 8 * u);
      D += lo_bf(x.x) * lo_bf(y.x) + hi_bf(x.x) * hi_bf(y.x) + lo_bf(x.y) * lo_bf(y.y) + hi_bf(x.y) * hi_bf(y.y) +
           lo_bf(x.z) * lo_bf(y.z) + hi_bf(x.z) * hi_bf(y.z) + lo_bf(x.w) * lo_bf(y.w) + hi_bf(x.w) * hi_bf(y.w);
    }
  }
  D += __shfl_xor(D, 16, 64);
  D += __shfl_xor(D, 32, 64);
  if (qok && g == 0) a.dsum[(long long)bh * L + q] = D;
  const float lse = qok ? a.lse[(long long)bh * L + q] : INFINITY;

  f32x4_t acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  TileRegs rk, rv;
  tile_load(rk, Kb, a.ldk, 0, L, tid);
  tile_load(rv, Vb, a.ldv, 0, L, tid);
  const int nkb = (L + 63) / 64;
  tile_store(sK2[0], rk, tid);
  tile_store(sV2[0], rv, tid);
  if (nkb > 1) {
    tile_load(rk, Kb, a.ldk, 64, L, tid);
    tile_load(rv, Vb, a.ldv, 64, L, tid);
  }
  __syncthreads();
  // this lane's u16 of the stored keep bits for key tile kb (Drop), prefetched with K/V
  constexpr bool kbits = DM == 1;
  const unsigned short* kp16 =
      reinterpret_cast<const unsigned short*>(a.keep + ((long long)bh * nkb * (nkb * 64) + (qok ? q : 0)) * 8 + 2 * g);
  const long long kstride = (long long)nkb * 64 * 4;   // u16 units per key tile
  unsigned knext = kbits ? kp16[0] : 0xFFFFu;
  for (int kb = 0; kb < nkb; ++kb) {
    const char* sK = sK2[kb & 1];
    const char* sV = sV2[kb & 1];
    unsigned bits = knext;
    if (kbits && kb + 1 < nkb) knext = kp16[(kb + 1) * kstride];
    if constexpr (DM == 2) bits = drop.bits16(q, kb * 64 + 4 * g);
    f32x4_t s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      s[t] = MFMA16(frag_rows(sK, 16 * t, 0, lane), qf0, s[t]);
      s[t] = MFMA16(frag_rows(sK, 16 * t, 1, lane), qf1, s[t]);
      dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dp[t] = MFMA16(frag_rows(sV, 16 * t, 0, lane), df0, dp[t]);
      dp[t] = MFMA16(frag_rows(sV, 16 * t, 1, lane), df1, dp[t]);
    }
    // dS = P (.) (dP (.) Z/(1-p) - D); bias / key tail only on the general path
    const bool gen = BIAS || kb * 64 + 64 > L;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kb * 64 + 16 * t + 4 * g + i;
        float p = 0.f;
        if (gen) {
          float v = s[t][i] * sl2;
          if (BIAS && key < L) v += bias[key] * LOG2E;
          if (key < L) p = fexp2(v - lse);
        } else {
          p = fexp2(fmaf(s[t][i], sl2, -lse));
        }
        if constexpr (DM != 0) {
          const float dpz = fmask(dp[t][i], bitmask(bits, 4 * t + i));
          s[t][i] = p * fmaf(dpz, drop.sc, -D);
        } else {
          s[t][i] = p * (dp[t][i] - D);
        }
      }
    const bf16x8_t d0 = pack_p(s[0], s[1]), d1 = pack_p(s[2], s[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      acc[d] = MFMA16(frag_tr(sK, 16 * d, 0, lane), d0, acc[d]);
      acc[d] = MFMA16(frag_tr(sK, 16 * d, 1, lane), d1, acc[d]);
    }
    if (kb + 1 < nkb) {
      tile_store(sK2[(kb + 1) & 1], rk, tid);
      tile_store(sV2[(kb + 1) & 1], rv, tid);
      if (kb + 2 < nkb) {
        tile_load(rk, Kb, a.ldk, (kb + 2) * 64, L, tid);
        tile_load(rv, Vb, a.ldv, (kb + 2) * 64, L, tid);
      }
      __syncthreads();
    }
  }
  if (qok) {
    bf16_t* op = a.dq + (long long)(b * L + q) * a.lddq + h * 64;
#pragma unroll
    for (int d = 0; d < 4; ++d) store4(op + 16 * d + 4 * g, acc[d], a.scale);
  }
}

// ------------------------------------------------------------------------------ backward: dK, dV
// DM / BIAS as k_attn_bwd_dq.  Without a bias the keys past L keep a zero bias: their dK / dV
// rows are never stored and no other key's rows read them.
template <int OCC, int DM, bool BIAS>
__global__ __launch_bounds__(256, OCC) void k_attn_bwd_dkv(AttnArgs a) {
  // double-buffered like k_attn_fwd: Q, dO, LSE, D and the keep bits of a query tile
  __shared__ __attribute__((aligned(16))) char sQ2[2][8192];
  __shared__ __attribute__((aligned(16))) char sO2[2][8192];  // dO tile
  __shared__ __attribute__((aligned(16))) float sL2[2][64];
  __shared__ __attribute__((aligned(16))) float sD2[2][64];
  // keep bits: the tile's 64 u64 words as two planes of 32-bit halves, sM2[j][half][q], so a
  // lane's four queries 16t + 4g + i are one ds_read_b128 (like LSE and D)
  __shared__ __attribute__((aligned(16))) unsigned sM2[2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  int xt, bh;
  attn_blk(a, xt, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int L = a.L;
  const int key = xt * 64 + 16 * w + (lane & 15);
  const bool kok = key < L;
  const bf16_t* Qb = a.q + (long long)b * L * a.ldq + h * 64;
  const bf16_t* Ob = a.dout + (long long)b * L * a.lddo + h * 64;
  const float sl2 = a.scale * LOG2E;
  const bf16_t* krow = a.k + (long long)(b * L + (kok ? key : 0)) * a.ldk + h * 64;
  const bf16_t* vrow = a.v + (long long)(b * L + (kok ? key : 0)) * a.ldv + h * 64;
  const bf16x8_t kf0 = load_frag_g(krow, 0, g, kok), kf1 = load_frag_g(krow, 1, g, kok);
  const bf16x8_t vf0 = load_frag_g(vrow, 0, g, kok), vf1 = load_frag_g(vrow, 1, g, kok);
  const float kb2 = BIAS ? (!kok ? -INFINITY : a.bias[(long long)b * L + key] * LOG2E) : 0.f;
  Drop drop;
  drop.init(a, bh);

  f32x4_t adk[4], adv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) { adk[d] = f32x4_t{0.f, 0.f, 0.f, 0.f}; adv[d] = adk[d]; }
  const int nqb = (L + 63) / 64;
  // stored keep bits (Drop): the 512-byte tile of words (q = qb*64.., this key tile) is
  // staged in LDS; this lane's key sits at bit kbit of each word
  constexpr bool kbits = DM == 1;
  const uint4* kw = reinterpret_cast<const uint4*>(a.keep + ((long long)bh * nqb + xt) * (nqb * 64) * 8);
  const int kl = 16 * w + (lane & 15), kbit = 16 * ((kl >> 2) & 3) + 4 * (kl >> 4) + (kl & 3);
  TileRegs rq, ro;
  float pl = 0.f, pd = 0.f;
  uint4 mnext = make_uint4(0, 0, 0, 0);
  auto fetch = [&](int qbn) {
    const int nq0 = qbn * 64;
    tile_load(rq, Qb, a.ldq, nq0, L, tid);
    tile_load(ro, Ob, a.lddo, nq0, L, tid);
    if (tid < 64) {
      const int qq = nq0 + tid;
      pl = qq < L ? a.lse[(long long)bh * L + qq] : INFINITY;
      pd = qq < L ? a.dsum[(long long)bh * L + qq] : 0.f;
    }
    if (kbits && tid < 32) mnext = kw[qbn * 32 + tid];
  };
  auto stage = [&](int j) {
    tile_store(sQ2[j], rq, tid);
    tile_store(sO2[j], ro, tid);
    if (tid < 64) { sL2[j][tid] = pl; sD2[j][tid] = pd; }
    if (kbits && tid < 32) {   // words 2tid, 2tid+1 = (mnext.x, .y), (mnext.z, .w)
      *reinterpret_cast<uint2*>(&sM2[j][0][2 * tid]) = make_uint2(mnext.x, mnext.z);
      *reinterpret_cast<uint2*>(&sM2[j][1][2 * tid]) = make_uint2(mnext.y, mnext.w);
    }
  };
  fetch(0);
  stage(0);
  if (nqb > 1) fetch(1);
  __syncthreads();
  for (int qb = 0; qb < nqb; ++qb) {
    const char* sQ = sQ2[qb & 1];
    const char* sO = sO2[qb & 1];
    const float* sL = sL2[qb & 1];
    const float* sD = sD2[qb & 1];
    const unsigned* sM = sM2[qb & 1][kbit >> 5];
    f32x4_t s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      s[t] = MFMA16(frag_rows(sQ, 16 * t, 0, lane), kf0, s[t]);
      s[t] = MFMA16(frag_rows(sQ, 16 * t, 1, lane), kf1, s[t]);
      dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dp[t] = MFMA16(frag_rows(sO, 16 * t, 0, lane), vf0, dp[t]);
      dp[t] = MFMA16(frag_rows(sO, 16 * t, 1, lane), vf1, dp[t]);
    }
    // s[t][i] = S[q = 16t + 4g + i][key]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 l4 = *reinterpret_cast<const float4*>(sL + 16 * t + 4 * g);
      const float4 d4 = *reinterpret_cast<const float4*>(sD + 16 * t + 4 * g);
      const uint4 m4 = kbits ? *reinterpret_cast<const uint4*>(sM + 16 * t + 4 * g) : make_uint4(0, 0, 0, 0);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
      const unsigned mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * t + 4 * g + i;
        const float p = fexp2(fmaf(s[t][i], sl2, BIAS ? kb2 - lv[i] : -lv[i]));
        if constexpr (DM != 0) {
          const int m = DM == 1 ? bitmask(mv[i], kbit & 31) : drop.keep1(qb * 64 + r, key);
          // dV takes P (.) Z (1/(1-p) applied at the store), dS = P (.) (dP (.) Z/(1-p) - D)
          s[t][i] = fmask(p, m);
          dp[t][i] = p * fmaf(fmask(dp[t][i], m), drop.sc, -dv[i]);
        } else {
          s[t][i] = p;
          dp[t][i] = p * (dp[t][i] - dv[i]);
        }
      }
    }
    const bf16x8_t p0 = pack_p(s[0], s[1]), p1 = pack_p(s[2], s[3]);
    const bf16x8_t d0 = pack_p(dp[0], dp[1]), d1 = pack_p(dp[2], dp[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      adv[d] = MFMA16(frag_tr(sO, 16 * d, 0, lane), p0, adv[d]);
      adv[d] = MFMA16(frag_tr(sO, 16 * d, 1, lane), p1, adv[d]);
      adk[d] = MFMA16(frag_tr(sQ, 16 * d, 0, lane), d0, adk[d]);
      adk[d] = MFMA16(frag_tr(sQ, 16 * d, 1, lane), d1, adk[d]);
    }
    if (qb + 1 < nqb) {   // buffer (qb+1)&1 last held tile qb-1: every wave left it at the last barrier
      stage((qb + 1) & 1);
      if (qb + 2 < nqb) fetch(qb + 2);
      __syncthreads();
    }
  }
  if (kok) {
    bf16_t* kp = a.dk + (long long)(b * L + key) * a.lddk + h * 64;
    bf16_t* vp = a.dv + (long long)(b * L + key) * a.lddv + h * 64;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      store4(kp + 16 * d + 4 * g, adk[d], a.scale);
      store4(vp + 16 * d + 4 * g, adv[d], drop.sc);
    }
  }
}

bool aligned16(const void* p) { return (((unsigned long long)p) & 15ull) == 0; }

}  // namespace

// q/k/v/out: token-major [B*L, ld*] bf16, head h at column 64h (head_dim must be 64)
// ctr/salt/pdrop: attention-probability dropout (ctr null or pdrop 0: none); keep: null or a
// [B*H, nkb, 64*nkb] u64 buffer (nkb = ceil(L/64)) that receives the keep bits (Drop)
KML_API int kml_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* out, float* lse,
                         const float* bias, int ldq, int ldk, int ldv, int ldout, int B, int H, int L, float scale,
                         const float* ctr, int salt, float pdrop, unsigned char* keep, hipStream_t s) {
  if (L <= 0 || B <= 0 || H <= 0 || ldq % 8 || ldk % 8 || ldv % 8 || ldout % 4) return (int)hipErrorInvalidValue;
  if (!aligned16(q) || !aligned16(k) || !aligned16(v)) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.out = out; a.lse = lse; a.bias = bias;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldout = ldout;
  a.B = B; a.H = H; a.L = L; a.scale = scale;
  a.ctr = ctr; a.salt = (unsigned)salt; a.pdrop = pdrop; a.xcd = 1; a.keep = keep;
  if (pdrop < 0.f || pdrop >= 1.f) return (int)hipErrorInvalidValue;
  const dim3 grid((L + 63) / 64, B * H);
  const bool dm = ctr != nullptr && pdrop > 0.f;
  if (bias) {
    if (dm) hipLaunchKernelGGL((k_attn_fwd<4, 1, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_attn_fwd<4, 0, true>), grid, dim3(256), 0, s, a);
  } else {
    if (dm) hipLaunchKernelGGL((k_attn_fwd<4, 1, false>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_attn_fwd<4, 0, false>), grid, dim3(256), 0, s, a);
  }
  KML_LAUNCH_CHECK();
}

// dq/dk/dv may point into one fused [B*L, 3*H*64] buffer (ld = 3*H*64); dsum: [B*H*L] fp32 scratch;
// keep: the forward's keep bits (read instead of re-hashing), or null
KML_API int kml_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                         const float* lse, float* dsum, const float* bias, bf16_t* dq, bf16_t* dk, bf16_t* dv,
                         int ldq, int ldk, int ldv, int ldo, int lddo, int lddq, int lddk, int lddv, int B, int H,
                         int L, float scale, const float* ctr, int salt, float pdrop, const unsigned char* keep,
                         hipStream_t s) {
  if (L <= 0 || ldq % 8 || ldk % 8 || ldv % 8 || ldo % 8 || lddo % 8 || lddq % 4 || lddk % 4 || lddv % 4)
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.o = o; a.dout = dout; a.lse = const_cast<float*>(lse); a.dsum = dsum;
  a.bias = bias; a.dq = dq; a.dk = dk; a.dv = dv;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo; a.lddo = lddo; a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  a.B = B; a.H = H; a.L = L; a.scale = scale;
  a.ctr = ctr; a.salt = (unsigned)salt; a.pdrop = pdrop; a.xcd = 1;
  a.keep = const_cast<unsigned char*>(keep);
  if (pdrop < 0.f || pdrop >= 1.f) return (int)hipErrorInvalidValue;
  const dim3 grid((L + 63) / 64, B * H);
  // occupancy from the register budgets (profiles/bert_base_r3.md): dQ at 4 waves per SIMD
  // (124 VGPRs, no spills), dKV at 2 (~211 VGPRs; 3 spills and doubles its time)
  const int dm = (ctr == nullptr || pdrop <= 0.f) ? 0 : (keep != nullptr ? 1 : 2);
  constexpr int DKV_OCC = 3;
#define KML_ATTN_BWD(DM, BI)                                              \
  do {                                                                    \
    hipLaunchKernelGGL((k_attn_bwd_dq<4, DM, BI>), grid, dim3(256), 0, s, a);  \
    hipLaunchKernelGGL((k_attn_bwd_dkv<DKV_OCC, DM, BI>), grid, dim3(256), 0, s, a); \
  } while (0)
  if (bias) {
    if (dm == 0) KML_ATTN_BWD(0, true);
    else if (dm == 1) KML_ATTN_BWD(1, true);
    else KML_ATTN_BWD(2, true);
  } else {
    if (dm == 0) KML_ATTN_BWD(0, false);
    else if (dm == 1) KML_ATTN_BWD(1, false);
    else KML_ATTN_BWD(2, false);
  }
#undef KML_ATTN_BWD
  KML_LAUNCH_CHECK();
}
