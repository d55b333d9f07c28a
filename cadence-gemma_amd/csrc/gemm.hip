// bf16 MFMA GEMMs for gfx950 with the fused epilogues of the CadenceGemma
// forward path.
//
//   C[M, N] = A[M, K] . W[N, K]^T       (both operands K-contiguous)
//
// Engines:
//  * big tile engine (prefill, M > 64): 256x256x64 block tile, 8 waves (2x4),
//    wave tile 128x64 of mfma_f32_16x16x32_bf16; operands go HBM -> LDS with
//    global_load_lds (LDS-DMA, no VGPR staging), the XOR chunk swizzle is
//    applied on the per-lane source address so ds_read_b128 stays
//    conflict-free; double-buffered, one barrier per k-tile; XCD-aware
//    bijective block remap + grouped tile order for L2 reuse.  Elementwise
//    epilogues are staged through the freed LDS and written as 16-B rows.
//  * stream engine (decode, M <= 32): every weight load of a block is issued
//    up front (latency-bound regime), optionally split over K with the
//    deterministic fp32 reduction below.
//  * skinny engine (decode fallback / logits): weight rows streamed straight
//    into MFMA B fragments, split-K over the grid, fp32 partial slabs reduced
//    in a fixed order (deterministic) by a second kernel that applies the
//    same epilogue.
//
// Epilogues replicate the reference rounding points:
//  EpiLinear      nn.Linear (+bias) [+GELU(erf)] [+residual], row remap
//  EpiGatedGelu   MLPBlock: gelu_tanh(x.Wg + bg) * (x.Wu + bu)  modules.py:754-756
//  EpiRglruGates  RG-LRU gate chain -> (a, normalized_x)       layers.py:345-365
//  EpiVitResid    timm residual: resid += gamma * (x.W + b)   (fp32 stream)
//  EpiPatch       patch-embed conv as GEMM + pos_embed at a prefix offset
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

constexpr int BK = 64;


// ---------------------------------------------------------------- epilogues

struct RowMap {
  int64_t div, mul, off;  // out_row = (m / div) * mul + (m % div) + off
  CADENCE_DEV int64_t operator()(int64_t m) const {
    // rows and divisors are < 2^31: 32-bit division (the 64-bit one is a
    // long inline sequence per call site in the unrolled epilogues)
    if (mul == 0 && off == 0 && m < div) return m;
    const uint32_t um = (uint32_t)m, ud = (uint32_t)div;
    const uint32_t q = um / ud;
    return (int64_t)q * mul + (int64_t)(um - q * ud) + off;
  }
};

// griffin.py:219-221 on bf16 logits: tanh(l / c) * c, each op rounded.
CADENCE_DEV float softcap(float l, float c) {
  const float t = rbf(l / c);
  return rbf(rbf(tanhf(t)) * c);
}

// Epilogue interface.
//  * Direct path (stream and split-K engines): apply(m, n, v, g)
//    / apply2(m, f, v_gate, v_up, g) write one element.
//  * Staged path (big engine, kStaged): bias_at() + stage() / stage2() take
//    one accumulator to its first bf16 rounding point (bias added); the
//    engine parks those in LDS and a ROLLED loop hands 8 consecutive staged
//    columns of one row to finish8(m, n, v8, g) (paired epilogues:
//    finish8p(m, f, gate8, up8, g)), which runs the rest of the element
//    chain and writes 16-B rows.  Keeping activations out of the unrolled
//    128-element accumulator loop keeps the kernel inside the instruction
//    cache (an unrolled gate chain made the kernel 160 KB and cost ~25 us of
//    instruction fetch per tile).
struct EpiLinear {
  struct Pref {};
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = true;
  static constexpr bool kTile = false;
  u16* out; int64_t ldo;
  const u16* bias;
  const u16* resid; int64_t ldr;
  int act;                 // 0 none, 1 gelu(erf), 2 soft-cap(cap), 3 gelu(tanh)
  RowMap map;
  float cap;
  CADENCE_DEV float activate(float r) const {
    if (act == 1) r = rbf(gelu_erf(r));
    if (act == 2) r = softcap(r, cap);
    if (act == 3) r = rbf(gelu_tanh(r));
    return r;
  }
  CADENCE_DEV float value(int64_t, int n, float v, int) const {
    // F.linear adds the bias in fp32 before the single bf16 rounding.
    if (bias) v = add_rn(v, bf2f(bias[n]));
    return activate(rbf(v));
  }
  CADENCE_DEV void apply(int64_t m, int n, float v, int g) const {
    float r = value(m, n, v, g);
    const int64_t orow = map(m);
    if (resid) r = badd(r, bf2f(resid[orow * ldr + n]));
    out[orow * ldo + n] = f2bf(r);
  }
  // staged path
  CADENCE_DEV float bias_at(bool, int n, int) const {
    return bias ? bf2f(bias[n]) : 0.0f;
  }
  CADENCE_DEV float stage(float v, float b) const {
    if (bias) v = add_rn(v, b);
    return rbf(v);
  }
  // stage() of two rows of one column, both bf16 in one word (kStage2)
  static constexpr bool kStage2 = true;
  CADENCE_DEV uint32_t stage2(f32x2 v, float b) const {
    if (bias) v = f32x2{add_rn(v.x, b), add_rn(v.y, b)};
    return pk2bf(v);
  }
  template <class Act>
  CADENCE_DEV void finish8_with(int64_t m, int n, uint4 v, Act&& f) const {
    const int64_t orow = map(m);
    float a[8];
    unpack8(v, a);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = f(a[i]);
    if (resid) {
      float b[8];
      unpack8(ld16(resid + orow * ldr + n), b);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = badd(a[i], b[i]);
    }
    st16(out + orow * ldo + n, pack8(a));
  }
  CADENCE_DEV void finish8(int64_t m, int n, uint4 v, int) const {
    finish8_with(m, n, v, [&](float r) { return activate(r); });
  }
};

// EpiLinear with the activation fixed at compile time (big engine).
template <int ACT>
struct EpiLinearA : EpiLinear {
  CADENCE_DEV void finish8(int64_t m, int n, uint4 v, int) const {
    if constexpr (ACT == 0) {
      if (!resid) {
        st16(out + map(m) * ldo + n, v);
        return;
      }
    }
    if constexpr (ACT == 1 || ACT == 3) {
      if (!resid) {             // GELU of 4 packed pairs (gelu_erf2 / gelu_tanh2)
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 a{__uint_as_float(w[k] << 16), __uint_as_float(w[k] & 0xffff0000u)};
          o[k] = pk2bf(ACT == 1 ? gelu_erf2(a) : gelu_tanh2(a));
        }
        st16(out + map(m) * ldo + n, make_uint4(o[0], o[1], o[2], o[3]));
        return;
      }
    }
    finish8_with(m, n, v, [&](float r) {
      if constexpr (ACT == 1) r = rbf(gelu_erf(r));
      if constexpr (ACT == 2) r = softcap(r, cap);
      if constexpr (ACT == 3) r = rbf(gelu_tanh(r));
      return r;
    });
  }
};

// act 0 with a residual (the Griffin output / down projections): the
// staged path loads the residual rows of every finish iteration before it
// stages the accumulators (kResidPref), so the finish loop waits on one
// memory trip instead of one per unrolled pair of iterations.  Same sums and
// roundings as EpiLinearA<0> with `resid` set.
template <>
struct EpiLinearA<4> : EpiLinear {
  static constexpr bool kResidPref = true;
  CADENCE_DEV uint4 resid_at(int64_t m, int n) const { return ld16(resid + map(m) * ldr + n); }
  CADENCE_DEV void finish8_r(int64_t m, int n, uint4 v, uint4 r) const {
    float a[8], b[8];
    unpack8(v, a);
    unpack8(r, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = badd(a[i], b[i]);
    st16(out + map(m) * ldo + n, pack8(a));
  }
  CADENCE_DEV void finish8(int64_t m, int n, uint4 v, int) const {
    finish8_r(m, n, v, resid_at(m, n));
  }
};

// Staged epilogues whose first rounding point takes two rows at once
// (stage2: one v_cvt_pk_bf16_f32 for both)
template <class E, class = void>
struct EpiStage2 { static constexpr bool value = false; };
template <class E>
struct EpiStage2<E, std::void_t<decltype(E::kStage2)>> {
  static constexpr bool value = E::kStage2;
};

template <class E, class = void>
struct EpiResidPref { static constexpr bool value = false; };
template <class E>
struct EpiResidPref<E, std::void_t<decltype(E::kResidPref)>> {
  static constexpr bool value = E::kResidPref;
};

// Decode yx projection fused with the Conv1D decode step of the x branch
// (stream engine only, M <= 32 rows = sequences): columns >= conv_lo are the
// x branch; their rounded linear output x_t enters the depthwise causal
// conv [state rows (TW-1) | x_t] (layers.py:478-483, same products, sums and
// roundings as conv1d_decode_kernel), the conv output replaces x_t in `out`
// and the state rows shift in place.  Each (row, channel) is owned by one
// thread; its conv operands are loaded at kernel start (kPrefetch) so they
// land while the weight stream is in flight.
template <int TW>
struct EpiLinearConv : EpiLinear {
  static constexpr bool kPrefetch = true;
  const u16* cw;         // [TW][E] conv weight
  const u16* cb;         // [E] conv bias
  u16* state;            // [M][TW-1][E], advanced in place
  int conv_lo, E;
  struct Pref { u16 w[TW], s[TW > 1 ? TW - 1 : 1], b; };
  CADENCE_DEV Pref prefetch(int64_t m, int n) const {
    // branch-free: y-branch columns read channel 0 (unused)
    Pref p{};
    const int c = n >= conv_lo ? n - conv_lo : 0;
    const u16* srow = state + m * (int64_t)(TW - 1) * E + c;
#pragma unroll
    for (int t = 0; t < TW; ++t) p.w[t] = cw[(int64_t)t * E + c];
#pragma unroll
    for (int r = 0; r < TW - 1; ++r) p.s[r] = srow[(int64_t)r * E];
    p.b = cb[c];
    return p;
  }
  CADENCE_DEV void apply_pf(int64_t m, int n, float v, int g, const Pref& p) const {
    const float x = value(m, n, v, g);          // act 0: bias + one rounding
    if (n < conv_lo) {
      out[m * ldo + n] = f2bf(x);
      return;
    }
    // [state rows | x_t] . w, newest first: conv1d_decode_kernel's order
    float acc = bmul(x, bf2f(p.w[TW - 1]));
#pragma unroll
    for (int s = 1; s < TW; ++s)
      acc = badd(acc, bmul(bf2f(p.s[TW - 1 - s]), bf2f(p.w[TW - 1 - s])));
    acc = badd(acc, bf2f(p.b));
    out[m * ldo + n] = f2bf(acc);
    u16* srow = state + m * (int64_t)(TW - 1) * E + (n - conv_lo);
#pragma unroll
    for (int r = 0; r + 1 < TW - 1; ++r) srow[(int64_t)r * E] = p.s[r + 1];
    if constexpr (TW > 1) srow[(int64_t)(TW - 2) * E] = f2bf(x);
  }
  CADENCE_DEV void apply(int64_t m, int n, float v, int g) const {
    apply_pf(m, n, v, g, prefetch(m, n));
  }
};

// Decode residual projection whose RMSNorm runs in the consuming GEMV
// (stream engine, M <= 32, in-kernel split-K combine): out = bias + resid +
// A.W^T as EpiLinear (act 0), written row-major and once more, unnormalised,
// in the packed decode layout the consumer loads.  Bias and residual are
// loaded at kernel start (kPrefetch), so the last-arriving split issues no
// dependent load after its partial-slab loads.
struct EpiResidRows : EpiLinear {
  static constexpr bool kPrefetch = true;
  u16* rows;                 // packed decode layout, mt = ceil(M / 16)
  int mt;
  struct Pref { u16 r, b; };
  CADENCE_DEV Pref prefetch(int64_t m, int n) const {
    const u16* zp = reinterpret_cast<const u16*>(kZeroPage);
    return Pref{*(resid ? resid + m * ldr + n : zp), *(bias ? bias + n : zp)};
  }
  CADENCE_DEV void apply_pf(int64_t m, int n, float v, int, const Pref& p) const {
    if (bias) v = add_rn(v, bf2f(p.b));
    float r = rbf(v);
    if (resid) r = badd(r, bf2f(p.r));
    const u16 o = f2bf(r);
    out[m * ldo + n] = o;
    rows[xpk((int)m, n, mt)] = o;
  }
  CADENCE_DEV void apply(int64_t m, int n, float v, int g) const {
    apply_pf(m, n, v, g, prefetch(m, n));
  }
};

// Raw fp32 dot products of one K split -- the split is the prefill engine's
// group index g -- to parts[g][m][n]: the split-K form of the prefill
// engine for small M (splitk_reduce_kernel then applies the real epilogue
// to the split-order sums).  Paired epilogues' packed gate / up columns are
// written as they are; the reduce kernel pairs them.
struct EpiPartial {
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = false;
  static constexpr bool kTile = false;
  float* parts;
  int64_t M, N;
  CADENCE_DEV void apply(int64_t m, int n, float v, int g) const {
    parts[((int64_t)g * M + m) * N + n] = v;
  }
};

// Decode q|k|v projection with RoPE in the epilogue (stream engine, M <= 32).
// The weight rows are pre-permuted so that each rotation pair (dims i and
// i + hd/4 of the rotated half of a q or k head) sits in adjacent columns
// 2i, 2i + 1: the two values of a pair are in neighbouring lanes of one
// wave (apply_pair gets the partner by a lane swap).  Columns hd/2.. of a
// head and the v head are unpermuted.  Output rows go to q [M][H*hd],
// k [M][hd], v [M][hd] in the natural dim order, with rope_qkv_kernel's
// products, sums and roundings (modules.py:73-81 via attention.hip).
struct EpiRopeQKV {
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = false;
  static constexpr bool kTile = false;
  static constexpr bool kPairLanes = true;
  u16* q; u16* k; u16* v;
  const int32_t* pos;
  const u16* table; int table_len;
  int H, hd;
  CADENCE_DEV float value(int64_t, int, float x, int) const { return rbf(x); }
  CADENCE_DEV void apply_pair(int64_t m, int n, float x, float y) const {
    const int h = n / hd, d = n % hd;
    const int half = hd / 2, quarter = hd / 4;
    u16* dst = h < H ? q + m * (int64_t)H * hd + (int64_t)h * hd
                     : (h == H ? k + m * hd : v + m * hd);
    if (h > H || d >= half) {            // v head / pass-through dims
      dst[d] = f2bf(x);
      return;
    }
    const int i = d >> 1;                 // rotation pair
    const int p = pos[m];
    float sn, cs;
    if (p >= 0 && p < table_len) {
      sn = bf2f(table[((int64_t)p * 2) * quarter + i]);
      cs = bf2f(table[((int64_t)p * 2 + 1) * quarter + i]);
    } else {
      rope_sincos(p, i, half, sn, cs);
    }
    if ((d & 1) == 0)                     // x = dim i, y = dim i + hd/4
      dst[i] = f2bf(bsub(bmul(x, cs), bmul(y, sn)));
    else                                  // x = dim i + hd/4, y = dim i
      dst[i + quarter] = f2bf(badd(bmul(x, cs), bmul(y, sn)));
  }
  CADENCE_DEV void apply(int64_t, int, float, int) const {}
};

// Prefill q|k|v projection with RoPE in the staged epilogue (big engine,
// one K split).  The weight rows are in qkv_rope_permutation order (as the
// decode EpiRopeQKV): in the rotated half of a q / k head, columns 2i, 2i + 1
// hold dims i, i + hd / 4, so every 8 staged columns carry 4 whole rotation
// pairs and finish8 rotates them with rope_qkv_kernel's products, sums and
// roundings (rounded GEMM output, bf16 sin / cos from the table) and writes
// dims i0..i0+3 and i0 + hd/4.. as two 8-B rows; pass-through dims and the v
// head are written as they are.  Outputs q [M][H*hd], k [M][hd], v [M][hd]
// in natural dim order (modules.py:73-81, :430-436).
struct EpiRopeQKVBig {
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = true;
  static constexpr bool kTile = false;
  static constexpr bool kRowPref = true;
  u16* q; u16* k; u16* v;
  const int32_t* pos;
  const u16* table; int table_len;
  int H, hd;
  struct RowPref { uint2 sn, cs; };
  CADENCE_DEV float bias_at(bool, int, int) const { return 0.0f; }
  CADENCE_DEV float stage(float x, float) const { return rbf(x); }
  static constexpr bool kStage2 = true;
  CADENCE_DEV uint32_t stage2(f32x2 v, float) const { return pk2bf(v); }
  CADENCE_DEV int row_pos(int64_t m) const { return pos[m]; }
  // the table entries of columns n..n+7's four rotation pairs (rotated
  // columns inside the table only; the others read entry 0, unused)
  CADENCE_DEV RowPref row_prefetch(int p, int n) const {
    const int d = n % hd, quarter = hd / 4;
    const bool ok = d < hd / 2 && p >= 0 && p < table_len;
    const int64_t so = ok ? ((int64_t)p * 2) * quarter + (d >> 1) : 0;
    return RowPref{*reinterpret_cast<const uint2*>(table + so),
                   *reinterpret_cast<const uint2*>(table + so + (ok ? quarter : 0))};
  }
  CADENCE_DEV void finish8_pf(int64_t m, int n, uint4 v8, int p, const RowPref& pf) const {
    const int h = n / hd, d = n % hd, half = hd / 2, quarter = hd / 4;
    if (h > H) {
      st16(v + m * hd + d, v8);
      return;
    }
    u16* dst = h < H ? q + m * (int64_t)H * hd + (int64_t)h * hd : k + m * hd;
    if (d >= half) {
      st16(dst + d, v8);
      return;
    }
    const int i0 = d >> 1;                  // pairs i0 .. i0 + 3
    float sn[4], cs[4];
    if (p >= 0 && p < table_len) {
      const uint32_t sw[2] = {pf.sn.x, pf.sn.y}, cw[2] = {pf.cs.x, pf.cs.y};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sn[j] = __uint_as_float(j & 1 ? sw[j >> 1] & 0xffff0000u : sw[j >> 1] << 16);
        cs[j] = __uint_as_float(j & 1 ? cw[j >> 1] & 0xffff0000u : cw[j >> 1] << 16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) rope_sincos(p, i0 + j, half, sn[j], cs[j]);
    }
    float x[8];
    unpack8(v8, x);
    uint32_t lo[2], hi[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a0 = x[4 * j], b0 = x[4 * j + 1], a1 = x[4 * j + 2], b1 = x[4 * j + 3];
      const int j0 = 2 * j, j1 = 2 * j + 1;
      lo[j] = (uint32_t)f2bf(bsub(bmul(a0, cs[j0]), bmul(b0, sn[j0]))) |
              ((uint32_t)f2bf(bsub(bmul(a1, cs[j1]), bmul(b1, sn[j1]))) << 16);
      hi[j] = (uint32_t)f2bf(badd(bmul(b0, cs[j0]), bmul(a0, sn[j0]))) |
              ((uint32_t)f2bf(badd(bmul(b1, cs[j1]), bmul(a1, sn[j1]))) << 16);
    }
    *reinterpret_cast<uint2*>(dst + i0) = make_uint2(lo[0], lo[1]);
    *reinterpret_cast<uint2*>(dst + quarter + i0) = make_uint2(hi[0], hi[1]);
  }
  CADENCE_DEV void finish8(int64_t m, int n, uint4 v8, int g) const {
    const int p = pos[m];
    finish8_pf(m, n, v8, p, row_prefetch(p, n));
  }
};

template <class E, class = void>
struct EpiPairLanes { static constexpr bool value = false; };
template <class E>
struct EpiPairLanes<E, std::void_t<decltype(E::kPairLanes)>> {
  static constexpr bool value = E::kPairLanes;
};

// Epilogues that load per-element operands at kernel start (kPrefetch).
template <class E, class = void>
struct EpiPrefetch { static constexpr bool value = false; };
template <class E>
struct EpiPrefetch<E, std::void_t<decltype(E::kPrefetch)>> {
  static constexpr bool value = E::kPrefetch;
};

// Decode GEMVs whose A operand may arrive unnormalised (the RMSNorm of the
// producing residual projection applied on load, gemm_stream_kernel NORM).
// Staged epilogues with per-row operands (kRowPref): the rolled finish loop
// is unrolled and every iteration's row operands are loaded before the first
// finish (row_pos for all rows, then row_prefetch for all), so the loop pays
// two memory round trips in all instead of two per iteration.
template <class E, class = void>
struct EpiRowPref { static constexpr bool value = false; };
template <class E>
struct EpiRowPref<E, std::void_t<decltype(E::kRowPref)>> {
  static constexpr bool value = E::kRowPref;
};

// Paired staged epilogues that combine gate and up in registers (kRegPair):
// a lane's accumulator tiles j and j + 2 hold the gate and up columns of the
// same features, so the output is computed before staging and only outputs
// (half the values, no finish math) go through LDS.
template <class E, class = void>
struct EpiRegPair { static constexpr bool value = false; };
template <class E>
struct EpiRegPair<E, std::void_t<decltype(E::kRegPair)>> {
  static constexpr bool value = E::kRegPair;
};

template <class E> struct EpiNormIn { static constexpr bool value = false; };

struct EpiGatedGelu {
  static constexpr bool kPaired = true;
  static constexpr bool kStaged = true;
  static constexpr bool kTile = false;
  u16* out; int64_t ldo;        // ldo == 0: packed rows (M <= 32)
  const u16* bias_g; const u16* bias_u;
  int mt;                        // ceil(M / 16)
  CADENCE_DEV float value2(int64_t, int f, float g, float u, int) const {
    // Einsum result is rounded, then `+ b` rounds again (layers.py:729).
    g = badd(rbf(g), bf2f(bias_g[f]));
    u = badd(rbf(u), bf2f(bias_u[f]));
    return bmul(rbf(gelu_tanh(g)), u);
  }
  CADENCE_DEV void apply2(int64_t m, int f, float g, float u, int gg) const {
    out[xoff((int)m, f, ldo, mt)] = f2bf(value2(m, f, g, u, gg));
  }
  // stream engine: the biases are loaded at kernel start (kPrefetch), so the
  // epilogue issues no dependent global load after the weight stream
  static constexpr bool kPrefetch = true;
  struct Pref { u16 bg, bu; };
  CADENCE_DEV Pref prefetch2(int64_t, int f, int) const { return Pref{bias_g[f], bias_u[f]}; }
  CADENCE_DEV void apply2_pf(int64_t m, int f, float g, float u, int, const Pref& p) const {
    g = badd(rbf(g), bf2f(p.bg));
    u = badd(rbf(u), bf2f(p.bu));
    out[xoff((int)m, f, ldo, mt)] = f2bf(bmul(rbf(gelu_tanh(g)), u));
  }
  CADENCE_DEV float bias_at(bool up, int f, int) const {
    return bf2f((up ? bias_u : bias_g)[f]);
  }
  CADENCE_DEV float stage(float v, float b) const { return badd(rbf(v), b); }
  CADENCE_DEV void finish8p(int64_t m, int f, uint4 g8, uint4 u8, int) const {
    float gv[8], uv[8];
    unpack8(g8, gv);
    unpack8(u8, uv);
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = bmul(rbf(gelu_tanh(gv[i])), uv[i]);
    st16(out + xoff((int)m, f, ldo, mt), pack8(gv));
  }
  // big engine: gate x up of two rows in registers (big_epilogue kRegPair),
  // the rounding points of stage() then finish8p(); packed bf16 pair out
  static constexpr bool kRegPair = true;
  CADENCE_DEV uint32_t out2(f32x2 g, f32x2 u, float bg, float bu) const {
    const f32x2 gs = badd2(rbf2(g), f32x2{bg, bg});
    const f32x2 us = badd2(rbf2(u), f32x2{bu, bu});
    const f32x2 gl = rbf2(gelu_tanh2(gs));
    return pk2bf(f32x2{mul_rn(gl.x, us.x), mul_rn(gl.y, us.y)});
  }
  CADENCE_DEV void store8(int64_t m, int f, uint4 v) const {
    st16(out + xoff((int)m, f, ldo, mt), v);
  }
};

template <int TW> struct EpiNormIn<EpiLinearConv<TW>> { static constexpr bool value = true; };
template <> struct EpiNormIn<EpiRopeQKV> { static constexpr bool value = true; };
template <> struct EpiNormIn<EpiGatedGelu> { static constexpr bool value = true; };

// Tile epilogues (kTile): the big engine hands the whole wave tile
// (acc[MR][4], rows mbase + 16 i + 4 (lane >> 4) + r, columns
// nbase + 16 j + (lane & 15)) to `tile`, which issues its global loads in
// batches ahead of the stores (element-wise load -> store through possibly
// aliasing pointers serialises one load latency per element).
template <int MR>
using AccTile = f32x4[MR][4];

// RG-LRU gate chain (layers.py:345-365) on the block-diagonal gate GEMM.
struct EpiRglruGates {
  static constexpr bool kPaired = true;
  static constexpr bool kStaged = true;
  static constexpr bool kTile = false;
  const u16* x; int64_t ldx;         // conv1d output (RG-LRU input)
  const u16* bias_x; const u16* bias_a;
  const u16* softplus_a;             // bf16(softplus(a_param)), [E]
  const int32_t* segpos;             // [M]
  u16* a_out; u16* nx_out; int64_t ldo;
  int bw;                            // block width (256)
  // Single-token step (decode): when h != nullptr the scan step is fused
  // here instead of writing (a, nx): h = a*h + nx (fp32, layers.py:175-182),
  // y = bf16(h) [* gate], state updated in place.
  float* h; int64_t ldh;
  const u16* gate; int64_t ldg;
  u16* y_out; int64_t ldy;           // ldy == 0: packed rows (M <= 32)
  int mt;                            // ceil(M / 16)
  // gx_pre / ga_pre are the bf16 BDL outputs (einsum rounded, + b rounded).
  CADENCE_DEV void chain(float gx_pre, float ga_pre, float xv, float sp,
                         bool reset, float& av, float& nx) const {
    const float gx = rbf(hw_sigmoid(gx_pre));
    const float ga = rbf(hw_sigmoid(ga_pre));
    // -8 ga and 2 log_a scale a bf16 value by a power of two: exact in bf16,
    // so the reference's rounding of them is the identity (not re-done here)
    const float log_a = bmul(-8.0f * ga, sp);
    const float a = rbf(hw_exp(log_a));
    const float a_sq = rbf(hw_exp(2.0f * log_a));
    const float gated = bmul(xv, gx);
    const float mult = reset ? 1.0f : rbf(hw_sqrt(rbf(1.0f - a_sq)));
    av = reset ? 0.0f : a;
    nx = bmul(gated, mult);
  }
  // Two elements at once (the prefill gates kernel's channel pair): the
  // same operations and rounding points as chain(), each rounding point one
  // v_cvt_pk_bf16_f32 for both values; bit-identical to two chain() calls.
  CADENCE_DEV void chain2(f32x2 gx_pre, f32x2 ga_pre, f32x2 xv, f32x2 sp, bool reset,
                          f32x2& av, f32x2& nx) const {
    const f32x2 gx = rbf2(f32x2{hw_sigmoid(gx_pre.x), hw_sigmoid(gx_pre.y)});
    const f32x2 ga = rbf2(f32x2{hw_sigmoid(ga_pre.x), hw_sigmoid(ga_pre.y)});
    const f32x2 log_a = bmul2(f32x2{-8.0f * ga.x, -8.0f * ga.y}, sp);   // exact scalings
    const f32x2 a = rbf2(f32x2{hw_exp(log_a.x), hw_exp(log_a.y)});
    const f32x2 l2 = f32x2{2.0f * log_a.x, 2.0f * log_a.y};
    const f32x2 a_sq = rbf2(f32x2{hw_exp(l2.x), hw_exp(l2.y)});
    const f32x2 gated = bmul2(xv, gx);
    const f32x2 om = rbf2(f32x2{sub_rn(1.0f, a_sq.x), sub_rn(1.0f, a_sq.y)});
    const f32x2 mult = reset ? f32x2{1.0f, 1.0f}
                             : rbf2(f32x2{hw_sqrt(om.x), hw_sqrt(om.y)});
    av = reset ? f32x2{0.0f, 0.0f} : a;
    nx = bmul2(gated, mult);
  }
  CADENCE_DEV void apply2(int64_t m, int j, float accx, float acca, int g) const {
    const int e = g * bw + j;
    float av, nx;
    chain(badd(rbf(accx), bf2f(bias_x[e])), badd(rbf(acca), bf2f(bias_a[e])),
          bf2f(x[m * ldx + e]), bf2f(softplus_a[e]), segpos[m] == 0, av, nx);
    if (h) {
      float* hp = h + m * ldh + e;
      const float hn = add_rn(mul_rn(av, *hp), nx);
      *hp = hn;
      float y = rbf(hn);
      if (gate) y = bmul(y, bf2f(gate[m * ldg + e]));
      y_out[xoff((int)m, e, ldy, mt)] = f2bf(y);
      return;
    }
    a_out[m * ldo + e] = f2bf(av);
    nx_out[m * ldo + e] = f2bf(nx);
  }
  // stream engine: every per-element operand is loaded at kernel start
  // (kPrefetch) and lands while the weight stream is in flight
  static constexpr bool kPrefetch = true;
  struct Pref { u16 bx, ba, xv, sp, gt; int reset; float h; };
  CADENCE_DEV Pref prefetch2(int64_t m, int j, int g) const {
    const int e = g * bw + j;
    Pref p;
    p.bx = bias_x[e];
    p.ba = bias_a[e];
    p.xv = x[m * ldx + e];
    p.sp = softplus_a[e];
    p.reset = segpos[m] == 0;
    // branch-free: absent operands read the zero page
    const float* hp = h ? h + m * ldh + e : reinterpret_cast<const float*>(kZeroPage);
    const u16* gp = (h && gate) ? gate + m * ldg + e : reinterpret_cast<const u16*>(kZeroPage);
    p.h = *hp;
    p.gt = *gp;
    return p;
  }
  CADENCE_DEV void apply2_pf(int64_t m, int j, float accx, float acca, int g,
                             const Pref& p) const {
    const int e = g * bw + j;
    float av, nx;
    chain(badd(rbf(accx), bf2f(p.bx)), badd(rbf(acca), bf2f(p.ba)), bf2f(p.xv),
          bf2f(p.sp), p.reset != 0, av, nx);
    if (h) {
      const float hn = add_rn(mul_rn(av, p.h), nx);
      h[m * ldh + e] = hn;
      float y = rbf(hn);
      if (gate) y = bmul(y, bf2f(p.gt));
      y_out[xoff((int)m, e, ldy, mt)] = f2bf(y);
      return;
    }
    a_out[m * ldo + e] = f2bf(av);
    nx_out[m * ldo + e] = f2bf(nx);
  }
  CADENCE_DEV float bias_at(bool up, int j, int g) const {
    return bf2f((up ? bias_a : bias_x)[g * bw + j]);
  }
  CADENCE_DEV float stage(float v, float b) const { return badd(rbf(v), b); }
  CADENCE_DEV void finish8p(int64_t m, int j, uint4 gx8, uint4 ga8, int g) const {
    const int e = g * bw + j;
    float gx[8], ga[8], xv[8], sp[8];
    unpack8(gx8, gx);
    unpack8(ga8, ga);
    unpack8(ld16(x + m * ldx + e), xv);
    unpack8(ld16(softplus_a + e), sp);
    const bool reset = segpos[m] == 0;
    float av[8], nx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) chain(gx[i], ga[i], xv[i], sp[i], reset, av[i], nx[i]);
    if (h) {
      float* hp = h + m * ldh + e;
      float y[8], gv[8];
      if (gate) unpack8(ld16(gate + m * ldg + e), gv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float hn = add_rn(mul_rn(av[i], hp[i]), nx[i]);
        hp[i] = hn;
        y[i] = rbf(hn);
        if (gate) y[i] = bmul(y[i], gv[i]);
      }
      st16(y_out + xoff((int)m, e, ldy, mt), pack8(y));
      return;
    }
    st16(a_out + m * ldo + e, pack8(av));
    st16(nx_out + m * ldo + e, pack8(nx));
  }
};

// Decode recurrent-block front in ONE launch (verdict r05 item 3): the y|x
// projection + Conv1D step (EpiLinearConv), then, in the same workgroups,
// the RG-LRU gate GEMV + scan step of EpiRglruGates (layers.py:345-365,
// :175-182) -- no second launch.  Each head's 2 bw / 32 gate items (the
// paired 16-channel blocks of gemm_stream_kernel<32, 1, 1, EpiRglruGates>)
// are taken one each by the head's 2 bw / 32 y|x workgroups (its y-branch
// and x-branch column pairs), after all of them have published their
// outputs: y|x outputs are stored write-through (sc1), each workgroup
// drains its stores, arrives on the head's counter and polls it (one lane,
// s_sleep) until every workgroup of the head has arrived, then reads the
// conv outputs and the y gate with sc1 loads (MI355X_MICROARCH.md
// "inter-workgroup visibility", first protocol row; the y|x grid is one
// round, so the awaited workgroups are running or about to be).  The gate
// weights and the epilogue's other operands are loaded before the wait.
// Same fragments, k order, reduction order and epilogue as the two
// launches: bitwise equal (tests/test_recurrent_front_gpu.py).  Measured
// SLOWER than the two launches in the graph-replayed decode (15.3 us against
// 9.1 + 5.0, +21..54 us per token: profiles/r06t_front/): the hand-off chain
// after the last y|x workgroup of a head -- drain 0.5 us, arrival seen 1.2,
// cross-XCD x reload + MFMA 1.1, epilogue 0.55 -- costs what the launch
// boundary and the gate kernel's own ramp cost.  Off by default
// (ops.FRONT_ONE_LAUNCH).  Counters:
// cnt[32 head] counts arrivals, cnt[32 (heads + head)] departures; the head's last
// workgroup to depart zeroes both (every workgroup departs only after its
// own wait saw all arrivals), so the buffer is left as it was found.
template <class E, class = void>
struct EpiPost { static constexpr bool value = false; };
template <class E>
struct EpiPost<E, std::void_t<decltype(E::kPost)>> {
  static constexpr bool value = E::kPost;
};

// write-through (sc1) accesses of the hand-off: 16-B buffer stores / loads
// with aux = sc1, 4-B agent-scope relaxed loads (global_load_dword sc1)
CADENCE_DEV __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// element i of a bf16 array through `r` (its base): the aligned dword that
// holds it, loaded sc1 (buffer_load_dword), then its half
CADENCE_DEV float ld_sc1_bf(__amdgpu_buffer_rsrc_t r, int64_t i) {
  const uint32_t w = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)((i & ~(int64_t)1) * 2), 0, 16);
  return bf2f((i & 1) ? (u16)(w >> 16) : (u16)(w & 0xffff));
}

template <int TW>
struct EpiLinearConvGates : EpiLinearConv<TW> {
  static constexpr bool kPost = true;
  EpiRglruGates ge;     // x = out + conv_lo (ldx = ldo), gate = out (ldg = ldo), packed y
  const u16* wg;        // decode-packed gate weights [H][2 bw / 16][bw / 32][64][8]
  // [2 H] arrive / depart counters, zero before and after, one per 128-B
  // line (polled by every workgroup of the head: one shared line for all
  // heads put the arrivals 4-5 us behind: profiles/r06t_front/)
  static constexpr int kCntStride = 32;
  int32_t* cnt;
  int32_t* err;         // set to 1 if an arrival wait gave up (never expected)
  using Pref = typename EpiLinearConv<TW>::Pref;
  // this workgroup's [32 rows][32 columns] of `out`, staged so that the
  // hand-off leaves in 16-B write-through stores (post, step 1)
  CADENCE_DEV static u16* stage() {
    __shared__ __attribute__((aligned(16))) u16 buf[32 * 32];
    return buf;
  }
  CADENCE_DEV void put(int64_t m, int n, u16 v) const {
    stage()[m * 32 + (n & 31)] = v;
  }
  // EpiLinearConv::apply_pf with `out` staged in LDS
  CADENCE_DEV void apply_pf(int64_t m, int n, float v, int g, const Pref& p) const {
    const float x = this->value(m, n, v, g);
    if (n < this->conv_lo) {
      put(m, n, f2bf(x));
      return;
    }
    float acc = bmul(x, bf2f(p.w[TW - 1]));
#pragma unroll
    for (int s = 1; s < TW; ++s)
      acc = badd(acc, bmul(bf2f(p.s[TW - 1 - s]), bf2f(p.w[TW - 1 - s])));
    acc = badd(acc, bf2f(p.b));
    put(m, n, f2bf(acc));
    u16* srow = this->state + m * (int64_t)(TW - 1) * this->E + (n - this->conv_lo);
#pragma unroll
    for (int r = 0; r + 1 < TW - 1; ++r) srow[(int64_t)r * this->E] = p.s[r + 1];
    if constexpr (TW > 1) srow[(int64_t)(TW - 2) * this->E] = f2bf(x);
  }
  CADENCE_DEV void apply(int64_t m, int n, float v, int g) const {
    apply_pf(m, n, v, g, this->prefetch(m, n));
  }
  // the gate item of this workgroup; `red` = the stream kernel's 8 x 1024
  // float reduction buffer (idle again), M <= 32 rows
  // this workgroup's gate item: head, rank among the head's 2 bw / 32
  // workgroups, the two packed gate-weight column blocks, the channel of
  // thread t (its row is t / 16)
  struct Item { int head, per, colg[2], e; };
  CADENCE_DEV Item item() const {
    const int bw = ge.bw, El = this->conv_lo;
    const int col0 = blockIdx.x * 32;                       // this workgroup's y|x columns
    const bool xb = col0 >= El;
    const int c0 = xb ? col0 - El : col0;
    Item it;
    it.head = c0 / bw;
    const int rank = (c0 % bw) / 32 + (xb ? bw / 32 : 0);
    it.per = 2 * bw / 32;
    const int grp = rank >> 1, half = rank & 1;
    it.colg[0] = grp * 64 + half * 16;
    it.colg[1] = grp * 64 + 32 + half * 16;
    it.e = it.head * bw + grp * 32 + half * 16 + (threadIdx.x & 15);
    return it;
  }
  // operands of the gate stage that do not depend on this launch (gate
  // weights: k-step = wave, K = bw; bias / softplus / position / state),
  // loaded at kernel start, ahead of the y|x stream
  struct PostPref { uint4 wb[2]; u16 bx, ba, sp; int reset; float h; };
  CADENCE_DEV PostPref pre(int M) const {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, bw = ge.bw;
    const Item it = item();
    const int k = wave * 32;
    const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
    const u16* W = wg + (int64_t)it.head * 2 * bw * bw;
    PostPref p;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      p.wb[j] = ld16_nt(k < bw ? W + (((int64_t)(it.colg[j] >> 4) * (bw >> 5) + (k >> 5)) * 64 +
                                      lane) * 8
                               : zpage);
    const int pm = min((int)(threadIdx.x >> 4), M - 1);
    p.bx = ge.bias_x[it.e];
    p.ba = ge.bias_a[it.e];
    p.sp = ge.softplus_a[it.e];
    p.reset = ge.segpos[pm] == 0;
    p.h = ge.h[(int64_t)pm * ge.ldh + it.e];
    return p;
  }
  // the gate item of this workgroup; `red` = the stream kernel's 8 x 1024
  // float reduction buffer (idle again), M <= 32 rows
  CADENCE_DEV void post(float* red, int M, const PostPref& pp) const {
    constexpr int MS = 32, MR = 2, NREP = 2, S = MS * 16 * NREP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bw = ge.bw, heads = this->conv_lo / bw;
    const int col0 = blockIdx.x * 32;
    const Item it = item();
    const int head = it.head, per = it.per, e = it.e;
    // 1. this workgroup's y|x outputs leave write-through (16-B sc1 stores:
    //    4 per row), are out of its queue, then the workgroup arrives
    __syncthreads();
    if (tid < M * 4) {
      const int r = tid >> 2, q = tid & 3;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *reinterpret_cast<const u32x4*>(stage() + r * 32 + q * 8);
      __builtin_amdgcn_raw_buffer_store_b128(
          v, rsrc_of(this->out), (int)(((int64_t)r * this->ldo + col0 + q * 8) * 2), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_add(cnt + kCntStride * head, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int K = bw;
    const int k = wave * 32, koff = 8 * (lane >> 4);
    const bool ok = k < K;
    const int pm = min(tid >> 4, M - 1);
    const uint4* wb = pp.wb;
    const u16 pbx = pp.bx, pba = pp.ba, psp = pp.sp;
    const int preset = pp.reset;
    const float ph = pp.h;
    // 3. every workgroup of the head has published
    if (tid == 0) {
      int n = 0;
      while (__hip_atomic_load(cnt + kCntStride * head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < per) {
        __builtin_amdgcn_s_sleep(1);
        if (++n == (1 << 24)) {   // give up rather than hang the queue (never expected)
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    // 4. the conv outputs (A operand) and this thread's x / gate values, sc1
    const __amdgpu_buffer_rsrc_t xr = rsrc_of(ge.x);
    uint4 xa[MR];
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = i * 16 + (lane & 15);
      const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
          xr, (int)(((int64_t)min(m, M - 1) * ge.ldx + head * bw + k + koff) * 2), 0, 16));
      xa[i] = (ok && m < M) ? v : make_uint4(0, 0, 0, 0);
    }
    const float pxv = ld_sc1_bf(xr, (int64_t)pm * ge.ldx + e);
    const float pgt = ld_sc1_bf(rsrc_of(ge.gate), (int64_t)pm * ge.ldg + e);
    f32x4 acc[MR][NREP];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[i]), __builtin_bit_cast(bf16x8, wb[j]),
            f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[wave * S + ((i * 16 + rsub + r) * NREP + j) * 16 + csub] = acc[i][j][r];
    __syncthreads();
    // 5. fixed-order reduction and the paired epilogue (EpiRglruGates::apply2_pf)
    const int m = tid >> 4, c = tid & 15;
    if (m < M) {
      float v[NREP];
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const float* rr = red + (m * NREP + j) * 16 + c;
        v[j] = ((rr[0] + rr[S]) + (rr[2 * S] + rr[3 * S])) +
               ((rr[4 * S] + rr[5 * S]) + (rr[6 * S] + rr[7 * S]));
      }
      float av, nx;
      ge.chain(badd(rbf(v[0]), bf2f(pbx)), badd(rbf(v[NREP - 1]), bf2f(pba)), pxv, bf2f(psp),
               preset != 0, av, nx);
      const float hn = add_rn(mul_rn(av, ph), nx);
      ge.h[(int64_t)m * ge.ldh + e] = hn;
      ge.y_out[xoff(m, e, ge.ldy, ge.mt)] = f2bf(bmul(rbf(hn), pgt));
    }
    // 6. depart; the head's last workgroup to depart zeroes both counters
    if (tid == 0) {
      const int d = __hip_atomic_fetch_add(cnt + kCntStride * (heads + head), 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (d == per - 1) {
        __hip_atomic_store(cnt + kCntStride * head, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + kCntStride * (heads + head), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
};
template <int TW> struct EpiNormIn<EpiLinearConvGates<TW>> { static constexpr bool value = true; };

struct EpiVitResid {
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = false;
  static constexpr bool kTile = true;
  float* resid; int64_t ldr;
  const u16* bias; const u16* gamma;
  CADENCE_DEV void apply(int64_t m, int n, float v, int) const {
    v += bf2f(bias[n]);
    if (gamma) v *= bf2f(gamma[n]);
    resid[m * ldr + n] += v;
  }
  // resid += gamma * (acc + bias): the residual rows are read two row
  // groups (32 values per lane) at a time ahead of their stores.
  template <int MR>
  CADENCE_DEV void tile(const AccTile<MR>& acc, int64_t mbase, int nbase,
                        int lane, int M, int N, int) const {
    const int rsub = (lane >> 4) * 4, csub = lane & 15;
    int col[4];
    float bv[4], gv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      col[j] = min(nbase + j * 16 + csub, N - 1);
      bv[j] = bf2f(bias[col[j]]);
      gv[j] = gamma ? bf2f(gamma[col[j]]) : 1.0f;
    }
#pragma unroll
    for (int i0 = 0; i0 < MR; i0 += 2) {
      float rv[2][4][4];
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = min<int64_t>(mbase + (i0 + ii) * 16 + rsub + r, M - 1);
#pragma unroll
          for (int j = 0; j < 4; ++j) rv[ii][j][r] = resid[row * ldr + col[j]];
        }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mbase + (i0 + ii) * 16 + rsub + r;
          if (row >= M) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (nbase + j * 16 + csub >= N) continue;
            float v = acc[i0 + ii][j][r] + bv[j];
            if (gamma) v *= gv[j];
            resid[row * ldr + col[j]] = rv[ii][j][r] + v;
          }
        }
    }
  }
};

struct EpiPatch {
  static constexpr bool kPaired = false;
  static constexpr bool kStaged = false;
  static constexpr bool kTile = true;
  float* resid;                      // [B, ntok, N] fp32
  const u16* bias; const u16* pos;   // pos [P, N]
  int64_t P, ntok, prefix, N;
  CADENCE_DEV void apply(int64_t m, int n, float v, int) const {
    const int64_t b = m / P, p = m % P;
    v += bf2f(bias[n]);
    v += bf2f(pos[p * N + n]);
    resid[(b * ntok + prefix + p) * N + n] = v;
  }
  template <int MR>
  CADENCE_DEV void tile(const AccTile<MR>& acc, int64_t mbase, int nbase,
                        int lane, int M, int Ncols, int) const {
    const int rsub = (lane >> 4) * 4, csub = lane & 15;
    int col[4];
    float bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      col[j] = min(nbase + j * 16 + csub, Ncols - 1);
      bv[j] = bf2f(bias[col[j]]);
    }
#pragma unroll
    for (int i0 = 0; i0 < MR; i0 += 2) {
      float pv[2][4][4];
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = min<int64_t>(mbase + (i0 + ii) * 16 + rsub + r, M - 1);
          const uint32_t pr = (uint32_t)row % (uint32_t)P;
#pragma unroll
          for (int j = 0; j < 4; ++j) pv[ii][j][r] = bf2f(pos[(int64_t)pr * N + col[j]]);
        }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mbase + (i0 + ii) * 16 + rsub + r;
          if (row >= M) continue;
          const uint32_t b = (uint32_t)row / (uint32_t)P;
          const uint32_t p = (uint32_t)row - b * (uint32_t)P;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (nbase + j * 16 + csub >= Ncols) continue;
            float v = acc[i0 + ii][j][r];
            v += bv[j];
            v += pv[ii][j][r];
            resid[((int64_t)b * ntok + prefix + p) * N + col[j]] = v;
          }
        }
    }
  }
};

// Paired epilogues take the (gate, up) halves of each 64-column group:
// packed column 64g + w (w < 32) pairs with 64g + 32 + w -> logical 32g + w.

// ------------------------------------------------- big tile engine (DMA)
//
// 256x256x64 block tile, 8 waves (2 M x 4 N), wave tile 128x64 =
// 8x4 mfma_f32_16x16x32_bf16.  Operands go HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4: one wave instruction = 1 KiB = 8 rows of 128 B,
// no VGPR staging, no ds_write), two LDS buffers (128 KiB), one barrier
// per K tile.  The XOR chunk swizzle is applied on the per-lane SOURCE
// address (LDS image stays lane-linear) and again on the ds_read address
// (it is an involution), which keeps the 16-lane ds_read_b128 groups
// conflict-free.  Rows past M / N are clamped on load and masked at the
// store, so any M and any N % 64 == 0 work.

typedef const void __attribute__((address_space(1)))* gptr_t;
typedef void __attribute__((address_space(3)))* lptr_t;

// BM x 256 output tile of this workgroup: consecutive workgroups go to
// consecutive XCDs, so each XCD takes a contiguous range of tiles, walked in
// groups of 4 M-tiles (the W column panel is reused from that XCD's L2).
template <int BM>
CADENCE_DEV void big_tile_origin(int M, int N, int& m0, int& n0) {
  constexpr int BN = 256, GM = 4;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN, nt = ntm * ntn;
  int t = blockIdx.x;
  {
    const int xcd = t & 7, q = nt >> 3, r = nt & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    t = base + (t >> 3);
  }
  const int grp = t / (GM * ntn), fm = grp * GM;
  const int gs = min(ntm - fm, GM);
  const int within = t % (GM * ntn);
  const int tm = fm + within % gs, tn = within / gs;
  m0 = tm * BM;
  n0 = tn * BN;
}

// Epilogue of one wave's (16 MR) x 64 accumulator block (rows mbase..,
// columns nbase..; paired: 32 gate + 32 up packed columns).  Staged
// epilogues use `st`, 16 KiB of idle operand LDS owned by this wave; the
// caller has synchronised the workgroup and skipped padding column blocks.
template <class Epi, int MR>
CADENCE_DEV void big_epilogue(const Epi& epi, f32x4 (&acc)[MR][4], u16* st, int mbase,
                              int nbase, int lane, int M, int N, int g) {
  constexpr int NR = 4;
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
  if constexpr (Epi::kStaged && EpiRegPair<Epi>::value) {
    // Gate x up in registers: output features obase + 16 h + csub, h = 0, 1
    // (gate tiles 0 / 1, up tiles 2 / 3), rows taken in pairs (r, r + 1) so
    // every rounding point rounds two values with one v_cvt_pk_bf16_f32; the
    // bf16 outputs go to [16 MR rows][32 features] of the wave's LDS (16-B
    // chunk XOR (row / 4) & 3: the 4 row groups of a write land on distinct
    // banks), then 16-B row segments out.  Same operations and rounding
    // points as stage() + finish8p(): bit-identical.
    const int obase = nbase / 2;
    float bgv[2], buv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bgv[h] = epi.bias_at(false, obase + h * 16 + csub, g);
      buv[h] = epi.bias_at(true, obase + h * 16 + csub, g);
    }
    auto oidx = [](int r, int c) { return r * 32 + ((((c >> 3) ^ (r >> 2)) & 3) << 3) + (c & 7); };
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const uint32_t w = epi.out2(f32x2{acc[i][h][r], acc[i][h][r + 1]},
                                      f32x2{acc[i][2 + h][r], acc[i][2 + h][r + 1]}, bgv[h],
                                      buv[h]);
          const int row = i * 16 + rsub + r, c = h * 16 + csub;
          st[oidx(row, c)] = (u16)w;
          st[oidx(row + 1, c)] = (u16)(w >> 16);
        }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // 4 chunks of 8 features per row, 16 rows per pass
    const int ch = lane & 3;
#pragma unroll
    for (int it = 0; it < MR; ++it) {
      const int lr = it * 16 + (lane >> 2);
      const int row = mbase + lr;
      const uint4 v = *reinterpret_cast<const uint4*>(&st[oidx(lr, ch * 8)]);
      if (row < M) epi.store8(row, obase + ch * 8, v);
    }
  } else if constexpr (Epi::kStaged) {
    // Stage the wave's first-rounding-point bf16 values in its own 16 KiB of
    // the (now idle) operand LDS, [128 rows][64 cols] with a 16-B chunk XOR
    // swizzle (paired: cols 0..31 gate half, 32..63 up half of the same 32
    // logical columns), then a rolled loop finishes 8 columns of one row per
    // lane and writes 16-B row segments.
    constexpr int OC = Epi::kPaired ? 32 : 64;     // output columns per wave
    constexpr int CPRW = OC / 8;                   // 16-B output chunks per row
    constexpr int RPI = 64 / CPRW;                 // rows per finish iteration
    auto sidx = [&](int r, int c) {
      return r * 64 + (((c >> 3) ^ (r & 7)) << 3) + (c & 7);
    };
    // kResidPref: every finish iteration's residual row segment is in flight
    // while the accumulators are staged (rows / columns clamped in bounds)
    constexpr bool kRP = EpiResidPref<Epi>::value;
    constexpr int RIT = kRP ? MR * 16 / RPI : 1;
    uint4 rpf[RIT];
    if constexpr (kRP) {
      const int col = min(nbase + (lane % CPRW) * 8, N - 8);
#pragma unroll
      for (int it = 0; it < RIT; ++it)
        rpf[it] = epi.resid_at(min(mbase + it * RPI + lane / CPRW, M - 1), col);
    }
    float bcol[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if constexpr (Epi::kPaired)
        bcol[j] = epi.bias_at(j >= 2, nbase / 2 + (j & 1) * 16 + csub, g);
      else
        bcol[j] = epi.bias_at(false, min(nbase + j * 16 + csub, N - 1), g);
    }
    // stage() returns bf16-rounded values: their bits are the top half of
    // the fp32 word (no third conversion), and the swizzled column of
    // (j, r) does not depend on i (rows i * 16 + ... keep row & 7)
    int soff[NR][4];
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) soff[j][r] = sidx(rsub + r, j * 16 + csub);
    if constexpr (!Epi::kPaired && EpiStage2<Epi>::value) {
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const uint32_t w = epi.stage2(f32x2{acc[i][j][r], acc[i][j][r + 1]}, bcol[j]);
            st[i * 16 * 64 + soff[j][r]] = (u16)w;
            st[i * 16 * 64 + soff[j][r + 1]] = (u16)(w >> 16);
          }
    } else {
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st[i * 16 * 64 + soff[j][r]] =
                (u16)(__float_as_uint(epi.stage(acc[i][j][r], bcol[j])) >> 16);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int obase = Epi::kPaired ? nbase / 2 : nbase;
    const int ch = lane % CPRW;
    if constexpr (kRP) {
      const int col = obase + ch * 8;
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        const int lr = it * RPI + lane / CPRW;
        const int row = mbase + lr;
        const uint4 v = *reinterpret_cast<const uint4*>(&st[lr * 64 + ((ch ^ (lr & 7)) << 3)]);
        if (row < M && col < N) epi.finish8_r(row, col, v, rpf[it]);
      }
      return;
    }
    if constexpr (EpiRowPref<Epi>::value) {
      constexpr int IT = MR * 16 / RPI;
      const int col = obase + ch * 8;
      int rp[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it)
        rp[it] = epi.row_pos(min(mbase + it * RPI + lane / CPRW, M - 1));
      typename Epi::RowPref pf[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) pf[it] = epi.row_prefetch(rp[it], min(col, N - 8));
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int lr = it * RPI + lane / CPRW;
        const int row = mbase + lr;
        const uint4 v = *reinterpret_cast<const uint4*>(&st[lr * 64 + ((ch ^ (lr & 7)) << 3)]);
        if (row < M && col < N) epi.finish8_pf(row, col, v, rp[it], pf[it]);
      }
      return;
    }
#pragma unroll 2
    for (int it = 0; it < MR * 16 / RPI; ++it) {
      const int lr = it * RPI + lane / CPRW;
      const int row = mbase + lr;
      const int col = obase + ch * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(&st[lr * 64 + ((ch ^ (lr & 7)) << 3)]);
      if constexpr (Epi::kPaired) {
        const uint4 u = *reinterpret_cast<const uint4*>(
            &st[lr * 64 + (((ch + 4) ^ (lr & 7)) << 3)]);
        if (row < M) epi.finish8p(row, col, v, u, g);
      } else {
        if (row < M && col < N) epi.finish8(row, col, v, g);
      }
    }
  } else if constexpr (Epi::kTile) {
    epi.template tile<MR>(acc, mbase, nbase, lane, M, N, g);
  } else if constexpr (Epi::kPaired) {
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mbase + i * 16 + rsub + r;
          if (row < M && nbase < N)
            epi.apply2(row, nbase / 2 + j * 16 + csub, acc[i][j][r],
                       acc[i][j + 2][r], g);
        }
  } else {
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mbase + i * 16 + rsub + r;
          const int col = nbase + j * 16 + csub;
          if (row < M && col < N) epi.apply(row, col, acc[i][j][r], g);
        }
  }
}

// 8-phase schedule (P8, K % 128 == 0).  The two LDS buffers (even / odd
// K-tile) are each cut into four 16 KiB half-tiles by the wave sub-tile they
// feed: A-h0 = rows {0..63, 128..191} (first 64 rows of each M-wave), A-h1 =
// {64..127, 192..255}, B-h0 / B-h1 = first / second 32 columns of each
// N-wave.  An iteration computes two K-tiles in 8 phases; phase p computes
// one 64x32 quadrant of the wave tile (16 MFMAs) from fragments read at the
// phase start and stages ONE half-tile (2 LDS-DMA instructions per lane):
//   p  reads            quadrant    stages
//   1  E.A-h0, E.B-h0   (m0, n0)    O.A-h1 <- K-tile 2i+1
//   2  E.B-h1           (m0, n1)    E.A-h0 <- 2i+2
//   3  E.A-h1           (m1, n1)    E.B-h0 <- 2i+2
//   4  -                (m1, n0)    E.B-h1 <- 2i+2; vmcnt(6) retires O
//   5  O.A-h0, O.B-h0   (m0, n0)    E.A-h1 <- 2i+2
//   6  O.B-h1           (m0, n1)    O.A-h0 <- 2i+3
//   7  O.A-h1           (m1, n1)    O.B-h0 <- 2i+3
//   8  -                (m1, n0)    O.B-h1 <- 2i+3; vmcnt(6) retires E
// Every half-tile is restaged >= 1 phase after its last read (a phase's
// reads feed its own MFMAs, so they are retired by the phase-end barrier) and
// read >= 1 phase after the counted vmcnt that retires it, so three
// half-tiles of DMA stay in flight across every barrier (no vmcnt(0) in the
// loop; raw s_barrier, since __syncthreads() would drain the DMA).
CADENCE_DEV void p8_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MR = 7 (BM = 224, P8 only): the second m-half of each wave holds 3
// fragments (48 rows); its half-tile DMA re-loads the last of those rows
// into the unused 16 rows, so every wave issues the same DMA count.
template <class Epi, int P8, int MR = 8>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ W,
    int64_t ldw, int M, int N, int K, int64_t a_goff, int64_t w_goff,
    Epi epi) {
  constexpr int BM = 32 * MR, BN = 256, NR = 4;
  static_assert(MR == 8 || (P8 && MR >= 5 && MR < 8), "BM < 256 needs the 8-phase schedule");
  constexpr int ROWS = 256 + BN;              // LDS rows per buffer (128 B)
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * ROWS * 8];

  const int g = blockIdx.y;
  A += g * a_goff;
  W += g * w_goff;

  int m0, n0;
  big_tile_origin<BM>(M, N, m0, n0);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // DMA mapping: lane l of an 8-row piece lands at LDS row 8*piece + l/8,
  // slot l%8, so it loads source chunk (l%8) ^ (l/8) (XOR swizzle).
  const int src_chunk = (lane & 7) ^ (lane >> 3);
  if constexpr (P8) {
    constexpr int HT = 128 * 8;                 // uint4 per half-tile
    // wave w moves pieces 2w, 2w+1 (8 rows each) of every half-tile
    const u16* sa[2][2];
    const u16* sb[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const int r = (2 * wave + pc) * 8 + (lane >> 3);   // half-tile row
        const int rr = h ? min(r & 63, MR * 16 - 65) : (r & 63);
        const int gm = min(m0 + (r >> 6) * (MR * 16) + h * 64 + rr, M - 1);
        const int gn = min(n0 + (r >> 5) * 64 + h * 32 + (r & 31), N - 1);
        sa[h][pc] = A + (int64_t)gm * lda + src_chunk * 8;
        sb[h][pc] = W + (int64_t)gn * ldw + src_chunk * 8;
      }
    auto stage = [&](int buf, int kind, const u16* p0, const u16* p1, int k0) {
      uint4* dst = &smem[(buf * 4 + kind) * HT + (2 * wave) * 64];
      __builtin_amdgcn_global_load_lds((gptr_t)(p0 + k0), (lptr_t)dst, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gptr_t)(p1 + k0), (lptr_t)(dst + 64), 16, 0, 0);
    };
    const int xr = lane & 7;   // row & 7 of every fragment row this lane reads
    // Each phase's fragments are read one phase ahead where the data is
    // already retired: B-h1 with phase 1's reads (b1 is idle in phase 1),
    // and -- given the registers for a second A set (MR < 8) -- A-h1 in
    // phase 2, so phases 2-4 (6-8) start their MFMAs on fragments already in
    // registers and only phases 1 and 5 wait for the LDS.
    constexpr bool PFA = MR < 8;
    bf16x8 af[4][2], b0[2][2], b1[2][2];
    [[maybe_unused]] bf16x8 ag[4][2];
    auto readA = [&](int buf, int mh, bf16x8 (&a)[4][2], int i0 = 0, int i1 = 4) {
      const uint4* base = &smem[(buf * 4 + mh) * HT];
#pragma unroll
      for (int i = i0; i < min(i1, mh ? MR - 4 : 4); ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          a[i][ks] = __builtin_bit_cast(
              bf16x8, base[(wm * 64 + i * 16 + (lane & 15)) * 8 +
                           ((ks * 4 + (lane >> 4)) ^ xr)]);
    };
    auto readB = [&](int buf, int nh, bf16x8 (&bf)[2][2]) {
      const uint4* base = &smem[(buf * 4 + 2 + nh) * HT];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bf[j][ks] = __builtin_bit_cast(
              bf16x8, base[(wn * 32 + j * 16 + (lane & 15)) * 8 +
                           ((ks * 4 + (lane >> 4)) ^ xr)]);
    };
    auto mma_rows = [&](int mh, int nh, const bf16x8 (&a)[4][2], const bf16x8 (&bf)[2][2],
                        int i0, int i1) {
#pragma unroll
      for (int i = i0; i < i1; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            acc[mh * 4 + i][nh * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                a[i][ks], bf[j][ks], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
    };
    auto mma = [&](int mh, int nh, const bf16x8 (&a)[4][2], const bf16x8 (&bf)[2][2]) {
      __builtin_amdgcn_s_setprio(1);
      mma_rows(mh, nh, a, bf, 0, mh ? MR - 4 : 4);
      __builtin_amdgcn_s_setprio(0);
    };
    // The compiler waits for every outstanding LDS read (lgkmcnt(0)) before
    // the first MFMA that consumes one, so a read meant for a later phase
    // goes out AFTER the wait of the phase it is issued in: behind the
    // quadrant's first MFMAs (sched_barrier keeps it there).
    // Phases 1 / 5 (fragments retired only by the previous barrier): rows
    // 0-1 of A-h0 + B-h0, their 8 MFMAs, then rows 2-3 + B-h1 (phase 2's).
    auto quad0 = [&](int buf) {
      readA(buf, 0, af, 0, 2);
      readB(buf, 0, b0);
      __builtin_amdgcn_s_setprio(1);
      mma_rows(0, 0, af, b0, 0, 2);
      __builtin_amdgcn_sched_barrier(0);
      readA(buf, 0, af, 2, 4);
      readB(buf, 1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma_rows(0, 0, af, b0, 2, 4);
      __builtin_amdgcn_s_setprio(0);
    };
    // Phases 2 / 6: with a second A set, A-h1 (phase 3's) behind row 0.
    auto quad1 = [&](int buf) {
      __builtin_amdgcn_s_setprio(1);
      if constexpr (PFA) {
        mma_rows(0, 1, af, b1, 0, 1);
        __builtin_amdgcn_sched_barrier(0);
        readA(buf, 1, ag);
        __builtin_amdgcn_sched_barrier(0);
        mma_rows(0, 1, af, b1, 1, 4);
      } else {
        mma_rows(0, 1, af, b1, 0, 4);
      }
      __builtin_amdgcn_s_setprio(0);
    };
    auto& a1 = PFA ? ag : af;   // the A-h1 fragments
    const int nk = K / BK;
    // prologue: even <- tile 0 (all four), odd <- tile 1 (A-h0, B-h0, B-h1)
    stage(0, 0, sa[0][0], sa[0][1], 0);
    stage(0, 1, sa[1][0], sa[1][1], 0);
    stage(0, 2, sb[0][0], sb[0][1], 0);
    stage(0, 3, sb[1][0], sb[1][1], 0);
    stage(1, 0, sa[0][0], sa[0][1], BK);
    stage(1, 2, sb[0][0], sb[0][1], BK);
    stage(1, 3, sb[1][0], sb[1][1], BK);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    p8_barrier();
    for (int it = 0; it < nk / 2; ++it) {
      const int kO1 = (2 * it + 1) * BK, kE = (2 * it + 2) * BK, kO = (2 * it + 3) * BK;
      const bool more = 2 * it + 2 < nk;         // tiles 2i+2 and 2i+3 exist
      // phase 1
      stage(1, 1, sa[1][0], sa[1][1], kO1);
      quad0(0); p8_barrier();
      // phase 2
      if (more) stage(0, 0, sa[0][0], sa[0][1], kE);
      quad1(0); p8_barrier();
      // phase 3
      if constexpr (!PFA) readA(0, 1, af);
      if (more) stage(0, 2, sb[0][0], sb[0][1], kE);
      mma(1, 1, a1, b1); p8_barrier();
      // phase 4
      if (more) {
        stage(0, 3, sb[1][0], sb[1][1], kE);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      mma(1, 0, a1, b0); p8_barrier();
      // phase 5
      if (more) stage(0, 1, sa[1][0], sa[1][1], kE);
      quad0(1); p8_barrier();
      // phase 6
      if (more) stage(1, 0, sa[0][0], sa[0][1], kO);
      quad1(1); p8_barrier();
      // phase 7
      if constexpr (!PFA) readA(1, 1, af);
      if (more) stage(1, 2, sb[0][0], sb[0][1], kO);
      mma(1, 1, a1, b1); p8_barrier();
      // phase 8
      if (more) {
        stage(1, 3, sb[1][0], sb[1][1], kO);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      mma(1, 0, a1, b0); p8_barrier();
    }
  } else {
  // 2-buffer schedule: wave w moves pieces 8w..8w+7 of the 64 pieces of a
  // K tile (pieces 0..31 = A rows, 32..63 = W rows).
  const u16* src[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = wave * 8 + i;
    if (piece < 32) {
      const int r = min(m0 + piece * 8 + (lane >> 3), M - 1);
      src[i] = A + (int64_t)r * lda + src_chunk * 8;
    } else {
      const int r = min(n0 + (piece - 32) * 8 + (lane >> 3), N - 1);
      src[i] = W + (int64_t)r * ldw + src_chunk * 8;
    }
  }
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int piece = wave * 8 + i;
      __builtin_amdgcn_global_load_lds(
          (gptr_t)(src[i] + k0),
          (lptr_t)(&smem[(buf * ROWS + piece * 8) * 8]), 16, 0, 0);
    }
  };

  const int nk = K / BK;
  const int sw = lane & 7;  // (row & 7) of every row this lane reads
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const uint4* As = &smem[cur * ROWS * 8];
    const uint4* Bs = &smem[(cur * ROWS + BM) * 8];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = (s * 4 + (lane >> 4)) ^ sw;
      bf16x8 bfr[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bfr[j] = __builtin_bit_cast(
            bf16x8, Bs[(wn * 64 + j * 16 + (lane & 15)) * 8 + ch]);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8 af = __builtin_bit_cast(
            bf16x8, As[(wm * 128 + i * 16 + (lane & 15)) * 8 + ch]);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j],
                                                              acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();   // waits this wave's DMA (vmcnt) + all waves' reads
  }
  }

  const int mbase = m0 + wm * (MR * 16), nbase = n0 + wn * 64;
  if constexpr (Epi::kStaged) {
    __syncthreads();   // every wave is done reading the operand buffers
    if (nbase >= N) return;   // wave-uniform: this wave's columns are padding
  }
  big_epilogue<Epi, MR>(epi, acc, reinterpret_cast<u16*>(smem) + wave * (128 * 64), mbase,
               nbase, lane, M, N, g);
}

// 4-wave engine: 256 x 256 x 64 block tile, 4 waves (2 M x 2 N) of one
// wave per SIMD, wave tile 128 x 128 = 8 x 8 mfma_f32_16x16x32_bf16
// (256 accumulator registers).  Per K-tile a wave reads 32 KiB of fragments
// for 128 MFMAs, a third less LDS traffic per MFMA than the 8-wave 128 x 64
// layout.  Operands go HBM -> LDS by LDS-DMA into two 64 KiB buffers with
// the same swizzled image as gemm_big_kernel (waves 0-1 move the 256 A rows,
// waves 2-3 the 256 W rows: 16 pieces of 8 rows x 128 B each).  One barrier
// per K-tile, placed between the tile's two 32-deep k-steps:
//   read k-step 1 of tile t | MFMAs k-step 0 | retire reads + DMA of t+1 |
//   barrier | DMA t+2 into this buffer, read k-step 0 of t+1 | MFMAs k-step 1
// so every MFMA block starts on fragments already in registers and each
// DMA has a whole K-tile of MFMAs to land in.
template <class Epi, int MR>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ W,
    int64_t ldw, int M, int N, int K, int64_t a_goff, int64_t w_goff,
    Epi epi) {
  constexpr int BM = 32 * MR, TILE = 512 * 8;  // uint4 per K-tile buffer
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * TILE];

  const int g = blockIdx.y;
  A += g * a_goff;
  W += g * w_goff;
  int m0, n0;
  big_tile_origin<BM>(M, N, m0, n0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // DMA sources: wave w moves buffer rows 128 w + 8 i + lane / 8 (i < 16);
  // lane l of a piece lands at slot l % 8, so it loads source chunk
  // (l % 8) ^ (l / 8) (the XOR swizzle, an involution)
  const int src_chunk = (lane & 7) ^ (lane >> 3);
  const bool isA = wave < 2;
  const u16* base = isA ? A : W;
  const int64_t ld = isA ? lda : ldw;
  // A halves hold 16 MR rows (pieces past them re-load the half's last row)
  const int half0 = (isA ? m0 + (wave & 1) * 16 * MR : n0 + (wave & 1) * 128);
  const int hlim = min((isA ? M : N) - 1, half0 + (isA ? 16 * MR : 128) - 1);
  // 32-bit byte offsets from a wave-uniform base: saddr + voffset loads,
  // no 64-bit address arithmetic per piece
  uint32_t soff[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    soff[i] = (uint32_t)(((int64_t)min(half0 + 8 * i + (lane >> 3), hlim) * ld +
                          src_chunk * 8) * 2);
  auto dma = [&](int buf, int k0) {
    uint4* dst = &smem[buf * TILE + wave * 16 * 64];
    const char* bk = reinterpret_cast<const char*>(base + k0);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(bk + soff[i]), (lptr_t)(dst + i * 64), 16,
                                       0, 0);
  };
  const int xr = lane & 7;
  // fragment read r of a k-step: r < MR = A row block r, else B column block
  // r - MR (ds_read_b128, XOR-swizzled chunk)
  auto rd1 = [&](int buf, int ks, int r, bf16x8& f) {
    const uint4* sp = &smem[buf * TILE];
    const int ch = (ks * 4 + (lane >> 4)) ^ xr;
    const int row = r < MR ? wm * 128 + r * 16 : 256 + wn * 128 + (r - MR) * 16;
    f = __builtin_bit_cast(bf16x8, sp[(row + (lane & 15)) * 8 + ch]);
  };
  f32x4 acc[MR][8];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // One segment = the MR x 8 MFMAs of one 32-deep k-step, with the next
  // k-step's MR + 8 fragment reads (after MFMAs 0, 3, 6, ...) and, when
  // `dma`, the 16 LDS-DMA pieces of a later K-tile (after MFMAs 1, 4, ...)
  // threaded between them.  The MFMAs are inline asm tied to their AGPR
  // accumulators ("+a"): with the builtin, hipcc re-allocates some
  // accumulators every iteration of this 224-256-accumulator loop and
  // shuffles them through v_accvgpr_mov / VGPR copies; an asm statement with
  // side effects also keeps the interleave in source order.  (hipcc inserts
  // no wait states for asm MFMAs: the loop's operands are only ds_read /
  // MFMA results, and the epilogue below waits explicitly.)
  const int nk = K / BK;
  // past the last K-tile the DMA pieces read the zero page (lane-linear
  // 16 B each) instead of branching around them
  const uint32_t zoff = lane * 16;
  const char* zpage = reinterpret_cast<const char*>(kZeroPage);
  auto segment = [&](const bf16x8 (&a)[MR], const bf16x8 (&b)[8], bf16x8 (&na)[MR],
                     bf16x8 (&nb)[8], int rbuf, int rks, bool dma_on, int dbuf,
                     int dtile) {
    uint4* dst = &smem[dbuf * TILE + wave * 16 * 64];
    const bool live = dtile < nk;
    const char* bk = live ? reinterpret_cast<const char*>(base + dtile * BK) : zpage;
    int nr = 0, nd = 0;
#pragma unroll
    for (int n = 0; n < MR * 8; ++n) {
      const int i = n / 8, j = n % 8;
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                   : "+a"(acc[i][j]) : "v"(a[i]), "v"(b[j]));
      if (n % 3 == 0 && nr < MR + 8) {
        if (nr < MR) rd1(rbuf, rks, nr, na[nr]);
        else rd1(rbuf, rks, nr, nb[nr - MR]);
        ++nr;
      }
      if (dma_on && n % 3 == 1 && nd < 16) {
        __builtin_amdgcn_global_load_lds((gptr_t)(bk + (live ? soff[nd] : zoff)),
                                         (lptr_t)(dst + nd * 64), 16, 0, 0);
        ++nd;
      }
    }
#pragma unroll
    for (; nr < MR + 8; ++nr) {
      if (nr < MR) rd1(rbuf, rks, nr, na[nr]);
      else rd1(rbuf, rks, nr, nb[nr - MR]);
    }
#pragma unroll
    for (; nd < 16; ++nd) {
      if (!dma_on) break;
      __builtin_amdgcn_global_load_lds((gptr_t)(bk + (live ? soff[nd] : zoff)),
                                       (lptr_t)(dst + nd * 64), 16, 0, 0);
    }
  };

  bf16x8 a0[MR], b0[8], a1[MR], b1[8];
  dma(0, 0);
  if (nk > 1) {
    dma(1, BK);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  p8_barrier();
#pragma unroll
  for (int r = 0; r < MR; ++r) rd1(0, 0, r, a0[r]);
#pragma unroll
  for (int r = 0; r < 8; ++r) rd1(0, 0, MR + r, b0[r]);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 4" ::: "memory");
  // K-tile t: segment A = MFMAs of k-step 0 with the reads of k-step 1;
  // every read of `cur` retired and this wave's DMA of tile t + 1 landed,
  // then the barrier publishes both; segment B = MFMAs of k-step 1 with
  // tile t + 2's DMA into the buffer just released and the reads of k-step
  // 0 of tile t + 1 (past the end: zero-page DMA and reads of dead data,
  // so the loop stays one branch-free body and hipcc keeps every
  // accumulator in one AGPR quad throughout -- a peeled tail made it copy
  // them at the loop exit, reading asm-MFMA results it cannot see pending).
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    segment(a0, b0, a1, b1, cur, 1, false, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(0)" ::: "memory");
    p8_barrier();
    segment(a1, b1, a0, b0, cur ^ 1, 0, true, cur, t + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // the zero-page DMA of the last tile lands before the epilogue reuses the
  // LDS, and the last asm MFMAs' results before the epilogue reads them
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15"
               ::: "memory");

  const int mbase = m0 + wm * 16 * MR;
  __syncthreads();   // every wave is done reading the operand buffers
  u16* st = reinterpret_cast<u16*>(smem) + wave * 2 * (128 * 64);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int nbase = n0 + wn * 128 + h * 64;
    if (nbase < N) {   // wave-uniform: these columns are not padding
      f32x4 half[MR][4];
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) half[i][j] = acc[i][h * 4 + j];
      big_epilogue<Epi, MR>(epi, half, st + h * (128 * 64), mbase, nbase, lane, M, N, g);
    }
  }
}

// Weight-streaming decode GEMM (M <= 32).  One workgroup = NTW x 16 output
// columns (paired: 16 gate + 16 up packed columns) x one K split; wave w owns
// k-steps w, w+8, ..., at most KSW of them, and issues ALL of its weight and
// activation loads before the first MFMA, so a workgroup waits for HBM once.
// NTW = 2 reuses every activation fragment for two column tiles (the
// activation loads, not the weight stream, bound the NTW = 1 form on the
// wide shapes); fragment-packed weights are read once, non-temporal.
// parts == nullptr: fixed-order LDS reduction + fused epilogue.  Otherwise
// raw fp32 partials go to parts[split][M][N]: for splitk_reduce_kernel /
// reduce_rmsnorm_kernel, or (counters != nullptr) combined in-kernel by the
// last K split of each column tile to arrive (write-through slabs, one
// agent-scope ticket per workgroup: MI355X_MICROARCH "inter-workgroup
// visibility", first protocol row), in split order -- the same sums as the
// reduce kernels -- then the epilogue.
//
// NORM: A holds unnormalised packed rows x, W's columns carry the RMSNorm
// scale (W[n][k] (1 + scale[k]) in bf16, ops.fold_norm), and the workgroup
// covers all of K (one split).  Each row's sum of squares comes from the
// MFMA pipe -- diag(X X^T) of the fragments already in registers, the
// products exact in fp32 -- and rsqrt(mean + eps), rounded as layers.py:70-78
// rounds var / var + eps / rsqrt, scales the fp32 dot products before the
// epilogue.  (The reference rounds x rsqrt and its product with 1 + scale to
// bf16 per element; doing that here made every workgroup re-normalise the
// whole activation on the VALU: +7..13 us per GEMV, measured.)
template <int MS, int KSW, int NTW, class Epi, bool NORM = false>
__global__ __launch_bounds__(512) void gemm_stream_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ W,
    int64_t ldw, int M, int N, int K, int klen, int64_t a_goff, int64_t w_goff,
    float* __restrict__ parts, Epi epi, int packed, int32_t* __restrict__ counters,
    float neps) {
  constexpr int MR = MS / 16;
  static_assert(!Epi::kPaired || NTW == 1, "paired epilogues pair gate/up tiles");
  constexpr int NREP = Epi::kPaired ? 2 : NTW;
  __shared__ float red[8][MS * 16 * NREP];
  __shared__ float nss[NORM ? 8 : 1][MS];
  __shared__ int ticket;
  const int g = blockIdx.z;
  A += g * a_goff;
  W += g * w_goff;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int col[NREP];
  if constexpr (Epi::kPaired) {
    const int grp = blockIdx.x >> 1, half = blockIdx.x & 1;
    col[0] = grp * 64 + half * 16;
    col[NREP - 1] = grp * 64 + 32 + half * 16;
  } else {
#pragma unroll
    for (int t = 0; t < NTW; ++t) col[t] = (blockIdx.x * NTW + t) * 16;
  }
  // prefetching epilogues: this thread's epilogue elements are row tid / 16,
  // columns col[j] + tid % 16 (the epilogue loop below runs once per thread)
  // (paired: one (gate, up) element per thread, column grp * 32 + half * 16 +
  // tid % 16 of the epilogue's output)
  constexpr bool kPf = EpiPrefetch<Epi>::value;
  [[maybe_unused]] typename std::conditional<kPf, Epi, EpiLinear>::type::Pref pf[NREP];
  // (unconditional, rows clamped to M - 1: a load under a branch would cost
  // a vmcnt(0) at the join before the weight stream is even issued)
  if constexpr (kPf) {
    static_assert(MS * 16 <= 512, "one epilogue element per thread");
    const int pm = min((int)(threadIdx.x >> 4), M - 1);
    if constexpr (Epi::kPaired) {
      pf[0] = epi.prefetch2(pm, (blockIdx.x >> 1) * 32 + (blockIdx.x & 1) * 16 + (threadIdx.x & 15),
                            g);
    } else {
#pragma unroll
      for (int j = 0; j < NREP; ++j) pf[j] = epi.prefetch(pm, col[j] + (threadIdx.x & 15));
    }
  }
  // a second stage's own operands (EpiLinearConvGates), ahead of the stream
  [[maybe_unused]] auto post_pf = [&] {
    if constexpr (EpiPost<Epi>::value) return epi.pre(M);
    else return 0;
  }();
  const int koff = 8 * (lane >> 4);
  const int kbeg = blockIdx.y * klen;
  const int kend = min(K, kbeg + klen);
  const uint4 zero = make_uint4(0, 0, 0, 0);
  // Branch-free issue: every load is unconditional; a fragment that must be
  // zero (k past the split, rows past M) is read from a zero page instead of
  // being masked after the load.  A load under a branch makes the waitcnt
  // pass put a vmcnt(0) at the join, and a select on the loaded value waits
  // for it: either costs a full memory round trip per k-step instead of one
  // per workgroup.
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  uint4 wb[KSW][NREP], xa[KSW][MR];
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kbeg + (wave + 8 * u) * 32;
    const bool ok = k < kend;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = i * 16 + (lane & 15);
      // packed rows (common.hpp xpk, mt == MR here) or row-major
      const int64_t off = lda == 0 ? ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3)
                                   : (int64_t)m * lda + k + koff;
      xa[u][i] = ld16((ok && (lda == 0 || m < M)) ? A + off : zpage);
    }
  }
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kbeg + (wave + 8 * u) * 32;
    const bool ok = k < kend;
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      // fragment-packed [N/16][K/32][64 lanes][8]: 1 KiB per load
      const int64_t off = packed
          ? (((int64_t)(col[j] >> 4) * (K >> 5) + (k >> 5)) * 64 + lane) * 8
          : (int64_t)(col[j] + (lane & 15)) * ldw + k + koff;
      wb[u][j] = ld16_nt(ok ? W + off : zpage);
    }
  }
  if constexpr (NORM) {
    // row sums of squares: diag of the 16 x 16 blocks X_i X_i^T; lane l
    // holds C[4 (l / 16) + r][l % 16], a diagonal element when
    // (l % 16) / 4 == l / 16 (row l % 16, r = l % 4)
    f32x4 dg[MR];
#pragma unroll
    for (int i = 0; i < MR; ++i) dg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < KSW; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i)
        dg[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[u][i]), __builtin_bit_cast(bf16x8, xa[u][i]),
            dg[i], 0, 0, 0);
    const int r4 = lane & 3;
    if (((lane & 15) >> 2) == (lane >> 4)) {
#pragma unroll
      for (int i = 0; i < MR; ++i)
        nss[wave][i * 16 + (lane & 15)] =
            r4 == 0 ? dg[i][0] : r4 == 1 ? dg[i][1] : r4 == 2 ? dg[i][2] : dg[i][3];
    }
  }
  f32x4 acc[MR][NREP];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KSW; ++u)
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[u][i]),
            __builtin_bit_cast(bf16x8, wb[u][j]), acc[i][j], 0, 0, 0);
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][((i * 16 + rsub + r) * NREP + j) * 16 + csub] = acc[i][j][r];
  __syncthreads();
  if constexpr (!Epi::kPaired && !EpiPairLanes<Epi>::value) {
    if (counters) {
      // in-kernel split-K combine: thread o owns (row o / 16, column o % 16)
      // of each of the NREP column tiles (MS * 16 <= 512 threads).
      // Visibility without fences: this is the first measured hand-off row
      // of MI355X_MICROARCH.md "Workgroup dispatch, XCD placement &
      // inter-workgroup visibility" -- every slab byte stored `sc1`
      // (relaxed agent-scope stores, write-through), every storing wave's
      // `s_waitcnt vmcnt(0)` before the workgroup barrier, ONE lane's agent
      // atomic add per workgroup on one unsharded counter, and the
      // workgroup whose add returned S - 1 reading every slab byte with
      // `sc1` loads (relaxed agent-scope loads, L1 bypass) only after that
      // add returned and a barrier.  A release / acquire fence pair would
      // cost ~1.7 us each (same guide, price table) on the critical path of
      // 51 launches per decode step.

      const int o = threadIdx.x, m = o / 16, c = o % 16;
      const bool mine = o < MS * 16 && m < M;
      const int64_t sstride = (int64_t)gridDim.z * M * N;
      // (rows past M, which only load, read row M - 1: inside the slab)
      float* slab = parts + (int64_t)g * M * N + (int64_t)min(m, M - 1) * N;
      float v[NREP];
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const int idx = (min(m, MS - 1) * NREP + j) * 16 + c;
        v[j] = ((red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx])) +
               ((red[4][idx] + red[5][idx]) + (red[6][idx] + red[7][idx]));
        if (mine)
          __hip_atomic_store(slab + blockIdx.y * sstride + col[j] + c, v[j],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        ticket = __hip_atomic_fetch_add(counters + g * gridDim.x + blockIdx.x, 1,
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (ticket != (int)gridDim.y - 1) return;
      constexpr int SMAX = 4;
      const int S = gridDim.y;
      float p[SMAX][NREP];
#pragma unroll
      for (int sp = 0; sp < SMAX; ++sp)
#pragma unroll
        for (int j = 0; j < NREP; ++j)
          p[sp][j] = __hip_atomic_load(slab + min(sp, S - 1) * sstride + col[j] + c,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (mine) {
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          float t = 0.0f;
#pragma unroll
          for (int sp = 0; sp < SMAX; ++sp)
            if (sp < S) t += sp == (int)blockIdx.y ? v[j] : p[sp][j];
          if constexpr (EpiPrefetch<Epi>::value)
            epi.apply_pf(m, col[j] + c, t, g, pf[j]);
          else
            epi.apply(m, col[j] + c, t, g);
        }
      }
      if (threadIdx.x == 0)
        __hip_atomic_store(counters + g * gridDim.x + blockIdx.x, 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  for (int o = threadIdx.x; o < MS * 16; o += 512) {
    const int m = o / 16, c = o % 16;
    if (m >= M) continue;
    float v[NREP];
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      const int idx = (m * NREP + j) * 16 + c;
      v[j] = ((red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx])) +
             ((red[4][idx] + red[5][idx]) + (red[6][idx] + red[7][idx]));
    }
    if constexpr (NORM) {
      const float ss = ((nss[0][m] + nss[1][m]) + (nss[2][m] + nss[3][m])) +
                       ((nss[4][m] + nss[5][m]) + (nss[6][m] + nss[7][m]));
      const float var = rbf(ss / (float)K);
      const float rs = rbf(1.0f / sqrtf(rbf(var + neps)));
#pragma unroll
      for (int j = 0; j < NREP; ++j) v[j] *= rs;
    }
    if (parts) {
      float* dst = parts + ((int64_t)blockIdx.y * gridDim.z + g) * (int64_t)M * N +
                   (int64_t)m * N;
#pragma unroll
      for (int j = 0; j < NREP; ++j) dst[col[j] + c] = v[j];
    } else if constexpr (Epi::kPaired) {
      const int grp = blockIdx.x >> 1, half = blockIdx.x & 1;
      if constexpr (kPf)
        epi.apply2_pf(m, grp * 32 + half * 16 + c, v[0], v[NREP - 1], g, pf[0]);
      else
        epi.apply2(m, grp * 32 + half * 16 + c, v[0], v[NREP - 1], g);
    } else if constexpr (EpiPairLanes<Epi>::value) {
      // lanes o and o ^ 1 hold the two columns of a pair (same row m)
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const float x = epi.value(m, col[j] + c, v[j], g);
        const float y = __shfl_xor(x, 1, 64);
        epi.apply_pair(m, col[j] + c, x, y);
      }
    } else if constexpr (kPf) {
#pragma unroll
      for (int j = 0; j < NREP; ++j) epi.apply_pf(m, col[j] + c, v[j], g, pf[j]);
    } else {
#pragma unroll
      for (int j = 0; j < NREP; ++j) epi.apply(m, col[j] + c, v[j], g);
    }
  }
  // a second stage in the same workgroups (EpiLinearConvGates: the RG-LRU
  // gate item), reusing the reduction buffer
  if constexpr (EpiPost<Epi>::value) epi.post(&red[0][0], M, post_pf);
}

// Decode residual projection of one K split (1..32 packed rows in MR = 1 or 2 16-row tiles,
// fragment-packed W, K <= 16 waves x KSW x 32): the 13 MB output projection
// (K = 2560).  One workgroup = 16 output columns over all of K, 16 waves
// streaming their k-steps in chunks of CH with INF chunks of weight +
// activation fragments in flight; the EpiResidRows epilogue straight from the
// fixed-order LDS reduction (no split, no combine trip).  Cold-weight lab
// (tools/gemv_lab2.hip): 6.45-6.52 us against 6.98-7.06 for the 2-split
// stream kernel with its in-kernel combine; the 39 MB down projection stays on
// the split engine (per-CU bound unsplit: 15 us against 11.3).
template <int NW, int KSW, int CH, int INF, int MR>
__global__ __launch_bounds__(NW * 64) void gemm_resid_pipe_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, int M, int K, EpiResidRows epi) {
  constexpr int NC = KSW / CH, MS = 16 * MR;     // MR 16-row tiles of packed rows
  static_assert(KSW % CH == 0 && INF <= NC && NW * 64 >= MS * 16, "chunking / epilogue");
  __shared__ float red[NW][MS * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  const int ks32 = K >> 5;
  const int col0 = blockIdx.x * 16;
  // epilogue operands first: thread t < 512 owns (row t / 16, column t % 16)
  const int pm = min((int)(threadIdx.x >> 4) & (MS - 1), M - 1);
  const EpiResidRows::Pref pf = epi.prefetch(pm, col0 + (threadIdx.x & 15));
  uint4 wb[INF][CH], xa[INF][CH][MR];
  auto issue = [&](int c, int slot) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = (wave + NW * (c * CH + u)) * 32;
      const bool ok = k < K;
      wb[slot][u] = ld16_nt(ok ? W + (((int64_t)blockIdx.x * ks32 + (k >> 5)) * 64 + lane) * 8
                               : zpage);
#pragma unroll
      for (int i = 0; i < MR; ++i)
        xa[slot][u][i] = ld16(ok ? A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3) : zpage);
    }
  };
  f32x4 acc[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < INF; ++c) issue(c, c);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int slot = c % INF;
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[slot][u][i]), __builtin_bit_cast(bf16x8, wb[slot][u]),
            acc[i], 0, 0, 0);
    if (c + INF < NC) issue(c + INF, slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][(i * 16 + rsub + r) * 16 + csub] = acc[i][r];
  __syncthreads();
  const int o = threadIdx.x;
  if (o >= MS * 16) return;
  const int m = o >> 4;
  if (m >= M) return;
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) v += red[w][o];
  epi.apply_pf(m, col0 + (o & 15), v, 0, pf);
}

// Decode gated up-projection (1..32 packed rows in MR 16-row tiles, fragment-packed W, one K
// split): TWO gate / up pairs -- 64 packed columns, 32 features -- per
// workgroup, so F = 7680 takes 240 workgroups, one round on the CUs (the
// one-pair stream kernel needs 480: two rounds, each paying the memory
// latency once), and each wave streams its KSW k-steps in chunks of CH with
// INF chunks of weight + activation fragments in flight: chunk c + INF's
// loads go out right after chunk c's MFMAs, into the registers those just
// released (a sched_barrier pins that order; the scheduler otherwise sinks
// loads to their first use).  Cold-weight lab (tools/gemv_lab.hip): 17.2 ->
// 14.0 us on the 2F = 15360, K = 2560 shape.  Same products and fixed-order
// LDS reduction as gemm_stream_kernel; NORM as there.
template <int KSW, int CH, int INF, bool NORM, int MR>
__global__ __launch_bounds__(512) void gemm_gated_pipe_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, int M, int K,
    EpiGatedGelu epi, float neps) {
  constexpr int MS = 16 * MR, NREP = 4, NC = KSW / CH;   // MR 16-row tiles
  static_assert(KSW % CH == 0 && INF <= NC, "chunking");
  __shared__ float red[8][MS * 16 * NREP];
  __shared__ float nss[NORM ? 8 : 1][MS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = blockIdx.x;               // 64-row group: 32 features
  // epilogue operands first: thread t owns row t / 16, features
  // grp * 32 + h * 16 + t % 16 (h = 0, 1)
  const int pm = min((int)(threadIdx.x >> 4) & (MS - 1), M - 1);
  EpiGatedGelu::Pref pf[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    pf[h] = epi.prefetch2(pm, grp * 32 + h * 16 + (threadIdx.x & 15), 0);
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  const int ks32 = K >> 5;
  uint4 wb[INF][CH][NREP], xa[INF][CH][MR];
  auto issue = [&](int c, int slot) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = (wave + 8 * (c * CH + u)) * 32;
      const bool ok = k < K;
#pragma unroll
      for (int j = 0; j < NREP; ++j)   // gate halves 0 / 1, up halves 0 / 1
        wb[slot][u][j] = ld16_nt(ok ? W + (((int64_t)(grp * 4 + j) * ks32 + (k >> 5)) * 64 + lane) * 8
                                    : zpage);
#pragma unroll
      for (int i = 0; i < MR; ++i)
        xa[slot][u][i] = ld16(ok ? A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3) : zpage);
    }
  };
  f32x4 acc[MR][NREP];
  [[maybe_unused]] f32x4 dg[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    dg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int c = 0; c < INF; ++c) issue(c, c);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int slot = c % INF;
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8 af = __builtin_bit_cast(bf16x8, xa[slot][u][i]);
#pragma unroll
        for (int j = 0; j < NREP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af, __builtin_bit_cast(bf16x8, wb[slot][u][j]), acc[i][j], 0, 0, 0);
        if constexpr (NORM) dg[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, af, dg[i], 0, 0, 0);
      }
    if (c + INF < NC) issue(c + INF, slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (NORM) {
    const int r4 = lane & 3;
    if (((lane & 15) >> 2) == (lane >> 4)) {
#pragma unroll
      for (int i = 0; i < MR; ++i)
        nss[wave][i * 16 + (lane & 15)] =
            r4 == 0 ? dg[i][0] : r4 == 1 ? dg[i][1] : r4 == 2 ? dg[i][2] : dg[i][3];
    }
  }
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][((i * 16 + rsub + r) * NREP + j) * 16 + csub] = acc[i][j][r];
  __syncthreads();
  const int m = threadIdx.x >> 4, c = threadIdx.x & 15;
  if (m >= M) return;
  float rs = 1.0f;
  if constexpr (NORM) {
    const float ss = ((nss[0][m] + nss[1][m]) + (nss[2][m] + nss[3][m])) +
                     ((nss[4][m] + nss[5][m]) + (nss[6][m] + nss[7][m]));
    const float var = rbf(ss / (float)K);
    rs = rbf(1.0f / sqrtf(rbf(var + neps)));
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float v[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {   // p = 0 gate, 1 up
      const int idx = (m * NREP + 2 * p + h) * 16 + c;
      v[p] = ((red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx])) +
             ((red[4][idx] + red[5][idx]) + (red[6][idx] + red[7][idx]));
      if constexpr (NORM) v[p] *= rs;
    }
    epi.apply2_pf(m, grp * 32 + h * 16 + c, v[0], v[1], 0, pf[h]);
  }
}

// Prefill RG-LRU gates (layers.py:321-365): both BlockDiagonalLinear GEMMs
// of one head block g plus the gate chain, as a block-bound grouped GEMM.
// K = BW is short (256 at 2B), so the block engine's per-tile prologue /
// epilogue dominated it.  Here a workgroup is bound to one block g for its
// whole life: its NW = BW / 32 waves each hold 64 of the block's 2 BW packed
// output columns (32 x-gate + 32 a-gate rows of the same 32 channels, the
// PackCache interleave) for all of K in registers, loaded once, and the
// workgroup walks row tiles of 32 rows (t = blockIdx.x, + gridDim.x, ...).
// The X tile (32 x BW bf16) is register-staged one tile ahead into the other
// half of a double LDS buffer (XOR chunk swizzle on the row, so the
// A-fragment ds_read_b128 of 16 rows is conflict-free); the chain's x operand
// is read back from it.  The gate chain (seven transcendentals and fourteen
// bf16 rounding points per element) is VALU-bound and sets the kernel's time;
// each lane runs its two channels' chains as pairs (chain2: one
// v_cvt_pk_bf16_f32 per rounding point of both).  Same MFMA k order as the
// block engine (k-steps 0..BW/32-1 chained per accumulator), same rounding
// points (EpiRglruGates::chain): bit-identical.
template <int BW>
__global__ __launch_bounds__(BW * 2) void rglru_gates_stream_kernel(
    const u16* __restrict__ X, int64_t ldx, const u16* __restrict__ Wp, int M,
    EpiRglruGates epi) {
  constexpr int NW = BW / 32, KS = BW / 32, RT = 32, CPR = BW / 8;   // chunks per row
  constexpr int RF = RT / 16;                                        // row fragments
  constexpr int NT = NW * 64, LPT = RT * CPR / NT;                   // 16-B loads per thread
  constexpr int SWM = CPR >= 16 ? 15 : CPR - 1;                      // chunk swizzle mask
  static_assert(RT * CPR % NT == 0, "tile staging");
  __shared__ uint4 xs[2][RT * CPR];
  __shared__ int rs_[2][RT];
  const int g = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntiles = (M + RT - 1) / RT;
  X += (int64_t)g * BW;
  // this wave's weight fragments: tile j = 0, 1 x-gate rows (channels
  // 32 wave + 16 j + lane % 16), j = 2, 3 a-gate rows of the same channels
  const u16* wg = Wp + (int64_t)g * 2 * BW * BW;
  uint4 wf[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[j][ks] = ld16(wg + (int64_t)(64 * wave + 16 * j + (lane & 15)) * BW + ks * 32 +
                       8 * (lane >> 4));
  // one use of every weight register before the loop (a never-true test on
  // their XOR): the waitcnt pass then knows them landed, and the tile loop's
  // MFMAs wait for nothing -- otherwise it counts the previous tile's stores
  // down in front of them, every tile
  {
    uint32_t chk = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) chk ^= wf[j][ks].x ^ wf[j][ks].y ^ wf[j][ks].z ^ wf[j][ks].w;
    if (chk == 0x6b43a9b5u && M < 0) epi.a_out[0] = 0;
  }
  // per-channel operands of the chain (constant over rows)
  const int ch0 = 32 * wave + (lane & 15);
  const int e0 = g * BW + ch0;
  const f32x2 bx{bf2f(epi.bias_x[e0]), bf2f(epi.bias_x[e0 + 16])};
  const f32x2 ba{bf2f(epi.bias_a[e0]), bf2f(epi.bias_a[e0 + 16])};
  const f32x2 sp{bf2f(epi.softplus_a[e0]), bf2f(epi.softplus_a[e0 + 16])};
  // register staging of one X tile: thread slot c -> (row c / CPR, chunk c %
  // CPR), plus the tile's reset flags (thread c < RT: row c).  Branch-free:
  // rows past M (and the tile after the last) read row M - 1, so a load
  // never sits under a branch (that costs a vmcnt(0) at the join, i.e. the
  // next tile's latency on this one's first MFMA).
  uint4 st[LPT];
  int sg;
  auto fetch = [&](int t) {
    t = min(t, ntiles - 1);
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = threadIdx.x + i * NT;
      const int r = min(t * RT + c / CPR, M - 1);
      st[i] = ld16(X + (int64_t)r * ldx + (c % CPR) * 8);
    }
    sg = epi.segpos[min(t * RT + (int)(threadIdx.x % RT), M - 1)];
  };
  auto stash = [&](int b) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = threadIdx.x + i * NT;
      const int r = c / CPR, cc = c % CPR;
      xs[b][r * CPR + (cc ^ (r & SWM))] = st[i];
    }
    if (threadIdx.x < RT) rs_[b][threadIdx.x] = sg == 0;
  };
  int t = blockIdx.x;
  if (t >= ntiles) return;
  fetch(t);
  stash(0);
  int buf = 0;
  for (; t < ntiles; t += gridDim.x) {
    fetch(t + gridDim.x);                // lands while this tile computes
    __syncthreads();                     // xs[buf] written by every thread
    f32x4 acc[RF][4];
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[RF];
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        const int r = 16 * i + (lane & 15), cc = 4 * ks + (lane >> 4);
        af[i] = __builtin_bit_cast(bf16x8, xs[buf][r * CPR + (cc ^ (r & SWM))]);
      }
#pragma unroll
      for (int i = 0; i < RF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i], __builtin_bit_cast(bf16x8, wf[j][ks]), acc[i][j], 0, 0, 0);
    }
    // epilogue: lane holds rows 16 i + 4 (lane / 16) + r of channels ch0,
    // ch0 + 16 (gx in tiles 0 / 1, ga in 2 / 3): one chain pair per row;
    // rows past M recompute row M - 1 from its clamped copy and store the
    // same values there (no store under a branch)
    const u16* xl = reinterpret_cast<const u16*>(xs[buf]);
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = 16 * i + 4 * (lane >> 4) + r;
        const int64_t m = min(t * RT + rl, M - 1);
        const f32x2 xv{bf2f(xl[(rl * CPR + ((ch0 >> 3) ^ (rl & SWM))) * 8 + (ch0 & 7)]),
                       bf2f(xl[(rl * CPR + (((ch0 + 16) >> 3) ^ (rl & SWM))) * 8 + (ch0 & 7)])};
        f32x2 av, nx;
        epi.chain2(badd2(rbf2(f32x2{acc[i][0][r], acc[i][1][r]}), bx),
                   badd2(rbf2(f32x2{acc[i][2][r], acc[i][3][r]}), ba), xv, sp,
                   rs_[buf][rl] != 0, av, nx);
        u16* ap = epi.a_out + m * epi.ldo + e0;
        u16* np = epi.nx_out + m * epi.ldo + e0;
        const uint32_t ab = pk2bf(av), nb = pk2bf(nx);
        ap[0] = (u16)ab;
        ap[16] = (u16)(ab >> 16);
        np[0] = (u16)nb;
        np[16] = (u16)(nb >> 16);
      }
    buf ^= 1;
    stash(buf);                          // the other buffer: last read a tile ago
  }
}

// Prefill RG-LRU with the scan fused in (layers.py:321-375: both
// BlockDiagonalLinear GEMMs, the gate chain, then rnn_scan :145-199 and the
// `x * y` join of modules.py:652): the (a, normalised x) pair never goes to
// HBM.  A workgroup owns one sequence b and 128 channels of one head block g
// (4 waves x 32 channels) for the whole sequence, and walks it in chunks of
// RT time steps (RT = 16 at BW 256, 32 at BW 128: a 32-row chunk's
// accumulators would spill beside BW 256's weight fragments).  The chunk's X
// rows (the block's BW conv outputs) and y-gate rows come by LDS-DMA
// (glds16_asm, 16 B per lane) into a ring of NB = 3 chunk buffers, issued
// two chunks ahead: every wave issues NDMA pieces per chunk, so a counted
// vmcnt(NDMA) -- the next chunk's pieces may stay in flight -- plus a
// barrier retires chunk c before it is read, and the buffer refilled at
// chunk c (c + 2's) was last read at chunk c - 1, behind that barrier.  Each
// wave runs rglru_gates_stream_kernel's MFMAs (same fragments, same k order)
// and chain2 for its 32 channels, parks the bf16 (a, nx) pairs in its own
// LDS slab, and its lanes 0..31 then scan the chunk's 32 steps, one channel
// per lane, in rnn_scan_kernel's op order (h = a h + nx in fp32, y =
// bf16(h) [* gate]); the chunk's outputs leave as 16-B row segments.  Every
// value and rounding point is the two-kernel path's: bitwise equal to
// rglru_gates_stream_kernel + rnn_scan_kernel.  HBM traffic: x and the gate
// in, y out (6 B per element) instead of 14; the gate chain's VALU (7
// transcendentals, 14 bf16 rounding points per element) bounds it.
// Workgroup n: unit (n / 16) * 8 + n % 8, half (n / 8) % 2 -- the two
// halves of a (sequence, block) unit sit on one XCD (blocks n and n + 8) and
// share its X rows through that XCD's L2.
// LDS-DMA of 16 B per lane into M0 + 16 * lane, hidden from hipcc's waitcnt
// pass (cdna_hip_programming.md §5.7: M0 is written and restored in the same
// statement); the caller retires it with its own vmcnt wait + barrier.
CADENCE_DEV void glds16_asm(const void* gsrc, uint32_t lds_byte) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_byte) : "memory");
}
CADENCE_DEV uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)(p));
}

constexpr int kRglruScanMaxL = 4096;   // reset flags held in LDS

struct RglruScanArgs {
  const u16* x; int64_t ldx;          // conv output rows [B * L][E]
  const u16* w;                       // packed gate weights [H][2 BW][BW]
  const u16* bias_x; const u16* bias_a; const u16* softplus_a;
  const int32_t* segpos;              // [B * L]
  const float* h0;                    // [B][E] fp32 or null
  const u16* gate; int64_t ldg;       // linear_y branch rows or null
  u16* out; int64_t ldo;
  float* h_last;                      // [B][E] fp32 or null
  int B, L, E, H;
};

template <int BW, bool GATE, int RT>
__global__ __launch_bounds__(256, 2) void rglru_scan_fused_kernel(RglruScanArgs p) {
  constexpr int KS = BW / 32, CPR = BW / 8, RF = RT / 16;
  constexpr int SWM = CPR >= 16 ? 15 : CPR - 1;
  constexpr int NQ = BW / 128;                    // workgroups per block row
  constexpr int AS = 33;                          // (a, nx) slab row stride (u32)
  constexpr int NB = 3;                           // chunk buffers: DMA two chunks ahead
  __shared__ uint4 xs[NB][RT * CPR];              // X rows of a chunk (swizzled)
  __shared__ uint4 ys[NB][RT * 16];               // y-gate rows, this WG's 128 channels
  __shared__ uint32_t an[4][RT * AS];             // per wave: bf16 a | nx << 16
  __shared__ uint4 ob[4][RT * 4];                 // per wave: RT rows x 32 bf16 outputs
  __shared__ uint8_t rs_[kRglruScanMaxL];         // reset flag of every step
  const int n = blockIdx.x;
  const int unit = (n >> 4) * 8 + (n & 7), q = (n >> 3) & 1;
  if (unit >= p.B * p.H || q >= NQ) return;       // grid padding (workgroup-uniform)
  const int b = unit / p.H, g = unit % p.H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wih = 4 * q + wave;                   // wave's 32-channel group in the block
  const int L = p.L;
  const int64_t row0 = (int64_t)b * L;
  const u16* X = p.x + (int64_t)g * BW;
  const u16* wg = p.w + (int64_t)g * 2 * BW * BW;
  const int nch = (L + RT - 1) / RT;
  // chunk c's X / y-gate rows go HBM -> LDS by LDS-DMA (one wave instruction
  // = 1 KiB of lane-linear LDS), rows clamped into the sequence (branch-free:
  // every wave issues the same NDMA pieces per chunk, which the counted waits
  // below rely on), issued by inline asm: hipcc would otherwise treat every
  // later ds_read as possibly aliasing the DMA and wait vmcnt(0) in front of
  // it.  The XOR chunk swizzle is applied to the per-lane source address (an
  // involution: the fragment reads apply it again).  Wave w moves X pieces
  // w, w + 4, ... and y pieces RF w .. RF w + RF - 1 (4 rows each).
  constexpr int XRP = 1024 / (CPR * 16);          // X rows per 1 KiB piece
  constexpr int XPC = RT / XRP;                   // X pieces per chunk
  constexpr int NDMA = XPC / 4 + (GATE ? RF : 0); // DMA instructions per wave per chunk
  static_assert(XPC % 4 == 0, "X pieces per wave");
  const uint32_t xs0 = lds_addr(&xs[0][0]), ys0 = lds_addr(&ys[0][0]);
  auto dma = [&](int c, int bfd) {
    c = min(c, nch - 1);
#pragma unroll
    for (int i = 0; i < XPC / 4; ++i) {
      const int pc = wave + 4 * i;
      const int r = pc * XRP + lane / CPR, slot = lane % CPR;
      const int t = min(c * RT + r, L - 1);
      glds16_asm(X + (row0 + t) * p.ldx + 8 * (slot ^ (r & SWM)),
                 xs0 + (uint32_t)(bfd * RT * CPR + pc * 64) * 16);
    }
    if constexpr (GATE) {
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        const int pc = RF * wave + i;
        const int r = pc * 4 + lane / 16;
        const int t = min(c * RT + r, L - 1);
        glds16_asm(p.gate + (row0 + t) * p.ldg + g * BW + 128 * q + 8 * (lane % 16),
                   ys0 + (uint32_t)(bfd * RT * 16 + pc * 64) * 16);
      }
    }
  };
  // the first two chunks' DMA flies under the weight loads and the flags
  dma(0, 0);
  dma(1, 1);
  uint4 wf[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[j][ks] = ld16(wg + (int64_t)(64 * wih + 16 * j + (lane & 15)) * BW + ks * 32 +
                       8 * (lane >> 4));
  // reset flags of the whole sequence (positions read once, coalesced)
  for (int t = threadIdx.x; t < L; t += 256) rs_[t] = p.segpos[row0 + t] == 0;
  const int ch0 = 32 * wih + (lane & 15);         // channel in the block
  const int e0 = g * BW + ch0;
  const f32x2 bx{bf2f(p.bias_x[e0]), bf2f(p.bias_x[e0 + 16])};
  const f32x2 ba{bf2f(p.bias_a[e0]), bf2f(p.bias_a[e0 + 16])};
  const f32x2 sp{bf2f(p.softplus_a[e0]), bf2f(p.softplus_a[e0 + 16])};
  float h = 0.0f;
  const int es = g * BW + 32 * wih + (lane & 31);  // the channel this lane scans
  if (p.h0) h = p.h0[(int64_t)b * p.E + es];
  // every register load above has landed before the loop (one use of each
  // weight register: rglru_gates_stream_kernel's note), so the only vector
  // memory operations the loop waits for are its own, counted below
  {
    uint32_t chk = __float_as_uint(h) ^ __float_as_uint(bx.x + ba.y + sp.x);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) chk ^= wf[j][ks].x ^ wf[j][ks].y ^ wf[j][ks].z ^ wf[j][ks].w;
    if (chk == 0x6b43a9b5u && L < 0) p.out[0] = 0;
  }
  const EpiRglruGates ep{};
  uint32_t* al = an[wave];
  u16* ol = reinterpret_cast<u16*>(ob[wave]);
  int bf = 0;
  for (int c = 0; c < nch; ++c) {
    // chunk c's DMA (issued two chunks ago) retired: only the NDMA younger
    // pieces of chunk c + 1 stay in flight; then every wave's, by the barrier
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NDMA) : "memory");
    __syncthreads();
    f32x4 acc[RF][4];
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[RF];
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        const int r = 16 * i + (lane & 15), cc = 4 * ks + (lane >> 4);
        af[i] = __builtin_bit_cast(bf16x8, xs[bf][r * CPR + (cc ^ (r & SWM))]);
      }
#pragma unroll
      for (int i = 0; i < RF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i], __builtin_bit_cast(bf16x8, wf[j][ks]), acc[i][j], 0, 0, 0);
    }
    // gate chain of rows 16 i + 4 (lane / 16) + r, channels ch0 / ch0 + 16
    // (rows past the sequence: the clamped last row's values, never scanned)
    const u16* xl = reinterpret_cast<const u16*>(xs[bf]);
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = 16 * i + 4 * (lane >> 4) + r;
        const f32x2 xv{bf2f(xl[(rl * CPR + ((ch0 >> 3) ^ (rl & SWM))) * 8 + (ch0 & 7)]),
                       bf2f(xl[(rl * CPR + (((ch0 + 16) >> 3) ^ (rl & SWM))) * 8 + (ch0 & 7)])};
        f32x2 av, nx;
        ep.chain2(badd2(rbf2(f32x2{acc[i][0][r], acc[i][1][r]}), bx),
                  badd2(rbf2(f32x2{acc[i][2][r], acc[i][3][r]}), ba), xv, sp,
                  rs_[min(c * RT + rl, L - 1)] != 0, av, nx);
        const uint32_t ab = pk2bf(av), nb = pk2bf(nx);
        al[rl * AS + (lane & 15)] = (ab & 0xffffu) | (nb << 16);
        al[rl * AS + (lane & 15) + 16] = (ab >> 16) | (nb & 0xffff0000u);
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // the scan: lane c < 32 carries channel 32 wih + c through the chunk
    // (a full chunk unrolled, so its LDS reads issue ahead of the chain)
    const int nr = min(RT, L - c * RT);
    if (lane < 32) {
      const u16* yl = reinterpret_cast<const u16*>(ys[bf]) + 32 * wave + lane;
      auto step = [&](int r) {
        const uint32_t v = al[r * AS + lane];
        h = add_rn(mul_rn(__uint_as_float(v << 16), h), __uint_as_float(v & 0xffff0000u));
        float y = rbf(h);
        if constexpr (GATE) y = bmul(y, bf2f(yl[r * 128]));
        ol[r * 32 + lane] = f2bf(y);
      };
      if (nr == RT) {
#pragma unroll
        for (int r = 0; r < RT; ++r) step(r);
      } else {
        for (int r = 0; r < nr; ++r) step(r);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // RT rows x 32 channels out: lane l stores 16 B of rows l / 4 (+ 16)
#pragma unroll
    for (int k = 0; k < RF; ++k) {
      const int r = 16 * k + (lane >> 2), cc = lane & 3;
      if (r < nr)
        st16(p.out + (row0 + c * RT + r) * p.ldo + g * BW + 32 * wih + 8 * cc, ob[wave][r * 4 + cc]);
    }
    // chunk c + 2 into the buffers chunk c - 1 used (every wave passed this
    // chunk's barrier after its last read of them); always issued (clamped
    // past the end) so the counted wait above sees NDMA per chunk
    dma(c + 2, bf == 0 ? 2 : bf - 1);
    bf = bf == NB - 1 ? 0 : bf + 1;
  }
  // no LDS-DMA may still land once the workgroup's LDS is handed on
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p.h_last && lane < 32) p.h_last[(int64_t)b * p.E + es] = h;
}

// torch.argmax order: NaN beats every number, ties (and NaN vs NaN) go to
// the lowest index -- a NaN row still yields an index inside the vocabulary
CADENCE_DEV bool argmax_better(float ov, int oi, float v, int i) {
  const bool on = ov != ov, n = v != v;
  if (on != n) return on;
  if (!on && ov != v) return ov > v;
  return oi < i;
}

// ---------------------------------------------------------- skinny engine

// One block: 64 output columns x MS rows over one K split; 4 waves split the
// K range round-robin in 32-deep steps and are summed through LDS.
template <int MS, bool ARGMAX = false>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ W,
    int64_t ldw, int M, int N, int K, int klen, float* __restrict__ part,
    int64_t a_goff, int64_t w_goff, int packed, float cap = 0.0f,
    u16* __restrict__ logits = nullptr, float* __restrict__ bval = nullptr,
    int* __restrict__ bidx = nullptr) {
  // ARGMAX (one K split): the logits epilogue runs here -- rounding,
  // soft-cap, optional bf16 logits, and the (max, lowest index) of this
  // block's 64 columns per row -- instead of fp32 partials + a reduce launch
  constexpr int MR = MS / 16;
  constexpr int UNROLL = 2;
  __shared__ float red[4][MS * 64];
  const int g = blockIdx.z;
  A += g * a_goff;
  W += g * w_goff;
  const int n0 = blockIdx.x * 64;
  const int kbeg = blockIdx.y * klen;
  const int kend = min(K, kbeg + klen);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int koff = 8 * (lane >> 4);

  f32x4 acc[MR][4];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint4 zero = make_uint4(0, 0, 0, 0);
  for (int kk = kbeg + 32 * wave; kk < kend; kk += 32 * 4 * UNROLL) {
    uint4 wb[UNROLL][4];
    uint4 xa[UNROLL][MR];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = kk + u * 128;
      const bool ok = k < kend;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wb[u][j] = !ok ? zero
                   : packed ? ld16_nt(W + (((int64_t)((n0 >> 4) + j) * (K >> 5) + (k >> 5)) * 64 + lane) * 8)
                            : ld16(W + (int64_t)(n0 + j * 16 + (lane & 15)) * ldw + k + koff);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const int m = i * 16 + (lane & 15);
        if (lda == 0)   // packed rows, mt == MR
          xa[u][i] = ok ? ld16(A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3)) : zero;
        else
          xa[u][i] = (ok && m < M) ? ld16(A + (int64_t)m * lda + k + koff) : zero;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, xa[u][i]),
              __builtin_bit_cast(bf16x8, wb[u][j]), acc[i][j], 0, 0, 0);
  }
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][(i * 16 + rsub + r) * 64 + j * 16 + csub] = acc[i][j][r];
  __syncthreads();
  if constexpr (ARGMAX) {
    // 64 consecutive idx = one row, one wave: lane = column
    for (int idx = tid; idx < MS * 64; idx += 256) {
      const int m = idx / 64, n = idx % 64;
      if (m >= M) continue;   // wave-uniform
      float l = rbf((red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx]));
      if (cap > 0.0f) l = softcap(l, cap);
      if (logits) logits[(int64_t)m * N + n0 + n] = f2bf(l);
      float v = l;
      int ix = n0 + n;
      for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(v, off, 64);
        const int oi = __shfl_xor(ix, off, 64);
        if (argmax_better(ov, oi, v, ix)) { v = ov; ix = oi; }
      }
      if (n == 0) {
        bval[(int64_t)m * gridDim.x + blockIdx.x] = v;
        bidx[(int64_t)m * gridDim.x + blockIdx.x] = ix;
      }
    }
    return;
  }
  float* dst = part + ((int64_t)blockIdx.y * gridDim.z + g) * (int64_t)M * N;
  for (int idx = tid; idx < MS * 64; idx += 256) {
    const int m = idx / 64, n = idx % 64;
    if (m < M) {
      const float s = (red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx]);
      dst[(int64_t)m * N + n0 + n] = s;
    }
  }
}

// Sums the split-K slabs in split order and applies the epilogue.
template <class Epi>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(
    const float* __restrict__ part, int splits, int groups, int M, int N,
    Epi epi) {
  const int g = blockIdx.y;
  const int64_t slab = (int64_t)M * N;
  if constexpr (Epi::kPaired) {
    const int half = N / 2;
    for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < (int64_t)M * half;
         idx += (int64_t)gridDim.x * 256) {
      const int m = idx / half, oc = idx % half;
      const int c0 = (oc / 32) * 64 + (oc % 32), c1 = c0 + 32;
      float v0 = 0.f, v1 = 0.f;
      for (int s = 0; s < splits; ++s) {
        const float* p = part + ((int64_t)s * groups + g) * slab + (int64_t)m * N;
        v0 += p[c0];
        v1 += p[c1];
      }
      epi.apply2(m, oc, v0, v1, g);
    }
  } else {
    for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < (int64_t)M * N;
         idx += (int64_t)gridDim.x * 256) {
      const int m = idx / N, n = idx % N;
      float v = 0.f;
      for (int s = 0; s < splits; ++s)
        v += part[((int64_t)s * groups + g) * slab + (int64_t)m * N + n];
      epi.apply(m, n, v, g);
    }
  }
}


// Logits reduce: one block = 256 vocabulary columns of one row.  Applies the
// soft-cap chain, optionally stores bf16 logits, and emits the block's
// (max, lowest index) pair.
__global__ __launch_bounds__(256) void logits_reduce_kernel(
    const float* __restrict__ part, int splits, int M, int V, float cap,
    u16* __restrict__ logits, float* __restrict__ bval, int* __restrict__ bidx) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int m = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  if (n < V) {
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += part[((int64_t)s * M + m) * V + n];
    float l = rbf(acc);
    if (cap > 0.0f) l = softcap(l, cap);
    if (logits) logits[(int64_t)m * V + n] = f2bf(l);
    v = l;
    idx = n;
  }
  // wave argmax (ties -> lowest index)
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, 64);
    const int oi = __shfl_xor(idx, off, 64);
    if (argmax_better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[wave] = v; si[wave] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (argmax_better(sv[w], si[w], v, idx)) { v = sv[w]; idx = si[w]; }
    bval[(int64_t)m * gridDim.x + blockIdx.x] = v;
    bidx[(int64_t)m * gridDim.x + blockIdx.x] = idx;
  }
}

__global__ __launch_bounds__(256) void argmax_final_kernel(
    const float* __restrict__ bval, const int* __restrict__ bidx, int nblk,
    int32_t* __restrict__ out) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int m = blockIdx.x;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  // 16 (value, index) pairs per thread per pass, every load issued before
  // the first compare; indices past nblk re-read the last pair (a duplicate
  // never changes the argmax)
  constexpr int PER = 16;
  for (int base = 0; base < nblk; base += 256 * PER) {
    float ov[PER];
    int oi[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t i = (int64_t)m * nblk + min(base + u * 256 + (int)threadIdx.x, nblk - 1);
      ov[u] = bval[i];
      oi[u] = bidx[i];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u)
      if (argmax_better(ov[u], oi[u], v, idx)) { v = ov[u]; idx = oi[u]; }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, 64);
    const int oi = __shfl_xor(idx, off, 64);
    if (argmax_better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[wave] = v; si[wave] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (argmax_better(sv[w], si[w], v, idx)) { v = sv[w]; idx = si[w]; }
    out[m] = idx;
  }
}

// The decode step's tail (cadence_logits_argmax_tail): argmax_final_kernel's
// reduction for row m, then decode_advance_kernel's bookkeeping for that row
// and embed_kernel's gather of the token written, into the next replay's
// input rows (row-major and packed).  *step is read by every workgroup before
// it arrives on the counter; the last arrival advances it and ANDs the done
// flags (written through to L2 before each arrival: the split-K hand-off of
// gemm_stream_kernel, MI355X_MICROARCH.md "inter-workgroup visibility").
__global__ __launch_bounds__(256) void argmax_tail_kernel(
    const float* __restrict__ bval, const int* __restrict__ bidx, int nblk,
    int32_t* __restrict__ next_out, CadenceDecodeTail a, int M, int D) {
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ int tok;
  const int m = blockIdx.x;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  constexpr int PER = 16;
  for (int base = 0; base < nblk; base += 256 * PER) {
    float ov[PER];
    int oi[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t i = (int64_t)m * nblk + min(base + u * 256 + (int)threadIdx.x, nblk - 1);
      ov[u] = bval[i];
      oi[u] = bidx[i];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u)
      if (argmax_better(ov[u], oi[u], v, idx)) { v = ov[u]; idx = oi[u]; }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, 64);
    const int oi = __shfl_xor(idx, off, 64);
    if (argmax_better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[wave] = v; si[wave] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (argmax_better(sv[w], si[w], v, idx)) { v = sv[w]; idx = si[w]; }
    next_out[m] = idx;
    // decode_advance_kernel for row m
    const int s = *a.step;
    int32_t t = idx;
    if (a.done) {
      const int d = a.done[m];
      if (d) t = a.pad_id;
      __hip_atomic_store(a.done + m, d | (t == a.eos_id && s >= a.eos_from), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    a.tokens_out[(int64_t)m * a.ld_out + s] = t;
    a.positions[m] += 1;
    if (a.cur_out) a.cur_out[m] = t;
    tok = t;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int n = __hip_atomic_fetch_add(a.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n == M - 1) {
      int all = 1;
      if (a.done) {
        for (int b = 0; b < M; ++b)
          all &= __hip_atomic_load(a.done + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.done[M] = all;
      }
      *a.step = s + 1;
      __hip_atomic_store(a.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  // embed_kernel for the token written (the next replay's input row)
  const int64_t t = tok;
  const u16* src = static_cast<const u16*>(a.embed) + (t >= 0 && t < a.vocab ? t : 0) * D;
  u16* xo = static_cast<u16*>(a.x_out) + (int64_t)m * a.ldx_out;
  u16* po = static_cast<u16*>(a.packed_out);
  const int mt = (M + 15) / 16;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    uint4 w = ld16(src + c);
    if (a.scale != 1.0f) {
      float f[8];
      unpack8(w, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = bmul(f[i], a.scale);
      w = pack8(f);
    }
    st16(xo + c, w);
    st16(po + xoff(m, c, 0, mt), w);
  }
}

constexpr int kSkinnyMaxM = 64;

// Split-K finish of a residual GEMM that feeds an RMSNorm (decode): one
// workgroup per output row.  out[m, :] = EpiLinear(sum_s part[s][m][:]) (bias,
// rounding, + resid), then nout[m, :] = RMSNorm(out[m, :]) with the rounding
// chain of rmsnorm_kernel (layers.py:73-78).  RC 8-column chunks per thread
// stay in registers between the two passes.
template <int RC, int S>
__global__ __launch_bounds__(512) void reduce_rmsnorm_kernel(
    const float* __restrict__ part, int M, int N, EpiLinear epi,
    const u16* __restrict__ scale, float eps, u16* __restrict__ nout,
    int64_t ldn) {
  __shared__ float wsum[8];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int64_t orow = epi.map(m);
  // issue every load of the row first (S splits x RC chunks, resid, scale)
  // (bias / residual chunks are read from the zero page when absent: a load
  // under a branch, or one per element in the epilogue, would serialise a
  // memory round trip each)
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + (tid & 63));
  float4 pa[RC][S][2];
  uint4 rq[RC], sq[RC], bq[RC];
#pragma unroll
  for (int c = 0; c < RC; ++c) {
    const int n0 = min((tid + c * 512) * 8, N - 8);
#pragma unroll
    for (int sp = 0; sp < S; ++sp) {
      const float4* src = reinterpret_cast<const float4*>(
          part + ((int64_t)sp * M + m) * N + n0);
      pa[c][sp][0] = src[0];
      pa[c][sp][1] = src[1];
    }
    rq[c] = ld16(epi.resid ? epi.resid + orow * epi.ldr + n0 : zpage);
    bq[c] = ld16(epi.bias ? epi.bias + n0 : zpage);
    sq[c] = ld16(scale + n0);
  }
  float o[RC][8];
  float ss = 0.0f;
#pragma unroll
  for (int c = 0; c < RC; ++c) {
    const int n0 = (tid + c * 512) * 8;
    if (n0 < N) {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < S; ++sp) {
        const float4 a = pa[c][sp][0], b = pa[c][sp][1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
      float r[8], bb[8];
      unpack8(rq[c], r);
      unpack8(bq[c], bb);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // EpiLinear::value with the bias chunk preloaded
        float y = v[i];
        if (epi.bias) y = add_rn(y, bb[i]);
        y = epi.activate(rbf(y));
        if (epi.resid) y = badd(y, r[i]);
        o[c][i] = y;
        ss += rbf(y * y);
      }
      st16(epi.out + orow * epi.ldo + n0, pack8(o[c]));
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) wsum[tid >> 6] = ss;
  __syncthreads();
  ss = ((wsum[0] + wsum[1]) + (wsum[2] + wsum[3])) +
       ((wsum[4] + wsum[5]) + (wsum[6] + wsum[7]));
  const float var = rbf(ss / (float)N);
  const float rs = rbf(1.0f / sqrtf(rbf(var + eps)));
#pragma unroll
  for (int c = 0; c < RC; ++c) {
    const int n0 = (tid + c * 512) * 8;
    if (n0 < N) {
      float sc[8];
      unpack8(sq[c], sc);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[c][i] = bmul(bmul(o[c][i], rs), badd(sc[i], 1.0f));
      st16(nout + xoff((int)orow, n0, ldn, (M + 15) >> 4), pack8(o[c]));
    }
  }
}

// Weight-streaming plan for M <= 32: k-steps per wave (KSW) and K splits so
// that one split is <= 8 * KSW steps.
int stream_plan(int64_t M, int64_t K, int* ksw, int* splits) {
  if (M > 32 || K % 32) return 0;
  const int64_t ks = K / 32;
  if (ks <= 8) { *ksw = 1; *splits = 1; }
  else if (ks <= 16) { *ksw = 2; *splits = 1; }
  else if (ks <= 32) { *ksw = 4; *splits = 1; }
  else { *ksw = 10; *splits = (int)((ks + 79) / 80); }
  return 1;
}

// Decode residual GEMM feeding an RMSNorm: the split-K plan whose row-owned
// reduce kernel also does the norm.  K > 2560 is split anyway; a one-split
// K (the 2560-wide output projections) is split in two as well: 32
// columns x one K half per workgroup halve the activation bytes each
// workgroup pulls, and the reduce kernel replaces the norm launch (decode
// step -50 us).
int rmsnorm_stream_plan(int64_t M, int64_t K, int* ksw, int* splits) {
  if (!stream_plan(M, K, ksw, splits)) return 0;
  if (*splits >= 2 && *splits <= 4) return 1;
  if (*splits == 1 && *ksw == 10 && K == 2560) {
    *ksw = 5;
    *splits = 2;
    return 1;
  }
  return 0;
}

int skinny_splits(int64_t N, int64_t K, int64_t groups) {
  const int64_t tiles = (N / 64) * groups;
  const int64_t ksteps = K / 32;
  // aim for ~512 blocks, keep >= 8 k-steps (2 per wave) per split
  int64_t splits = (512 + tiles - 1) / tiles;
  splits = splits < 1 ? 1 : splits;
  const int64_t maxs = ksteps / 8 > 0 ? ksteps / 8 : 1;
  if (splits > maxs) splits = maxs;
  return (int)splits;
}

int64_t skinny_klen(int64_t K, int splits) {
  int64_t klen = (K + splits - 1) / splits;
  klen = (klen + 31) / 32 * 32;
  return klen;
}

// Column tiles per stream-engine workgroup: two when that still leaves >= 150
// workgroups (cold-weight sweep, tools/gemv_lab.py: xy 12.7 -> 8.9 us, down
// 18.6 -> 13).
template <class Epi>
int stream_ntw(int64_t N, int ksw, int splits, int64_t groups) {
  return (!Epi::kPaired && (ksw == 10 || ksw == 5) && N % 32 == 0 &&
          (N / 32) * splits * groups >= 150) ? 2 : 1;
}

template <class Epi, bool NORM>
void launch_stream_t(const u16* A, int64_t lda, const u16* W, int64_t ldw,
                     int64_t M, int64_t N, int64_t K, int64_t groups,
                     int64_t a_goff, int64_t w_goff, const Epi& epi, int ksw,
                     int splits, float* parts, int packed, hipStream_t st,
                     int32_t* counters, float neps) {
  const int ntw = stream_ntw<Epi>(N, ksw, splits, groups);
  const unsigned nblk = (unsigned)(Epi::kPaired ? N / 32 : N / 16 / ntw);
  const int64_t ks = K / 32;
  const int klen = (int)((ks + splits - 1) / splits) * 32;
  dim3 grid(nblk, (unsigned)splits, (unsigned)groups);
#define CADENCE_STREAM(MS_, KSW_, NTW_)                                               \
  hipLaunchKernelGGL((gemm_stream_kernel<MS_, KSW_, NTW_, Epi, NORM>), grid, dim3(512), \
                     0, st, A, lda, W, ldw, (int)M, (int)N, (int)K, klen, a_goff,      \
                     w_goff, parts, epi, packed, counters, neps)
  if (M <= 16) {
    if (ksw == 1) CADENCE_STREAM(16, 1, 1);
    else if (ksw == 2) CADENCE_STREAM(16, 2, 1);
    else if (ksw == 4) CADENCE_STREAM(16, 4, 1);
    else if (ksw == 5) {
      if constexpr (std::is_same_v<Epi, EpiLinear> || std::is_same_v<Epi, EpiResidRows>) {
        if (ntw == 2) CADENCE_STREAM(16, 5, 2);
        else CADENCE_STREAM(16, 5, 1);   // N too narrow for 2 tiles per block
      }
    }
    else if (ntw == 2) { if constexpr (!Epi::kPaired) CADENCE_STREAM(16, 10, 2); }
    else CADENCE_STREAM(16, 10, 1);
  } else {
    if (ksw == 1) CADENCE_STREAM(32, 1, 1);
    else if (ksw == 2) CADENCE_STREAM(32, 2, 1);
    else if (ksw == 4) CADENCE_STREAM(32, 4, 1);
    else if (ksw == 5) {
      if constexpr (std::is_same_v<Epi, EpiLinear> || std::is_same_v<Epi, EpiResidRows>) {
        if (ntw == 2) CADENCE_STREAM(32, 5, 2);
        else CADENCE_STREAM(32, 5, 1);   // N too narrow for 2 tiles per block
      }
    }
    else if (ntw == 2) { if constexpr (!Epi::kPaired) CADENCE_STREAM(32, 10, 2); }
    else CADENCE_STREAM(32, 10, 1);
  }
#undef CADENCE_STREAM
}

// Stream engine launch: `splits` K splits (raw fp32 partials to `parts`
// [split][group][M][N] when > 1: reduced by a second kernel, or in-kernel
// when `counters` is given, else the epilogue runs in-kernel).  `norm`: A is
// unnormalised packed rows and W carries the norm scale; the rows' rsqrt is
// applied in-kernel (gemm_stream_kernel NORM; one split only).
template <class Epi>
void launch_stream(const u16* A, int64_t lda, const u16* W, int64_t ldw,
                   int64_t M, int64_t N, int64_t K, int64_t groups,
                   int64_t a_goff, int64_t w_goff, const Epi& epi, int ksw,
                   int splits, float* parts, int packed, hipStream_t st,
                   int32_t* counters = nullptr, int norm = 0,
                   float neps = 0.0f) {
  if constexpr (EpiNormIn<Epi>::value) {
    if (norm) {
      launch_stream_t<Epi, true>(A, lda, W, ldw, M, N, K, groups, a_goff, w_goff, epi,
                                 ksw, splits, parts, packed, st, counters, neps);
      return;
    }
  }
  launch_stream_t<Epi, false>(A, lda, W, ldw, M, N, K, groups, a_goff, w_goff, epi, ksw,
                              splits, parts, packed, st, counters, 0.0f);
}

// lab A/B switch of the prefill engines, a bit mask: bit 0 = the 4-wave
// gemm_w4_kernel on its plans, bit 1 = rglru_gates_stream_kernel, bit 2 =
// the residual-prefetching linear epilogue EpiLinearA<4>, bit 3 = the
// streaming ViT attention kernel vit_flash_attn_kernel for every tower size
// (0 = the 8-wave block engine with the plain epilogues for everything, and
// the round-3 ViT attention kernels)
int g_engine = 15;

// The 4-wave engine runs the wide long-K GEMMs (the gated MLP up-projection,
// N = 2F = 15360, K = 2560) on 224 / 256-row tile plans.  Measured A/B in
// the bench pipeline (tools/bench_engine_ab.sh, profiles/r03f_*): gated
// 717 vs 734 us; the N = 2560..5120 projections ran 10 % SLOWER on it there
// (288 vs 263 us) although 4 % faster in isolation with warm operands: one
// wave per SIMD and one K-tile of DMA lookahead expose the cold weight
// panels' HBM latency that the 8-wave engine's two waves per SIMD and 1.5
// K-tiles in flight hide.  A 5-slot 32-deep ring with 1.5 K-tiles of
// lookahead was slower still (barrier per 32-deep step; profiles/r03g_*).
// Short K keeps the 8-wave engine, whose 8 waves also finish element-wise
// epilogues twice as fast (fc1's erf-GELU at K = 1024: 0.87x on 4 waves).
bool use_w4(int64_t N, int64_t K, int rows) {
  // lab A/B: CADENCE_W4_MIN_N lowers the N threshold
  static const int64_t min_n = [] {
    const char* e = getenv("CADENCE_W4_MIN_N");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v > 0 ? v : 8192);
  }();
  return (g_engine & 1) && K >= 2048 && N >= min_n && (rows == 224 || rows == 256);
}

// Tile height of the 4-wave engine: 256 rows up to kW4TallMaxM rows of A,
// 224 beyond (its round-count model picks 256 at C2's M = 65536 and 224 at
// the bench's 10208, the opposite of what runs faster).  Measured at the gated MLP shape
// (N = 15360, K = 2560; profiles/r05k_w4_tile_rows.log): M = 10208 (the
// bench) 642 vs 650-652 us in the bench pipeline (734.9-735.8 vs 739.0-739.9
// ms per step) and 687-691 vs 703 us isolated, M = 20448 (C4) 1343-1350 vs
// 1381-1388 us, but M = 65536 (C2) 4320-4334 vs 4209-4213 us for 224 rows.
// CADENCE_W4_ROWS = 224 / 256 forces one (lab A/B).
constexpr int64_t kW4TallMaxM = 32768;
int w4_tile_rows(int64_t M, int64_t N) {
  static const int forced = [] {
    const char* e = getenv("CADENCE_W4_ROWS");
    const int r = e ? atoi(e) : 0;
    return (r == 224 || r == 256) ? r : 0;
  }();
  if (forced) return forced;
  if (N < 8192) return 224;   // the narrower projections (lab: CADENCE_W4_MIN_N)
  return M <= kW4TallMaxM ? 256 : 224;
}

// Prefill engine plan for M > kSkinnyMaxM: 0 = 2-buffer 256-row kernel,
// 160 / 192 / 224 / 256 = 8-phase kernel with that tile height.
//  * 8-phase when K splits into pairs of 64-deep tiles (an A/B of the
//    guide's two-barrier phase -- reads, barrier, lgkmcnt(0), MFMAs,
//    barrier -- ran 1-5 % slower on every prefill shape);
//  * tile height 256 or 224 rows, whichever needs fewer (rounds x rows) on
//    the CUs (M = 10208 = 32 x 319: 460 tiles of 224 in 2 rounds beat 400 of
//    256 in 2 rounds);
//  * 192 or 160 rows where that saves > 5 % of rounds x (MR + 2), MR =
//    rows / 32 (a tile's time: its MR MFMA row blocks plus ~2 blocks' worth
//    of fixed prologue / DMA / epilogue) -- the narrow ViT GEMMs (N = 1024 /
//    1152: 4-5 column panels, 152-185 tiles of 224 rows for 256 CUs) and the
//    ViT MLP up-projections (608 tiles: 3 rounds of 224, or 3 of 192).
int big_tile_rows(int64_t M, int64_t N, int64_t K, int64_t groups) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    return n;
  }();
  if (K % (2 * BK) != 0) return 0;
  // lab A/B: CADENCE_TILE_ROWS = 160 / 192 / 224 / 256 forces the block
  // engine's tile height for every shape
  static const int forced = [] {
    const char* e = getenv("CADENCE_TILE_ROWS");
    const int r = e ? atoi(e) : 0;
    return (r == 160 || r == 192 || r == 224 || r == 256) ? r : 0;
  }();
  if (forced) return forced;
  const int64_t ntn = (N + 255) / 256;
  auto rounds = [&](int64_t bm) {
    const int64_t t = ((M + bm - 1) / bm) * ntn * groups;
    return (t + cus - 1) / cus;
  };
  int best = rounds(224) * 224 < rounds(256) * 256 ? 224 : 256;
  double cost = (double)rounds(best) * (best / 32 + 2);
  for (int mr = 6; mr >= 5; --mr) {
    const double c = (double)rounds(32 * mr) * (mr + 2);
    if (c < 0.95 * cost) {
      best = 32 * mr;
      cost = c;
    }
  }
  return best;
}

// K splits of the prefill engine when its output tiles would leave most CUs
// idle (one image / one prompt: M = 261..319 rows give 2 x N/256 tiles):
// the largest S <= 8 with tiles x S <= CUs whose split length is a whole
// number of >= 2 K-tile pairs (the 8-phase loop's unit, 128).  Ungrouped
// launches only; 1 = no split.
int big_splits(int64_t M, int64_t N, int64_t K, int64_t groups, int rows) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    return n;
  }();
  if (groups != 1 || rows == 0) return 1;
  const int64_t tiles = ((M + rows - 1) / rows) * ((N + 255) / 256);
  if (tiles * 2 > cus) return 1;
  for (int sp = 8; sp >= 2; --sp)
    if (tiles * sp <= cus && K % (128 * sp) == 0 && K / sp >= 256) return sp;
  return 1;
}

template <class Epi>
int launch_gemm(const u16* A, int64_t lda, const u16* W, int64_t ldw, int64_t M,
                int64_t N, int64_t K, int64_t groups, int64_t a_goff,
                int64_t w_goff, const Epi& epi, void* ws, int64_t ws_bytes,
                hipStream_t st, int norm = 0, float neps = 0.0f) {
  if (M <= 0) return 0;
  // norm (normalise-on-load) needs packed rows and one weight-stream split
  if (norm) {
    int ksw = 0, ss = 0;
    if (lda != 0 || !stream_plan(M, K, &ksw, &ss) || ss != 1)
      return (int)hipErrorInvalidValue;
  }
  // ldw == 0: W is fragment-packed (see cadence_kernels.h), decode engines only
  const int packed = ldw == 0 ? 1 : 0;
  if (packed && (M > kSkinnyMaxM || N % 16 || K % 32)) return (int)hipErrorInvalidValue;
  if (lda == 0 && (M > 32 || K % 32)) return (int)hipErrorInvalidValue;   // packed rows
  if (M > kSkinnyMaxM) {
    if (N % 64 || K % BK) return (int)hipErrorInvalidValue;
    const int rows = big_tile_rows(M, N, K, groups);
    const bool p8 = rows != 0;
    const int64_t bm = p8 ? rows : 256;
    const int64_t tiles = ((M + bm - 1) / bm) * ((N + 255) / 256);
    const int sk = big_splits(M, N, K, groups, rows);
    if (sk > 1 && ws && ws_bytes >= (int64_t)sk * M * N * 4) {
      // split-K: split s = group s (A and W advance klen columns per
      // group), raw fp32 partials, then the epilogue on the split-order sums
      const int64_t klen = K / sk;
      float* parts = static_cast<float*>(ws);
      const EpiPartial ep{parts, M, N};
      const dim3 sgrid((unsigned)tiles, (unsigned)sk);
#define CADENCE_BIG_PART(MR_)                                                              \
  hipLaunchKernelGGL((gemm_big_kernel<EpiPartial, 1, MR_>), sgrid, dim3(512), 0, st, A, lda, \
                     W, ldw, (int)M, (int)N, (int)klen, klen, klen, ep)
      switch (rows) {
        case 160: CADENCE_BIG_PART(5); break;
        case 192: CADENCE_BIG_PART(6); break;
        case 224: CADENCE_BIG_PART(7); break;
        default: CADENCE_BIG_PART(8); break;
      }
#undef CADENCE_BIG_PART
      int64_t outs = M * N;
      int rblocks = (int)((outs + 255) / 256);
      if (rblocks > 4096) rblocks = 4096;
      hipLaunchKernelGGL((splitk_reduce_kernel<Epi>), dim3(rblocks, 1), dim3(256), 0, st,
                         parts, sk, 1, (int)M, (int)N, epi);
      return (int)hipGetLastError();
    }
    if (use_w4(N, K, rows)) {
      const int wrows = w4_tile_rows(M, N);
      const dim3 wgrid((unsigned)(((M + wrows - 1) / wrows) * ((N + 255) / 256)),
                       (unsigned)groups);
      if constexpr (std::is_same_v<Epi, EpiLinear>) {
#define CADENCE_W4_ACT(ACT_)                                                              \
  if (wrows == 224)                                                                       \
    hipLaunchKernelGGL((gemm_w4_kernel<EpiLinearA<ACT_>, 7>), wgrid, dim3(256), 0, st, A,   \
                       lda, W, ldw, (int)M, (int)N, (int)K, a_goff, w_goff,               \
                       EpiLinearA<ACT_>{epi});                                            \
  else                                                                                    \
    hipLaunchKernelGGL((gemm_w4_kernel<EpiLinearA<ACT_>, 8>), wgrid, dim3(256), 0, st, A,   \
                       lda, W, ldw, (int)M, (int)N, (int)K, a_goff, w_goff,               \
                       EpiLinearA<ACT_>{epi})
        if (epi.act == 0 && epi.resid && (g_engine & 4)) {
          CADENCE_W4_ACT(4);
        } else {
          switch (epi.act) {
            case 0: CADENCE_W4_ACT(0); break;
            case 1: CADENCE_W4_ACT(1); break;
            case 2: CADENCE_W4_ACT(2); break;
            case 3: CADENCE_W4_ACT(3); break;
            default: return (int)hipErrorInvalidValue;
          }
        }
#undef CADENCE_W4_ACT
      } else if (wrows == 224) {
        hipLaunchKernelGGL((gemm_w4_kernel<Epi, 7>), wgrid, dim3(256), 0, st, A, lda, W, ldw,
                           (int)M, (int)N, (int)K, a_goff, w_goff, epi);
      } else {
        hipLaunchKernelGGL((gemm_w4_kernel<Epi, 8>), wgrid, dim3(256), 0, st, A, lda, W, ldw,
                           (int)M, (int)N, (int)K, a_goff, w_goff, epi);
      }
      return (int)hipGetLastError();
    }
    dim3 grid((unsigned)tiles, (unsigned)groups);
    if constexpr (std::is_same_v<Epi, EpiLinear>) {
#define CADENCE_BIG_ACT(ACT_)                                                          \
  if (rows == 160) hipLaunchKernelGGL((gemm_big_kernel<EpiLinearA<ACT_>, 1, 5>), grid, \
                             dim3(512), 0, st, A, lda, W, ldw, (int)M, (int)N, (int)K,  \
                             a_goff, w_goff, EpiLinearA<ACT_>{epi});                    \
  else if (rows == 192) hipLaunchKernelGGL((gemm_big_kernel<EpiLinearA<ACT_>, 1, 6>), grid, \
                             dim3(512), 0, st, A, lda, W, ldw, (int)M, (int)N, (int)K,  \
                             a_goff, w_goff, EpiLinearA<ACT_>{epi});                    \
  else if (rows == 224) hipLaunchKernelGGL((gemm_big_kernel<EpiLinearA<ACT_>, 1, 7>), grid, \
                             dim3(512), 0, st, A, lda, W, ldw, (int)M, (int)N, (int)K,  \
                             a_goff, w_goff, EpiLinearA<ACT_>{epi});                    \
  else if (p8) hipLaunchKernelGGL((gemm_big_kernel<EpiLinearA<ACT_>, 1>), grid,         \
                             dim3(512), 0, st, A, lda, W, ldw, (int)M, (int)N, (int)K,  \
                             a_goff, w_goff, EpiLinearA<ACT_>{epi});                    \
  else hipLaunchKernelGGL((gemm_big_kernel<EpiLinearA<ACT_>, 0>), grid, dim3(512),      \
                          0, st, A, lda, W, ldw, (int)M, (int)N, (int)K, a_goff,        \
                          w_goff, EpiLinearA<ACT_>{epi})
      switch (epi.act) {
        case 0:
          if (epi.resid && (g_engine & 4)) CADENCE_BIG_ACT(4);
          else CADENCE_BIG_ACT(0);
          break;
        case 1: CADENCE_BIG_ACT(1); break;
        case 2: CADENCE_BIG_ACT(2); break;
        case 3: CADENCE_BIG_ACT(3); break;
        default: return (int)hipErrorInvalidValue;
      }
#undef CADENCE_BIG_ACT
    } else if (rows == 160) {
      hipLaunchKernelGGL((gemm_big_kernel<Epi, 1, 5>), grid, dim3(512), 0, st, A, lda, W,
                         ldw, (int)M, (int)N, (int)K, a_goff, w_goff, epi);
    } else if (rows == 192) {
      hipLaunchKernelGGL((gemm_big_kernel<Epi, 1, 6>), grid, dim3(512), 0, st, A, lda, W,
                         ldw, (int)M, (int)N, (int)K, a_goff, w_goff, epi);
    } else if (rows == 224) {
      hipLaunchKernelGGL((gemm_big_kernel<Epi, 1, 7>), grid, dim3(512), 0, st, A, lda, W,
                         ldw, (int)M, (int)N, (int)K, a_goff, w_goff, epi);
    } else if (p8) {
      hipLaunchKernelGGL((gemm_big_kernel<Epi, 1>), grid, dim3(512), 0, st, A, lda, W,
                         ldw, (int)M, (int)N, (int)K, a_goff, w_goff, epi);
    } else {
      hipLaunchKernelGGL((gemm_big_kernel<Epi, 0>), grid, dim3(512), 0, st, A, lda, W,
                         ldw, (int)M, (int)N, (int)K, a_goff, w_goff, epi);
    }
    return (int)hipGetLastError();
  }
  if (N % 64 || K % 32) return (int)hipErrorInvalidValue;
  int ksw = 0, ssplits = 0;
  if (stream_plan(M, K, &ksw, &ssplits)) {
    float* parts = nullptr;
    if (ssplits > 1) {
      const int64_t need = (int64_t)ssplits * groups * M * N * 4;
      if (!ws || ws_bytes < need) return (int)hipErrorInvalidValue;
      parts = static_cast<float*>(ws);
    }
    launch_stream(A, lda, W, ldw, M, N, K, groups, a_goff, w_goff, epi, ksw,
                  ssplits, parts, packed, st, nullptr, norm, neps);
    if (ssplits > 1) {
      int64_t outs = M * N;
      int rblocks = (int)((outs + 255) / 256);
      if (rblocks > 4096) rblocks = 4096;
      hipLaunchKernelGGL((splitk_reduce_kernel<Epi>), dim3(rblocks, (unsigned)groups),
                         dim3(256), 0, st, parts, ssplits, (int)groups, (int)M,
                         (int)N, epi);
    }
    return (int)hipGetLastError();
  }
  const int splits = skinny_splits(N, K, groups);
  const int64_t klen = skinny_klen(K, splits);
  const int64_t need = (int64_t)splits * groups * M * N * 4;
  if (!ws || ws_bytes < need) return (int)hipErrorInvalidValue;
  float* part = static_cast<float*>(ws);
  dim3 grid((unsigned)(N / 64), (unsigned)splits, (unsigned)groups);
  if (M <= 16)
    hipLaunchKernelGGL((gemm_skinny_kernel<16>), grid, dim3(256), 0, st, A, lda, W,
                       ldw, (int)M, (int)N, (int)K, (int)klen, part, a_goff, w_goff,
                       packed);
  else if (M <= 32)
    hipLaunchKernelGGL((gemm_skinny_kernel<32>), grid, dim3(256), 0, st, A, lda, W,
                       ldw, (int)M, (int)N, (int)K, (int)klen, part, a_goff, w_goff,
                       packed);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<64>), grid, dim3(256), 0, st, A, lda, W,
                       ldw, (int)M, (int)N, (int)K, (int)klen, part, a_goff, w_goff,
                       packed);
  int64_t outs = M * N;
  int rblocks = (int)((outs + 255) / 256);
  if (rblocks > 4096) rblocks = 4096;
  hipLaunchKernelGGL((splitk_reduce_kernel<Epi>), dim3(rblocks, (unsigned)groups),
                     dim3(256), 0, st, part, splits, (int)groups, (int)M, (int)N, epi);
  return (int)hipGetLastError();
}

}  // namespace

// the lab switch's bits for the other translation units (attention.hip)
__attribute__((visibility("hidden"))) int cadence_engine_bits() { return g_engine; }

extern "C" {

int cadence_abi_version(void) { return 18; }

int cadence_gemm_set_engine(int engine) {
  const int prev = g_engine;
  if (engine >= 0) g_engine = engine;   // engine < 0: query only
  return prev;
}

int cadence_gemm_big_splits(int64_t M, int64_t N, int64_t K, int64_t groups) {
  if (M <= kSkinnyMaxM || M <= 0) return 1;
  const int64_t g = groups > 0 ? groups : 1;
  return big_splits(M, N, K, g, big_tile_rows(M, N, K, g));
}

int cadence_gemm_engine(int64_t M, int64_t N, int64_t K, int64_t groups) {
  if (M <= kSkinnyMaxM || M <= 0) return 0;
  const int64_t g = groups > 0 ? groups : 1;
  const int rows = big_tile_rows(M, N, K, g);
  if (big_splits(M, N, K, g, rows) > 1) return 0;
  return use_w4(N, K, rows) ? 1 : 0;
}

int cadence_gemm_tile_rows(int64_t M, int64_t N, int64_t K, int64_t groups) {
  if (M <= kSkinnyMaxM || M <= 0) return 0;
  const int64_t g = groups > 0 ? groups : 1;
  const int r = big_tile_rows(M, N, K, g);
  if (big_splits(M, N, K, g, r) == 1 && use_w4(N, K, r)) return w4_tile_rows(M, N);
  return r ? r : 256;
}

int64_t cadence_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K,
                                     int64_t groups) {
  if (M > kSkinnyMaxM) {
    const int sk = big_splits(M, N, K, groups, big_tile_rows(M, N, K, groups));
    return sk > 1 ? (int64_t)sk * M * N * 4 : 0;
  }
  int ksw = 0, ss = 0;
  if (M > 0 && stream_plan(M, K, &ksw, &ss))
    return ss > 1 ? (int64_t)ss * groups * M * N * 4 : 0;
  if (M > kSkinnyMaxM || M <= 0) return 0;
  const int splits = skinny_splits(N, K, groups);
  return (int64_t)splits * groups * M * N * 4;
}

int cadence_gemm_linear(const void* A, int64_t lda, const void* W, int64_t ldw,
                        const void* bias, const void* resid, int64_t ld_resid,
                        void* out, int64_t ldo, int64_t M, int64_t N, int64_t K,
                        int act, int64_t row_div, int64_t row_mul,
                        int64_t row_off, void* workspace, int64_t ws_bytes,
                        void* stream) {
  if (row_div <= 0) return (int)hipErrorInvalidValue;
  EpiLinear epi{static_cast<u16*>(out), ldo, static_cast<const u16*>(bias),
                static_cast<const u16*>(resid), ld_resid, act,
                RowMap{row_div, row_mul, row_off}, 0.0f};
  return launch_gemm(static_cast<const u16*>(A), lda, static_cast<const u16*>(W),
                     ldw, M, N, K, 1, 0, 0, epi, workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

int cadence_gemm_linear_conv1d(const void* A, int64_t lda, const void* W,
                               int64_t ldw, const void* bias, void* out,
                               int64_t ldo, int64_t M, int64_t N, int64_t K,
                               int64_t conv_lo, const void* conv_w,
                               const void* conv_b, void* conv_state,
                               int64_t temporal_width, int norm,
                               float norm_eps, void* stream) {
  if (M <= 0) return 0;
  const int64_t E = N - conv_lo;
  if (norm && lda != 0) return (int)hipErrorInvalidValue;
  int ksw = 0, ss = 0;
  if (M > 32 || N % 64 || K % 32 || ldo < N || conv_lo < 0 || E <= 0 ||
      temporal_width < 1 || temporal_width > 4 || !conv_w || !conv_b ||
      (temporal_width > 1 && !conv_state) || (ldw != 0 && ldw < K) ||
      (lda != 0 && lda < K) || !stream_plan(M, K, &ksw, &ss) || ss != 1)
    return (int)hipErrorInvalidValue;
  const EpiLinear base{static_cast<u16*>(out), ldo, static_cast<const u16*>(bias),
                       nullptr, 0, 0, RowMap{M, 0, 0}, 0.0f};
  auto run = [&](auto tw_tag) {
    constexpr int TW = decltype(tw_tag)::value;
    EpiLinearConv<TW> epi{};
    static_cast<EpiLinear&>(epi) = base;
    epi.cw = static_cast<const u16*>(conv_w);
    epi.cb = static_cast<const u16*>(conv_b);
    epi.state = static_cast<u16*>(conv_state);
    epi.conv_lo = (int)conv_lo;
    epi.E = (int)E;
    launch_stream(static_cast<const u16*>(A), lda, static_cast<const u16*>(W), ldw, M,
                  N, K, 1, 0, 0, epi, ksw, 1, nullptr, ldw == 0 ? 1 : 0,
                  static_cast<hipStream_t>(stream), nullptr, norm, norm_eps);
  };
  switch (temporal_width) {   // Griffin uses 4; 1-3 for API parity
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 3: run(std::integral_constant<int, 3>{}); break;
    default: run(std::integral_constant<int, 4>{}); break;
  }
  return (int)hipGetLastError();
}

int cadence_recurrent_decode_front_plan(int64_t M, int64_t E, int64_t K, int64_t heads,
                                        int64_t bw) {
  int ksw = 0, ss = 0;
  // the one instantiation the gate stage is written for: packed rows of 17..32
  // sequences, 32 y|x columns per workgroup (ten 32-deep k-steps per wave, one
  // K split), 2 bw / 32 workgroups per head = the head's gate items, the
  // whole grid resident at once (<= 256 workgroups: one round).  (Two column
  // tiles per workgroup whatever stream_ntw picks for the plain launch: a
  // column's k-steps, waves and reduction order do not depend on NTW.)
  return (M > 16 && M <= 32 && bw > 0 && bw % 64 == 0 && bw <= 256 && heads * bw == E &&
          K % 32 == 0 && stream_plan(M, K, &ksw, &ss) && ksw == 10 && ss == 1 &&
          2 * E / 32 <= 256) ? 1 : 0;
}

int cadence_recurrent_decode_front(const void* A, const void* Wyx, const void* bias,
                                   void* yx_out, int64_t M, int64_t E, int64_t K,
                                   const void* conv_w, const void* conv_b, void* conv_state,
                                   int norm, float norm_eps, const void* Wgates,
                                   const void* bias_x, const void* bias_a,
                                   const void* softplus_a, const int32_t* segment_pos,
                                   float* h, void* y_out, int64_t heads, int64_t bw,
                                   int32_t* counters, int32_t* err, void* stream) {
  if (M <= 0) return 0;
  const int64_t N = 2 * E;
  if (!cadence_recurrent_decode_front_plan(M, E, K, heads, bw) || !Wyx || !Wgates ||
      !conv_w || !conv_b || !conv_state || !h || !y_out || !yx_out || !counters || !err ||
      !segment_pos)
    return (int)hipErrorInvalidValue;
  EpiLinearConvGates<4> epi{};
  static_cast<EpiLinear&>(epi) = EpiLinear{static_cast<u16*>(yx_out), N,
                                           static_cast<const u16*>(bias), nullptr, 0, 0,
                                           RowMap{M, 0, 0}, 0.0f};
  epi.cw = static_cast<const u16*>(conv_w);
  epi.cb = static_cast<const u16*>(conv_b);
  epi.state = static_cast<u16*>(conv_state);
  epi.conv_lo = (int)E;
  epi.E = (int)E;
  u16* yx = static_cast<u16*>(yx_out);
  epi.ge = EpiRglruGates{yx + E, N, static_cast<const u16*>(bias_x),
                         static_cast<const u16*>(bias_a), static_cast<const u16*>(softplus_a),
                         segment_pos, nullptr, nullptr, 0, (int)bw, h, E, yx, N,
                         static_cast<u16*>(y_out), 0, (int)((M + 15) / 16)};
  epi.wg = static_cast<const u16*>(Wgates);
  epi.cnt = counters;
  epi.err = err;
  const int klen = (int)K;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (norm)
    hipLaunchKernelGGL((gemm_stream_kernel<32, 10, 2, EpiLinearConvGates<4>, true>),
                       dim3((unsigned)(N / 32), 1, 1), dim3(512), 0, st,
                       static_cast<const u16*>(A), (int64_t)0, static_cast<const u16*>(Wyx),
                       (int64_t)0, (int)M, (int)N, (int)K, klen, (int64_t)0, (int64_t)0,
                       nullptr, epi, 1, nullptr, norm_eps);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<32, 10, 2, EpiLinearConvGates<4>, false>),
                       dim3((unsigned)(N / 32), 1, 1), dim3(512), 0, st,
                       static_cast<const u16*>(A), (int64_t)0, static_cast<const u16*>(Wyx),
                       (int64_t)0, (int)M, (int)N, (int)K, klen, (int64_t)0, (int64_t)0,
                       nullptr, epi, 1, nullptr, 0.0f);
  return (int)hipGetLastError();
}

int cadence_qkv_rope_decode(const void* A, int64_t lda, const void* Wperm,
                            int64_t ldw, const int32_t* positions, void* q_out,
                            void* k_out, void* v_out, int64_t M, int64_t H,
                            int64_t hd, int64_t K, const void* table,
                            int64_t table_len, int norm,
                            float norm_eps, void* stream) {
  if (M <= 0) return 0;
  if (norm && lda != 0) return (int)hipErrorInvalidValue;
  const int64_t N = (H + 2) * hd;
  int ksw = 0, ss = 0;
  if (M > 32 || hd % 64 || H < 1 || K % 32 || (ldw != 0 && ldw < K) ||
      (lda != 0 && lda < K) || !positions || !stream_plan(M, K, &ksw, &ss) || ss != 1)
    return (int)hipErrorInvalidValue;
  EpiRopeQKV epi{static_cast<u16*>(q_out), static_cast<u16*>(k_out),
                 static_cast<u16*>(v_out), positions, static_cast<const u16*>(table),
                 table ? (int)table_len : 0, (int)H, (int)hd};
  launch_stream(static_cast<const u16*>(A), lda, static_cast<const u16*>(Wperm), ldw,
                M, N, K, 1, 0, 0, epi, ksw, 1, nullptr, ldw == 0 ? 1 : 0,
                static_cast<hipStream_t>(stream), nullptr, norm, norm_eps);
  return (int)hipGetLastError();
}

int cadence_qkv_rope_prefill(const void* A, int64_t lda, const void* Wperm,
                             int64_t ldw, const int32_t* positions, void* q_out,
                             void* k_out, void* v_out, int64_t M, int64_t H, int64_t hd,
                             int64_t K, const void* table, int64_t table_len,
                             void* stream) {
  if (M <= 0) return 0;
  const int64_t N = (H + 2) * hd;
  if (M <= kSkinnyMaxM || hd % 64 || H < 1 || K % BK || N % 64 || lda < K || ldw < K ||
      !positions || big_splits(M, N, K, 1, big_tile_rows(M, N, K, 1)) > 1 ||
      use_w4(N, K, big_tile_rows(M, N, K, 1)))
    return (int)hipErrorInvalidValue;
  const EpiRopeQKVBig epi{static_cast<u16*>(q_out), static_cast<u16*>(k_out),
                          static_cast<u16*>(v_out), positions,
                          static_cast<const u16*>(table), table ? (int)table_len : 0,
                          (int)H, (int)hd};
  const u16* a = static_cast<const u16*>(A);
  const u16* w = static_cast<const u16*>(Wperm);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int rows = big_tile_rows(M, N, K, 1);
  const int64_t bm = rows ? rows : 256;
  const dim3 grid((unsigned)(((M + bm - 1) / bm) * ((N + 255) / 256)), 1);
#define CADENCE_ROPE_BIG(P8_, MR_)                                                        \
  hipLaunchKernelGGL((gemm_big_kernel<EpiRopeQKVBig, P8_, MR_>), grid, dim3(512), 0, st,  \
                     a, lda, w, ldw, (int)M, (int)N, (int)K, (int64_t)0, (int64_t)0, epi)
  switch (rows) {
    case 160: CADENCE_ROPE_BIG(1, 5); break;
    case 192: CADENCE_ROPE_BIG(1, 6); break;
    case 224: CADENCE_ROPE_BIG(1, 7); break;
    case 256: CADENCE_ROPE_BIG(1, 8); break;
    default: CADENCE_ROPE_BIG(0, 8); break;
  }
#undef CADENCE_ROPE_BIG
  return (int)hipGetLastError();
}

int64_t cadence_gemm_rmsnorm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  int ksw = 0, ss = 0;
  if (M <= 0 || N > 4096 || N % 64 || !rmsnorm_stream_plan(M, K, &ksw, &ss)) return 0;
  return (int64_t)ss * M * N * 4;
}

int cadence_gemm_linear_rmsnorm(const void* A, int64_t lda, const void* W,
                                int64_t ldw, const void* bias,
                                const void* resid, int64_t ld_resid, void* out,
                                int64_t ldo, int64_t M, int64_t N, int64_t K,
                                const void* norm_scale, float eps,
                                void* norm_out, int64_t ld_norm,
                                void* workspace, int64_t ws_bytes,
                                void* stream) {
  if (M <= 0) return 0;
  if (N % 8 || ldo % 8 || ld_norm % 8 || (resid && ld_resid % 8))
    return (int)hipErrorInvalidValue;
  if (ld_norm == 0 && (M > 32 || N % 32)) return (int)hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  EpiLinear epi{static_cast<u16*>(out), ldo, static_cast<const u16*>(bias),
                static_cast<const u16*>(resid), ld_resid, 0,
                RowMap{M, 0, 0}, 0.0f};
  int ksw = 0, ss = 0;
  if (N <= 4096 && N % 64 == 0 && rmsnorm_stream_plan(M, K, &ksw, &ss)) {
    // decode GEMM split over K (rmsnorm_stream_plan): the row-owned reduce +
    // residual + RMSNorm kernel replaces the split-K reduce and the norm.
    const int splits = ss;
    const int64_t need = (int64_t)splits * M * N * 4;
    if (!workspace || ws_bytes < need) return (int)hipErrorInvalidValue;
    float* parts = static_cast<float*>(workspace);
    launch_stream(static_cast<const u16*>(A), lda, static_cast<const u16*>(W), ldw,
                  M, N, K, 1, 0, 0, epi, ksw, splits, parts, ldw == 0 ? 1 : 0, st);
    const u16* sc = static_cast<const u16*>(norm_scale);
    u16* no = static_cast<u16*>(norm_out);
    const dim3 g((unsigned)M), b(512);
#define CADENCE_RN(RC_, S_) \
  hipLaunchKernelGGL((reduce_rmsnorm_kernel<RC_, S_>), g, b, 0, st, parts, (int)M, \
                     (int)N, epi, sc, eps, no, ld_norm)
    const bool one = N <= 4096;
    switch (splits) {
      case 2: if (one) CADENCE_RN(1, 2); else CADENCE_RN(2, 2); break;
      case 3: if (one) CADENCE_RN(1, 3); else CADENCE_RN(2, 3); break;
      case 4: if (one) CADENCE_RN(1, 4); else CADENCE_RN(2, 4); break;
      default: return (int)hipErrorInvalidValue;
    }
#undef CADENCE_RN
    return (int)hipGetLastError();
  }
  const int rc = launch_gemm(static_cast<const u16*>(A), lda,
                             static_cast<const u16*>(W), ldw, M, N, K, 1, 0, 0,
                             epi, workspace, ws_bytes, st);
  if (rc) return rc;
  return cadence_rmsnorm(out, ldo, norm_scale, norm_out, ld_norm, M, N, eps, stream);
}

int cadence_gemm_linear_residual_rows(const void* A, int64_t lda, const void* W,
                                      int64_t ldw, const void* bias,
                                      const void* resid, int64_t ld_resid,
                                      void* out, int64_t ldo, void* out_rows,
                                      int64_t M, int64_t N, int64_t K,
                                      void* workspace, int64_t ws_bytes,
                                      int32_t* counters, void* stream) {
  if (M <= 0) return 0;
  int ksw = 0, ss = 0;
  if (M > 32 || N % 64 || N > 4096 || ldo < N || (resid && ld_resid < N) ||
      !out_rows || !counters || (ldw != 0 && ldw < K) || (lda != 0 && lda < K) ||
      !rmsnorm_stream_plan(M, K, &ksw, &ss))
    return (int)hipErrorInvalidValue;
  if (!workspace || ws_bytes < (int64_t)ss * M * N * 4) return (int)hipErrorInvalidValue;
  EpiResidRows epi{};
  static_cast<EpiLinear&>(epi) =
      EpiLinear{static_cast<u16*>(out), ldo, static_cast<const u16*>(bias),
                static_cast<const u16*>(resid), ld_resid, 0, RowMap{M, 0, 0}, 0.0f};
  epi.rows = static_cast<u16*>(out_rows);
  epi.mt = (int)((M + 15) / 16);
  if (K == 2560 && lda == 0 && ldw == 0 && N % 16 == 0) {
    // the output projection: unsplit, 16 waves per 16 columns (one or two
    // 16-row tiles of packed rows)
    if (M > 16)
      hipLaunchKernelGGL((gemm_resid_pipe_kernel<16, 5, 1, 5, 2>), dim3((unsigned)(N / 16)),
                         dim3(1024), 0, static_cast<hipStream_t>(stream),
                         static_cast<const u16*>(A), static_cast<const u16*>(W), (int)M,
                         (int)K, epi);
    else
      hipLaunchKernelGGL((gemm_resid_pipe_kernel<16, 5, 1, 5, 1>), dim3((unsigned)(N / 16)),
                         dim3(1024), 0, static_cast<hipStream_t>(stream),
                         static_cast<const u16*>(A), static_cast<const u16*>(W), (int)M,
                         (int)K, epi);
    return (int)hipGetLastError();
  }
  launch_stream(static_cast<const u16*>(A), lda, static_cast<const u16*>(W), ldw, M, N,
                K, 1, 0, 0, epi, ksw, ss, static_cast<float*>(workspace),
                ldw == 0 ? 1 : 0, static_cast<hipStream_t>(stream), counters);
  return (int)hipGetLastError();
}

int cadence_gemm_gated_gelu(const void* A, int64_t lda, const void* Wpacked,
                            int64_t ldw, const void* bias_gate,
                            const void* bias_up, void* out, int64_t ldo,
                            int64_t M, int64_t F, int64_t K, void* workspace,
                            int64_t ws_bytes, int norm,
                            float norm_eps, void* stream) {
  if (F % 64 || (ldw != 0 && ldw < K)) return (int)hipErrorInvalidValue;
  if (ldo == 0 && M > 32) return (int)hipErrorInvalidValue;   // packed rows
  EpiGatedGelu epi{static_cast<u16*>(out), ldo,
                   static_cast<const u16*>(bias_gate),
                   static_cast<const u16*>(bias_up), (int)((M + 15) / 16)};
  if (M <= 32 && ldw == 0 && lda == 0 && K % 32 == 0 && K <= 2560) {
    // decode (packed rows, one or two 16-row tiles): the two-pair pipelined
    // kernel (one round)
    const dim3 grid((unsigned)(F / 32));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const u16* a = static_cast<const u16*>(A);
    const u16* w = static_cast<const u16*>(Wpacked);
#define CADENCE_GP(NORM_, MR_, EPS_)                                                        \
  hipLaunchKernelGGL((gemm_gated_pipe_kernel<10, 2, 3, NORM_, MR_>), grid, dim3(512), 0, st, a, \
                     w, (int)M, (int)K, epi, EPS_)
    if (M > 16) {
      if (norm) CADENCE_GP(true, 2, norm_eps);
      else CADENCE_GP(false, 2, 0.0f);
    } else {
      if (norm) CADENCE_GP(true, 1, norm_eps);
      else CADENCE_GP(false, 1, 0.0f);
    }
#undef CADENCE_GP
    return (int)hipGetLastError();
  }
  return launch_gemm(static_cast<const u16*>(A), lda,
                     static_cast<const u16*>(Wpacked), ldw, M, 2 * F, K, 1, 0, 0,
                     epi, workspace, ws_bytes, static_cast<hipStream_t>(stream),
                     norm, norm_eps);
}

// The prefill gates plan: the block-bound streaming kernel, or (lab switch
// engine bit 1 clear, a width it has no instance for, packed decode weights,
// M <= 32, unaligned rows) the block engine's grouped GEMM with EpiRglruGates.
static bool gates_stream_plan(const void* X, int64_t ldx, const void* Wpacked,
                              int64_t ldw, int64_t ldo, int64_t M, int64_t bw) {
  return (g_engine & 2) && ldw == bw && M > 32 && (bw == 64 || bw == 128 || bw == 256) &&
         ldx % 8 == 0 && ldo % 8 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0 &&
         reinterpret_cast<uintptr_t>(Wpacked) % 16 == 0;
}

int cadence_rglru_gates_stream_plan(const void* X, int64_t ldx, const void* Wpacked,
                                    int64_t ldw, int64_t ldo, int64_t M, int64_t bw) {
  return gates_stream_plan(X, ldx, Wpacked, ldw, ldo, M, bw) ? 1 : 0;
}

int cadence_rglru_gates(const void* X, int64_t ldx, const void* Wpacked,
                        int64_t ldw, const void* bias_x, const void* bias_a,
                        const void* softplus_a, const int32_t* segment_pos,
                        void* a_out, void* nx_out, int64_t ldo, int64_t M,
                        int64_t heads, int64_t bw, void* workspace,
                        int64_t ws_bytes, void* stream) {
  if (bw % 64 || (ldw != 0 && ldw != bw)) return (int)hipErrorInvalidValue;
  EpiRglruGates epi{static_cast<const u16*>(X), ldx,
                    static_cast<const u16*>(bias_x),
                    static_cast<const u16*>(bias_a),
                    static_cast<const u16*>(softplus_a), segment_pos,
                    static_cast<u16*>(a_out), static_cast<u16*>(nx_out), ldo,
                    (int)bw, nullptr, 0, nullptr, 0, nullptr, 0, 1};
  hipStream_t st = static_cast<hipStream_t>(stream);
  // (lab switch: engine 0 keeps the block engine, for the bitwise A/B test)
  if (gates_stream_plan(X, ldx, Wpacked, ldw, ldo, M, bw)) {
    // prefill: the block-bound streaming kernel, ~256 / heads workgroups per
    // block (2 / 4 per CU for the narrower blocks' smaller waves counts)
    const int64_t ntiles = (M + 31) / 32;
    const int64_t per = std::max<int64_t>(1, (256 * (256 / bw)) / heads);
    const dim3 grid((unsigned)std::min(ntiles, per), (unsigned)heads);
    if (bw == 256)
      hipLaunchKernelGGL(rglru_gates_stream_kernel<256>, grid, dim3(512), 0, st,
                         static_cast<const u16*>(X), ldx, static_cast<const u16*>(Wpacked),
                         (int)M, epi);
    else if (bw == 128)
      hipLaunchKernelGGL(rglru_gates_stream_kernel<128>, grid, dim3(256), 0, st,
                         static_cast<const u16*>(X), ldx, static_cast<const u16*>(Wpacked),
                         (int)M, epi);
    else
      hipLaunchKernelGGL(rglru_gates_stream_kernel<64>, grid, dim3(128), 0, st,
                         static_cast<const u16*>(X), ldx, static_cast<const u16*>(Wpacked),
                         (int)M, epi);
    return (int)hipGetLastError();
  }
  return launch_gemm(static_cast<const u16*>(X), ldx,
                     static_cast<const u16*>(Wpacked), ldw, M, 2 * bw, bw, heads,
                     bw, 2 * bw * bw, epi, workspace, ws_bytes, st);
}

// Fused prefill gates + scan plan: block widths with a 128-channel split
// (128, 256), row-major packed weights, enough (sequence, block half) units
// to fill the chip (the sequential walk over L is each workgroup's latency),
// 16-B aligned rows.
static bool rglru_scan_plan(const void* X, int64_t ldx, const void* gate, int64_t ldg,
                            int64_t ldo, int64_t B, int64_t L, int64_t heads, int64_t bw) {
  return (bw == 128 || bw == 256) && L >= 16 && L <= kRglruScanMaxL &&
         B * heads * (bw / 128) >= 512 &&
         ldx % 8 == 0 && ldo % 8 == 0 && (gate == nullptr || ldg % 8 == 0) &&
         reinterpret_cast<uintptr_t>(X) % 16 == 0 &&
         reinterpret_cast<uintptr_t>(gate) % 16 == 0;
}

int cadence_rglru_scan_plan(const void* X, int64_t ldx, const void* gate, int64_t ldg,
                            int64_t ldo, int64_t B, int64_t L, int64_t heads, int64_t bw) {
  return rglru_scan_plan(X, ldx, gate, ldg, ldo, B, L, heads, bw) ? 1 : 0;
}

int cadence_rglru_scan(const void* X, int64_t ldx, const void* Wpacked,
                       const void* bias_x, const void* bias_a, const void* softplus_a,
                       const int32_t* segment_pos, const float* h0, const void* gate,
                       int64_t ldg, void* out, int64_t ldo, float* h_last, int64_t B,
                       int64_t L, int64_t heads, int64_t bw, void* stream) {
  if (!rglru_scan_plan(X, ldx, gate, ldg, ldo, B, L, heads, bw) ||
      B * L > INT32_MAX || heads * bw > INT32_MAX)
    return (int)hipErrorInvalidValue;
  RglruScanArgs a{static_cast<const u16*>(X), ldx, static_cast<const u16*>(Wpacked),
                  static_cast<const u16*>(bias_x), static_cast<const u16*>(bias_a),
                  static_cast<const u16*>(softplus_a), segment_pos, h0,
                  static_cast<const u16*>(gate), ldg, static_cast<u16*>(out), ldo, h_last,
                  (int)B, (int)L, (int)(heads * bw), (int)heads};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((B * heads + 7) / 8 * 16));
  // 16-step chunks at BW 256 (its K = 256 weight fragments take 128 VGPRs;
  // a 32-row tile's accumulators would spill), 32-step chunks at BW 128
  if (bw == 256) {
    if (gate) hipLaunchKernelGGL((rglru_scan_fused_kernel<256, true, 16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((rglru_scan_fused_kernel<256, false, 16>), grid, dim3(256), 0, st, a);
  } else {
    if (gate) hipLaunchKernelGGL((rglru_scan_fused_kernel<128, true, 32>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((rglru_scan_fused_kernel<128, false, 32>), grid, dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

int cadence_rglru_step(const void* X, int64_t ldx, const void* Wpacked,
                       int64_t ldw, const void* bias_x, const void* bias_a,
                       const void* softplus_a, const int32_t* segment_pos,
                       float* h, const void* gate, int64_t ldg, void* y_out,
                       int64_t ldy, int64_t M, int64_t heads, int64_t bw,
                       void* workspace, int64_t ws_bytes, void* stream) {
  if (bw % 64 || (ldw != 0 && ldw != bw) || !h || !y_out)
    return (int)hipErrorInvalidValue;
  if (ldy == 0 && M > 32) return (int)hipErrorInvalidValue;   // packed rows
  EpiRglruGates epi{static_cast<const u16*>(X), ldx,
                    static_cast<const u16*>(bias_x),
                    static_cast<const u16*>(bias_a),
                    static_cast<const u16*>(softplus_a), segment_pos,
                    nullptr, nullptr, 0, (int)bw, h, heads * bw,
                    static_cast<const u16*>(gate), ldg, static_cast<u16*>(y_out),
                    ldy, (int)((M + 15) / 16)};
  return launch_gemm(static_cast<const u16*>(X), ldx,
                     static_cast<const u16*>(Wpacked), ldw, M, 2 * bw, bw, heads,
                     bw, 2 * bw * bw, epi, workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

int cadence_gemm_vit_residual(const void* A, int64_t lda, const void* W,
                              int64_t ldw, const void* bias, const void* gamma,
                              float* resid, int64_t ld_resid, int64_t M,
                              int64_t N, int64_t K, void* workspace,
                              int64_t ws_bytes, void* stream) {
  EpiVitResid epi{resid, ld_resid, static_cast<const u16*>(bias),
                  static_cast<const u16*>(gamma)};
  return launch_gemm(static_cast<const u16*>(A), lda, static_cast<const u16*>(W),
                     ldw, M, N, K, 1, 0, 0, epi, workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

int cadence_gemm_patch_embed(const void* patches, int64_t ldp, const void* W,
                             int64_t ldw, const void* bias, const void* pos,
                             float* resid, int64_t B, int64_t P, int64_t ntok,
                             int64_t prefix, int64_t N, int64_t K,
                             void* workspace, int64_t ws_bytes, void* stream) {
  EpiPatch epi{resid, static_cast<const u16*>(bias),
               static_cast<const u16*>(pos), P, ntok, prefix, N};
  return launch_gemm(static_cast<const u16*>(patches), ldp,
                     static_cast<const u16*>(W), ldw, B * P, N, K, 1, 0, 0, epi,
                     workspace, ws_bytes, static_cast<hipStream_t>(stream));
}

int64_t cadence_logits_scratch_bytes(int64_t M, int64_t V, int64_t D) {
  const int splits = skinny_splits(V, D, 1);
  const int64_t nblk = (V + 255) / 256;
  return (int64_t)splits * M * V * 4 + M * nblk * 8 + 256;
}

int cadence_logits_argmax(const void* X, int64_t ldx, const void* E,
                          int64_t lde, int64_t M, int64_t V, int64_t D,
                          float soft_cap, void* logits_out, int32_t* next_token,
                          void* scratch, int64_t scratch_bytes, void* stream) {
  if (M <= 0) return 0;
  if (M > kSkinnyMaxM || V % 64 || D % 32 || (lde != 0 && lde < D))
    return (int)hipErrorInvalidValue;
  if (scratch_bytes < cadence_logits_scratch_bytes(M, V, D))
    return (int)hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int packed = lde == 0 ? 1 : 0;
  const int splits = skinny_splits(V, D, 1);
  const int64_t klen = skinny_klen(D, splits);
  float* part = static_cast<float*>(scratch);
  const int64_t nblk = (V + 255) / 256;
  float* bval = part + (int64_t)splits * M * V;
  int* bidx = reinterpret_cast<int*>(bval + M * nblk);   // split path
  const u16* A = static_cast<const u16*>(X);
  const u16* W = static_cast<const u16*>(E);
  dim3 grid((unsigned)(V / 64), (unsigned)splits, 1);
  if (splits == 1) {
    // one pass: the skinny kernel emits per-64-column (max, index) pairs
    // (into the partial-slab area of the scratch, unused without a split)
    const int64_t nb64 = V / 64;
    u16* lo = static_cast<u16*>(logits_out);
    bval = part;
    bidx = reinterpret_cast<int*>(part + M * nb64);
#define CADENCE_LGA(MS_)                                                                 \
  hipLaunchKernelGGL((gemm_skinny_kernel<MS_, true>), grid, dim3(256), 0, st, A, ldx, W, \
                     lde, (int)M, (int)V, (int)D, (int)klen, part, (int64_t)0, (int64_t)0, \
                     packed, soft_cap, lo, bval, bidx)
    if (M <= 16) CADENCE_LGA(16);
    else if (M <= 32) CADENCE_LGA(32);
    else CADENCE_LGA(64);
#undef CADENCE_LGA
    if (next_token)
      hipLaunchKernelGGL(argmax_final_kernel, dim3((unsigned)M), dim3(256), 0, st,
                         bval, bidx, (int)nb64, next_token);
    return (int)hipGetLastError();
  }
  if (M <= 16)
    hipLaunchKernelGGL((gemm_skinny_kernel<16>), grid, dim3(256), 0, st, A, ldx, W,
                       lde, (int)M, (int)V, (int)D, (int)klen, part, (int64_t)0, (int64_t)0,
                       packed);
  else if (M <= 32)
    hipLaunchKernelGGL((gemm_skinny_kernel<32>), grid, dim3(256), 0, st, A, ldx, W,
                       lde, (int)M, (int)V, (int)D, (int)klen, part, (int64_t)0, (int64_t)0,
                       packed);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<64>), grid, dim3(256), 0, st, A, ldx, W,
                       lde, (int)M, (int)V, (int)D, (int)klen, part, (int64_t)0, (int64_t)0,
                       packed);
  hipLaunchKernelGGL(logits_reduce_kernel, dim3((unsigned)nblk, (unsigned)M),
                     dim3(256), 0, st, part, splits, (int)M, (int)V, soft_cap,
                     static_cast<u16*>(logits_out), bval, bidx);
  if (next_token)
    hipLaunchKernelGGL(argmax_final_kernel, dim3((unsigned)M), dim3(256), 0, st,
                       bval, bidx, (int)nblk, next_token);
  return (int)hipGetLastError();
}

// the descriptor's layout as the ctypes mirror declares it (cadence._lib.DecodeTail)
static_assert(sizeof(CadenceDecodeTail) == 120 && offsetof(CadenceDecodeTail, counter) == 64 &&
                  offsetof(CadenceDecodeTail, scale) == 88 &&
                  offsetof(CadenceDecodeTail, packed_out) == 112,
              "CadenceDecodeTail layout");

int cadence_logits_argmax_tail(const void* X, int64_t ldx, const void* E, int64_t lde,
                               int64_t M, int64_t V, int64_t D, float soft_cap,
                               int32_t* next_token, void* scratch, int64_t scratch_bytes,
                               const CadenceDecodeTail* tail, void* stream) {
  if (M <= 0) return 0;
  if (!tail || !next_token || M > 32 || D % 32 || !tail->counter || !tail->step ||
      !tail->positions || !tail->tokens_out || !tail->embed || !tail->x_out ||
      !tail->packed_out || tail->ldx_out < D || tail->vocab <= 0)
    return (int)hipErrorInvalidValue;
  // the logits and the per-block (max, index) pairs, no argmax launch
  const int rc = cadence_logits_argmax(X, ldx, E, lde, M, V, D, soft_cap, nullptr, nullptr,
                                       scratch, scratch_bytes, stream);
  if (rc != 0) return rc;
  // where cadence_logits_argmax left the pairs (its scratch layout)
  const int splits = skinny_splits(V, D, 1);
  float* part = static_cast<float*>(scratch);
  const float* bval;
  const int* bidx;
  int nb;
  if (splits == 1) {
    nb = (int)(V / 64);
    bval = part;
    bidx = reinterpret_cast<const int*>(part + M * nb);
  } else {
    nb = (int)((V + 255) / 256);
    bval = part + (int64_t)splits * M * V;
    bidx = reinterpret_cast<const int*>(bval + M * nb);
  }
  hipLaunchKernelGGL(argmax_tail_kernel, dim3((unsigned)M), dim3(256), 0,
                     static_cast<hipStream_t>(stream), bval, bidx, nb, next_token, *tail,
                     (int)M, (int)D);
  return (int)hipGetLastError();
}

int cadence_gemm_logits(const void* X, int64_t ldx, const void* E, int64_t lde,
                        int64_t M, int64_t V, int64_t D, float soft_cap, void* out,
                        int64_t ldo, void* workspace, int64_t ws_bytes,
                        void* stream) {
  EpiLinear epi{static_cast<u16*>(out), ldo, nullptr, nullptr, 0,
                soft_cap > 0.0f ? 2 : 0, RowMap{M > 0 ? M : 1, 0, 0}, soft_cap};
  return launch_gemm(static_cast<const u16*>(X), ldx, static_cast<const u16*>(E),
                     lde, M, V, D, 1, 0, 0, epi, workspace, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

}  // extern "C"
