// Attention kernels for gfx950.
//
// flash_attn_kernel<HD, MODE>: one workgroup = 4 waves = 64 query rows of one
// (batch, head); each wave owns 16 rows.  Key tiles of 32 are staged in LDS
// (K row-major with an XOR chunk swizzle, V transposed so PV B-fragments are
// 16-byte reads), S = Q.K^T and O += P.V run on mfma_f32_16x16x32_bf16,
// softmax is online in fp32, P goes through a 1 KiB per-wave LDS tile to
// become the next MFMA's A operand.
//   MODE_LOCAL: Griffin local attention (modules.py:466-480): logits rounded
//     to bf16 then * hd^-0.5, mask = same segment & causal & window; key
//     tiles outside [max(seg_start, q0 - W), q_last] are skipped.  MQA: every
//     head reads the single K/V head.
//   MODE_VIT: timm bidirectional SDPA (fp32 logits, no mask but the tail);
//     not instantiated: cadence_vit_attention runs vit_attention.hip /
//     vit_stream_attn_kernel for every shape it accepts.
// decode_attn_kernel: one wave per sequence, 16 rows = the query heads,
// keys = ring-buffer slots (positions of _compute_cache_mask) + the new key,
// then the in-place slot update of _update_attention_cache.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

int vit_attention_lds_launch(const void* qkv, void* out, int64_t B, int64_t N,
                             int64_t H, int64_t hd, void* stream);  // vit_attention.hip
int griffin_attention_launch(const void* q, const void* k, const void* v,
                             const int32_t* seg_start, void* out, int64_t B,
                             int64_t L, int64_t H, int64_t hd, int64_t window,
                             void* stream);  // griffin_attention.hip
int vit_stream_attention_launch(const void* qkv, void* out, int64_t B, int64_t N,
                                int64_t H, int64_t hd, void* stream);
int vit_flash_attention_launch(const void* qkv, void* out, int64_t B, int64_t N,
                               int64_t H, int64_t hd, void* stream);  // vit_flash.hip
int cadence_engine_bits();                                            // gemm.hip
int generic_attention_launch(const void* q, const void* k, const void* v,
                             const void* cache_k, const void* cache_v,
                             const int32_t* num_tokens, const int32_t* seg_start,
                             void* out, int64_t B, int64_t T, int64_t H,
                             int64_t hd, int64_t window, void* stream);
int rope_qkv_generic_launch(const void* qkv, int64_t ld, const int32_t* positions,
                            void* q_out, void* k_out, void* v_out, int64_t M,
                            int64_t H, int64_t hd, void* stream);  // attention_generic.hip

namespace {

constexpr int MODE_LOCAL = 0;
constexpr int MODE_VIT = 1;
constexpr int KT = 32;  // keys per tile
constexpr int kDecodeSplitsMax = 32;  // window ranges of the decode attention
// ranges per sequence: enough workgroups to cover the CUs at any batch
// fewest keys per range (a multiple of 16; see decode_attn_kernel's plan)
constexpr int kDecodeMinRange = 64;
inline int decode_splits(int64_t B) {
  const int64_t ns = 256 / (B > 0 ? B : 1);
  return (int)(ns < 1 ? 1 : ns > kDecodeSplitsMax ? kDecodeSplitsMax : ns);
}

struct AttnArgs {
  const u16* q; int64_t q_bs, q_rs, q_hs;   // batch / row / head strides
  const u16* k; int64_t k_bs, k_rs, k_hs;
  const u16* v; int64_t v_bs, v_rs, v_hs;
  u16* o; int64_t o_bs, o_rs, o_hs;
  const int32_t* seg; const int32_t* seg_start;
  int L;          // query rows == key rows per sequence
  int H, hd;      // heads, true head dim (<= HD)
  int window;
  float scale;
};

// XOR swizzle of a 16-B chunk index inside one K row; stays inside the row
// for any chunks-per-row that is a multiple of 4 (HD = 96 -> 12 chunks).
template <int CPR>
CADENCE_DEV int swz(int ch, int row) {
  return (CPR % 8 == 0) ? (ch ^ (row & 7)) : (ch ^ (row & 3));
}

template <int HD>
struct Smem {
  uint4 k[KT * HD / 8];        // [key][HD] swizzled 16-B chunks
  u16 vt[HD * KT];             // [dim][key]
  u16 p[4][16 * KT];           // per-wave P tile [row][key]
};

template <int HD, int MODE>
__global__ __launch_bounds__(256) void flash_attn_kernel(AttnArgs a) {
  constexpr int KS = HD / 32;   // k-steps for Q.K^T
  constexpr int NO = HD / 16;   // output column reps
  constexpr int CPR = HD / 8;   // 16-B chunks per K row
  __shared__ Smem<HD> sm;

  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qw = q0 + wave * 16;

  const u16* qb = a.q + b * a.q_bs + h * a.q_hs;
  const u16* kb = a.k + b * a.k_bs + h * a.k_hs;
  const u16* vb = a.v + b * a.v_bs + h * a.v_hs;

  // Q fragments: lane holds Q[row lane&15][32*ks + 8*(lane>>4) + j]
  bf16x8 qf[KS];
  {
    const int r = qw + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 32 + 8 * (lane >> 4);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < a.L && d < a.hd) v = ld16(qb + (int64_t)r * a.q_rs + d);
      qf[ks] = __builtin_bit_cast(bf16x8, v);
    }
  }

  f32x4 o[NO];
#pragma unroll
  for (int j = 0; j < NO; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_run[r] = -INFINITY;
    l_run[r] = 0.0f;
  }

  // key range for the whole workgroup
  int kbeg = 0, kend = a.L;
  if (MODE == MODE_LOCAL) {
    const int qlast = min(q0 + 63, a.L - 1);
    int lo = a.seg_start[(int64_t)b * a.L + q0];
    lo = max(lo, q0 - a.window);
    kbeg = (max(lo, 0) / KT) * KT;
    kend = qlast + 1;
  }
  const int rowq0 = qw + 4 * (lane >> 4);  // + r
  // same segment and causal <=> seg_start(q) <= key <= q (segments are
  // contiguous runs of seg = cumsum(pos == 0)): one start per query row,
  // no per-key segment loads in the tile loop
  int sstart[4];
  if (MODE == MODE_LOCAL) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = min(rowq0 + r, a.L - 1);
      sstart[r] = a.seg_start[(int64_t)b * a.L + qi];
    }
  }

  // K / V tile staging: all of this thread's chunks of a tile are loaded
  // (unconditional loads from clamped rows, masked after the load) before
  // the first LDS store -- one memory round trip per tile.  (Prefetching
  // the next tile across the compute kept 32 more VGPRs live and halved the
  // occupancy: 193 -> 238 us.)
  constexpr int NIT = (KT * CPR + 255) / 256;
  uint4 kreg[NIT], vreg[NIT];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int c = tid + i * 256;
      const int kr = c / CPR, ch = c % CPR;
      const int key = k0 + kr;
      const int kc = min(key, a.L - 1), d = min(ch * 8, a.hd - 8);
      const uint4 kv = ld16(kb + (int64_t)kc * a.k_rs + d);
      const uint4 vv = ld16(vb + (int64_t)kc * a.v_rs + d);
      const uint32_t mk = (key < a.L && ch * 8 < a.hd && c < KT * CPR) ? 0xffffffffu : 0u;
      kreg[i] = make_uint4(kv.x & mk, kv.y & mk, kv.z & mk, kv.w & mk);
      vreg[i] = make_uint4(vv.x & mk, vv.y & mk, vv.z & mk, vv.w & mk);
    }
  };
  for (int k0 = kbeg; k0 < kend; k0 += KT) {
    load_tile(k0);
    __syncthreads();  // previous tile fully consumed
    // store the staged K tile (swizzled) and V^T tile
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int c = tid + i * 256;
      if (c < KT * CPR) {
        const int kr = c / CPR, ch = c % CPR;
        const int d = ch * 8;
        sm.k[kr * CPR + swz<CPR>(ch, kr)] = kreg[i];
        const uint4 vv = vreg[i];
        const u16* vs = reinterpret_cast<const u16*>(&vv);
#pragma unroll
        for (int e = 0; e < 8; ++e) sm.vt[(d + e) * KT + kr] = vs[e];
      }
    }
    __syncthreads();

    // S = Q K^T  (2 column reps of 16 keys)
    f32x4 s[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const int kr = jn * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = ks * 4 + (lane >> 4);
        const bf16x8 kf = __builtin_bit_cast(bf16x8, sm.k[kr * CPR + swz<CPR>(ch, kr)]);
        s[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, s[jn], 0, 0, 0);
      }
    }

    // scale + mask, online softmax
    float p[2][4];
    float tmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tmax[r] = -INFINITY;
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const int key = k0 + jn * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v;
        bool ok;
        if (MODE == MODE_LOCAL) {
          v = rbf(s[jn][r]) * a.scale;
          const int qi = rowq0 + r;
          ok = key < a.L && key <= qi && qi <= key + a.window && key >= sstart[r];
        } else {
          v = s[jn][r] * a.scale;
          ok = key < a.L;
        }
        v = ok ? v : -INFINITY;
        p[jn][r] = v;
        tmax[r] = fmaxf(tmax[r], v);
      }
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t = tmax[r];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) t = fmaxf(t, __shfl_xor(t, off, 64));
      const float mn = fmaxf(m_run[r], t);
      alpha[r] = (mn == -INFINITY) ? 1.0f : expf(m_run[r] - mn);
      float rs = 0.0f;
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) {
        const float e = (mn == -INFINITY) ? 0.0f : expf(p[jn][r] - mn);
        p[jn][r] = e;
        rs += e;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l_run[r] = l_run[r] * alpha[r] + rs;
      m_run[r] = mn;
    }
#pragma unroll
    for (int j = 0; j < NO; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= alpha[r];

    // P (bf16) -> LDS [row][key] -> A fragments
    u16* pw = sm.p[wave];
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pw[(4 * (lane >> 4) + r) * KT + jn * 16 + (lane & 15)] = f2bf(p[jn][r]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const bf16x8 pf = __builtin_bit_cast(
        bf16x8, *reinterpret_cast<const uint4*>(pw + (lane & 15) * KT + 8 * (lane >> 4)));
#pragma unroll
    for (int j = 0; j < NO; ++j) {
      const bf16x8 vf = __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(&sm.vt[(j * 16 + (lane & 15)) * KT +
                                                        8 * (lane >> 4)]));
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[j], 0, 0, 0);
    }
  }

  // normalise and store
  u16* ob = a.o + b * a.o_bs + h * a.o_hs;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qi = rowq0 + r;
    if (qi >= a.L) continue;
    const float inv = l_run[r] > 0.0f ? 1.0f / l_run[r] : 0.0f;
#pragma unroll
    for (int j = 0; j < NO; ++j) {
      const int d = j * 16 + (lane & 15);
      if (d < a.hd) ob[(int64_t)qi * a.o_rs + d] = f2bf(o[j][r] * inv);
    }
  }
}

// ------------------------------------------------------------------ decode

struct DecodeArgs {
  const u16* q;           // [B, H*hd]
  const u16* k_new;       // [B, hd] (row stride knew_rs)
  const u16* v_new;
  int64_t new_rs;
  u16* ck; u16* cv;       // [B, W, hd]
  int32_t* num_tokens;    // [B]
  u16* o;                 // [B, H*hd] (ldo = H*hd) or packed rows (ldo = 0)
  int64_t ldo;
  int omt;                // ceil(B / 16) for packed rows
  int H, hd, W;
  float scale;
  float* parts;           // [B, NS, 32 + 16 * hd] fp32 split partials (NS > 1)
  int32_t* sems;          // [B] zeroed arrival counters (NS > 1)
  int cmin;               // fewest keys per range (a multiple of 16)
};

// Split over the window (gridDim.y = NS): the B x NS workgroups cover the
// sequence's non-empty keys -- ring slots [0, slot_hi) then the new key,
// nk = slot_hi + 1 in all -- in NS contiguous ranges of C = ceil(nk / NS)
// keys rounded up to 16, at least cmin = 64 (ranges past nk exit at once:
// every range costs the combine a partial, and the combine's trip is the
// dearest link of the chain -- tools/decode_attn_lab.sh, profiles/r03ad_*:
// B = 32 at 320 keys 15.6 -> 14.6 us, at 64 keys 13.5 -> 11.9; more, shorter
// ranges per sequence were slower at every context).  A range is streamed
// in tiles of 64 keys: every K and V byte of the tile is loaded up front into
// registers (the next tile's loads go out as soon as this one is in LDS), K
// is stored with the row swizzle of the QK^T fragment reads, V row-major with
// a 32-B-slot XOR for the transposed P.V reads (ds_read_b64_tr_b16: 4 keys x
// 16 dims per 16-lane group, two per MFMA B fragment), so no V transpose
// pass exists.  The 4 waves compute the 16 x 64 score tile redundantly (the
// query heads are the MFMA rows) and each owns a quarter of the head dim in
// P.V.  A range keeps its own online-softmax state and, with NS > 1,
// publishes (m, l, unnormalised o) of the H real heads with write-through
// stores; the last range to arrive at the sequence's counter combines the
// partials in range order (fixed, so replays are bit-identical), writes the
// output and performs the cache update.  Hand-off: MI355X_MICROARCH
// "inter-workgroup visibility", first protocol row (sc1 stores and loads,
// one relaxed agent atomic per workgroup, no fences).
constexpr int kDecodeKT = 64;   // keys per tile

// V image slot XOR: rows {0..3, 8..11} (and {4..7, 12..15}) of a 16-row
// block land on distinct 32-B slots of a 256-B bank row, so each
// ds_read_b64_tr_b16 (one 32-lane half = two 4-row blocks 8 rows apart) is
// conflict-free; a multiple of 2 keeps a row's two 16-B chunks of one 32-B
// slot together.
template <int CPR>
CADENCE_DEV int vswz(int row) {
  return CPR >= 16 ? 2 * ((row & 3) | (((row >> 3) & 1) << 2)) : 2 * (row & 3);
}

// Reductions over the 16 lanes of a DPP row (the 16 key columns of a score
// block) on the VALU's DPP lane moves -- quad xor 1, quad xor 2, half-row
// mirror, row mirror -- instead of four ds_bpermute round trips through the
// LDS pipe.  After the two quad steps every lane of a quad holds bitwise the
// same value (IEEE max / add are commutative), so pairing lane i with 7 - i
// and then 15 - i combines the same operands as xor 4 and xor 8: the same
// bits as the __shfl_xor butterfly.
template <int CTRL>
CADENCE_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
CADENCE_DEV float row16_max(float t) {
  t = fmaxf(t, dpp_f<0xb1>(t));    // quad_perm [1, 0, 3, 2]
  t = fmaxf(t, dpp_f<0x4e>(t));    // quad_perm [2, 3, 0, 1]
  t = fmaxf(t, dpp_f<0x141>(t));   // row_half_mirror
  return fmaxf(t, dpp_f<0x140>(t));  // row_mirror
}
CADENCE_DEV float row16_sum(float t) {
  t += dpp_f<0xb1>(t);
  t += dpp_f<0x4e>(t);
  t += dpp_f<0x141>(t);
  return t + dpp_f<0x140>(t);
}

template <int HD>
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeArgs a) {
  constexpr int KS = HD / 32, NO = HD / 64, CPR = HD / 8;
  constexpr int KT = kDecodeKT, LPT = KT * CPR / 256;   // 16-B loads per operand
  __shared__ uint4 ks_[KT * CPR];
  __shared__ uint4 vs_[KT * CPR];
  __shared__ u16 ptall[4][16 * KT];
  __shared__ int ticket;
  __shared__ __attribute__((aligned(16))) float ml[32];   // split m[16], l[16]
  __shared__ float mls[kDecodeSplitsMax * 32];            // combine: all ranges'
  const int b = blockIdx.x;
  const int split = blockIdx.y, NS = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  u16* pt = ptall[wave];
  const int dbase = wave * (HD / 4);
  const int nt = a.num_tokens[b];
  const int qpos = nt;
  const int kblk = nt / a.W;
  // slots with a non-negative position: all of them once the ring wrapped
  const int slot_hi = nt >= a.W ? a.W : nt;
  const int nk = slot_hi + 1;                   // + the new key
  const int C = max(a.cmin, (((nk + NS - 1) / NS) + 15) & ~15);
  const int nsp = (nk + C - 1) / C;             // active ranges
  if (split >= nsp) return;
  const int kb = split * C, ke = min(nk, kb + C);

  // branch-free loads throughout (absent rows / keys read the zero page)
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  const u16* ckb = a.ck + (int64_t)b * a.W * a.hd;
  const u16* cvb = a.cv + (int64_t)b * a.W * a.hd;
  const u16* knb = a.k_new + (int64_t)b * a.new_rs;
  const u16* vnb = a.v_new + (int64_t)b * a.new_rs;
  // the cache update's rows, loaded now so the update at the end waits for
  // nothing
  const uint4 knew = ld16(knb + min(tid * 8, HD - 8));
  const uint4 vnew = ld16(vnb + min(tid * 8, HD - 8));
  uint4 kreg[LPT], vreg[LPT];
  auto fetch = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + i * 256;
      const int j = t0 + c / CPR, d = (c % CPR) * 8;
      const bool ring = j < slot_hi, fresh = j == slot_hi && j < ke;
      const int64_t roff = (int64_t)j * a.hd + d;
      kreg[i] = ld16(ring && j < ke ? ckb + roff : fresh ? knb + d : zpage);
      vreg[i] = ld16(ring && j < ke ? cvb + roff : fresh ? vnb + d : zpage);
    }
  };
  fetch(kb);
  bf16x8 qf[KS];
  {
    const int hrow = lane & 15;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 32 + 8 * (lane >> 4);
      qf[ks] = __builtin_bit_cast(
          bf16x8, ld16(hrow < a.H ? a.q + (int64_t)b * a.H * a.hd + hrow * a.hd + d : zpage));
    }
  }
  f32x4 o[NO];
#pragma unroll
  for (int j = 0; j < NO; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_run[r] = -INFINITY;
    l_run[r] = 0.0f;
  }
  const uint32_t vlds = (uint32_t)(uintptr_t)vs_;
  // transposed-read addresses: lane 4q+p of a 16-lane group reads key row
  // q of its 4-row block, dims 4p..4p+3 of the 16-dim column block
  const int tq = (lane & 15) >> 2, tp = lane & 3, g = lane >> 4;
  for (int t0 = kb; t0 < ke; t0 += KT) {
    __syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + i * 256;
      const int kr = c / CPR, ch = c % CPR;
      ks_[kr * CPR + swz<CPR>(ch, kr)] = kreg[i];
      vs_[kr * CPR + (ch ^ vswz<CPR>(kr))] = vreg[i];
    }
    __syncthreads();
    if (t0 + KT < ke) fetch(t0 + KT);
    const int nblk = min(4, (ke - t0 + 15) / 16);   // live 16-key blocks
    f32x4 s[4];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      s[jn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (jn >= nblk) continue;
      const int kr = jn * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = ks * 4 + (lane >> 4);
        const bf16x8 kf = __builtin_bit_cast(bf16x8, ks_[kr * CPR + swz<CPR>(ch, kr)]);
        s[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, s[jn], 0, 0, 0);
      }
    }
    float p[4][4], tmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tmax[r] = -INFINITY;
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      const int j = t0 + jn * 16 + (lane & 15);
      // _compute_cache_mask: slot positions from num_tokens; j == slot_hi
      // is the new key at the query's own position
      int kpos;
      if (j < slot_hi) {
        const int now = j + kblk * a.W;
        kpos = now < nt ? now : j + (kblk - 1) * a.W;
      } else {
        kpos = qpos;
      }
      const bool ok = j < ke && kpos >= 0 && qpos >= kpos && qpos <= kpos + a.W;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = ok ? rbf(s[jn][r]) * a.scale : -INFINITY;
        p[jn][r] = v;
        tmax[r] = fmaxf(tmax[r], v);
      }
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t = tmax[r];
      t = row16_max(t);
      const float mn = fmaxf(m_run[r], t);
      alpha[r] = (mn == -INFINITY) ? 1.0f : expf(m_run[r] - mn);
      float rs = 0.0f;
#pragma unroll
      for (int jn = 0; jn < 4; ++jn) {
        const float e = (mn == -INFINITY) ? 0.0f : expf(p[jn][r] - mn);
        p[jn][r] = e;
        rs += e;
      }
      rs = row16_sum(rs);
      l_run[r] = l_run[r] * alpha[r] + rs;
      m_run[r] = mn;
    }
#pragma unroll
    for (int j = 0; j < NO; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= alpha[r];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pt[(4 * (lane >> 4) + r) * KT + jn * 16 + (lane & 15)] = f2bf(p[jn][r]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // O += P . V over each live 32-key half: P fragment (head row, keys
    // 32 kk + 8 g ..), V^T fragment by two transposed reads (keys 32 kk +
    // 8 g + {0..3} and {4..7}, dims of this wave's column block)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk * 32 >= nblk * 16) continue;
      const bf16x8 pf = __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(pt + (lane & 15) * KT + kk * 32 + 8 * g));
      const int r1 = kk * 32 + 8 * g + tq, r2 = r1 + 4;
#pragma unroll
      for (int j = 0; j < NO; ++j) {
        const int ch = (dbase + j * 16) / 8 + (tp >> 1);
        const uint32_t a1 = vlds + (r1 * CPR + (ch ^ vswz<CPR>(r1))) * 16 + 8 * (tp & 1);
        const uint32_t a2 = vlds + (r2 * CPR + (ch ^ vswz<CPR>(r2))) * 16 + 8 * (tp & 1);
        uint2 w1, w2;
        asm volatile(
            "ds_read_b64_tr_b16 %0, %2\n"
            "ds_read_b64_tr_b16 %1, %3\n"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(w1), "=&v"(w2)
            : "v"(a1), "v"(a2)
            : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(w1.x, w1.y, w2.x, w2.y));
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[j], 0, 0, 0);
      }
    }
  }
  if (nsp == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hrow = 4 * (lane >> 4) + r;
      if (hrow >= a.H) continue;
      const float inv = l_run[r] > 0.0f ? 1.0f / l_run[r] : 0.0f;
#pragma unroll
      for (int j = 0; j < NO; ++j) {
        const int d = dbase + j * 16 + (lane & 15);
        a.o[xoff(b, hrow * a.hd + d, a.ldo, a.omt)] = f2bf(o[j][r] * inv);
      }
    }
  } else {
    constexpr int PS = 32 + 16 * HD;            // floats per split partial
    float* part = a.parts + ((int64_t)b * NS + split) * PS;
    float* stage = reinterpret_cast<float*>(ks_);   // [16][HD] fp32 <= sizeof(ks_)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hrow = 4 * (lane >> 4) + r;
#pragma unroll
      for (int j = 0; j < NO; ++j)
        stage[hrow * HD + dbase + j * 16 + (lane & 15)] = o[j][r];
      if (wave == 0 && (lane & 15) == 0) {
        ml[hrow] = m_run[r];
        ml[16 + hrow] = l_run[r];
      }
    }
    __syncthreads();
    // m, l of all 16 rows, o of the H real head rows
    for (int q = tid * 4; q < 32 + a.H * HD; q += 1024) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(q < 32 ? ml + q : stage + (q - 32));
      float* dst = part + q;
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(dst), "v"(v) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      ticket = __hip_atomic_fetch_add(&a.sems[b], 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (ticket != nsp - 1) return;
    const float* pb = a.parts + (int64_t)b * NS * PS;
    // One memory round trip for up to 8 ranges: every range's (m, l) rows go
    // through LDS (one load per thread), and each thread's float4 chunks of
    // the H x HD output (up to HD / 64 per thread) of all 8
    // ranges are loaded with 16-B write-through-side (sc1) loads before the
    // first use; ranges past 8 (only B <= 16) take another trip per 8.
    constexpr int GS = 8, QP = HD / 64;   // QP x 256 float4 >= 16 heads x HD
    const int nq = a.H * HD / 4;
    // the running rescale's factors depend on (head row, range) only: one
    // lane per head row walks the ranges once (the same operations in the
    // same order as a per-element walk, so the same bits) and every thread
    // applies them -- per-thread, the walk cost 2 expf per (chunk, range),
    // 3.5-5 us of the combine at B = 32 (profiles/r06v_decode_attn_phases/)
    __shared__ float2 fac[kDecodeSplitsMax * 16];   // (scale of the sum so far, of range u)
    __shared__ float lfin[16];
    f32x4 acc[QP];
#pragma unroll
    for (int p = 0; p < QP; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int idx = tid; idx < nsp * 32; idx += 256)
      mls[idx] = __hip_atomic_load(pb + (idx >> 5) * PS + (idx & 31), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    for (int s0 = 0; s0 < nsp; s0 += GS) {
      f32x4 w[QP][GS];
#pragma unroll
      for (int p = 0; p < QP; ++p)
#pragma unroll
        for (int u = 0; u < GS; ++u) {
          const int c = min(tid + 256 * p, nq - 1);
          const float* src = pb + min(s0 + u, nsp - 1) * PS + 32 + 4 * c;
          asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(w[p][u]) : "v"(src)
                       : "memory");
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // the (m, l) rows are in LDS
      if (s0 == 0) {
        if (tid < 16) {
          // running rescale in range order, head row tid
          float mx = -INFINITY, l = 0.0f;
          for (int u = 0; u < nsp; ++u) {
            const float mu = mls[u * 32 + tid], lu = mls[u * 32 + 16 + tid];
            const float mn = fmaxf(mx, mu);
            const float sa = mx == -INFINITY ? 0.0f : expf(mx - mn);
            const float sb = mu == -INFINITY ? 0.0f : expf(mu - mn);
            l = l * sa + lu * sb;
            fac[u * 16 + tid] = make_float2(sa, sb);
            mx = mn;
          }
          lfin[tid] = l;
        }
        __syncthreads();
      }
#pragma unroll
      for (int p = 0; p < QP; ++p) {
        const int hrow = min(tid + 256 * p, nq - 1) * 4 / HD;
#pragma unroll
        for (int u = 0; u < GS; ++u) {
          if (s0 + u >= nsp) continue;
          const float2 f = fac[(s0 + u) * 16 + hrow];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[p][e] = acc[p][e] * f.x + w[p][u][e] * f.y;
        }
      }
    }
#pragma unroll
    for (int p = 0; p < QP; ++p) {
      const int c = tid + 256 * p;
      if (c >= nq) continue;
      const float lp = lfin[c * 4 / HD];
      const float inv = lp > 0.0f ? 1.0f / lp : 0.0f;
      u16* dst = a.o + xoff(b, 4 * c, a.ldo, a.omt);
      const uint32_t lo = (uint32_t)f2bf(acc[p][0] * inv) | ((uint32_t)f2bf(acc[p][1] * inv) << 16);
      const uint32_t hi = (uint32_t)f2bf(acc[p][2] * inv) | ((uint32_t)f2bf(acc[p][3] * inv) << 16);
      *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
    }
    if (tid == 0)
      __hip_atomic_store(&a.sems[b], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // _update_attention_cache: write the new key/value into slot nt % W, then
  // bump num_tokens (all reads of this sequence's cache are done: with NS > 1
  // every range has arrived before the last one gets here).
  __syncthreads();
  const int slot = nt % a.W;
  if (tid * 8 < HD) {
    st16(a.ck + ((int64_t)b * a.W + slot) * a.hd + tid * 8, knew);
    st16(a.cv + ((int64_t)b * a.W + slot) * a.hd + tid * 8, vnew);
  }
  if (tid == 0) a.num_tokens[b] = nt + 1;
}

// ------------------------------------------------------------------- RoPE

// sin / cos table (common.hpp rope_sincos) for positions [0, P).
__global__ __launch_bounds__(256) void rope_table_kernel(u16* __restrict__ t,
                                                         int P, int hd) {
  const int quarter = hd / 4, half = hd / 2;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < (int64_t)P * quarter;
       idx += (int64_t)gridDim.x * 256) {
    const int p = idx / quarter, i = idx % quarter;
    float sn, cs;
    rope_sincos(p, i, half, sn, cs);
    t[((int64_t)p * 2) * quarter + i] = f2bf(sn);
    t[((int64_t)p * 2 + 1) * quarter + i] = f2bf(cs);
  }
}

// One thread: 8 rotation pairs (16-B loads) of one head of one row, plus
// the matching 16 pass-through dims.  Heads 0..H-1 are queries, head H is
// the key; v is copied by head H's threads.
__global__ __launch_bounds__(256) void rope_qkv_kernel(
    const u16* __restrict__ qkv, int64_t ld, const int32_t* __restrict__ pos,
    u16* __restrict__ qo, u16* __restrict__ ko, u16* __restrict__ vo, int64_t M,
    int H, int hd, const u16* __restrict__ table, int table_len) {
  const int half = hd / 2, quarter = hd / 4;  // rope dims, pairs
  const int cpq = quarter / 8;                // threads per head
  const int64_t total = M * (H + 1) * cpq;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % cpq;
    const int64_t mh = idx / cpq;
    const int hh = mh % (H + 1);
    const int64_t m = mh / (H + 1);
    const u16* src = qkv + m * ld + hh * hd;
    u16* dst = hh < H ? qo + m * (int64_t)H * hd + hh * hd : ko + m * hd;
    const int i0 = c * 8;
    // every load independent of the position issued first: the rotated
    // pair, this thread's 16 pass-through dims (hd / 2 / cpq == 16 for
    // every hd) and, for the K head, its 32 dims of V (hd / cpq == 32)
    const int p = pos[m];
    const uint4 r1 = ld16(src + i0), r2 = ld16(src + quarter + i0);
    const int pt0 = half + c * 16;
    const uint4 pt[2] = {ld16(src + pt0), ld16(src + pt0 + 8)};
    uint4 vv[4];
    const u16* vs = qkv + m * ld + (H + 1) * hd + c * 32;
    if (hh == H) {
#pragma unroll
      for (int j = 0; j < 4; ++j) vv[j] = ld16(vs + 8 * j);
    }
    float x1[8], x2[8];
    float sn[8], cs[8];
    if (p >= 0 && p < table_len) {
      unpack8(ld16(table + ((int64_t)p * 2) * quarter + i0), sn);
      unpack8(ld16(table + ((int64_t)p * 2 + 1) * quarter + i0), cs);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) rope_sincos(p, i0 + i, half, sn[i], cs[i]);
    }
    unpack8(r1, x1);
    unpack8(r2, x2);
    float o1[8], o2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o1[i] = bsub(bmul(x1[i], cs[i]), bmul(x2[i], sn[i]));
      o2[i] = badd(bmul(x2[i], cs[i]), bmul(x1[i], sn[i]));
    }
    st16(dst + i0, pack8(o1));
    st16(dst + quarter + i0, pack8(o2));
    st16(dst + pt0, pt[0]);
    st16(dst + pt0 + 8, pt[1]);
    if (hh == H) {
#pragma unroll
      for (int j = 0; j < 4; ++j) st16(vo + m * hd + c * 32 + 8 * j, vv[j]);
    }
  }
}

// KV cache from the prompt: slot (i + num_tokens) % W <- key L - w + i.
__global__ __launch_bounds__(256) void kv_fill_kernel(
    const u16* __restrict__ k, const u16* __restrict__ v,
    const int32_t* __restrict__ pos, u16* __restrict__ ck, u16* __restrict__ cv,
    int32_t* __restrict__ ntok, int B, int L, int hd, int W) {
  const int cpr = hd / 8;
  const int64_t total = (int64_t)B * W * cpr;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % cpr;
    const int64_t bs = idx / cpr;
    const int slot = bs % W, b = bs / W;
    const int nt = pos[(int64_t)b * L + L - 1] + 1;
    const int w = L < W ? L : W;
    // rolled[slot] = keys_tail[(slot - shift) mod w] for slot < w, else 0
    uint4 kv = make_uint4(0, 0, 0, 0), vv = kv;
    if (slot < w) {
      const int shift = ((nt % W) + W) % W;
      int src = (slot - shift) % w;
      if (src < 0) src += w;
      const int64_t row = (int64_t)b * L + (L - w) + src;
      kv = ld16(k + row * hd + c * 8);
      vv = ld16(v + row * hd + c * 8);
    }
    st16(ck + ((int64_t)b * W + slot) * hd + c * 8, kv);
    st16(cv + ((int64_t)b * W + slot) * hd + c * 8, vv);
    if (slot == 0 && c == 0) ntok[b] = nt;
  }
}

int grid_cap(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

template <int HD, int MODE>
void launch_flash(const AttnArgs& a, int B, hipStream_t st) {
  dim3 grid((unsigned)((a.L + 63) / 64), (unsigned)a.H, (unsigned)B);
  hipLaunchKernelGGL((flash_attn_kernel<HD, MODE>), grid, dim3(256), 0, st, a);
}

}  // namespace

extern "C" {

int cadence_rope_qkv(const void* qkv, int64_t ldqkv, const int32_t* positions,
                     void* q_out, void* k_out, void* v_out, int64_t M,
                     int64_t H, int64_t hd, const void* table,
                     int64_t table_len, void* stream) {
  if (hd % 64)   // head dims the vectorised kernel does not tile
    return rope_qkv_generic_launch(qkv, ldqkv, positions, q_out, k_out, v_out,
                                   M, H, hd, stream);
  if (ldqkv % 8) return (int)hipErrorInvalidValue;
  if (M <= 0) return 0;
  const int cpq = (int)(hd / 4 / 8);
  hipLaunchKernelGGL(rope_qkv_kernel, dim3(grid_cap(M * (H + 1) * cpq)), dim3(256),
                     0, static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(qkv), ldqkv, positions,
                     static_cast<u16*>(q_out), static_cast<u16*>(k_out),
                     static_cast<u16*>(v_out), M, (int)H, (int)hd,
                     static_cast<const u16*>(table), table ? (int)table_len : 0);
  return (int)hipGetLastError();
}

int cadence_rope_table(void* table, int64_t positions, int64_t hd,
                       void* stream) {
  if (hd % 64 || positions <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rope_table_kernel, dim3(grid_cap(positions * (hd / 4))),
                     dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<u16*>(table), (int)positions, (int)hd);
  return (int)hipGetLastError();
}

int cadence_local_attention(const void* q, const void* k, const void* v,
                            const int32_t* seg_id, const int32_t* seg_start,
                            void* out, int64_t B, int64_t L, int64_t H,
                            int64_t hd, int64_t window, void* stream) {
  if (hd != 256 && hd != 128 && hd != 64)      // any other head dim
    return generic_attention_launch(q, k, v, nullptr, nullptr, nullptr,
                                    seg_start, out, B, L, H, hd, window, stream);
  if (B <= 0 || L <= 0) return 0;
  // MQA workgroups (all heads per K/V tile, griffin_attention.hip) where
  // they apply; the per-head streaming kernel otherwise
  {
    const int rc = griffin_attention_launch(q, k, v, seg_start, out, B, L, H,
                                            hd, window, stream);
    if (rc >= 0) return rc;
  }
  AttnArgs a{};
  a.q = static_cast<const u16*>(q); a.q_bs = L * H * hd; a.q_rs = H * hd; a.q_hs = hd;
  a.k = static_cast<const u16*>(k); a.k_bs = L * hd; a.k_rs = hd; a.k_hs = 0;
  a.v = static_cast<const u16*>(v); a.v_bs = L * hd; a.v_rs = hd; a.v_hs = 0;
  a.o = static_cast<u16*>(out); a.o_bs = L * H * hd; a.o_rs = H * hd; a.o_hs = hd;
  a.seg = seg_id; a.seg_start = seg_start;
  a.L = (int)L; a.H = (int)H; a.hd = (int)hd; a.window = (int)window;
  a.scale = 1.0f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hd == 256) launch_flash<256, MODE_LOCAL>(a, (int)B, st);
  else if (hd == 128) launch_flash<128, MODE_LOCAL>(a, (int)B, st);
  else launch_flash<64, MODE_LOCAL>(a, (int)B, st);
  return (int)hipGetLastError();
}

// The ViT attention plan: the streaming kernel with MFMA-computed softmax
// sums (vit_flash.hip) for every shape but DINO's 224-px one (N = 261, hd
// 64), where the LDS-resident kernel is faster (25.7 vs 29.2 us at bs 32;
// SigLIP 224 px 24.4 vs 28.7, 336 px 78 / 86 vs 97 / 112:
// profiles/r04g_vit_flash_ab.log); with the lab switch's bit 3 clear, the
// round-3 kernels (LDS-resident up to 288 tokens, streaming above).
static int vit_plan(int64_t N, int64_t hd) {
  if ((hd != 64 && hd != 72) || N <= 0) return -1;
  if ((cadence_engine_bits() & 8) && !(hd == 64 && N <= 288)) return 2;
  if (N <= 288) return 0;
  return 1;
}

int cadence_vit_attention_kernel(int64_t N, int64_t hd) { return vit_plan(N, hd); }

int cadence_vit_attention(const void* qkv, void* out, int64_t B, int64_t N,
                          int64_t H, int64_t hd, void* stream) {
  if (hd != 64 && hd != 72) return (int)hipErrorInvalidValue;
  if (B <= 0 || N <= 0) return 0;
  if (vit_plan(N, hd) == 2) {
    const int rc = vit_flash_attention_launch(qkv, out, B, N, H, hd, stream);
    if (rc >= 0) return rc;
  }
  // LDS-resident swapped-QK^T kernel (vit_attention.hip) for short sequences
  {
    const int rc = vit_attention_lds_launch(qkv, out, B, N, H, hd, stream);
    if (rc >= 0) return rc;
  }
  // longer sequences (336 / 384 px towers): K/V tiles streamed by LDS-DMA;
  // it takes every shape but a qkv / out pointer that is not 16-B aligned,
  // which the contract excludes (cadence_kernels.h)
  const int rc = vit_stream_attention_launch(qkv, out, B, N, H, hd, stream);
  return rc >= 0 ? rc : (int)hipErrorInvalidValue;
}

int cadence_kv_cache_fill(const void* k, const void* v,
                          const int32_t* segment_pos, void* cache_k,
                          void* cache_v, int32_t* num_tokens, int64_t B,
                          int64_t L, int64_t hd, int64_t window, void* stream) {
  if (hd % 8) return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  hipLaunchKernelGGL(kv_fill_kernel, dim3(grid_cap(B * window * (hd / 8))), dim3(256),
                     0, static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(k), static_cast<const u16*>(v),
                     segment_pos, static_cast<u16*>(cache_k),
                     static_cast<u16*>(cache_v), num_tokens, (int)B, (int)L,
                     (int)hd, (int)window);
  return (int)hipGetLastError();
}

int64_t cadence_local_attention_decode_workspace_bytes(int64_t B, int64_t hd) {
  return B * decode_splits(B) * (32 + 16 * hd) * 4;
}

int cadence_local_attention_decode(const void* q, const void* k_new,
                                   const void* v_new, void* cache_k,
                                   void* cache_v, int32_t* num_tokens,
                                   void* out, int64_t ld_out, int64_t B, int64_t H,
                                   int64_t hd, int64_t window, void* workspace,
                                   int64_t ws_bytes, int32_t* sems, void* stream) {
  if ((hd != 256 && hd != 128 && hd != 64) || H > 16)
    return (int)hipErrorInvalidValue;
  if (ld_out == 0 && B > 32) return (int)hipErrorInvalidValue;   // packed rows
  if (ld_out != 0 && ld_out < H * hd) return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  const bool split = workspace && sems &&
                     ws_bytes >= cadence_local_attention_decode_workspace_bytes(B, hd);
  DecodeArgs a{static_cast<const u16*>(q), static_cast<const u16*>(k_new),
               static_cast<const u16*>(v_new), hd,
               static_cast<u16*>(cache_k), static_cast<u16*>(cache_v),
               num_tokens, static_cast<u16*>(out), ld_out, (int)((B + 15) / 16),
               (int)H, (int)hd,
               (int)window, 1.0f / sqrtf((float)hd),
               static_cast<float*>(workspace), sems, kDecodeMinRange};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)B, split ? decode_splits(B) : 1);
  if (hd == 256)
    hipLaunchKernelGGL(decode_attn_kernel<256>, grid, dim3(256), 0, st, a);
  else if (hd == 128)
    hipLaunchKernelGGL(decode_attn_kernel<128>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(decode_attn_kernel<64>, grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

}  // extern "C"
