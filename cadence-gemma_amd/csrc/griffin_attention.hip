// Griffin local multi-query attention, prefill (recurrentgemma/torch/
// modules.py:402-483 with the mask of :90-152) on gfx950.
//
// MQA: all H query heads read the one K/V head, so a workgroup takes 16
// queries of one sequence with ALL heads -- wave w = head w -- and every
// K / V tile it stages is used H times (the per-head streaming kernel staged
// each K/V tile once per head).  Key tiles of 64 keys stream through two
// LDS buffers by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no
// ds_write); the next tile's DMA is in flight while the current one is
// computed, one workgroup barrier per tile.
//
// Per wave (one head, 16 queries), "swapped" QK^T as in vit_attention.hip:
// S^T = K . Q^T on mfma_f32_16x16x32_bf16, so a lane owns ONE query and
// four keys of each 16-key group; the score tile is directly the B operand
// of O^T = V^T . P^T under the key-slot permutation
//   slot 8g + j  <->  key 4g + j (j < 4),  16 + 4g + (j - 4) (j >= 4),
// and the V^T operand comes from the row-major V image by two
// ds_read_b64_tr_b16 per fragment (4 keys x 16 dims each, transposed by the
// LDS), so V needs no transposing write pass.
//
// LDS images (512-B rows of 32 16-B chunks, swizzled through the per-lane
// DMA source address, XOR being an involution):
//   K: chunk c of key row r at slot c ^ (r & 15)  -- the ds_read_b128 groups
//      of an A-fragment read are conflict-free;
//   V: chunk c of key row r at slot c ^ ((r & 7) << 1) -- the 32-lane halves
//      of a transposed read touch 8 rows x 2 chunks at 16 distinct slots.
//
// Mask (modules.py:90-152): key k is visible to query q iff
//   max(seg_start(q), q - W) <= k <= q
// (same segment = same run of positions since the last 0; window: q <= k +
// W).  Logits are rounded to bf16 before the exact * hd^-1/2 (the
// reference's bf16 einsum), softmax in fp32 (exp2, scale folded in), P in
// bf16, online over tiles with a deferred rescale.  Only tiles that straddle
// a bound carry masking code; a masked key (-inf) weighs exactly 0, also
// while its query has no visible key yet (running max -inf).
#include <type_traits>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef const void __attribute__((address_space(1)))* ga_gptr_t;
typedef void __attribute__((address_space(3)))* ga_lptr_t;

constexpr int GA_KT = 64;      // keys per tile
constexpr int GA_QB = 16;      // queries per workgroup
constexpr int GA_MAXW = 10;    // waves (= heads) per workgroup, at most

// Compiler-visible maxes (not inline asm): the hazard recognizer must see
// these reads of fresh MFMA results and the permlane reads of their outputs
// (an asm VALU reading an MFMA's D within ~12 wait states reads stale
// accumulators -- seen as run-to-run output differences in the ViT kernel).
CADENCE_DEV float ga_max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
CADENCE_DEV float ga_max2(float a, float b) { return __builtin_fmaxf(a, b); }
// max over lanes l, l ^ 16, l ^ 32, l ^ 48 (the four key groups of a query)
CADENCE_DEV float ga_max_rows(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float m = ga_max2(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const uint32_t w = __float_as_uint(m);
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return ga_max2(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
CADENCE_DEV uint32_t ga_pk2bf(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

struct GAArgs {
  const u16* q;               // [B*L, H*HD] (RoPE applied)
  const u16* k;               // [B*L, HD]
  const u16* v;               // [B*L, HD]
  const int32_t* seg_start;   // [B*L] first index of each row's segment
  u16* o;                     // [B*L, H*HD]
  int B, L, H, W;
  float scale_log2;           // log2(e) / sqrt(HD)
};

template <int HD>
__global__ __launch_bounds__(GA_MAXW * 64) void griffin_attn_kernel(GAArgs a) {
  constexpr int CPR = HD / 8;          // 16-B chunks per K / V row
  constexpr int KS = HD / 32;          // k-steps of S^T
  constexpr int NDT = HD / 16;         // 16-dim tiles of O^T
  constexpr int TILE = GA_KT * CPR;    // uint4 per image (K or V) of a tile
  constexpr int NDMA = 2 * TILE / 64;  // 1-KiB DMA pieces per tile (K then V)
  static_assert(CPR == 32, "the LDS swizzles assume 512-B rows");
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * 2 * TILE];   // [buf][K|V]

  const int nw = blockDim.x >> 6;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;

  // XCD-aware, longest-first order: consecutive dispatch indices go to
  // consecutive XCDs, so remap bijectively to give each XCD a contiguous
  // range of (sequence, query block) pairs (the blocks of a sequence share
  // its K / V rows in that XCD's L2), walking query blocks from the last
  // (the most keys under the causal mask) to the first.
  const int nqb = (a.L + GA_QB - 1) / GA_QB;
  int b, qb;
  {
    const int total = gridDim.x;
    const int lin = blockIdx.x;
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int p = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    b = p / nqb;
    qb = nqb - 1 - p % nqb;
  }
  const int q0 = qb * GA_QB;
  const int64_t row0 = (int64_t)b * a.L;
  const int qi = min(q0 + c16, a.L - 1);        // rows past L: computed, not stored
  const int lo = max(a.seg_start[row0 + qi], qi - a.W);
  // bounds over the 16 queries (the c16 lanes of each 16-lane group)
  int lo_min = lo, lo_max = lo;
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    lo_min = min(lo_min, __shfl_xor(lo_min, off, 64));
    lo_max = max(lo_max, __shfl_xor(lo_max, off, 64));
  }
  const int q_last = min(q0 + GA_QB - 1, a.L - 1);
  const int kbeg = lo_min & ~(GA_KT - 1);
  const int ntiles = (q_last + 1 - kbeg + GA_KT - 1) / GA_KT;

  // DMA sources of this wave's pieces: piece i covers key rows 2i, 2i+1 of
  // the K image (i < TILE/64) or the V image; lane l writes row 2i + l/32,
  // slot l%32, so it loads the chunk that slot holds under the swizzle
  const int dma_row = lane >> 5, dma_slot = lane & 31;
  auto stage = [&](int t, int buf) {
    uint4* kdst = smem + (buf * 2) * TILE;
    uint4* vdst = smem + (buf * 2 + 1) * TILE;
    const int c0 = kbeg + t * GA_KT;
    for (int i = wave; i < NDMA; i += nw) {
      const bool isv = i >= TILE / 64;
      const int pi = isv ? i - TILE / 64 : i;
      const int r = 2 * pi + dma_row;
      const int ch = isv ? (dma_slot ^ ((r & 7) << 1)) : (dma_slot ^ (r & 15));
      const int key = min(c0 + r, a.L - 1);    // past L: masked (key > q)
      const u16* src = (isv ? a.v : a.k) + (row0 + key) * HD + ch * 8;
      uint4* dst = (isv ? vdst : kdst) + pi * 64;
      __builtin_amdgcn_global_load_lds((ga_gptr_t)src, (ga_lptr_t)dst, 16, 0, 0);
    }
  };
  stage(0, 0);

  // Q^T fragments of this head: B[k = dim 32 ks + 8 g + i][n = query c16]
  const int h = wave;
  bf16x8 qf[KS];
  {
    const u16* qrow = a.q + (row0 + qi) * (int64_t)a.H * HD + (int64_t)h * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[ks] = __builtin_bit_cast(bf16x8, ld16(qrow + ks * 32 + 8 * g));
  }
  f32x4 o[NDT];
#pragma unroll
  for (int j = 0; j < NDT; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;
  constexpr float kThr = 8.0f;        // deferred rescale (see vit_attention.hip)

  __syncthreads();                    // tile 0 landed (each wave's vmcnt) for all
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) stage(t + 1, buf ^ 1);
    const int c0 = kbeg + t * GA_KT;
    const uint4* kimg = smem + (buf * 2) * TILE;
    const uint32_t vlds = (uint32_t)(uintptr_t)(smem + (buf * 2 + 1) * TILE);
    // S^T = K . Q^T: s[tt][r] = S[key c0 + 16 tt + 4 g + r][query q0 + c16]
    // K fragments QG k-steps at a time, each group read before its MFMAs
    // (one LDS wait per group; the compiler otherwise waits per fragment)
    constexpr int QG = 2;
    f32x4 s[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      s[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = 16 * tt + c16;
#pragma unroll
      for (int k0 = 0; k0 < KS; k0 += QG) {
        bf16x8 kf[QG];
#pragma unroll
        for (int u = 0; u < QG; ++u)
          kf[u] = __builtin_bit_cast(bf16x8, kimg[kr * CPR + ((4 * (k0 + u) + g) ^ (kr & 15))]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < QG; ++u)
          s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[u], qf[k0 + u], s[tt], 0, 0, 0);
      }
    }
    // logits: bf16-rounded dot (the scale 2^-k is exact), masked where the
    // tile straddles a bound of any of the 16 queries
    const bool full = c0 >= lo_max && c0 + GA_KT - 1 <= q0;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = rbf(s[tt][r]);
        if (!full) {
          const int key = c0 + 16 * tt + 4 * g + r;
          if (key < lo || key > qi) v = -INFINITY;
        }
        s[tt][r] = v;
      }
    float smax = ga_max3(s[0][0], s[0][1], s[0][2]);
    smax = ga_max3(smax, s[0][3], s[1][0]);
    smax = ga_max3(smax, s[1][1], s[1][2]);
    smax = ga_max3(smax, s[1][3], s[2][0]);
    smax = ga_max3(smax, s[2][1], s[2][2]);
    smax = ga_max3(smax, s[2][3], s[3][0]);
    smax = ga_max3(smax, s[3][1], s[3][2]);
    smax = ga_max2(smax, s[3][3]);
    smax = ga_max_rows(smax);
    const float mt = smax * a.scale_log2;
    const bool need = mt > m + kThr;
    if (__any(need)) {
      const float mn = need ? mt : m;
      // rows that do not rescale keep alpha 1 (exp2(m - m) is NaN while a
      // row has no visible key yet, m = -inf); m = -inf -> mn: alpha 0
      const float alpha = need ? __builtin_amdgcn_exp2f(m - mn) : 1.0f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
      l *= alpha;
      m = mn;
    }
    // a row with no visible key so far (m = -inf) exponentiates against 0:
    // its masked scores (-inf) give exactly 0, and it has no finite score
    const float nm = m == -INFINITY ? 0.0f : -m;
    bf16x8 pf[2];
    float ps0 = 0.0f, ps1 = 0.0f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int tt = 2 * kk + (j >> 2), r = j & 3;
        const float e0 = __builtin_amdgcn_exp2f(fmaf(s[tt][r], a.scale_log2, nm));
        const float e1 = __builtin_amdgcn_exp2f(fmaf(s[tt][r + 1], a.scale_log2, nm));
        ps0 += e0;
        ps1 += e1;
        pk[j >> 1] = ga_pk2bf(f32x2{e0, e1});
      }
      pf[kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    }
    l += ps0 + ps1;
    // O^T += V^T . P^T: the V^T fragment of dims 16 dt.., keys (slot order)
    // 32 kk + {4g..4g+3, 16+4g..16+4g+3}: two transposed 4 x 16 reads; lane
    // 4q+p addresses key row q of the block, dims 4p..4p+3.  The reads are
    // inline asm with their own lgkmcnt wait: the compiler's builtin for
    // them is followed by a vmcnt(0) (it waits for the next tile's DMA).
    const int tq = c16 >> 2, tp = c16 & 3;
    // software-pipelined: the four reads of step s + 1 go out before step
    // s's MFMAs, and a counted wait (LDS returns in order) retires only step
    // s's -- one LDS latency per tile instead of one per two dim tiles
    constexpr int NSTEP = 2 * (NDT / 2);    // (key half, dim-tile pair)
    auto vaddr = [&](int step, uint32_t (&ad)[4]) {
      const int kk = step / (NDT / 2), d0 = 2 * (step % (NDT / 2));
      const int r1 = 32 * kk + 4 * g + tq, r2 = r1 + 16;
      const uint32_t a1 = vlds + r1 * 512 + 8 * (tp & 1);
      const uint32_t a2 = vlds + r2 * 512 + 8 * (tp & 1);
      const int x1 = (r1 & 7) << 1, x2 = (r2 & 7) << 1;
      const int ch0 = 2 * d0 + (tp >> 1), ch1 = ch0 + 2;
      ad[0] = a1 + 16 * (ch0 ^ x1);
      ad[1] = a2 + 16 * (ch0 ^ x2);
      ad[2] = a1 + 16 * (ch1 ^ x1);
      ad[3] = a2 + 16 * (ch1 ^ x2);
    };
    // step s + 1's reads and step s's counted wait are ONE asm statement
    // (outputs: the new registers; in/out: the pending ones), so no
    // compiler-placed copy of a still-loading register can sit between them
    uint2 wv[2][4];
    {
      uint32_t ad[4];
      vaddr(0, ad);
      asm volatile(
          "ds_read_b64_tr_b16 %0, %4\n"
          "ds_read_b64_tr_b16 %1, %5\n"
          "ds_read_b64_tr_b16 %2, %6\n"
          "ds_read_b64_tr_b16 %3, %7"
          : "=&v"(wv[0][0]), "=&v"(wv[0][1]), "=&v"(wv[0][2]), "=&v"(wv[0][3])
          : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3])
          : "memory");
    }
#pragma unroll
    for (int step = 0; step < NSTEP; ++step) {
      uint2 (&cur)[4] = wv[step & 1];
      if (step + 1 < NSTEP) {
        uint2 (&nx)[4] = wv[(step + 1) & 1];
        uint32_t ad[4];
        vaddr(step + 1, ad);
        asm volatile(
            "ds_read_b64_tr_b16 %0, %8\n"
            "ds_read_b64_tr_b16 %1, %9\n"
            "ds_read_b64_tr_b16 %2, %10\n"
            "ds_read_b64_tr_b16 %3, %11\n"
            "s_waitcnt lgkmcnt(4)"
            : "=&v"(nx[0]), "=&v"(nx[1]), "=&v"(nx[2]), "=&v"(nx[3]),
              "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3])
            : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3])
            : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3])
                     :
                     : "memory");
      }
      const int kk = step / (NDT / 2), d0 = 2 * (step % (NDT / 2));
      // cur[0] / cur[1]: dims of d0 (rows r1 / r2), cur[2] / cur[3]: d0 + 1
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16x8 vf = __builtin_bit_cast(
            bf16x8, make_uint4(cur[2 * u].x, cur[2 * u].y, cur[2 * u + 1].x, cur[2 * u + 1].y));
        o[d0 + u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[kk], o[d0 + u], 0, 0, 0);
      }
    }
    __syncthreads();   // this wave's DMA landed (vmcnt) + every wave done with buf
  }

  // out[q][h*HD + d]: lane holds dims 16 dt + 4 g + 0..3 of query q0 + c16
  float lt = l;
  lt += __shfl_xor(lt, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float inv = lt > 0.0f ? 1.0f / lt : 0.0f;
  if (q0 + c16 < a.L) {
    u16* orow = a.o + (row0 + q0 + c16) * (int64_t)a.H * HD + (int64_t)h * HD;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const uint32_t lo2 = ga_pk2bf(f32x2{o[dt][0] * inv, o[dt][1] * inv});
      const uint32_t hi2 = ga_pk2bf(f32x2{o[dt][2] * inv, o[dt][3] * inv});
      *reinterpret_cast<uint2*>(orow + dt * 16 + 4 * g) = make_uint2(lo2, hi2);
    }
  }
}

// ------------------------------------------------ ViT, long sequences
//
// timm bidirectional SDPA (dino_siglip.py:85-86,149-151 via timm Attention)
// for the towers at 336 / 384 px (N = 576..734 tokens), where the whole K /
// V^T of a head no longer fits the LDS-resident kernel of vit_attention.hip.
// Same tile machinery as griffin_attn_kernel: K / V tiles of 64 keys by
// LDS-DMA into two buffers, swapped QK^T, V^T fragments by transposed LDS
// reads.  One workgroup = (image, head, 128 queries): wave w takes query
// tile w (16 queries); K and V of the head are read once per workgroup.
// Rows are padded to 16 chunks (128 dims): hd 64 uses chunks 0-7; hd 72
// uses 9 real chunks, and the k-step / dim-tile padding (chunks 9-11 of K,
// 9 of V) is DMA'd from chunk 8 of the same row -- finite, multiplied by a
// zero Q fragment, or landing in output dims that are not stored.  fp32
// scores (the reference tower is fp32); only the tail tile is masked.

template <int KS, int NDT, int CPR, int NB, int NW, int QT>
__global__ __launch_bounds__(NW * 64, 2) void vit_stream_attn_kernel(
    const u16* __restrict__ qkv, u16* __restrict__ out, int N, int H, int hd,
    float scale_log2) {
  // CPR 16-B chunks per LDS row: 8 (128 B) for hd 64, 16 (256 B) for hd 72;
  // NB tile buffers (tile t + NB - 1 is fetched while tile t is computed);
  // NW waves per workgroup, QT 16-query tiles per wave: every K fragment and
  // V^T fragment a wave reads from LDS feeds QT query tiles' MFMAs (the LDS
  // reads of shared K / V^T, 8 waves x 16 queries per tile, bounded the
  // QT = 1 form, not the MFMA pipe)
  constexpr int TILE = GA_KT * CPR;   // uint4 per K or V image
  constexpr int NP = TILE / 64;       // 1-KiB DMA pieces per image
  constexpr int DPW = 2 * NP / NW;    // DMA instructions per wave per tile
  constexpr int RPP = 64 / CPR;       // rows per DMA piece
  static_assert(4 * KS <= CPR && 2 * NDT <= CPR && 2 * NP % NW == 0, "row padding");
  static_assert(NB == 2 || (NB == 3 && (DPW == 2 || DPW == 4)), "vmcnt below");
  __shared__ __attribute__((aligned(16))) uint4 smem[NB * 2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int nqb = (N + NW * 16 * QT - 1) / (NW * 16 * QT);
  int b, h, qb;
  {
    const int total = gridDim.x, lin = blockIdx.x;
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int p = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    qb = p % nqb;
    h = (p / nqb) % H;
    b = p / (nqb * H);
  }
  const int D = H * hd;
  const int64_t rs = 3 * (int64_t)D;
  const u16* base = qkv + (int64_t)b * N * rs + (int64_t)h * hd;
  const int real = hd / 8;            // stored chunks of a row
  // V^T image swizzle (even, so a lane's two 8-B halves stay in one chunk):
  // the 8 rows a 32-lane transposed read touches land on 8 distinct 32-B
  // bank slots -- (r & 7) << 1 over 256-B rows, ((r >> 1) & 3) << 1 over
  // 128-B rows (two rows per bank row)
  auto vx = [](int r) { return CPR == 16 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1); };

  // DMA: piece i covers RPP rows (lane l -> row RPP i + l / CPR, slot l % CPR)
  const int drow = lane / CPR, dslot = lane % CPR;
  auto stage = [&](int t, int buf) {
    const int c0 = t * GA_KT;
#pragma unroll
    for (int i = wave; i < 2 * NP; i += NW) {
      const bool isv = i >= NP;
      const int pi = isv ? i - NP : i;
      const int r = RPP * pi + drow;
      int ch = isv ? (dslot ^ vx(r)) : (dslot ^ (r & (CPR - 1)));
      ch = min(ch, real - 1);
      const int key = min(c0 + r, N - 1);
      const u16* src = base + key * rs + (isv ? 2 * D : D) + ch * 8;
      uint4* dst = smem + (buf * 2 + (isv ? 1 : 0)) * TILE + pi * 64;
      __builtin_amdgcn_global_load_lds((ga_gptr_t)src, (ga_lptr_t)dst, 16, 0, 0);
    }
  };
  const int ntiles = (N + GA_KT - 1) / GA_KT;

  // this wave's query tiles u: queries q0[u] .. q0[u] + 15
  int q0[QT];
  bf16x8 qf[QT][KS];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    q0[u] = ((qb * NW + wave) * QT + u) * 16;
    const int qi = min(q0[u] + c16, N - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 32 + 8 * g;
      qf[u][ks] = __builtin_bit_cast(bf16x8, d < hd ? ld16(base + qi * rs + d)
                                                    : make_uint4(0, 0, 0, 0));
    }
  }
  // q in registers before any DMA is issued, by a wait the compiler sees
  // (otherwise it keeps the q loads pending and puts a vmcnt(0) -- a wait
  // for every tile in flight -- before each tile's first MFMA)
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
  for (int t = 0; t < NB - 1 && t < ntiles; ++t) stage(t, t);
  f32x4 o[QT][NDT];
  float m[QT], l[QT];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
#pragma unroll
    for (int j = 0; j < NDT; ++j) o[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[u] = -INFINITY;
    l[u] = 0.0f;
  }
  constexpr float kThr = 8.0f;
  const int tq = c16 >> 2, tp = c16 & 3;

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t % NB;
    // tile t landed (this wave's DMA: tiles > t may stay in flight), then
    // every wave's: raw s_barrier (__syncthreads would drain all DMA)
    if (NB == 3 && t + 1 < ntiles) {
      if constexpr (DPW == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the buffer of tile t - 1, which every wave is done reading
    if (t + NB - 1 < ntiles) stage(t + NB - 1, (t + NB - 1) % NB);
    const int c0 = t * GA_KT;
    const uint4* kimg = smem + (buf * 2) * TILE;
    const uint32_t vlds = (uint32_t)(uintptr_t)(smem + (buf * 2 + 1) * TILE);
    // every K fragment of the tile read before the first QK^T MFMA (one
    // LDS wait instead of one per 16-key group)
    bf16x8 kf[4][KS];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int kr = 16 * tt + c16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[tt][ks] = __builtin_bit_cast(bf16x8, kimg[kr * CPR + ((4 * ks + g) ^ (kr & (CPR - 1)))]);
    }
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 pf[QT][2];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      f32x4 s[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        s[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[tt][ks], qf[u][ks], s[tt], 0, 0, 0);
      }
      if (c0 + GA_KT > N) {              // tail tile: keys past N
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + 16 * tt + 4 * g + r >= N) s[tt][r] = -INFINITY;
      }
      float smax = ga_max3(s[0][0], s[0][1], s[0][2]);
      smax = ga_max3(smax, s[0][3], s[1][0]);
      smax = ga_max3(smax, s[1][1], s[1][2]);
      smax = ga_max3(smax, s[1][3], s[2][0]);
      smax = ga_max3(smax, s[2][1], s[2][2]);
      smax = ga_max3(smax, s[2][3], s[3][0]);
      smax = ga_max3(smax, s[3][1], s[3][2]);
      smax = ga_max2(smax, s[3][3]);
      smax = ga_max_rows(smax);
      const float mt = smax * scale_log2;
      const bool need = mt > m[u] + kThr;
      if (__any(need)) {
        const float mn = need ? mt : m[u];
        const float alpha = need ? __builtin_amdgcn_exp2f(m[u] - mn) : 1.0f;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[u][dt][r] *= alpha;
        l[u] *= alpha;
        m[u] = mn;
      }
      const float nm = -m[u];            // every query has a key in tile 0
      float ps0 = 0.0f, ps1 = 0.0f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int tt = 2 * kk + (j >> 2), r = j & 3;
          const float e0 = __builtin_amdgcn_exp2f(fmaf(s[tt][r], scale_log2, nm));
          const float e1 = __builtin_amdgcn_exp2f(fmaf(s[tt][r + 1], scale_log2, nm));
          ps0 += e0;
          ps1 += e1;
          pk[j >> 1] = ga_pk2bf(f32x2{e0, e1});
        }
        pf[u][kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
      }
      l[u] += ps0 + ps1;
    }
    // V^T fragments by the transposing LDS read: all 2 NDT of a key half in
    // ONE asm statement with one lgkmcnt wait (the compiler's builtin for the
    // read is preceded by a vmcnt(0), i.e. it would wait for the next tile's
    // DMA; a statement per pair waited once per pair), each fragment feeding
    // the QT query tiles' P.V MFMAs
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r1 = 32 * kk + 4 * g + tq, r2 = r1 + 16;
      const uint32_t a1 = vlds + r1 * (CPR * 16) + 8 * (tp & 1);
      const uint32_t a2 = vlds + r2 * (CPR * 16) + 8 * (tp & 1);
      const int x1 = vx(r1), x2 = vx(r2);
      uint32_t ad[2 * NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int ch = 2 * dt + (tp >> 1);
        ad[2 * dt] = a1 + 16 * (ch ^ x1);
        ad[2 * dt + 1] = a2 + 16 * (ch ^ x2);
      }
      uint2 w[2 * NDT];
      if constexpr (NDT == 4) {
        asm volatile(
            "ds_read_b64_tr_b16 %0, %8\n" "ds_read_b64_tr_b16 %1, %9\n"
            "ds_read_b64_tr_b16 %2, %10\n" "ds_read_b64_tr_b16 %3, %11\n"
            "ds_read_b64_tr_b16 %4, %12\n" "ds_read_b64_tr_b16 %5, %13\n"
            "ds_read_b64_tr_b16 %6, %14\n" "ds_read_b64_tr_b16 %7, %15\n"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]),
              "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7])
            : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]),
              "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7])
            : "memory");
      } else {
        static_assert(NDT == 5, "hd 64 / 72");
        asm volatile(
            "ds_read_b64_tr_b16 %0, %10\n" "ds_read_b64_tr_b16 %1, %11\n"
            "ds_read_b64_tr_b16 %2, %12\n" "ds_read_b64_tr_b16 %3, %13\n"
            "ds_read_b64_tr_b16 %4, %14\n" "ds_read_b64_tr_b16 %5, %15\n"
            "ds_read_b64_tr_b16 %6, %16\n" "ds_read_b64_tr_b16 %7, %17\n"
            "ds_read_b64_tr_b16 %8, %18\n" "ds_read_b64_tr_b16 %9, %19\n"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]),
              "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]), "=&v"(w[8]), "=&v"(w[9])
            : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]),
              "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(ad[8]), "v"(ad[9])
            : "memory");
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 vf = __builtin_bit_cast(
            bf16x8, make_uint4(w[2 * dt].x, w[2 * dt].y, w[2 * dt + 1].x, w[2 * dt + 1].y));
#pragma unroll
        for (int u = 0; u < QT; ++u)
          o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[u][kk], o[u][dt], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    float lt = l[u];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const float inv = 1.0f / lt;
    if (q0[u] + c16 < N) {
      u16* orow = out + ((int64_t)b * N + q0[u] + c16) * D + (int64_t)h * hd;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < hd) {
          const uint32_t lo2 = ga_pk2bf(f32x2{o[u][dt][0] * inv, o[u][dt][1] * inv});
          const uint32_t hi2 = ga_pk2bf(f32x2{o[u][dt][2] * inv, o[u][dt][3] * inv});
          *reinterpret_cast<uint2*>(orow + d0) = make_uint2(lo2, hi2);
        }
      }
    }
  }
}

}  // namespace

// The MQA workgroup form covers hd = 256 with up to 10 heads (one wave per
// head): the RecurrentGemma-2B preset (10 x 256).  Returns -1 when the
// caller should use the per-head streaming kernel instead.
__attribute__((visibility("hidden"))) int griffin_attention_launch(
    const void* q, const void* k, const void* v, const int32_t* seg_start,
    void* out, int64_t B, int64_t L, int64_t H, int64_t hd, int64_t window,
    void* stream) {
  if (hd != 256 || H < 1 || H > GA_MAXW) return -1;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) % 16) return -1;
  GAArgs a{static_cast<const u16*>(q), static_cast<const u16*>(k),
           static_cast<const u16*>(v), seg_start, static_cast<u16*>(out),
           (int)B, (int)L, (int)H, (int)window,
           1.4426950408889634f / sqrtf((float)hd)};
  const int64_t nqb = (L + GA_QB - 1) / GA_QB;
  hipLaunchKernelGGL(griffin_attn_kernel<256>, dim3((unsigned)(B * nqb)),
                     dim3((unsigned)(H * 64)), 0, static_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

// ViT attention for sequences longer than the LDS-resident kernel holds
// (hd 64 / 72).  Returns -1 for other shapes.
__attribute__((visibility("hidden"))) int vit_stream_attention_launch(
    const void* qkv, void* out, int64_t B, int64_t N, int64_t H, int64_t hd,
    void* stream) {
  if ((hd != 64 && hd != 72) || N < 1) return -1;
  if (((uintptr_t)qkv | (uintptr_t)out) % 16) return -1;
  // 128 queries per workgroup: hd 64 as 4 waves x 2 query tiles (each K /
  // V^T fragment read from LDS feeds two tiles' MFMAs), hd 72 as 8 waves x
  // 1 tile.  Same-box A/B (profiles/r03q_vit_stream_qt_ab.log): hd 64
  // 4 x 2 is 3-8 % faster at 336 / 384 px, hd 72 the same or slower.
  const float sl2 = 1.4426950408889634f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
  const int64_t nqb = (N + 127) / 128;
  const dim3 grid((unsigned)(B * H * nqb));
  if (hd == 64)
    hipLaunchKernelGGL((vit_stream_attn_kernel<2, 4, 8, 3, 4, 2>), grid, dim3(256), 0, st, in,
                       o, (int)N, (int)H, (int)hd, sl2);
  else
    hipLaunchKernelGGL((vit_stream_attn_kernel<3, 5, 16, 2, 8, 1>), grid, dim3(512), 0, st,
                       in, o, (int)N, (int)H, (int)hd, sl2);
  return (int)hipGetLastError();
}
