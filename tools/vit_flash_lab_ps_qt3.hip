// LAB VARIANT (not built; kept for the record of profiles/r04p_*): the
// round-4 flash kernel plus two measured-and-rejected options, selected in
// the launcher by lab bits of cadence_gemm_set_engine when this file
// replaces csrc/vit_flash.hip: bit 4 (16) = PS, Q pre-multiplied by
// scale*log2(e) and the running max subtracted by the MFMA accumulator's
// start value (no fma per score); bit 5 (32) = PS with three query tiles per
// wave at two waves per SIMD.  PS: 2-6 % faster at 336 / 384 px, rel-L2 to
// fp32 2.06e-3 -> 3.6e-3 (the extra bf16 rounding of Q); QT 3: dino 384 px
// -8 %, 336 px unchanged.  The attention.hip plan needs bit 4 to let DINO
// 224 px through as well (r04p used that).
// ViT (bidirectional) attention, streaming form for every tower size
// (timm Attention.forward -> F.scaled_dot_product_attention, scale hd^-1/2,
// reached through recurrentgemma/vit/dino_siglip.py:85-86,149-151; timm not
// vendored) on gfx950.
//
// One workgroup = (image, head, block of 16-query tiles); NW waves, wave w
// owning QT query tiles.  64-key tiles of K and V stream through two LDS
// buffers by buffer_load ... lds (one 1-KiB LDS-DMA piece per wave
// instruction, the source rows addressed by a per-lane offset fixed for the
// kernel's life and a scalar tile offset: no per-tile address arithmetic;
// rows past the image batch read as zeros by the buffer's range check).
//
// The issue budget is what bounds this kernel: per 16 queries x 64 keys a
// wave issues 16-18 MFMAs (256 cycles of the SIMD's matrix pipe, each
// holding its vector issue for 8 of 16 cycles) and the online softmax of
// 1024 scores.  So everything the MFMA pipe can do instead of the VALU, it
// does, and every per-tile address is an immediate:
//  * the K image is stored in MFMA A-fragment order (fragment (16-key group,
//    32-dim k-step) = one 1-KiB DMA piece, lane i <- key i % 16, dims
//    8 (i / 16)..): each fragment is one conflict-free ds_read_b128 at
//    lane * 16 + a constant;
//  * the V image is chunk-major (16-B chunk ch of key row r at slot
//    64 ch + (r ^ 8 (ch & 1))): every transposing read of a V^T fragment
//    (ds_read_b64_tr_b16, 4 keys x 16 dims per 16 lanes) is one lane base
//    plus 2048 dt + 512 kk (+ 256), and each 32-lane half touches 64
//    distinct banks;
//  * the softmax denominator is an MFMA: P^T multiplied by a row of ones
//    (hd 64: an all-ones A operand in registers; hd 72: dims 72..79 of the
//    last V^T tile, whose LDS chunk holds ones) -- the sum of the bf16 P
//    that the P.V MFMAs use, so O and l agree exactly;
//  * the running max is checked lane-locally (one compare and a wave vote
//    per query tile); the cross-lane max and the O rescale run only when a
//    row's max grew by more than 2^8 (deferred rescale, kThr): on the first
//    tile and rarely after it.
// Swapped QK^T as in vit_attention.hip: S^T = K . Q^T, a lane owns one query
// and 4 keys of each 16-key group, and the score tile is the B operand of
// O^T = V^T . P^T under the key-slot permutation
//   slot 8g + j <-> key 4g + j (j < 4), 16 + 4g + (j - 4) (j >= 4).
// fp32 scores and softmax (the reference tower is fp32), P in bf16.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* vf_lptr_t;

constexpr int VF_KT = 64;      // keys per tile
constexpr uint32_t kBf16Ones = 0x3F803F80u;

CADENCE_DEV float vf_max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
// max over lanes l, l ^ 16, l ^ 32, l ^ 48 (the four key groups of a query)
CADENCE_DEV float vf_max_rows(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float m = __builtin_fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const uint32_t w = __float_as_uint(m);
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __builtin_fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// Per head-dim layout of one LDS buffer (uint4 units):
//   [0, 512)          K fragments (tt, ks) for dims 0..63, 64 uint4 each
//   [512, KEND)       hd 72: dims 64..71 of the 64 keys (one "compact" piece)
//   [KEND, +64 VCH)   V image, chunk-major; hd 72: chunk 9 = bf16 ones
template <int HD>
struct VFLayout {
  static constexpr bool kWide = HD == 72;
  static constexpr int KS = kWide ? 3 : 2;        // QK^T k-steps
  static constexpr int NDT = kWide ? 5 : 4;       // O^T dim tiles read from V
  static constexpr int KEND = kWide ? 576 : 512;
  static constexpr int VCH = kWide ? 9 : 8;       // V chunks loaded per tile
  static constexpr int VSLOTS = kWide ? 10 : 8;   // V chunks stored (+ ones)
  static constexpr int BUF = KEND + 64 * VSLOTS;  // uint4 per buffer
  static constexpr int KPIECES = kWide ? 9 : 8;
  static constexpr int PIECES = KPIECES + VCH;    // DMA pieces per tile
};

template <int HD, int NW, int QT, int NB, bool PS>
__global__ __launch_bounds__(NW * 64, QT == 2 ? 3 : 2) void vit_flash_attn_kernel(
    const u16* __restrict__ qkv, u16* __restrict__ out, int B, int N, int H,
    int nqb, float scale_log2) {
  using L = VFLayout<HD>;
  constexpr int KS = L::KS, NDT = L::NDT;
  constexpr int NO = NDT + (L::kWide ? 0 : 1);   // accumulators (+ ones tile)
  __shared__ __attribute__((aligned(16))) uint4 smem[NB * L::BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform (an SGPR): the DMA's LDS base and the per-tile branches
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  // XCD-aware order: consecutive dispatch indices go to consecutive XCDs,
  // so remap bijectively to give each XCD a contiguous range of (image,
  // head, query block): the blocks of a head share its K / V rows in that
  // XCD's L2
  int b, h, qb;
  {
    const int total = gridDim.x, lin = blockIdx.x;
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int p = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    qb = p % nqb;
    h = (p / nqb) % H;
    b = p / (nqb * H);
  }
  const int D = H * HD;
  const int rsb = 3 * D * 2;                       // qkv row stride, bytes
  const u16* img = qkv + (int64_t)b * N * (3 * D);
  // buffer resource over the rest of the batch from this image on: key rows
  // past the last image read as zeros (finite; masked, weighted 0)
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<u16*>(img), 0, (int)((int64_t)(B - b) * N * rsb), 0x00020000);
  const int kcol = (D + h * HD) * 2, vcol = (2 * D + h * HD) * 2;

  // query tiles of this block: a balanced share of the image's ceil(N / 16)
  const int ntq = (N + 15) >> 4;
  const int tq0 = qb * ntq / nqb, tq1 = (qb + 1) * ntq / nqb;
  int qt[QT];
  bool act[QT];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    qt[u] = tq0 + wave + NW * u;
    act[u] = qt[u] < tq1;
  }

  // hd 72: the V chunk holding dims 72..79 is bf16 ones in every buffer
  if constexpr (L::kWide) {
    if (wave == 0) {
      const uint4 ones = make_uint4(kBf16Ones, kBf16Ones, kBf16Ones, kBf16Ones);
#pragma unroll
      for (int i = 0; i < NB; ++i) smem[i * L::BUF + L::KEND + 9 * 64 + lane] = ones;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // before tile 0's barrier
    }
  }

  // per-lane DMA source offsets (bytes from the tile's first key row)
  const int voff_k = (lane & 15) * rsb + (lane >> 4) * 16;   // K fragment pieces
  const int voff_r = lane * rsb;                              // one row per lane
  const int voff_x = (lane ^ 8) * rsb;                        // odd V chunks
  // wave w stages the K fragments of key group tt = w (k-steps 0, 1) and V
  // chunks 2w, 2w + 1; hd 72 adds the dims-64..71 piece (wave 0) and V chunk
  // 8 (wave 1): no per-piece branches on the wave index
  static_assert(NW == 4, "one 16-key group of K per wave");
  auto stage = [&](int t, int buf) {
    const int c0b = t * VF_KT * rsb;
    uint4* base = smem + buf * L::BUF;
    const int kso = c0b + 16 * wave * rsb + kcol;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)(base + 128 * wave), 16,
                                             voff_k, kso, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)(base + 128 * wave + 64), 16,
                                             voff_k, kso + 64, 0, 0);
    const int vso = c0b + vcol + 32 * wave;
    uint4* vb = base + L::KEND + 128 * wave;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)vb, 16, voff_r, vso, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)(vb + 64), 16, voff_x, vso + 16,
                                             0, 0);
    if constexpr (L::kWide) {
      if (wave == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)(base + 512), 16, voff_r,
                                                 c0b + kcol + 128, 0, 0);
      else if (wave == 1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (vf_lptr_t)(base + L::KEND + 512), 16,
                                                 voff_r, c0b + vcol + 128, 0, 0);
    }
  };

  // Q^T fragments: B[k = dim 32 ks + 8 g + i][n = query c16], zero past hd
  bf16x8 qf[QT][KS];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    const int q = min(qt[u] * 16 + c16, N - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 32 + 8 * g;
      qf[u][ks] = __builtin_bit_cast(
          bf16x8, d < HD ? ld16(img + (int64_t)q * (3 * D) + h * HD + d) : make_uint4(0, 0, 0, 0));
    }
  }
  // Q in registers before the first DMA: an asm that "modifies" every
  // fragment makes the compiler wait for the loads here; a Q load still
  // pending in the loop would put a vmcnt wait -- one that also waits for
  // the next tile's DMA -- in front of the first MFMA reading it
#pragma unroll
  for (int u = 0; u < QT; ++u)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qf[u][ks]));
  // PS: Q pre-multiplied by scale * log2(e) (rounded to bf16 once more), so
  // a score is exp2's argument once the running max is subtracted -- and the
  // max is subtracted by the MFMA itself, its accumulator starting at -m
  if constexpr (PS) {
#pragma unroll
    for (int u = 0; u < QT; ++u)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        uint4 w = __builtin_bit_cast(uint4, qf[u][ks]);
        uint32_t* p = &w.x;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          p[i] = pk2bf(f32x2{__uint_as_float(p[i] << 16) * scale_log2,
                             __uint_as_float(p[i] & 0xffff0000u) * scale_log2});
        qf[u][ks] = __builtin_bit_cast(bf16x8, w);
      }
  }
  const int ntiles = (N + VF_KT - 1) / VF_KT;
  // NB - 1 tiles in flight before the first is computed
#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < ntiles) stage(i, i);

  f32x4 o[QT][NO];
  float m[QT];
  f32x4 nm4[QT];     // PS: the score accumulators' start, -(max they hold)
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    m[u] = -INFINITY;
    nm4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NO; ++j) o[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr float kThr = 8.0f;
  const bf16x8 ones8 = __builtin_bit_cast(
      bf16x8, make_uint4(kBf16Ones, kBf16Ones, kBf16Ones, kBf16Ones));
  // LDS byte address of this lane's transposing V^T reads in buffer 0
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  const int tq = c16 >> 2, tp = c16 & 3, tp1 = tp >> 1;
  const uint32_t va = sbase + 16 * L::KEND + 1024 * tp1 +
                      16 * ((4 * g + tq) ^ (8 * tp1)) + 8 * (tp & 1);   // + 2048 dt + 512 kk (+ 256)

  // V^T fragments of key half kk: two transposing reads per 16-dim tile, all
  // in one asm statement with one wait (the compiler's builtin for this read
  // waits vmcnt(0) first -- for the DMA of the tiles in flight)
  auto vread = [&](uint32_t a, uint2 (&w)[2 * NDT]) {
    if constexpr (NDT == 4) {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n" "ds_read_b64_tr_b16 %1, %8 offset:256\n"
          "ds_read_b64_tr_b16 %2, %8 offset:2048\n" "ds_read_b64_tr_b16 %3, %8 offset:2304\n"
          "ds_read_b64_tr_b16 %4, %8 offset:4096\n" "ds_read_b64_tr_b16 %5, %8 offset:4352\n"
          "ds_read_b64_tr_b16 %6, %8 offset:6144\n" "ds_read_b64_tr_b16 %7, %8 offset:6400\n"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]),
            "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7])
          : "v"(a)
          : "memory");
    } else {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %10\n" "ds_read_b64_tr_b16 %1, %10 offset:256\n"
          "ds_read_b64_tr_b16 %2, %10 offset:2048\n" "ds_read_b64_tr_b16 %3, %10 offset:2304\n"
          "ds_read_b64_tr_b16 %4, %10 offset:4096\n" "ds_read_b64_tr_b16 %5, %10 offset:4352\n"
          "ds_read_b64_tr_b16 %6, %10 offset:6144\n" "ds_read_b64_tr_b16 %7, %10 offset:6400\n"
          "ds_read_b64_tr_b16 %8, %10 offset:8192\n" "ds_read_b64_tr_b16 %9, %10 offset:8448\n"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]),
            "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]), "=&v"(w[8]), "=&v"(w[9])
          : "v"(a)
          : "memory");
    }
  };

  // the same reads without their wait (hd 64: issued before the QK^T MFMAs,
  // waited for before the first P.V MFMA by vwait)
  auto vissue = [&](uint32_t a, uint2 (&w)[2 * NDT]) {
    static_assert(NDT == 4 || !PS, "hd 64 only");
    if constexpr (NDT == 4)
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n" "ds_read_b64_tr_b16 %1, %8 offset:256\n"
          "ds_read_b64_tr_b16 %2, %8 offset:2048\n" "ds_read_b64_tr_b16 %3, %8 offset:2304\n"
          "ds_read_b64_tr_b16 %4, %8 offset:4096\n" "ds_read_b64_tr_b16 %5, %8 offset:4352\n"
          "ds_read_b64_tr_b16 %6, %8 offset:6144\n" "ds_read_b64_tr_b16 %7, %8 offset:6400"
          : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]),
            "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7])
          : "v"(a)
          : "memory");
  };
  auto vwait = [&](uint2 (&w0)[2 * NDT], uint2 (&w1)[2 * NDT]) {
    if constexpr (NDT == 4)
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(w0[0]), "+v"(w0[1]), "+v"(w0[2]), "+v"(w0[3]), "+v"(w0[4]),
                     "+v"(w0[5]), "+v"(w0[6]), "+v"(w0[7]), "+v"(w1[0]), "+v"(w1[1]),
                     "+v"(w1[2]), "+v"(w1[3]), "+v"(w1[4]), "+v"(w1[5]), "+v"(w1[6]),
                     "+v"(w1[7])
                   :
                   : "memory");
  };

  // one key tile for the wave's NA active query tiles (a compile-time count:
  // no per-MFMA predicates)
  auto tile = [&](int t, auto tail_tag, auto na_tag) __attribute__((always_inline)) {
    constexpr bool tail = decltype(tail_tag)::value;
    constexpr int NA = decltype(na_tag)::value;
    const int buf = t % NB;
    const uint32_t bo = buf * (L::BUF * 16);
    const int nk = N - t * VF_KT;        // keys in this tile (tail: < 64)
    // every LDS read of the tile's K and (hd 64) V^T issued at its start,
    // under one wait: one LDS latency per tile instead of three
    const uint4* kb = smem + buf * L::BUF;
    bf16x8 kf[4][KS];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        kf[tt][ks] = __builtin_bit_cast(bf16x8, kb[64 * (2 * tt + ks) + lane]);
      if constexpr (KS == 3)
        kf[tt][2] = __builtin_bit_cast(bf16x8, kb[512 + 16 * tt + c16]);
    }
    // key halves read up front (hd 72: none, its fragments would spill);
    // PS: after every QK^T MFMA, into the K fragments' registers, their wait
    // at the first P.V MFMA (the softmax covers the LDS latency)
    constexpr int VPRE = L::kWide ? 0 : 2;
    uint2 w[2][2 * NDT];
    if constexpr (!PS) {
#pragma unroll
      for (int kk = 0; kk < VPRE; ++kk)
        if (!(tail && 32 * kk >= nk)) vread(va + bo + 512 * kk, w[kk]);
    }
    bf16x8 pf[QT][2];
    auto qk = [&](int u, f32x4 (&s)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        s[tt] = PS ? nm4[u] : f32x4{0.f, 0.f, 0.f, 0.f};
        if (tail && 16 * tt >= nk) continue;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[tt][ks], qf[u][ks], s[tt], 0, 0, 0);
      }
    };
    auto softmax = [&](int u, f32x4 (&s)[4]) __attribute__((always_inline)) {
      if constexpr (tail) {
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * tt + 4 * g + r >= nk) s[tt][r] = -INFINITY;
      }
      // lane-local max; the row max and the rescale only when some row grew
      float lm;
      if constexpr (PS) {   // a tree: depth 3 instead of a chain of 8
        const float a0 = vf_max3(s[0][0], s[0][1], s[0][2]);
        const float a1 = vf_max3(s[0][3], s[1][0], s[1][1]);
        const float a2 = vf_max3(s[1][2], s[1][3], s[2][0]);
        const float a3 = vf_max3(s[2][1], s[2][2], s[2][3]);
        const float a4 = vf_max3(s[3][0], s[3][1], s[3][2]);
        lm = __builtin_fmaxf(vf_max3(a0, a1, a2), vf_max3(a3, a4, s[3][3]));
      } else {
        lm = vf_max3(s[0][0], s[0][1], s[0][2]);
        lm = vf_max3(lm, s[0][3], s[1][0]);
        lm = vf_max3(lm, s[1][1], s[1][2]);
        lm = vf_max3(lm, s[1][3], s[2][0]);
        lm = vf_max3(lm, s[2][1], s[2][2]);
        lm = vf_max3(lm, s[2][3], s[3][0]);
        lm = vf_max3(lm, s[3][1], s[3][2]);
        lm = __builtin_fmaxf(lm, s[3][3]);
      }
      if constexpr (PS) {
        // s = scaled score - mo (mo = -nm4, the max the accumulators started
        // from); every row starts at m = -inf, so tile 0 always decides
        if (t == 0 || __any(lm > kThr)) {
          const float mo = -nm4[u][0];
          const float mt = vf_max_rows(lm) + mo;
          const bool need = mt > m[u] + kThr;
          const float mn = need ? mt : m[u];
          const float alpha = need ? __builtin_amdgcn_exp2f(m[u] - mn) : 1.0f;
#pragma unroll
          for (int j = 0; j < NO; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[u][j][r] *= alpha;
          // this tile's scores move to the new max; later tiles start there
          const float d = need ? mn - mo : 0.0f;
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[tt][r] -= d;
          const float nmn = need ? -mn : nm4[u][0];
          nm4[u] = f32x4{nmn, nmn, nmn, nmn};
          m[u] = mn;
        }
      } else if (__any(lm * scale_log2 > m[u] + kThr)) {
        const float mt = vf_max_rows(lm) * scale_log2;
        const bool need = mt > m[u] + kThr;
        const float mn = need ? mt : m[u];
        // rows that keep their max keep alpha 1; m = -inf -> alpha 0
        const float alpha = need ? __builtin_amdgcn_exp2f(m[u] - mn) : 1.0f;
#pragma unroll
        for (int j = 0; j < NO; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[u][j][r] *= alpha;
        m[u] = mn;
      }
      const float nm = -m[u];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (tail && 32 * kk >= nk) continue;   // its P.V is skipped below
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int tt = 2 * kk + (j >> 2), r = j & 3;
          const float e0 = __builtin_amdgcn_exp2f(PS ? s[tt][r] : fmaf(s[tt][r], scale_log2, nm));
          const float e1 =
              __builtin_amdgcn_exp2f(PS ? s[tt][r + 1] : fmaf(s[tt][r + 1], scale_log2, nm));
          pk[j >> 1] = pk2bf(f32x2{e0, e1});
        }
        pf[u][kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
      }
    };
    if constexpr (PS) {
      f32x4 sa[QT][4];
#pragma unroll
      for (int u = 0; u < NA; ++u) qk(u, sa[u]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        if (!(tail && 32 * kk >= nk)) vissue(va + bo + 512 * kk, w[kk]);
#pragma unroll
      for (int u = 0; u < NA; ++u) softmax(u, sa[u]);
    } else {
#pragma unroll
      for (int u = 0; u < NA; ++u) {
        f32x4 s[4];
        qk(u, s);
        softmax(u, s);
      }
    }
    // O^T += V^T . P^T (and, hd 64, l += ones . P^T)
    if constexpr (PS) vwait(w[0], w[1]);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (tail && 32 * kk >= nk) continue;
      if (kk >= VPRE) vread(va + bo + 512 * kk, w[kk]);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 vf = __builtin_bit_cast(
            bf16x8, make_uint4(w[kk][2 * dt].x, w[kk][2 * dt].y, w[kk][2 * dt + 1].x,
                               w[kk][2 * dt + 1].y));
#pragma unroll
        for (int u = 0; u < NA; ++u)
          o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[u][kk], o[u][dt], 0, 0, 0);
      }
      if constexpr (!L::kWide) {
#pragma unroll
        for (int u = 0; u < NA; ++u)
          o[u][NDT] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pf[u][kk], o[u][NDT], 0, 0, 0);
      }
    }
  };

  // tile t landed: this wave's DMA (the pieces of the NB - 2 tiles after it
  // may stay in flight: every wave issues PPW pieces per tile), then every
  // wave's: a raw s_barrier (__syncthreads would wait for all DMA).  The
  // barrier also retires the buffer of tile t - 1, which the DMA of tile
  // t + NB - 1 then refills.
  constexpr int PPW = L::kWide ? 5 : 4;     // (hd 72: at most 5)
  auto wait_tile = [&](int t) {
    if (NB == 3 && t + 1 < ntiles) {
      static_assert(NB == 2 || !L::kWide, "hd 72's waves issue 4 or 5 pieces");
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  using F = std::false_type;
  using T = std::true_type;
  const bool ragged = (N % VF_KT) != 0;
  auto run = [&](auto na_tag) __attribute__((always_inline)) {
    // full tiles; the last tile peeled (the only one that can be ragged: the
    // loop body carries no masking)
    int t = 0;
    for (; t + 1 < ntiles; ++t) {
      wait_tile(t);
      if (t + NB - 1 < ntiles) stage(t + NB - 1, (t + NB - 1) % NB);
      tile(t, F{}, na_tag);
    }
    wait_tile(t);
    if (ragged) tile(t, T{}, na_tag);
    else tile(t, F{}, na_tag);
  };
  // the active tiles are a prefix of the wave's QT (qt[u] grows with u)
  static_assert(QT == 2 || QT == 3, "active-tile dispatch below");
  bool done = false;
  if constexpr (QT == 3) {
    if (act[2]) {
      run(std::integral_constant<int, QT == 3 ? 3 : 0>{});
      done = true;
    }
  }
  if (!done) {
    if (act[1]) run(std::integral_constant<int, 2>{});
    else if (act[0]) run(std::integral_constant<int, 1>{});
    else run(std::integral_constant<int, 0>{});   // DMA and barriers only
  }

  // out[q][h*HD + d]: lane holds dims 16 dt + 4 g + 0..3 of query c16
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    if (!act[u]) continue;
    float l;
    if constexpr (L::kWide) {
      // rows 8..15 of the last tile (dims 72..79 x ones) = l: lanes g >= 2
      const float x = o[u][4][0];
      const float y = __shfl_xor(x, 32, 64);
      l = g >= 2 ? x : y;
    } else {
      l = o[u][NDT][0];
    }
    const float inv = 1.0f / l;
    const int q = qt[u] * 16 + c16;
    if (q < N) {
      u16* orow = out + ((int64_t)b * N + q) * D + h * HD;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < HD) {
          const uint32_t lo2 = pk2bf(f32x2{o[u][dt][0] * inv, o[u][dt][1] * inv});
          const uint32_t hi2 = pk2bf(f32x2{o[u][dt][2] * inv, o[u][dt][3] * inv});
          *reinterpret_cast<uint2*>(orow + d0) = make_uint2(lo2, hi2);
        }
      }
    }
  }
}

}  // namespace

int cadence_engine_bits();   // gemm.hip (the lab switch)

// Streaming ViT attention for hd 64 / 72 and any N; returns -1 for other
// shapes (or a qkv / out pointer that is not 16-B aligned, or a batch whose
// byte size exceeds the buffer range).
__attribute__((visibility("hidden"))) int vit_flash_attention_launch(
    const void* qkv, void* out, int64_t B, int64_t N, int64_t H, int64_t hd,
    void* stream) {
  if ((hd != 64 && hd != 72) || N < 1 || B < 1 || H < 1) return -1;
  if (((uintptr_t)qkv | (uintptr_t)out) % 16) return -1;
  if (B * N * 3 * H * hd * 2 >= ((int64_t)1 << 31)) return -1;
  constexpr int NW = 4;
  const bool qt3 = hd == 64 && (cadence_engine_bits() & 32);   // lab
  const int QT = qt3 ? 3 : 2;
  const int64_t ntq = (N + 15) / 16;
  int64_t nqb = (ntq + NW * QT - 1) / (NW * QT);
  static const int lab_nqb = getenv("CADENCE_VF_NQB") ? atoi(getenv("CADENCE_VF_NQB")) : 0;
  if (lab_nqb > 0) nqb = std::max<int64_t>(nqb, (ntq * lab_nqb + 99) / 100);   // lab: blocks per 100 tiles
  const float sl2 = 1.4426950408889634f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(B * H * nqb));
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
  // hd 64: three tile buffers (48 KB, three workgroups per CU); hd 72's
  // 19-KB tiles fit two buffers at three workgroups per CU
  if (qt3)
    hipLaunchKernelGGL((vit_flash_attn_kernel<64, NW, 3, 3, true>), grid, dim3(NW * 64), 0, st,
                       in, o, (int)B, (int)N, (int)H, (int)nqb, sl2);
  else if (hd == 64 && (cadence_engine_bits() & 16))
    hipLaunchKernelGGL((vit_flash_attn_kernel<64, NW, 2, 3, true>), grid, dim3(NW * 64), 0, st,
                       in, o, (int)B, (int)N, (int)H, (int)nqb, sl2);
  else if (hd == 64)
    hipLaunchKernelGGL((vit_flash_attn_kernel<64, NW, 2, 3, false>), grid, dim3(NW * 64), 0, st,
                       in, o, (int)B, (int)N, (int)H, (int)nqb, sl2);
  else
    hipLaunchKernelGGL((vit_flash_attn_kernel<72, NW, 2, 2, false>), grid, dim3(NW * 64), 0, st,
                       in, o, (int)B, (int)N, (int)H, (int)nqb, sl2);
  return (int)hipGetLastError();
}
