// LAB KERNEL (round 6, measured and not shipped: tools/vit_fa32_lab.py,
// profiles/r06*_fa32_lab.log) -- not part of libcadence_hip.so.
//
// ViT (bidirectional) attention on the 32x32x16 MFMA (timm Attention.forward
// -> F.scaled_dot_product_attention, scale hd^-1/2, reached through
// recurrentgemma/vit/dino_siglip.py:85-86,149-151; timm not vendored, SURVEY
// §8c a4) for the tower head dims 64 (DINOv2-L) and 72 (SigLIP-so400m).
//
// Why this shape: at hd 64 a score costs 4 hd = 256 MFMA FLOP but ~3 VALU
// issues of softmax (exp, pack, max) -- as many issue cycles as the MFMAs
// take.  The 16x16x32 MFMA holds the SIMD's vector issue for 8 of its 16
// cycles, the 32x32x16 one for 8 of 32 (MI355X_MICROARCH.md, issue costs),
// so this kernel computes every product on 32 x 32 tiles and keeps the
// per-score VALU at one v_exp_f32, half a v_cvt_pk_bf16_f32 and half a
// v_max3_f32:
//  * Q is pre-multiplied by hd^-1/2 log2(e) (scores come out in log2 units)
//    and the QK^T accumulator starts from -m (the running row max, an MFMA
//    C operand), so a score is exp2(S) with no per-score scale / subtract;
//  * the running max is checked lane-locally (one v_max3 per two scores and
//    a wave vote); the row max and the O rescale run only when a row grew by
//    more than 2^8 (deferred rescale, kThr; forced on the first tile);
//  * the softmax denominator is an MFMA on the P fragments the P.V MFMAs
//    use: hd 64 -- a 16x16x32 MFMA whose constant A operand selects each
//    query's 16 keys of a k-step (rows 0-7: queries 0-15, rows 8-15: 16-31);
//    hd 72 -- row 72 of the third 32-dim output block, fed by a ones chunk.
// Swapped QK^T: S^T[32 keys][32 queries] = K . Q^T, lane l owns query l & 31
// and keys 8 (r / 4) + 4 (l / 32) + r % 4 of its 16 accumulators r, and the
// exp of accumulators 8j..8j+7 is directly the B operand of the P.V k-step j
// under the key-slot order  slot 8 hi + e <-> key 16 j + 4 hi + (e < 4 ? e :
// e + 4); the V^T A operand is read in that order by two transposing
// ds_read_b64_tr_b16 (keys +0..3 and +8..11 of the lane's half).
//
// Workgroup = (image, head, block of 32-query tiles): 4 waves, one 32-query
// tile each, two workgroups per CU (2 waves per SIMD from independent
// workgroups: their barriers do not phase-lock them).  64-key tiles of K and
// V stream through NB LDS buffers by buffer_load ... lds (1-KiB pieces, lane
// i <- 16 B at M0 + 16 i; per-lane source offsets fixed for the kernel's life
// and a scalar tile offset; rows past the batch read as zeros by the buffer
// range check), issued NB - 1 tiles ahead and retired by a counted vmcnt + one
// barrier per tile:
//  * K: piece (kh, ks) = keys 32 kh + (l & 31), dims 16 ks + 8 (l / 32): the
//    A fragment itself, one conflict-free ds_read_b128 at lane * 16;
//  * V: row-major [64 keys][8 chunks of 8 dims], chunk c of row r at slot
//    c ^ 4 ((r >> 1) & 1): each 32-lane half of a transposing read touches 4
//    rows x 4 chunks on 64 distinct banks;
//  * hd 72: dims 64..71 of K as a fifth k-step (the lanes of dims 72..79
//    re-read dims 64..71 against zero Q), dims 64..71 of V as a 1-KiB piece
//    [64 keys][16 B]; dim 72 reads a ones region shared by the buffers (the
//    row sum).
// fp32 scores and accumulation, P in bf16 (as the other ViT kernels).
#include <algorithm>
#include <type_traits>
#include "../cadence-gemma_amd/csrc/common.hpp"
#include "../include/cadence_kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* fa_lptr_t;
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int FA_KT = 64;                 // keys per tile
constexpr uint32_t kFaOnes = 0x3F803F80u;  // two bf16 1.0

template <int HD>
struct FALayout {
  static constexpr bool kWide = HD == 72;
  static constexpr int KS = kWide ? 5 : 4;    // QK^T k-steps of 16 dims
  static constexpr int NDB = kWide ? 3 : 2;   // 32-dim output blocks
  // uint4 offsets inside one buffer
  static constexpr int VOFF = 2 * KS * 64;    // V image, 512 uint4
  static constexpr int TOFF = VOFF + 512;     // hd 72: dims 64..71, 64 uint4
  static constexpr int BUF = kWide ? TOFF + 64 : TOFF;
  // hd 72: one ones region after the buffers, 8 uint4 (128 B) off the bank
  // alignment of TOFF (BUF and TOFF are multiples of 16 uint4 = 256 B)
  static constexpr int ONES = kWide ? 8 + 64 : 0;
  static constexpr int PIECES = 2 * KS + 8 + (kWide ? 1 : 0);
  static constexpr int PPW = (PIECES + 3) / 4;   // DMA pieces per wave per tile
};

CADENCE_DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
CADENCE_DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
CADENCE_DEV float fa_max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
// max of lanes l and l ^ 32 (v_permlane32_swap of a register with itself
// leaves {v[0..31], v[0..31]} and {v[32..63], v[32..63]}: the two results
// hold both halves' values in every lane)
CADENCE_DEV float fa_max_halves(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto s = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

// s_waitcnt lgkmcnt(n) that also "rewrites" the fragments it retires, so
// the MFMAs reading them stay below it (n is a compile-time constant after
// unrolling: one of 0, 2 NDB, 4 NDB, 6 NDB)
template <int NDB>
CADENCE_DEV void vwait(uint2 (&x)[NDB], uint2 (&y)[NDB], int n) {
#define CADENCE_FA_WAIT(N_)                                                             \
  if constexpr (NDB == 2) {                                                             \
    asm volatile("s_waitcnt lgkmcnt(%[c])"                                              \
                 : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]) : [c] "n"((N_) > 15 ? 15 : (N_)));         \
  } else {                                                                              \
    asm volatile("s_waitcnt lgkmcnt(%[c])"                                              \
                 : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]), "+v"(x[2]), "+v"(y[2])  \
                 : [c] "n"((N_) > 15 ? 15 : (N_)));                                                      \
  }
  if (n == 0) { CADENCE_FA_WAIT(0) }
  else if (n == 2 * NDB) { CADENCE_FA_WAIT(2 * NDB) }
  else if (n == 4 * NDB) { CADENCE_FA_WAIT(4 * NDB) }
  else { CADENCE_FA_WAIT(6 * NDB) }
#undef CADENCE_FA_WAIT
}

// LAB: measurement variants for tools/vit_fa32_lab.hip only (0 = the
// product kernel): bit 0 no per-tile DMA, bit 1 no exp (P = S), bit 2 no max
// check, bit 3 no P.V MFMAs, bit 4 no QK^T MFMAs, bit 5 no sched_group_barrier
template <int HD, int NB, bool QSCALED, int LAB = 0>
__global__ __launch_bounds__(256, (LAB & 64) ? 3 : 2) void vit_fa32_kernel(
    const u16* __restrict__ qkv, u16* __restrict__ out, int B, int N, int H,
    int nqb, float qscale) {
  using L = FALayout<HD>;
  constexpr int KS = L::KS, NDB = L::NDB, PPW = L::PPW;
  static_assert(NB >= 3 && NB <= 4, "tile t + 1 read while t + 2 lands");
  // output store instructions per wave and unit (d0 = 32 db + 8 rg + 4 hi < HD)
  constexpr int NST = 4 * (HD / 32) + (HD % 32 ? 1 : 0);
  // the next unit's Q loads fly under the current unit (hd 64; hd 72 has no
  // registers to spare and loads Q at the unit's start)
  constexpr bool QPRE = !L::kWide;
  __shared__ __attribute__((aligned(16))) uint4 smem[NB * L::BUF + L::ONES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hi = lane >> 5;
  // Persistent workgroups: unit u = (image, head, block of 32-query tiles),
  // U = B H nqb of them; gridDim.x (a multiple of 8) workgroups, each walking
  // its units with one continuous DMA stream of key tiles (the next unit's
  // first tiles land under the current unit's last ones).  Dispatch deals
  // blocks round robin over the 8 XCDs, so XCD x = blockIdx % 8 owns the
  // contiguous unit range [start(x), start(x) + cnt(x)) and its workgroups
  // take them in lockstep: at any time an XCD works on a few heads, whose
  // query blocks share the K / V rows in its L2.
  const int D = H * HD;
  const int rsb = 3 * D * 2;                           // qkv row stride, bytes
  const int ntq = (N + 31) >> 5;                       // 32-query tiles per image
  const int ntiles = (N + FA_KT - 1) / FA_KT;
  const bool ragged = (N % FA_KT) != 0;
  int nunits, ubase, ustep;
  {
    const int U = B * H * nqb, gx = gridDim.x >> 3, x = blockIdx.x & 7, i = blockIdx.x >> 3;
    const int q8 = U >> 3, r8 = U & 7;
    const int cnt = q8 + (x < r8 ? 1 : 0);
    ubase = x * q8 + min(x, r8) + i;
    ustep = gx;
    nunits = i < cnt ? (cnt - i + gx - 1) / gx : 0;
  }
  if (nunits == 0) return;                             // whole workgroup
  const int total = nunits * ntiles;                   // tiles in the DMA stream
  struct Unit { int b, h, qb; };
  auto unit = [&](int k) {
    const int u = ubase + k * ustep;
    return Unit{u / (nqb * H), (u / nqb) % H, u % nqb};
  };

  if constexpr (L::kWide) {
    // the ones region (V^T row 72 of the third output block: the row sums)
    smem[NB * L::BUF + L::ONES - 64 + lane] = make_uint4(kFaOnes, kFaOnes, kFaOnes, kFaOnes);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // before tile 0's barrier
  }

  // per-lane DMA source offsets (bytes from the tile's first key row)
  const int voff_k = l32 * rsb + hi * 16;                       // K fragments
  const int voff_kt = l32 * rsb;                                // hd 72: dims 64..71 twice
  const int voff_v = (lane >> 3) * rsb + 16 * ((lane & 7) ^ (4 * ((lane >> 4) & 1)));
  const int voff_t = lane * rsb;                                // hd 72: one row per lane
  // DMA source of a unit: a buffer resource over its image and the batch
  // after it (rows past the batch read as zeros) and its K / V column bytes.
  // (The resource is a plain local: a struct member of the opaque buffer
  // type makes the kernel template's instantiation fail without a
  // diagnostic.)
  auto src_rsrc = [&](int k) {
    const Unit un = unit(k);
    const u16* im = qkv + (int64_t)un.b * N * (3 * D);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(im), 0,
                                             (int)((int64_t)(B - un.b) * N * rsb), 0x00020000);
  };
  // The DMA producer walks the stream in order: tile dt of unit dk into
  // buffer dj % NB, its source switched when the stream enters the next unit
  __amdgpu_buffer_rsrc_t drsrc = src_rsrc(0);
  int dkcol, dvcol;
  {
    const Unit un = unit(0);
    dkcol = (D + un.h * HD) * 2;
    dvcol = (2 * D + un.h * HD) * 2;
  }
  int dj = 0, dk = 0, dt = 0;
  auto stage_next = [&]() {
    uint4* base = smem + (dj % NB) * L::BUF;
    const int r0 = dt * FA_KT * rsb;
    // K (kh, ks = wave) and V rows 8 wave.. / 32 + 8 wave..
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          drsrc, (fa_lptr_t)(base + 64 * (kh * KS + wave)), 16, voff_k,
          r0 + 32 * kh * rsb + dkcol + 32 * wave, 0, 0);
#pragma unroll
    for (int vh = 0; vh < 2; ++vh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          drsrc, (fa_lptr_t)(base + L::VOFF + 64 * (4 * vh + wave)), 16, voff_v,
          r0 + (32 * vh + 8 * wave) * rsb + dvcol, 0, 0);
    if constexpr (L::kWide) {
      // the fifth piece: K dims 64..71 of key half `wave` (waves 0, 1), V
      // dims 64..71 (waves 2, 3: the same bytes twice, so every wave issues
      // PPW pieces)
      if (wave < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            drsrc, (fa_lptr_t)(base + 64 * (wave * KS + 4)), 16, voff_kt,
            r0 + 32 * wave * rsb + dkcol + 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            drsrc, (fa_lptr_t)(base + L::TOFF), 16, voff_t, r0 + dvcol + 128, 0, 0);
    }
    ++dj;
    if (++dt == ntiles) {
      dt = 0;
      if (++dk < nunits) {
        drsrc = src_rsrc(dk);
        const Unit un = unit(dk);
        dkcol = (D + un.h * HD) * 2;
        dvcol = (2 * D + un.h * HD) * 2;
      }
    }
  };
  auto stage = [&](int j, int) {
    (void)j;                       // j == dj: the stream is staged in order
    stage_next();
  };

  // Q^T fragments of unit k: B[k = dim 16 ks + 8 hi + i][n = query l32],
  // scaled by hd^-1/2 log2(e) (already in memory when QSCALED), zero past hd;
  // qload issues the loads at the unit's start, qmake finishes them where
  // they are used
  uint4 qraw[KS];
  auto qload = [&](int k) {
    const Unit un = unit(k);
    const int tq0 = un.qb * ntq / nqb;
    const int q = min((tq0 + wave) * 32 + l32, N - 1);
    const u16* qrow = qkv + ((int64_t)un.b * N + q) * (3 * D) + un.h * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 16 + 8 * hi;
      qraw[ks] = d < HD ? ld16(qrow + d) : make_uint4(0, 0, 0, 0);
    }
  };
  bf16x8 qf[KS];
  auto qmake = [&]() {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 w = qraw[ks];
      if constexpr (!QSCALED) {
        float f[8];
        unpack8(w, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] *= qscale;
        w = make_uint4(pk2bf(f32x2{f[0], f[1]}), pk2bf(f32x2{f[2], f[3]}),
                       pk2bf(f32x2{f[4], f[5]}), pk2bf(f32x2{f[6], f[7]}));
      }
      qf[ks] = __builtin_bit_cast(bf16x8, w);
    }
  };
  // tiles 0 .. NB - 3 in flight before the first unit; a unit's start stages
  // one more (its tile NB - 2) and iteration t tile t + NB - 1, each into the
  // buffer of the stream tile two back (read for the last time before the
  // barrier that precedes the DMA)
#pragma unroll
  for (int i = 0; i < NB - 2; ++i)
    if (i < total) stage(i, 0);

  f32x16 o[NDB];
#pragma unroll
  for (int j = 0; j < NDB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[j][r] = 0.0f;
  f32x4 lsum = f32x4{0.f, 0.f, 0.f, 0.f};          // hd 64: 16x16 layout
  float m = 0.0f;                                   // running max (log2 units)
  f32x16 negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) negm[r] = 0.0f;
  constexpr float kThr = 8.0f;
  // hd 64's row-sum A operand: row i = lane & 15 takes k-group lane / 16 when
  // (i < 8) == (group even)
  const bf16x8 onesA = __builtin_bit_cast(
      bf16x8, (((lane & 15) < 8) == (((lane >> 4) & 1) == 0))
                  ? make_uint4(kFaOnes, kFaOnes, kFaOnes, kFaOnes)
                  : make_uint4(0, 0, 0, 0));

  // LDS byte addresses of this lane's transposing V^T reads in buffer 0:
  // lane 4 q + p of 16-lane group g reads key row 4 hi + q, dims 32 db +
  // 16 (g & 1) + 4 p..; + 2048 per k-step, + 1024 for keys + 8
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  const int g = lane >> 4, iq = (lane >> 2) & 3, ip = lane & 3;
  const int vrow = 4 * hi + iq;
  uint32_t va[NDB];
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    const int c = 4 * db + 2 * (g & 1) + (ip >> 1);
    va[db] = sbase + 16 * L::VOFF + 128 * vrow + 16 * (c ^ (4 * ((iq >> 1) & 1))) + 8 * (ip & 1);
  }
  // hd 72, third block: dims 64..71 from the buffer's TOFF piece (lanes
  // p < 2), dim 72.. from the shared ones region (p >= 2: no buffer offset);
  // dims 80..95 (g odd) read the same addresses and are discarded
  uint32_t bomask = 0;
  if constexpr (L::kWide) {
    va[2] = sbase + 16 * (ip < 2 ? L::TOFF : NB * L::BUF + L::ONES - 64) + 16 * vrow +
            8 * (ip & 1);
    bomask = ip < 2 ? 0xffffffffu : 0u;
  }

  // tile t's V^T fragments (k-step ksp = 2 kh + j: keys 16 ksp + 4 hi +
  // 0..3 and + 8..11 of the lane's half), issued by inline asm with no wait
  // (hipcc puts a vmcnt(0) -- a wait for the LDS-DMA in flight -- in front of
  // its own transposing-read builtin); vwait retires them
  typedef uint2 VFrag[4][NDB][2];
  auto vread = [&](int t, VFrag& v) {
    const uint32_t bo = (t % NB) * (L::BUF * 16);
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const uint32_t a = va[db] + (db == 2 ? (bo & bomask) : bo);
      if (db == 2) {
        asm volatile(
            "ds_read_b64_tr_b16 %0, %8 offset:0\n\t"
            "ds_read_b64_tr_b16 %1, %8 offset:128\n\t"
            "ds_read_b64_tr_b16 %2, %8 offset:256\n\t"
            "ds_read_b64_tr_b16 %3, %8 offset:384\n\t"
            "ds_read_b64_tr_b16 %4, %8 offset:512\n\t"
            "ds_read_b64_tr_b16 %5, %8 offset:640\n\t"
            "ds_read_b64_tr_b16 %6, %8 offset:768\n\t"
            "ds_read_b64_tr_b16 %7, %8 offset:896"
            : "=&v"(v[0][db][0]), "=&v"(v[0][db][1]), "=&v"(v[1][db][0]), "=&v"(v[1][db][1]),
              "=&v"(v[2][db][0]), "=&v"(v[2][db][1]), "=&v"(v[3][db][0]), "=&v"(v[3][db][1])
            : "v"(a)
            : "memory");
      } else {
        asm volatile(
            "ds_read_b64_tr_b16 %0, %8 offset:0\n\t"
            "ds_read_b64_tr_b16 %1, %8 offset:1024\n\t"
            "ds_read_b64_tr_b16 %2, %8 offset:2048\n\t"
            "ds_read_b64_tr_b16 %3, %8 offset:3072\n\t"
            "ds_read_b64_tr_b16 %4, %8 offset:4096\n\t"
            "ds_read_b64_tr_b16 %5, %8 offset:5120\n\t"
            "ds_read_b64_tr_b16 %6, %8 offset:6144\n\t"
            "ds_read_b64_tr_b16 %7, %8 offset:7168"
            : "=&v"(v[0][db][0]), "=&v"(v[0][db][1]), "=&v"(v[1][db][0]), "=&v"(v[1][db][1]),
              "=&v"(v[2][db][0]), "=&v"(v[2][db][1]), "=&v"(v[3][db][0]), "=&v"(v[3][db][1])
            : "v"(a)
            : "memory");
      }
    }
  };
  // every LDS read of this wave retired; the V^T fragments "rewritten" by it,
  // so the MFMAs reading them stay below it
  auto vwait = [&](VFrag& v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ksp = 0; ksp < 4; ++ksp)
#pragma unroll
      for (int db = 0; db < NDB; ++db) asm volatile("" : "+v"(v[ksp][db][0]), "+v"(v[ksp][db][1]));
  };

  // S^T = K . Q'^T - m of tile t (all K fragments read first: one LDS latency)
  auto qk = [&](int t, f32x16 (&s)[2]) {
    const uint4* kb = smem + (t % NB) * L::BUF;
    bf16x8 kf[2][KS];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[kh][ks] = __builtin_bit_cast(bf16x8, kb[64 * (kh * KS + ks) + lane]);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      s[kh] = negm;
      if constexpr (!(LAB & 16)) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[kh] = mfma32(kf[kh][ks], qf[ks], s[kh]);
      }
    }
  };
  // keys past N (the ragged last tile) -> -inf
  auto mask = [&](int t, f32x16 (&s)[2]) {
    // key of (kh, r) = 32 kh + 8 (r / 4) + r % 4 + 4 hi; the limit is made
    // opaque here, so the 32 compares are done at the (rare) use instead of
    // hoisted out of every loop as 32 live lane masks (64 SGPRs)
    int lim = N - t * FA_KT - 4 * hi;
    asm volatile("" : "+v"(lim));
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (32 * kh + 8 * (r >> 2) + (r & 3) >= lim) s[kh][r] = -INFINITY;
  };
  // lane-local max of the 32 scores (relative to m): four independent chains
  auto lanemax = [&](const f32x16 (&s)[2]) {
    float c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x16& x = s[i >> 1];
      const int r0 = 8 * (i & 1);
      float v = fa_max3(x[r0], x[r0 + 1], x[r0 + 2]);
      v = fa_max3(v, x[r0 + 3], x[r0 + 4]);
      v = fa_max3(v, x[r0 + 5], x[r0 + 6]);
      c[i] = __builtin_fmaxf(v, x[r0 + 7]);
    }
    return fa_max3(fa_max3(c[0], c[1], c[2]), c[3], c[3]);
  };
  // the deferred rescale: rows whose max grew by more than kThr (every row on
  // the first tile, from m = 0 with O and l still zero) move m to their max;
  // O and l were last written by the P.V MFMAs of the previous tile, whose P
  // used the old m (the order examples of T13 require)
  auto check = [&](f32x16 (&s)[2], bool first, float lm) {
    if (!(LAB & 4) && (first || __any(lm > kThr))) {
      const float rm = fa_max_halves(lm);   // the row's max
      const bool need = first || rm > kThr;
      const float delta = need ? rm : 0.0f;
      if (!first) {
        const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
        for (int j = 0; j < NDB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[j][r] *= alpha;
        if constexpr (!L::kWide) {
          // lsum's lane holds query (lane >> 5 ? 16 : 0) + (lane & 15)
          const int src = (lane >> 5) ? 16 + (lane & 15) : (lane & 15);
          const float al = __shfl(alpha, src, 64);
#pragma unroll
          for (int r = 0; r < 4; ++r) lsum[r] *= al;
        }
      }
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kh][r] -= delta;
      m += delta;
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[r] = -m;
    }
  };
  // P = exp2(S): the B operands of the P.V k-steps
  auto expp = [&](const f32x16 (&s)[2], bf16x8 (&pf)[4]) {
#pragma unroll
    for (int ksp = 0; ksp < 4; ++ksp) {
      const int kh = ksp >> 1, j = ksp & 1;
      uint32_t pk[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2)
        pk[e >> 1] = (LAB & 2) ? pk2bf(f32x2{s[kh][8 * j + e], s[kh][8 * j + e + 1]})
                               : pk2bf(f32x2{__builtin_amdgcn_exp2f(s[kh][8 * j + e]),
                                             __builtin_amdgcn_exp2f(s[kh][8 * j + e + 1])});
      pf[ksp] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    }
  };
  // O^T += V^T . P^T (hd 64: l += selector . P^T) for the k-steps below nk keys
  auto pv = [&](const bf16x8 (&pf)[4], const VFrag& v, int nk) {
#pragma unroll
    for (int ksp = 0; ksp < 4; ++ksp) {
      if (16 * ksp >= nk) continue;
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const bf16x8 vf = __builtin_bit_cast(
            bf16x8, make_uint4(v[ksp][db][0].x, v[ksp][db][0].y, v[ksp][db][1].x,
                               v[ksp][db][1].y));
        if constexpr (!(LAB & 8)) o[db] = mfma32(vf, pf[ksp], o[db]);
      }
      if constexpr (!L::kWide && !(LAB & 8)) lsum = mfma16(onesA, pf[ksp], lsum);
    }
  };

  // tile t landed: this wave's DMA pieces of tile t (those of the tiles after
  // it may stay in flight: every wave issues PPW per tile), then every
  // wave's: a raw s_barrier (__syncthreads would wait for all DMA).  No LDS
  // read of this wave may still be in flight across it (the buffer refilled
  // right after it was read last in the previous iteration).
  // `issued`: the last tile whose DMA this wave has issued so far
  // `stores`: the output stores issued since (the previous unit's, newer
  // than every DMA piece still in flight: NST of them, or none)
  auto wait_tile = [&](int t, int issued, bool stores = false) {
    const int ahead = min(issued, total - 1) - t;
    if (stores) {
      if (NB >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PPW + NST) : "memory");
      else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW + NST) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NST) : "memory");
    } else {
      if (NB >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PPW) : "memory");
      else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // Software pipeline over key tiles: iteration t reads tile t's V^T and
  // tile t + 1's K, issues tile t + 1's QK^T MFMAs beside tile t's exp (VALU
  // independent of them: one overlaps the other inside the wave), then tile
  // t's P.V MFMAs beside tile t + 1's lane max, then tile t + 1's max check
  // (its rescale touches O after tile t's P.V: T13's order).  Two tiles per
  // loop trip, so the score tiles trade roles without register copies.
  // Stream tile j = j0 + t of unit k (j0 = k ntiles) sits in buffer j % NB.
  f32x16 sa[2], sb[2];
  VFrag vc;
  bf16x8 pf[4];
  int j0 = 0;
  // one whole step: tile t's P.V with tile t + 1 (whole) in flight
  auto step = [&](int t, f32x16 (&sc)[2], f32x16 (&sn)[2]) {
    const int j = j0 + t;
    wait_tile(j + 1, j + NB - 2);
    if (!(LAB & 1) && j + NB - 1 < total) stage(j + NB - 1, j0);
    vread(j, vc);
    qk(j + 1, sn);
    expp(sc, pf);
    if constexpr (!(LAB & 32)) {
      // every K read first, then QK^T MFMAs with the exp / pack VALU (and
      // transcendentals: mask 0x400) beside them
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS, 0);
#pragma unroll
      for (int i = 0; i < 2 * KS; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x402, 6, 0);
      }
    }
    vwait(vc);
    pv(pf, vc, FA_KT);
    const float lm = lanemax(sn);
    if constexpr (!(LAB & 32)) {
#pragma unroll
      for (int i = 0; i < 4 * NDB + (L::kWide ? 0 : 4); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x402, 2, 0);
      }
    }
    check(sn, false, lm);
  };

  bool stored = false;
  if (QPRE) {
    const Unit u0 = unit(0);
    if (u0.qb * ntq / nqb + wave < (u0.qb + 1) * ntq / nqb) qload(0);
  }
  for (int k = 0; k < nunits; ++k, j0 += ntiles) {
    const Unit un = unit(k);
    const int tq0 = un.qb * ntq / nqb, tq1 = (un.qb + 1) * ntq / nqb;
    const int qt = tq0 + wave;
    const bool active = qt < tq1;
    // the unit's first tile (its DMA issued under the previous unit), then
    // the ring topped up
    if (!QPRE && active) qload(k);
    wait_tile(j0, j0 + NB - 3, stored);
    stored = false;
    if (!(LAB & 1) && j0 + NB - 2 < total) stage(j0 + NB - 2, j0);
    if (active) qmake();
    if (QPRE && k + 1 < nunits) {
      const Unit nx = unit(k + 1);
      if (nx.qb * ntq / nqb + wave < (nx.qb + 1) * ntq / nqb) qload(k + 1);
    }
    if (!active) {
      // DMA and barriers only (the workgroup's other waves read the
      // buffers): the same barrier sequence as the active waves' pipeline
      for (int t = 0; t + 1 < ntiles; ++t) {
        wait_tile(j0 + t + 1, j0 + t + NB - 2);
        if (!(LAB & 1) && j0 + t + NB - 1 < total) stage(j0 + t + NB - 1, j0);
      }
      continue;
    }
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] = 0.0f;
    lsum = f32x4{0.f, 0.f, 0.f, 0.f};
    m = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.0f;
    qk(j0, sa);
    if (ntiles == 1 && ragged) mask(0, sa);
    check(sa, true, lanemax(sa));
    int t = 0;
    // tiles t + 1 and t + 2 whole (the last tile is stepped to below)
    for (; t + 3 < ntiles; t += 2) {
      step(t, sa, sb);
      step(t + 1, sb, sa);
    }
    if (t + 2 < ntiles) {
      step(t, sa, sb);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) sa[kh] = sb[kh];
      ++t;
    }
    if (t + 1 < ntiles) {               // tile t + 1 is the unit's last one
      const int j = j0 + t;
      wait_tile(j + 1, j + NB - 2);
      if (!(LAB & 1) && j + NB - 1 < total) stage(j + NB - 1, j0);
      vread(j, vc);
      qk(j + 1, sb);
      expp(sa, pf);
      vwait(vc);
      pv(pf, vc, FA_KT);
      if (ragged) mask(t + 1, sb);
      check(sb, false, lanemax(sb));
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) sa[kh] = sb[kh];
      ++t;
    }
    // the last tile's P.V
    vread(j0 + t, vc);
    expp(sa, pf);
    vwait(vc);
    pv(pf, vc, N - t * FA_KT);

    // the row sum of query l32
    float l;
    if constexpr (L::kWide) {
      l = __shfl(o[2][4], l32, 64);   // O^T row 72 = lane (l32, hi 0), register 4
    } else {
      l = __shfl(lsum[0], l32 < 16 ? l32 : l32 + 16, 64);
    }
    const float inv = 1.0f / l;
    // O rows by buffer stores over this image's output rows: a query past N
    // falls outside the range and is dropped, so every wave issues exactly
    // NST store instructions (the next unit's counted waits rely on it)
    const int qrow = qt * 32 + l32;
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)un.b * N * D, 0, N * D * 2, 0x00020000);
    const int obase = (qrow * D + un.h * HD) * 2;
    typedef unsigned int u32x2 __attribute__((__vector_size__(8)));
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        if (32 * db + 8 * rg >= HD) continue;       // (hd 72: rg 0 of block 2 only)
        const int d0 = 32 * db + 8 * rg + 4 * hi;
        const u32x2 w = {pk2bf(f32x2{o[db][4 * rg] * inv, o[db][4 * rg + 1] * inv}),
                         pk2bf(f32x2{o[db][4 * rg + 2] * inv, o[db][4 * rg + 3] * inv})};
        __builtin_amdgcn_raw_buffer_store_b64(w, orsrc, obase + 2 * d0, 0, 0);
      }
    stored = true;
  }
}

}  // namespace

// 32x32x16-MFMA ViT attention for hd 64 / 72 and any N; `q_scaled` says the
// q columns of qkv already hold q * hd^-1/2 * log2(e) (rounded once, by the
// q|k|v GEMM's epilogue); otherwise the kernel scales the bf16 q itself (a
// second rounding of q).  Returns -1 for other shapes (or a qkv / out pointer
// that is not 16-B aligned, or a batch whose byte size exceeds the buffer
// range).
__attribute__((visibility("hidden"))) int vit_fa32_attention_launch(
    const void* qkv, void* out, int64_t B, int64_t N, int64_t H, int64_t hd, int q_scaled,
    void* stream) {
  if ((hd != 64 && hd != 72) || N < 1 || B < 1 || H < 1) return -1;
  if (((uintptr_t)qkv | (uintptr_t)out) % 16) return -1;
  if (B * N * 3 * H * hd * 2 >= ((int64_t)1 << 31)) return -1;
  const int64_t ntq = (N + 31) / 32;
  const int64_t nqb = (ntq + 3) / 4;
  const float qs = 1.4426950408889634f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  // persistent: two workgroups per CU (a multiple of 8: one share per XCD)
  const int64_t units = B * H * nqb;
  const dim3 grid((unsigned)std::min<int64_t>((units + 7) / 8 * 8, 2 * 256));
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
#define CADENCE_FA32(HD_, NB_, QS_)                                                   \
  hipLaunchKernelGGL((vit_fa32_kernel<HD_, NB_, QS_>), grid, dim3(256), 0, st, in, o, \
                     (int)B, (int)N, (int)H, (int)nqb, qs)
  if (hd == 64) {
    if (q_scaled) CADENCE_FA32(64, 4, true);
    else CADENCE_FA32(64, 4, false);
  } else {
    if (q_scaled) CADENCE_FA32(72, 4, true);
    else CADENCE_FA32(72, 4, false);
  }
#undef CADENCE_FA32
  return (int)hipGetLastError();
}
