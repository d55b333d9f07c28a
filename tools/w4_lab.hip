// LAB (round 6): where the gated GEMM's time goes -- gemm_w4_kernel (csrc/gemm.hip)
// copied at round 6 (commit of this file) with switches: 1 no per-K-tile vmcnt(0),
// 2 no per-K-tile barrier, 4 no epilogue, 8 no in-loop DMA, 16 no MFMA;
// 32 / 64: all / half of a K-tile's DMA issued ahead of the segment's MFMAs
// (correct results: schedule variants).
// Results are wrong for every switch but 0: timing only.  Not product code.
#include "../cadence-gemma_amd/csrc/gemm.hip"

namespace {
// lab epilogue (LAB & 128): the gated outputs stored straight from the
// accumulator layout, no LDS staging -- two 2-B stores per pair of rows
// (16 lanes = 32 contiguous bytes of one row per store instruction)
template <class Epi, int MR>
CADENCE_DEV void direct_gated_epilogue(const Epi& epi, f32x4 (&acc)[MR][4], int mbase,
                                       int nbase, int lane, int M, int g) {
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
  const int obase = nbase / 2;
  float bgv[2], buv[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bgv[h] = epi.bias_at(false, obase + h * 16 + csub, g);
    buv[h] = epi.bias_at(true, obase + h * 16 + csub, g);
  }
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const uint32_t w = epi.out2(f32x2{acc[i][h][r], acc[i][h][r + 1]},
                                    f32x2{acc[i][2 + h][r], acc[i][2 + h][r + 1]}, bgv[h],
                                    buv[h]);
        const int row = mbase + i * 16 + rsub + r, c = obase + h * 16 + csub;
        if (row < M) epi.out[(int64_t)row * epi.ldo + c] = (u16)w;
        if (row + 1 < M) epi.out[(int64_t)(row + 1) * epi.ldo + c] = (u16)(w >> 16);
      }
}

template <class Epi, int MR, int LAB>
__global__ __launch_bounds__(256, 1) void w4_lab_kernel(
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
    if constexpr ((LAB & 32) != 0) {
      // lab: the K-tile's 16 DMA pieces issued ahead of the segment's MFMAs
      if (dma_on) {
#pragma unroll
        for (; nd < 16; ++nd)
          __builtin_amdgcn_global_load_lds((gptr_t)(bk + (live ? soff[nd] : zoff)),
                                           (lptr_t)(dst + nd * 64), 16, 0, 0);
      }
    }
    if constexpr ((LAB & 64) != 0) {
      // lab: the first 8 pieces ahead, the rest interleaved
      if (dma_on) {
#pragma unroll
        for (; nd < 8; ++nd)
          __builtin_amdgcn_global_load_lds((gptr_t)(bk + (live ? soff[nd] : zoff)),
                                           (lptr_t)(dst + nd * 64), 16, 0, 0);
      }
    }
#pragma unroll
    for (int n = 0; n < MR * 8; ++n) {
      const int i = n / 8, j = n % 8;
      if constexpr (!(LAB & 16))
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i][j]) : "v"(a[i]), "v"(b[j]));
      if (n % 3 == 0 && nr < MR + 8) {
        if (nr < MR) rd1(rbuf, rks, nr, na[nr]);
        else rd1(rbuf, rks, nr, nb[nr - MR]);
        ++nr;
      }
      if (!(LAB & 8) && dma_on && n % 3 == 1 && nd < 16) {
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
      if (!dma_on || (LAB & 8)) break;
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
    if constexpr (LAB & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!(LAB & 2)) p8_barrier();
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
      if constexpr ((LAB & 128) != 0)
        direct_gated_epilogue<Epi, MR>(epi, half, mbase, nbase, lane, M, g);
      else if constexpr (!(LAB & 4))
        big_epilogue<Epi, MR>(epi, half, st + h * (128 * 64), mbase, nbase, lane, M, N, g);
      else if (acc[0][0][0] == 12345.0f)   // keep the accumulators live
        epi.out[0] = 1;
    }
  }
}


// epilogue variants (results wrong, timing only): V & 1 the gate x up math
// replaced by one add per pair, V & 2 no global stores (the LDS staging kept)
template <int V>
struct EpiGatedLab : EpiGatedGelu {
  CADENCE_DEV uint32_t out2(f32x2 g, f32x2 u, float bg, float bu) const {
    if constexpr ((V & 1) != 0) return pk2bf(f32x2{g.x + u.x, g.y + u.y});
    else return EpiGatedGelu::out2(g, u, bg, bu);
  }
  CADENCE_DEV void store8(int64_t m, int f, uint4 v) const {
    if constexpr ((V & 2) != 0) {
      if (v.x == 0x12345678u) out[0] = 1;
    } else {
      EpiGatedGelu::store8(m, f, v);
    }
  }
};

}  // namespace

extern "C" int w4_lab(const void* A, const void* W, const void* bg, const void* bu, void* out,
                      int64_t M, int64_t F, int64_t K, int lab, void* stream) {
  EpiGatedGelu epi{static_cast<u16*>(out), F, static_cast<const u16*>(bg),
                   static_cast<const u16*>(bu), (int)((M + 15) / 16)};
  const int64_t N = 2 * F;
  const dim3 grid((unsigned)(((M + 255) / 256) * ((N + 255) / 256)), 1);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const u16* a = static_cast<const u16*>(A);
  const u16* w = static_cast<const u16*>(W);
#define W4L(L_) case L_: hipLaunchKernelGGL((w4_lab_kernel<EpiGatedGelu, 8, L_>), grid, dim3(256), 0, st, \
                           a, K, w, K, (int)M, (int)N, (int)K, (int64_t)0, (int64_t)0, epi); break;
  switch (lab) {
    W4L(0) W4L(1) W4L(2) W4L(3) W4L(4) W4L(8) W4L(9) W4L(16) W4L(20) W4L(24) W4L(28)
    W4L(32) W4L(64) W4L(128)
#define W4E(L_, V_) case L_: hipLaunchKernelGGL((w4_lab_kernel<EpiGatedLab<V_>, 8, 0>), grid, dim3(256), 0, \
                           st, a, K, w, K, (int)M, (int)N, (int)K, (int64_t)0, (int64_t)0, \
                           EpiGatedLab<V_>{epi}); break;
    W4E(101, 1) W4E(102, 2) W4E(103, 3)
#undef W4E
    default: return -1;
  }
#undef W4L
  return (int)hipGetLastError();
}
