// LAB KERNEL (round 6): phase-locked 8-wave ViT attention, hd 64, for
// tools/vit_pp_lab.py -- not part of libcadence_hip.so.
//
// The 32x32x16 kernel of tools/vit_fa32_kernel.hip (same fragments, same
// math: q pre-scaled, S^T = K . Q'^T - m, deferred rescale, P = exp2(S), O^T
// += V^T . P^T, MFMA row sums) restructured after the guide's 8-wave
// attention: a workgroup holds two groups of 4 waves, each group walking its
// own units (image, head, block of 32-query tiles) with its own LDS-DMA ring,
// and every wave alternates an MFMA phase (QK^T of tile t with P.V of tile
// t - 1, operands already in registers) with a VALU / LDS phase (max check,
// rescale and exp of tile t, the K fragments of tile t + 1 and the V^T
// fragments of tile t), one workgroup barrier between phases.  Group 1 runs
// one phase behind group 0, so on each SIMD (waves w and w + 4) one wave is
// in its MFMA phase while its partner is in its softmax phase.
#include "vit_fa32_kernel.hip"

namespace {

// RA: the K(t + 1) / V(t) fragment reads move into the MFMA phase (issued
// behind the QK^T MFMAs, retired by the phase's closing barrier), leaving the
// softmax phase pure VALU
template <int NB, int LAB = 0, bool RA = false>
__global__ __launch_bounds__(512, 1) void vit_pp_kernel(const u16* __restrict__ qkv,
                                                        u16* __restrict__ out, int B, int N,
                                                        int H, int nqb) {
  constexpr int HD = 64;
  using L = FALayout<HD>;
  constexpr int KS = L::KS, NDB = L::NDB, PPW = L::PPW;
  constexpr int NST = 4 * (HD / 32);
  static_assert(NB == 4 || NB == 5, "vmcnt cases below cover 4 / 5-deep rings");
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * NB * L::BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gr = wave >> 2, wq = wave & 3;
  const int l32 = lane & 31, hi = lane >> 5;
  const int D = H * HD;
  const int rsb = 3 * D * 2;
  const int ntq = (N + 31) >> 5;
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
  const int niter = (nunits + 1) >> 1;                 // unit pairs
  const int gunits = (nunits - gr + 1) >> 1;           // this group's units 2 i + gr
  const int total = gunits * ntiles;                   // tiles in this group's stream
  struct Unit { int b, h, qb; };
  auto unit = [&](int i) {
    const int u = ubase + (2 * i + gr) * ustep;
    return Unit{u / (nqb * H), (u / nqb) % H, u % nqb};
  };
  uint4* const gsm = smem + gr * NB * L::BUF;

  const int voff_k = l32 * rsb + hi * 16;
  const int voff_v = (lane >> 3) * rsb + 16 * ((lane & 7) ^ (4 * ((lane >> 4) & 1)));
  auto src_rsrc = [&](int i) {
    const Unit un = unit(i);
    const u16* im = qkv + (int64_t)un.b * N * (3 * D);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(im), 0,
                                             (int)((int64_t)(B - un.b) * N * rsb), 0x00020000);
  };
  __amdgpu_buffer_rsrc_t drsrc = src_rsrc(0);
  int dkcol, dvcol;
  {
    const Unit un = unit(0);
    dkcol = (D + un.h * HD) * 2;
    dvcol = (2 * D + un.h * HD) * 2;
  }
  int dj = 0, dk = 0, dt = 0;
  // stream tile dj (tile dt of unit dk) into buffer dj % NB: PPW pieces per wave
  auto stage_next = [&]() {
    uint4* base = gsm + (dj % NB) * L::BUF;
    const int r0 = dt * FA_KT * rsb;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          drsrc, (fa_lptr_t)(base + 64 * (kh * KS + wq)), 16, voff_k,
          r0 + 32 * kh * rsb + dkcol + 32 * wq, 0, 0);
#pragma unroll
    for (int vh = 0; vh < 2; ++vh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          drsrc, (fa_lptr_t)(base + L::VOFF + 64 * (4 * vh + wq)), 16, voff_v,
          r0 + (32 * vh + 8 * wq) * rsb + dvcol, 0, 0);
    ++dj;
    if (++dt == ntiles) {
      dt = 0;
      if (++dk < gunits) {
        drsrc = src_rsrc(dk);
        const Unit un = unit(dk);
        dkcol = (D + un.h * HD) * 2;
        dvcol = (2 * D + un.h * HD) * 2;
      }
    }
  };
  // wait until at most n of this wave's VMEM operations are in flight (n
  // rounded DOWN to a supported count: a stricter wait is always safe)
  auto vm_wait = [&](int n) {
    if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // phase boundary: this wave's LDS reads retired, then every wave
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  uint4 qraw[KS];
  auto qload = [&](int i) {
    const Unit un = unit(i);
    const int tq0 = un.qb * ntq / nqb;
    const int q = min((tq0 + wq) * 32 + l32, N - 1);
    const u16* qrow = qkv + ((int64_t)un.b * N + q) * (3 * D) + un.h * HD;
    // inline-asm loads: hipcc would otherwise put a conservative vmcnt in
    // front of their first use, across the tile loop, draining the DMA ring;
    // the phase waits below retire them (every tile staged after them)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qraw[ks])
                   : "v"(qrow + ks * 16 + 8 * hi) : "memory");
  };
  bf16x8 qf[KS];

  f32x16 o[NDB];
  f32x4 lsum = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = 0.0f;
  f32x16 negm;
  constexpr float kThr = 8.0f;
  const bf16x8 onesA = __builtin_bit_cast(
      bf16x8, (((lane & 15) < 8) == (((lane >> 4) & 1) == 0))
                  ? make_uint4(kFaOnes, kFaOnes, kFaOnes, kFaOnes)
                  : make_uint4(0, 0, 0, 0));
  const uint32_t sbase = (uint32_t)(uintptr_t)gsm;
  const int g = lane >> 4, iq = (lane >> 2) & 3, ip = lane & 3;
  const int vrow = 4 * hi + iq;
  uint32_t va[NDB];
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    const int c = 4 * db + 2 * (g & 1) + (ip >> 1);
    va[db] = sbase + 16 * L::VOFF + 128 * vrow + 16 * (c ^ (4 * ((iq >> 1) & 1))) + 8 * (ip & 1);
  }
  typedef uint2 VFrag[4][NDB][2];
  auto vread = [&](int j, VFrag& v) {
    const uint32_t bo = (j % NB) * (L::BUF * 16);
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const uint32_t a = va[db] + bo;
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
  };
  auto vwait = [&](VFrag& v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ksp = 0; ksp < 4; ++ksp)
#pragma unroll
      for (int db = 0; db < NDB; ++db) asm volatile("" : "+v"(v[ksp][db][0]), "+v"(v[ksp][db][1]));
  };
  bf16x8 kf[2][KS];
  auto kread = [&](int j) {
    const uint4* kb = gsm + (j % NB) * L::BUF;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[kh][ks] = __builtin_bit_cast(bf16x8, kb[64 * (kh * KS + ks) + lane]);
  };
  auto qk = [&](f32x16 (&s)[2]) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      s[kh] = negm;
      if constexpr (!(LAB & 16)) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[kh] = mfma32(kf[kh][ks], qf[ks], s[kh]);
      }
    }
  };
  auto mask = [&](int t, f32x16 (&s)[2]) {
    int lim = N - t * FA_KT - 4 * hi;
    asm volatile("" : "+v"(lim));
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (32 * kh + 8 * (r >> 2) + (r & 3) >= lim) s[kh][r] = -INFINITY;
  };
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
  auto check = [&](f32x16 (&s)[2], bool first, float lm) {
    if (!(LAB & 4) && (first || __any(lm > kThr))) {
      const float rm = fa_max_halves(lm);
      const bool need = first || rm > kThr;
      const float delta = need ? rm : 0.0f;
      if (!first) {
        const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
        for (int j = 0; j < NDB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[j][r] *= alpha;
        const int src = (lane >> 5) ? 16 + (lane & 15) : (lane & 15);
        const float al = __shfl(alpha, src, 64);
#pragma unroll
        for (int r = 0; r < 4; ++r) lsum[r] *= al;
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
      if constexpr (!(LAB & 8)) lsum = mfma16(onesA, pf[ksp], lsum);
    }
  };
  auto init_unit = [&]() {
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] = 0.0f;
    lsum = f32x4{0.f, 0.f, 0.f, 0.f};
    m = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.0f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, qraw[ks]);
  };
  typedef unsigned int u32x2 __attribute__((__vector_size__(8)));
  auto store_unit = [&](const Unit& un, int qt) {
    const float l = __shfl(lsum[0], l32 < 16 ? l32 : l32 + 16, 64);
    const float inv = 1.0f / l;
    const int qrow = qt * 32 + l32;
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)un.b * N * D, 0, N * D * 2, 0x00020000);
    const int obase = (qrow * D + un.h * HD) * 2;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int d0 = 32 * db + 8 * rg + 4 * hi;
        const u32x2 w = {pk2bf(f32x2{o[db][4 * rg] * inv, o[db][4 * rg + 1] * inv}),
                         pk2bf(f32x2{o[db][4 * rg + 2] * inv, o[db][4 * rg + 3] * inv})};
        __builtin_amdgcn_raw_buffer_store_b64(w, orsrc, obase + 2 * d0, 0, 0);
      }
  };

  // prologue: stream tiles 0 .. NB - 2 and unit 0's Q, all landed
#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < total) stage_next();
  if (gunits > 0) qload(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (gr == 1) bar();   // group 1 runs one phase behind

  f32x16 s[2];
  VFrag vf;
  bf16x8 pf[4];
  bool stored = false;   // this wave's output stores of the previous unit issued
  Unit prev{0, 0, 0};
  int prev_qt = 0;
  bool prev_active = false;
  for (int i = 0; i < niter; ++i) {
    const bool gact = 2 * i + gr < nunits;          // this group has a unit
    const Unit un = gact ? unit(i) : Unit{0, 0, 0};
    const int tq0 = un.qb * ntq / nqb, tq1 = (un.qb + 1) * ntq / nqb;
    const int qt = tq0 + wq;
    const bool active = gact && qt < tq1;           // this wave has a query tile
    const int j0 = i * ntiles;                      // this unit's first stream tile
    // phase E / B_pre: the previous unit's output, this unit's K(0) and Q
    if (prev_active) store_unit(prev, prev_qt);
    stored = prev_active;   // stores issued in THIS phase (newer than the ring's older tiles)
    if (active) {
      init_unit();
      kread(j0);
    }
    if constexpr (RA) {
      if (gact && ntiles > 1) {
        // tile j0 + 1 landed (read in A(0)); newer: the tiles staged after it
        // (up to j0 + NB - 2) and this phase's stores
        const int issued = min(j0 + NB - 2, total - 1);
        vm_wait((issued - (j0 + 1)) * PPW + (stored ? NST : 0));
      }
    }
    bar();
    if constexpr (RA) {
      for (int t = 0; t < ntiles; ++t) {
        const int j = j0 + t;
        // ---- phase A(t): QK^T of tile t, P.V of tile t - 1, reads of
        // K(t + 1) and V(t) ----
        if (gact && j + NB - 1 < total) stage_next();
        if (active) {
          if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(1);
          qk(s);
          if (t + 1 < ntiles) kread(j + 1);
          if (t > 0) pv(pf, vf, FA_KT);
          vread(j, vf);
          vwait(vf);
          if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(0);
        }
        bar();
        // ---- phase B(t): max check, rescale, exp of tile t ----
        if (active) {
          if (t == ntiles - 1 && ragged) mask(t, s);
          const float lm = lanemax(s);
          check(s, t == 0, lm);
          expp(s, pf);
        }
        if (t == 0 && gact && i + 1 < gunits) {
          const Unit nx = unit(i + 1);
          if (nx.qb * ntq / nqb + wq < (nx.qb + 1) * ntq / nqb) qload(i + 1);
        }
        if (gact && t + 2 < ntiles) {
          // tile j + 2 landed (read in A(t + 1))
          const int issued = min(j + NB - 1, total - 1);
          vm_wait((issued - (j + 2)) * PPW + ((stored && t + 2 <= NB - 2) ? NST : 0));
        }
        bar();
      }
    } else
    for (int t = 0; t < ntiles; ++t) {
      const int j = j0 + t;
      // ---- phase A(t): QK^T of tile t, P.V of tile t - 1 ----
      if (gact && j + NB - 1 < total) stage_next();
      if (active) {
        if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(1);
        qk(s);
        if (t > 0) pv(pf, vf, FA_KT);
        if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(0);
      }
      if (gact && t + 1 < ntiles) {
        // tile j + 1 landed (read in B(t)); newer in flight: the tiles staged
        // after it, and the previous unit's stores when they followed it
        const int issued = min(j + NB - 1, total - 1);
        vm_wait((issued - (j + 1)) * PPW + ((stored && t + 1 <= NB - 2) ? NST : 0));
      }
      bar();
      // ---- phase B(t): max check, rescale, exp of tile t; K(t+1), V(t) ----
      if (active) {
        if (t == ntiles - 1 && ragged) mask(t, s);
        const float lm = lanemax(s);
        check(s, t == 0, lm);
        expp(s, pf);
        if (t + 1 < ntiles) kread(j + 1);
        vread(j, vf);
        vwait(vf);
      }
      if (t == 0 && gact && i + 1 < gunits) {
        // the next unit's Q (waited for by the vmcnt counts of the tiles
        // after it, at the latest by that unit's first phase)
        const Unit nx = unit(i + 1);
        if (nx.qb * ntq / nqb + wq < (nx.qb + 1) * ntq / nqb) qload(i + 1);
      }
      bar();
    }
    // ---- phase A(T): P.V of the last tile ----
    if (active) {
      if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(1);
      pv(pf, vf, N - (ntiles - 1) * FA_KT);
      if constexpr (!(LAB & 32)) __builtin_amdgcn_s_setprio(0);
    }
    if (gact && j0 + ntiles < total) {
      // the next unit's tile 0 landed (read in the next phase)
      const int issued = min(j0 + ntiles - 1 + NB - 1, total - 1);
      vm_wait((issued - (j0 + ntiles)) * PPW);
    }
    // (short streams: the next unit's Q may be newer than every tile left)
    if (ntiles < NB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    prev = un;
    prev_qt = qt;
    prev_active = active;
  }
  // final phase E
  if (prev_active) store_unit(prev, prev_qt);
  if (gr == 0) bar();
}

}  // namespace

extern "C" int pp_lab(const void* qkv, void* out, int64_t B, int64_t N, int64_t H, int64_t hd,
                      int lab, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (lab == -1) return vit_fa32_attention_launch(qkv, out, B, N, H, hd, 1, stream);
  if (hd != 64 || N < 1) return -1;
  const int64_t ntq = (N + 31) / 32, nqb = (ntq + 3) / 4;
  const int64_t units = B * H * nqb;
  // one workgroup per CU, a multiple of 8 (one share per XCD); two units per
  // workgroup at a time
  const unsigned grid = (unsigned)std::min<int64_t>(((units + 1) / 2 + 7) / 8 * 8, 256);
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
  // lab bits: as vit_fa32 (2 no exp, 8 no P.V, 16 no QK^T, 32 no setprio);
  // 256 = reads in the MFMA phase (RA), 512 = a 5-deep ring
#define PP_CASE(L_)                                                                      \
  case L_:                                                                               \
    hipLaunchKernelGGL((vit_pp_kernel<4, L_>), dim3(grid), dim3(512), 0, st, in, o,     \
                       (int)B, (int)N, (int)H, (int)nqb);                                 \
    break;                                                                               \
  case 256 + L_:                                                                         \
    hipLaunchKernelGGL((vit_pp_kernel<4, L_, true>), dim3(grid), dim3(512), 0, st, in, o, \
                       (int)B, (int)N, (int)H, (int)nqb);                                 \
    break;                                                                               \
  case 768 + L_:                                                                         \
    hipLaunchKernelGGL((vit_pp_kernel<5, L_, true>), dim3(grid), dim3(512), 0, st, in, o, \
                       (int)B, (int)N, (int)H, (int)nqb);                                 \
    break;
  switch (lab) {
    PP_CASE(0)
    PP_CASE(2)
    PP_CASE(8)
    PP_CASE(16)
    PP_CASE(24)
    PP_CASE(32)
    default: return -1;
  }
#undef PP_CASE
  return (int)hipGetLastError();
}
