// Recurrent-block kernels: Conv1D (temporal width 4) and the RG-LRU linear
// recurrence.
//
// Scan design (HBM-bound, SURVEY §8d: 8 B per (b,t,e) element here: x and a
// in, gate in, out):  one lane owns one (or two) channels of one sequence and
// walks the sequence in order, so h_t = a_t*h_{t-1} + x_t is evaluated with the
// reference's exact fp32 op order (separate mul, add; layers.py:195-197).
// Memory parallelism comes from a register ring: the next CH time steps of
// x / a / gate are in flight while the current CH steps are combined, so each
// wave keeps 3*CH loads (128-256 B each) outstanding.  Workgroups are a
// single wave so the B*E lanes spread over all 256 CUs.  The per-step dependent
// chain (two VALU ops) is far shorter than the HBM time per step.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

// ----------------------------------------------------------------- Conv1D

// One thread = 8 channels of one (b, t).
__global__ __launch_bounds__(256) void conv1d_prefill_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ bias, const int32_t* __restrict__ pos,
    u16* __restrict__ out, int64_t ldo, u16* __restrict__ cache_out, int B,
    int L, int E, int TW, int compat) {
  const int ch8 = E / 8;
  const int64_t total = (int64_t)B * L * ch8;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % ch8;
    const int64_t bt = idx / ch8;
    const int t = bt % L, b = bt / L;
    const int e0 = c * 8;
    float acc[8];
    const int nshift = TW < L ? TW : L;
    for (int s = 0; s < nshift; ++s) {
      float xv[8];
      const int ts = t - s;
      if (ts >= 0) {
        unpack8(ld16(x + ((int64_t)b * L + ts) * ldx + e0), xv);
        // document mask: product of (pos != 0) over the look-ahead taps
        const int look = compat ? s - 2 : s;
        bool keep = true;
        for (int k = 1; k <= look; ++k)
          keep = keep && (pos[(int64_t)b * L + ts + k] != 0);
        if (!keep)
#pragma unroll
          for (int i = 0; i < 8; ++i) xv[i] = 0.0f;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = 0.0f;
      }
      float wv[8];
      unpack8(ld16(w + (int64_t)(TW - 1 - s) * E + e0), wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float term = bmul(xv[i], wv[i]);
        acc[i] = s == 0 ? term : badd(acc[i], term);
      }
    }
    float bv[8];
    unpack8(ld16(bias + e0), bv);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = badd(acc[i], bv[i]);
    st16(out + ((int64_t)b * L + t) * ldo + e0, pack8(acc));
    // new state = last TW-1 inputs, left-padded with zeros when L < TW-1
    if (cache_out && t >= L - (TW - 1)) {
      const int slot = t - (L - (TW - 1));
      st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0,
           ld16(x + ((int64_t)b * L + t) * ldx + e0));
    }
    if (cache_out && t == 0 && L < TW - 1) {
      for (int slot = 0; slot < TW - 1 - L; ++slot)
        st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0,
             make_uint4(0, 0, 0, 0));
    }
  }
}

// Same arithmetic for a compile-time width: every load of the thread (TW
// input rows from clamped time indices, TW weight rows, the bias, the TW-1
// positions the document mask reads) is issued before the first multiply,
// instead of one dependent round trip per tap; terms accumulate in the same
// order (s = 0 .. TW-1, then + bias) with the same bf16 rounding.
template <int TW>
__global__ __launch_bounds__(256) void conv1d_prefill_tw_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ bias, const int32_t* __restrict__ pos,
    u16* __restrict__ out, int64_t ldo, u16* __restrict__ cache_out, int B,
    int L, int E, int compat) {
  const int ch8 = E / 8;
  const int64_t total = (int64_t)B * L * ch8;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % ch8;
    const int64_t bt = idx / ch8;
    const int t = bt % L, b = bt / L;
    const int e0 = c * 8;
    const int64_t row0 = (int64_t)b * L;
    uint4 xr[TW], wr[TW];
    bool nz[TW > 1 ? TW - 1 : 1];
#pragma unroll
    for (int s = 0; s < TW; ++s) {
      xr[s] = ld16(x + (row0 + max(t - s, 0)) * ldx + e0);
      wr[s] = ld16(w + (int64_t)(TW - 1 - s) * E + e0);
    }
#pragma unroll
    for (int j = 0; j + 1 < TW; ++j) nz[j] = pos[row0 + max(t - j, 0)] != 0;
    const uint4 br = ld16(bias + e0);
    float acc[8];
#pragma unroll
    for (int s = 0; s < TW; ++s) {
      if (s >= L) break;   // taps past the sequence are skipped, not added as 0
      // document mask: pos[t - s + k] != 0 for k = 1..look, i.e. nz[s - k]
      const int look = compat ? s - 2 : s;
      bool keep = t - s >= 0;
#pragma unroll
      for (int k = 1; k <= TW; ++k)
        if (k <= look) keep = keep && nz[s - k];
      float xv[8], wv[8];
      unpack8(xr[s], xv);
      unpack8(wr[s], wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float term = bmul(keep ? xv[i] : 0.0f, wv[i]);
        acc[i] = s == 0 ? term : badd(acc[i], term);
      }
    }
    float bv[8];
    unpack8(br, bv);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = badd(acc[i], bv[i]);
    st16(out + (row0 + t) * ldo + e0, pack8(acc));
    if (cache_out && t >= L - (TW - 1)) {
      const int slot = t - (L - (TW - 1));
      st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0, xr[0]);
    }
    if (cache_out && t == 0 && L < TW - 1) {
      for (int slot = 0; slot < TW - 1 - L; ++slot)
        st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0,
             make_uint4(0, 0, 0, 0));
    }
  }
}

// Single-token decode: full = [state (TW-1 rows), x]; no document mask
// (layers.py:478-483).  cache_out may alias cache_in (each thread reads its
// 8 channels of every state row before writing them).
template <int TW>
__global__ __launch_bounds__(256) void conv1d_decode_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ bias, const u16* cache_in, u16* out, int64_t ldo,
    u16* cache_out, int B, int E) {
  const int ch8 = E / 8;
  const int64_t total = (int64_t)B * ch8;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % ch8, b = idx / ch8;
    const int e0 = c * 8;
    uint4 rows[TW], wr[TW];
#pragma unroll
    for (int r = 0; r < TW - 1; ++r)
      rows[r] = ld16(cache_in + ((int64_t)b * (TW - 1) + r) * E + e0);
    rows[TW - 1] = ld16(x + (int64_t)b * ldx + e0);
#pragma unroll
    for (int r = 0; r < TW; ++r) wr[r] = ld16(w + (int64_t)r * E + e0);
    const uint4 bq = ld16(bias + e0);
    float acc[8];
#pragma unroll
    for (int s = 0; s < TW; ++s) {
      float xv[8], wv[8];
      unpack8(rows[TW - 1 - s], xv);
      unpack8(wr[TW - 1 - s], wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float term = bmul(xv[i], wv[i]);
        acc[i] = s == 0 ? term : badd(acc[i], term);
      }
    }
    float bv[8];
    unpack8(bq, bv);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = badd(acc[i], bv[i]);
    st16(out + (int64_t)b * ldo + e0, pack8(acc));
#pragma unroll
    for (int r = 0; r < TW - 1; ++r)
      st16(cache_out + ((int64_t)b * (TW - 1) + r) * E + e0, rows[r + 1]);
  }
}

// ------------------------------------------------------------------- scan

struct ScanArgs {
  const u16* x; int64_t ldx;
  const u16* a; int64_t lda;
  const int32_t* pos;
  const float* h0;
  const u16* gate; int64_t ldg;
  u16* out; int64_t ldo;
  float* h_last;
  int B, L, E;
};

// CPL channels (1 or 2, adjacent) of one sequence per lane; raw bf16 bits in
// the low (channel e) / high (channel e+1) half of a 32-bit register.
template <int CPL>
CADENCE_DEV uint32_t scan_ld(const u16* base) {
  if constexpr (CPL == 2) return *reinterpret_cast<const uint32_t*>(base);
  else return (uint32_t)*base;
}

// Per-lane row cursors of one sequence (row t of x is xp + t * ldx).
struct ScanLane {
  const u16* xp; const u16* ap; const u16* gp; const int32_t* pp; u16* op;
};

template <int CPL, int CH, bool GATE, bool POS>
struct ScanStage {
  uint32_t x[CH], a[CH], g[CH];
  int32_t pos[CH];
  // Unguarded: callers only pass full chunks, so the loads carry no branches
  // (a branch per load makes the compiler drain vmcnt at every join).
  CADENCE_DEV void load(const ScanArgs& p, const ScanLane& l, int t0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int64_t t = t0 + i;
      x[i] = scan_ld<CPL>(l.xp + t * p.ldx);
      a[i] = scan_ld<CPL>(l.ap + t * p.lda);
      if constexpr (GATE) g[i] = scan_ld<CPL>(l.gp + t * p.ldg);
      if constexpr (POS) pos[i] = l.pp[t];
    }
  }
};

template <int CPL, bool GATE, bool POS>
CADENCE_DEV void scan_one(const ScanArgs& p, const ScanLane& l, int64_t t,
                          float (&h)[CPL], uint32_t xs, uint32_t as,
                          uint32_t gs, int32_t ps) {
  const bool reset = POS && ps == 0;
  uint32_t packed = 0;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int sh = 16 * c;
    const float xv = __uint_as_float(((xs >> sh) & 0xffffu) << 16);
    const float av = __uint_as_float(((as >> sh) & 0xffffu) << 16);
    // layers.py:175-197: a *= ~reset; h = a * h + x in fp32, two roundings
    h[c] = add_rn(mul_rn(reset ? 0.0f : av, h[c]), xv);
    float y = rbf(h[c]);
    if constexpr (GATE) y = bmul(y, __uint_as_float(((gs >> sh) & 0xffffu) << 16));
    packed |= (uint32_t)f2bf(y) << sh;
  }
  if constexpr (CPL == 2) *reinterpret_cast<uint32_t*>(l.op + t * p.ldo) = packed;
  else l.op[t * p.ldo] = (u16)packed;
}

template <int CPL, int CH, bool GATE, bool POS>
CADENCE_DEV void scan_chunk(const ScanArgs& p, const ScanLane& l, int t0,
                            float (&h)[CPL],
                            const ScanStage<CPL, CH, GATE, POS>& s) {
#pragma unroll
  for (int i = 0; i < CH; ++i)
    scan_one<CPL, GATE, POS>(p, l, t0 + i, h, s.x[i], s.a[i],
                             GATE ? s.g[i] : 0u, POS ? s.pos[i] : 1);
}

// One wave per workgroup so the B*E/CPL lanes spread over every CU.  Full
// CH-step chunks are double-buffered in registers (the next chunk's loads are
// in flight while the current one is combined); the L % CH tail is guarded.
template <int CPL, int CH, bool GATE, bool POS>
__global__ __launch_bounds__(64) void rnn_scan_kernel(ScanArgs p) {
  const int groups = p.E / CPL;
  const int64_t gid = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (gid >= (int64_t)p.B * groups) return;
  const int b = gid / groups;
  const int e = (gid % groups) * CPL;
  const int64_t row0 = (int64_t)b * p.L;
  ScanLane l{p.x + row0 * p.ldx + e, p.a + row0 * p.lda + e,
             GATE ? p.gate + row0 * p.ldg + e : nullptr,
             POS ? p.pos + row0 : nullptr, p.out + row0 * p.ldo + e};
  float h[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) h[c] = p.h0 ? p.h0[(int64_t)b * p.E + e + c] : 0.0f;
  const int nfull = p.L / CH;
  ScanStage<CPL, CH, GATE, POS> sa, sb;
  if (nfull > 0) {
    sa.load(p, l, 0);
    for (int c = 0; c < nfull; c += 2) {
      sb.load(p, l, min(c + 1, nfull - 1) * CH);   // clamped: branch-free
      scan_chunk(p, l, c * CH, h, sa);
      if (c + 1 >= nfull) break;
      sa.load(p, l, min(c + 2, nfull - 1) * CH);
      scan_chunk(p, l, (c + 1) * CH, h, sb);
    }
  }
  for (int64_t t = (int64_t)nfull * CH; t < p.L; ++t)
    scan_one<CPL, GATE, POS>(p, l, t, h, scan_ld<CPL>(l.xp + t * p.ldx),
                             scan_ld<CPL>(l.ap + t * p.lda),
                             GATE ? scan_ld<CPL>(l.gp + t * p.ldg) : 0u,
                             POS ? l.pp[t] : 1);
  if (p.h_last) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) p.h_last[(int64_t)b * p.E + e + c] = h[c];
  }
}

// ---------------------------------------------- LDS-staged scan (prefill)
//
// One wave per (sequence, 64-channel group); lane = channel.  Time is cut
// into chunks of S steps; x / a / gate rows of a chunk (S x 128 B each) and
// its positions move HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: one
// instruction = 8 rows = 1 KiB), NB chunks in flight in an LDS ring.  That
// is what lifts the bytes in flight: a register-staged scan is capped at 63
// outstanding vector ops of 128-256 B per wave (~10 MB chip-wide), the DMA
// ops carry 1 KiB each.  The recurrence itself is the exact sequential fp32
// chain of layers.py:195-197; y rows are staged in LDS and leave as 16-B
// stores.  vmcnt is managed by hand: loads and stores retire in order, so
// "chunk c has landed" = at most (ops issued after it) outstanding.
// Measured against the register engine once that one filled the chip with
// one-wave workgroups, this variant is slower (4.4 vs 4.7 TB/s at NB=4; a
// deeper ring costs residency), so it is an A/B option, not the default.

typedef const void __attribute__((address_space(1)))* scan_gptr_t;
typedef void __attribute__((address_space(3)))* scan_lptr_t;

template <int N>
CADENCE_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0xf70);
  __asm__ volatile("" ::: "memory");
}

// wait for "BASE + k * NST ops still outstanding", k = 0..KMAX (runtime k)
template <int BASE, int NST, int K, int KMAX>
CADENCE_DEV void wait_sel(int k) {
  if constexpr (K == KMAX) {
    wait_vm<BASE + K * NST>();
  } else {
    if (k == K) wait_vm<BASE + K * NST>();
    else wait_sel<BASE, NST, K + 1, KMAX>(k);
  }
}

template <int S, int NB, bool GATE, bool POS>
__global__ __launch_bounds__(64) void rnn_scan_lds_kernel(ScanArgs p) {
  constexpr int RB = S * 64;                  // u16 per S x 64-channel slab
  constexpr int NARR = 2 + (GATE ? 1 : 0);    // x, a, [gate]
  constexpr int SLOT = NARR * RB + 128;       // u16 per ring slot (+ 64 pos)
  constexpr int NLD = NARR * (S / 8) + (POS ? 1 : 0);
  constexpr int NST = S / 8;
  static_assert(S == 16, "ring-read offsets below assume 16-step chunks");
  __shared__ __attribute__((aligned(16))) u16 lds[NB * SLOT];
  __shared__ __attribute__((aligned(16))) u16 ylds[RB];   // never a DMA target

  const int groups = p.E / 64;
  const int b = blockIdx.x / groups;
  const int e0 = (blockIdx.x % groups) * 64;
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)b * p.L;
  const int nch = (p.L + S - 1) / S;

  // per-lane DMA sources: row (lane / 8) of an 8-row piece, 16-B chunk lane % 8
  const int prow = lane >> 3, pcol = (lane & 7) * 8;
  auto issue = [&](int c) {
    u16* slot = lds + (c % NB) * SLOT;
#pragma unroll
    for (int i = 0; i < S / 8; ++i) {
      const int64_t t = min(c * S + i * 8 + prow, p.L - 1);   // clamp tail
      __builtin_amdgcn_global_load_lds(
          (scan_gptr_t)(p.x + (row0 + t) * p.ldx + e0 + pcol),
          (scan_lptr_t)(slot + i * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (scan_gptr_t)(p.a + (row0 + t) * p.lda + e0 + pcol),
          (scan_lptr_t)(slot + RB + i * 512), 16, 0, 0);
      if constexpr (GATE)
        __builtin_amdgcn_global_load_lds(
            (scan_gptr_t)(p.gate + (row0 + t) * p.ldg + e0 + pcol),
            (scan_lptr_t)(slot + 2 * RB + i * 512), 16, 0, 0);
    }
    if constexpr (POS) {
      const int64_t t = min(c * S + lane, p.L - 1);
      __builtin_amdgcn_global_load_lds((scan_gptr_t)(p.pos + row0 + t),
                                       (scan_lptr_t)(slot + NARR * RB), 4, 0, 0);
    }
  };

  // h0 rides the DMA queue ahead of chunk 0 (a register load here would make
  // the compiler drain the whole prologue before the loop).
  __shared__ float hlds[64];
  if (p.h0)
    __builtin_amdgcn_global_load_lds((scan_gptr_t)(p.h0 + (int64_t)b * p.E + e0 + lane),
                                     (scan_lptr_t)hlds, 4, 0, 0);
  float h = 0.0f;
#pragma unroll
  for (int c = 0; c < NB - 1; ++c)
    if (c < nch) issue(c);
  for (int c = 0; c < nch; ++c) {
    const bool more = c + NB - 1 < nch;
    if (more) issue(c + NB - 1);
    // chunk c landed: ops issued after it = NB-1 load groups + the store
    // groups of the last min(c, NB-1) chunks; once the ring drains, wait all.
    if (more) wait_sel<(NB - 1) * NLD, NST, 0, NB - 1>(min(c, NB - 1));
    else wait_vm<0>();
    // Ring reads go through inline asm: the compiler cannot tell ring slots
    // apart and would otherwise put vmcnt(0) before every ds_read.
    const uint32_t sbase =
        (uint32_t)(uintptr_t)(scan_lptr_t)(lds + (c % NB) * SLOT);
    const int steps = min(S, p.L - c * S);
    if (c == 0 && p.h0) {
      const uint32_t ha = (uint32_t)(uintptr_t)(scan_lptr_t)hlds + lane * 4;
      asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)"
                   : "=&v"(h) : "v"(ha) : "memory");
    }
    for (int i0 = 0; i0 < steps; i0 += 4) {
      uint32_t xv[4], av[4], gv[4] = {0, 0, 0, 0};
      int32_t pv[4] = {1, 1, 1, 1};
      const uint32_t va = sbase + i0 * 128 + lane * 2;
      asm volatile(
          "ds_read_u16 %0, %8 offset:0\n"
          "ds_read_u16 %1, %8 offset:128\n"
          "ds_read_u16 %2, %8 offset:256\n"
          "ds_read_u16 %3, %8 offset:384\n"
          "ds_read_u16 %4, %8 offset:2048\n"
          "ds_read_u16 %5, %8 offset:2176\n"
          "ds_read_u16 %6, %8 offset:2304\n"
          "ds_read_u16 %7, %8 offset:2432\n"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(xv[0]), "=&v"(xv[1]), "=&v"(xv[2]), "=&v"(xv[3]),
            "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3])
          : "v"(va) : "memory");
      if constexpr (GATE)
        asm volatile(
            "ds_read_u16 %0, %4 offset:4096\n"
            "ds_read_u16 %1, %4 offset:4224\n"
            "ds_read_u16 %2, %4 offset:4352\n"
            "ds_read_u16 %3, %4 offset:4480\n"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(gv[0]), "=&v"(gv[1]), "=&v"(gv[2]), "=&v"(gv[3])
            : "v"(va) : "memory");
      if constexpr (POS) {
        const uint32_t pa = sbase + NARR * RB * 2 + i0 * 4;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(*reinterpret_cast<int4*>(pv)) : "v"(pa) : "memory");
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (i0 + j < steps) {
          float a = __uint_as_float(av[j] << 16);
          if constexpr (POS) a = pv[j] == 0 ? 0.0f : a;   // a *= ~reset
          h = add_rn(mul_rn(a, h), __uint_as_float(xv[j] << 16));
          float y = rbf(h);
          if constexpr (GATE) y = bmul(y, __uint_as_float(gv[j] << 16));
          ylds[(i0 + j) * 64 + lane] = f2bf(y);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): y slab written
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < S / 8; ++i) {
      const int r = i * 8 + prow;
      const uint4 v = *reinterpret_cast<const uint4*>(ylds + r * 64 + pcol);
      if (r < steps)
        *reinterpret_cast<uint4*>(p.out + (row0 + c * S + r) * p.ldo + e0 + pcol) = v;
    }
  }
  if (p.h_last) p.h_last[(int64_t)b * p.E + e0 + lane] = h;
  wait_vm<0>();   // no DMA may land after the workgroup's LDS is released
}

template <int S, int NB>
bool launch_scan_lds(const ScanArgs& p, hipStream_t st) {
  const bool g = p.gate != nullptr, q = p.pos != nullptr;
  auto al = [](const void* ptr, int64_t ld) {
    return ((uintptr_t)ptr % 16 == 0) && ld % 8 == 0;
  };
  if (p.E % 64 || p.L < 2 * S || !al(p.x, p.ldx) || !al(p.a, p.lda) ||
      !al(p.out, p.ldo) || (g && !al(p.gate, p.ldg)))
    return false;
  const dim3 grid((unsigned)((int64_t)p.B * (p.E / 64))), block(64);
  if (g && q) hipLaunchKernelGGL((rnn_scan_lds_kernel<S, NB, true, true>), grid, block, 0, st, p);
  else if (g) hipLaunchKernelGGL((rnn_scan_lds_kernel<S, NB, true, false>), grid, block, 0, st, p);
  else if (q) hipLaunchKernelGGL((rnn_scan_lds_kernel<S, NB, false, true>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((rnn_scan_lds_kernel<S, NB, false, false>), grid, block, 0, st, p);
  return true;
}

template <int CPL, int CH>
void launch_scan(const ScanArgs& p, hipStream_t st) {
  const dim3 grid((unsigned)(((int64_t)p.B * (p.E / CPL) + 63) / 64)), block(64);
  const bool g = p.gate != nullptr, q = p.pos != nullptr;
  if (g && q) hipLaunchKernelGGL((rnn_scan_kernel<CPL, CH, true, true>), grid, block, 0, st, p);
  else if (g) hipLaunchKernelGGL((rnn_scan_kernel<CPL, CH, true, false>), grid, block, 0, st, p);
  else if (q) hipLaunchKernelGGL((rnn_scan_kernel<CPL, CH, false, true>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((rnn_scan_kernel<CPL, CH, false, false>), grid, block, 0, st, p);
}

int grid_for(int64_t work, int per_block = 256, int cap = 8192) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

extern "C" {

int cadence_conv1d(const void* x, int64_t ldx, const void* w, const void* b,
                   const int32_t* segment_pos, const void* cache_in,
                   void* out, int64_t ldo, void* cache_out, int64_t B,
                   int64_t L, int64_t E, int64_t temporal_width, int compat,
                   void* stream) {
  if (E % 8 || ldx % 8 || ldo % 8 || temporal_width < 1 || temporal_width > 8)
    return (int)hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (cache_in) {
    if (L != 1) return (int)hipErrorInvalidValue;
    const dim3 grid(grid_for(B * E / 8)), block(256);
    const u16* xp = static_cast<const u16*>(x);
    const u16* wp = static_cast<const u16*>(w);
    const u16* bp = static_cast<const u16*>(b);
    const u16* ci = static_cast<const u16*>(cache_in);
    u16* op = static_cast<u16*>(out);
    u16* co = static_cast<u16*>(cache_out);
    switch (temporal_width) {
#define CADENCE_CONV_TW(T) \
  case T: hipLaunchKernelGGL(conv1d_decode_kernel<T>, grid, block, 0, st, xp, ldx, wp, bp, ci, op, ldo, co, (int)B, (int)E); break;
      CADENCE_CONV_TW(1) CADENCE_CONV_TW(2) CADENCE_CONV_TW(3) CADENCE_CONV_TW(4)
      CADENCE_CONV_TW(5) CADENCE_CONV_TW(6) CADENCE_CONV_TW(7) CADENCE_CONV_TW(8)
#undef CADENCE_CONV_TW
    }
  } else {
    if (temporal_width == 4)
      hipLaunchKernelGGL(conv1d_prefill_tw_kernel<4>, dim3(grid_for(B * L * E / 8)),
                         dim3(256), 0, st, static_cast<const u16*>(x), ldx,
                         static_cast<const u16*>(w), static_cast<const u16*>(b),
                         segment_pos, static_cast<u16*>(out), ldo,
                         static_cast<u16*>(cache_out), (int)B, (int)L, (int)E,
                         compat);
    else
      hipLaunchKernelGGL(conv1d_prefill_kernel, dim3(grid_for(B * L * E / 8)),
                         dim3(256), 0, st, static_cast<const u16*>(x), ldx,
                         static_cast<const u16*>(w), static_cast<const u16*>(b),
                         segment_pos, static_cast<u16*>(out), ldo,
                         static_cast<u16*>(cache_out), (int)B, (int)L, (int)E,
                         (int)temporal_width, compat);
  }
  return (int)hipGetLastError();
}

int cadence_rnn_scan(const void* x, int64_t ldx, const void* a, int64_t lda,
                     const int32_t* segment_pos, const float* h0,
                     const void* gate, int64_t ldg, void* out, int64_t ldo,
                     float* h_last, int64_t B, int64_t L, int64_t E,
                     void* stream) {
  if (E % 2 || ldx % 2 || lda % 2 || ldo % 2 || (gate && ldg % 2))
    return (int)hipErrorInvalidValue;
  if (L <= 0 || B <= 0) return 0;
  ScanArgs p{static_cast<const u16*>(x), ldx, static_cast<const u16*>(a), lda,
             segment_pos, h0, static_cast<const u16*>(gate), ldg,
             static_cast<u16*>(out), ldo, h_last, (int)B, (int)L, (int)E};
  // Default: two channels per lane, 16-step register ring, one-wave
  // workgroups (4.7 TB/s at B=32, L=319/2048, E=2560 on MI355X).
  // CADENCE_SCAN=reg1|lds4|lds6|lds8|reg2c8|reg2c12 selects the A/B variants
  // (tools/scan_micro.py; the LDS-DMA ring measured 4.4 TB/s at NB=4 and
  // loses residency beyond it).
  hipStream_t st = static_cast<hipStream_t>(stream);
  static const int mode = [] {
    const char* v = getenv("CADENCE_SCAN");
    if (!v) return 0;
    const char* names[] = {"reg2", "reg1", "lds4", "lds6", "lds8", "reg2c8", "reg2c12"};
    for (int i = 0; i < 7; ++i)
      if (!strcmp(v, names[i])) return i;
    return 0;
  }();
  switch (mode) {
    case 1: launch_scan<1, 16>(p, st); break;
    case 2: if (!launch_scan_lds<16, 4>(p, st)) launch_scan<2, 16>(p, st); break;
    case 3: if (!launch_scan_lds<16, 6>(p, st)) launch_scan<2, 16>(p, st); break;
    case 4: if (!launch_scan_lds<16, 8>(p, st)) launch_scan<2, 16>(p, st); break;
    case 5: launch_scan<2, 8>(p, st); break;
    case 6: launch_scan<2, 12>(p, st); break;
    default: launch_scan<2, 16>(p, st);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
