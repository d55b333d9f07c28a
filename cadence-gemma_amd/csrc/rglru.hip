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
    // new state = last TW-1 inputs, left-padded with zeros when L < TW-1.
    // compat (Q4): the reference zeroes masked rows of x in place before
    // caching x[:, 1-TW:] (layers.py:506,524,542); cache row t = L - m was
    // zeroed by shift m - 1 iff pos[t + k] == 0 for some k in 1..m-3 (only
    // reachable for TW > 4)
    if (cache_out && t >= L - (TW - 1)) {
      const int slot = t - (L - (TW - 1));
      bool keep = true;
      if (compat)
        for (int k = 1; k <= L - t - 3; ++k)
          keep = keep && (pos[(int64_t)b * L + t + k] != 0);
      st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0,
           keep ? ld16(x + ((int64_t)b * L + t) * ldx + e0) : make_uint4(0, 0, 0, 0));
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

// conv1d_prefill_tw_kernel's arithmetic for TS consecutive time steps of one
// 8-channel chunk per thread: the TS + TW - 1 input rows, the TW weight rows
// and the bias are loaded and unpacked once (instead of TW row loads and
// unpacks per output), and the products / sums run on channel pairs
// (v_pk_mul / v_pk_add_f32 + one v_cvt_pk_bf16_f32 per rounding point of two
// channels: bmul2 / badd2).  Same terms in the same order (s = 0 .. TW-1,
// then + bias) with the same bf16 roundings, and a masked tap still adds
// bf16(0 * w) (signed zero included): bitwise equal to the one-step kernel.
// Threads whose outputs all keep every tap (no document start in reach: the
// common case) skip the mask selects.
template <int TW, int TS>
__global__ __launch_bounds__(256) void conv1d_prefill_ts_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ bias, const int32_t* __restrict__ pos,
    u16* __restrict__ out, int64_t ldo, u16* __restrict__ cache_out, int B,
    int L, int E, int compat) {
  constexpr int NR = TS + TW - 1;            // input rows t0 - (TW-1) .. t0 + TS - 1
  const int ch8 = E / 8;
  const int ng = (L + TS - 1) / TS;
  const int64_t total = (int64_t)B * ng * ch8;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % ch8;
    const int64_t bg = idx / ch8;
    const int t0 = (int)(bg % ng) * TS, b = (int)(bg / ng);
    const int e0 = c * 8;
    const int64_t row0 = (int64_t)b * L;
    // row r holds time t0 - (TW-1) + r, clamped into [0, L - 1]
    uint4 xr[NR], wr[TW];
    bool nz[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int tt = min(max(t0 - (TW - 1) + r, 0), L - 1);
      xr[r] = ld16(x + (row0 + tt) * ldx + e0);
    }
#pragma unroll
    for (int s = 0; s < TW; ++s) wr[s] = ld16(w + (int64_t)(TW - 1 - s) * E + e0);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int tt = min(max(t0 - (TW - 1) + r, 0), L - 1);
      nz[r] = pos[row0 + tt] != 0;
    }
    const uint4 br = ld16(bias + e0);
    // keep(i, s): output t = t0 + i, tap s reads row i + TW-1 - s; its mask
    // needs pos[t - s + k] != 0 for k = 1..look (rows i + TW-1 - s + k)
    bool keep[TS][TW];
    bool all = true;
#pragma unroll
    for (int i = 0; i < TS; ++i)
#pragma unroll
      for (int s = 0; s < TW; ++s) {
        const int look = compat ? s - 2 : s;
        bool k_ = t0 + i - s >= 0;
#pragma unroll
        for (int k = 1; k <= TW; ++k)
          if (k <= look) k_ = k_ && nz[i + TW - 1 - s + k];
        keep[i][s] = k_;
        if (t0 + i < L && s < L) all = all && k_;
      }
    f32x2 xv[NR][4], wv[TW][4], bv[4];
    auto unpack = [](uint4 q, f32x2 (&o)[4]) {
      const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = f32x2{__uint_as_float(u[j] << 16), __uint_as_float(u[j] & 0xffff0000u)};
    };
#pragma unroll
    for (int r = 0; r < NR; ++r) unpack(xr[r], xv[r]);
#pragma unroll
    for (int s = 0; s < TW; ++s) unpack(wr[s], wv[s]);
    unpack(br, bv);
    auto outputs = [&](auto masked) {
#pragma unroll
      for (int i = 0; i < TS; ++i) {
        const int t = t0 + i;
        f32x2 acc[4];
#pragma unroll
        for (int s = 0; s < TW; ++s) {
          if (s >= L) break;   // taps past the sequence are skipped, not added as 0
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f32x2 xs = xv[i + TW - 1 - s][j];
            if constexpr (decltype(masked)::value)
              xs = keep[i][s] ? xs : f32x2{0.0f, 0.0f};
            const f32x2 term = bmul2(xs, wv[s][j]);
            acc[j] = s == 0 ? term : badd2(acc[j], term);
          }
        }
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pk2bf(f32x2{add_rn(acc[j].x, bv[j].x),
                                                       add_rn(acc[j].y, bv[j].y)});
        if (t < L) st16(out + (row0 + t) * ldo + e0, make_uint4(o[0], o[1], o[2], o[3]));
      }
    };
    if (all) outputs(std::false_type{});
    else outputs(std::true_type{});
    if (cache_out) {
#pragma unroll
      for (int i = 0; i < TS; ++i) {
        const int t = t0 + i;
        if (t < L && t >= L - (TW - 1))
          st16(cache_out + ((int64_t)b * (TW - 1) + (t - (L - (TW - 1)))) * E + e0,
               xr[i + TW - 1]);
      }
      if (t0 == 0 && L < TW - 1)
        for (int slot = 0; slot < TW - 1 - L; ++slot)
          st16(cache_out + ((int64_t)b * (TW - 1) + slot) * E + e0, make_uint4(0, 0, 0, 0));
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

// ------------------------------------------- chunked (segmented) scan
//
// For batches too small to fill the chip with one lane per (sequence,
// channel pair) -- B * E / 2 lanes is 1280 at B = 1, E = 2560 -- time is cut
// into C chunks of S steps and every (sequence, 128-channel group, chunk)
// gets its own wave.  A wave loads its chunk's x / a / gate / reset rows
// into registers (all loads issued up front), then
//   1. scans the chunk from h = 0, giving the chunk's affine summary
//      h_end = P * h_in + H with P = prod(a * ~reset) (chunk 0 scans from h0
//      exactly and publishes P = 0, H = its exact end state);
//   2. publishes (P, H) per channel;
//   3. carries h_in = P_j * h_in + H_j over the summaries of chunks
//      j = 0 .. c-1 in that fixed order (deterministic: it never depends
//      on which chunks finished first);
//   4. rescans its register-resident chunk from h_in with the reference op
//      order (layers.py:195-197) and writes y (and h_last from the last
//      chunk).
// HBM traffic stays one read of the inputs and one write of y; the summary
// reads are L2 / MALL hits.  Chunks 0 and 1 are bit-exact with the
// sequential chain; later chunks differ only through the carry's rounding
// (the composed summaries round differently), which decays as a < 1.
//
// Publication needs no fence: the summary buffer starts as all-ones bits (a
// NaN) and every summary float is written and read with agent-scope atomic
// accesses (coherent across the XCDs' L2s); a reader spins per value until
// it is not NaN.  (A release / acquire fence per wave -- an L2 write-back
// plus invalidate -- cost ~40 us over 1600 waves.)  The waves of one
// (sequence, channel group) take their chunk index from a counter of that
// group in dispatch order, and chunk c only waits on chunks < c, so every
// wait is on a wave that is already running; the wait is also bounded so a
// fault cannot hang the GPU.

struct ChunkArgs {
  float* agg;           // [B][C][4][E/2]: (P0, H0, P1, H1) planes per chunk
  int32_t* ticket;      // [B][E/128] chunk counters, start at -1
  int C;
};

CADENCE_DEV float bflo(uint32_t v) { return __uint_as_float(v << 16); }
CADENCE_DEV float bfhi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }

CADENCE_DEV void agg_put(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
CADENCE_DEV float agg_get(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

template <int S, bool GATE, bool POS>
__global__ __launch_bounds__(64) void rnn_scan_chunk_kernel(ScanArgs p,
                                                            ChunkArgs c) {
  const int G = p.E / 128;
  const int BG = p.B * G;
  const int bg = blockIdx.x % BG;
  __shared__ int tk;
  if (threadIdx.x == 0) tk = atomicAdd(c.ticket + bg, 1) + 1;
  __syncthreads();
  const int chunk = tk;
  const int b = bg / G;
  const int e = (bg - b * G) * 128 + threadIdx.x * 2;
  const int lp = e >> 1;
  const int t0 = chunk * S;
  const int n = min(S, p.L - t0);
  const int64_t row0 = (int64_t)b * p.L;
  uint32_t xs[S], as[S], gs[S];
  int32_t ps[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {           // clamped rows: branch-free loads
    const int64_t t = row0 + t0 + min(i, n - 1);
    xs[i] = *reinterpret_cast<const uint32_t*>(p.x + t * p.ldx + e);
    as[i] = *reinterpret_cast<const uint32_t*>(p.a + t * p.lda + e);
    if constexpr (GATE) gs[i] = *reinterpret_cast<const uint32_t*>(p.gate + t * p.ldg + e);
    if constexpr (POS) ps[i] = p.pos[t];
  }
  float h0v = 0.f, h1v = 0.f;
  if (chunk == 0 && p.h0) {
    h0v = p.h0[(int64_t)b * p.E + e];
    h1v = p.h0[(int64_t)b * p.E + e + 1];
  }
  // component u of chunk j for this lane: agg[(j * 4 + u) * E/2] (lanes of
  // one wave are contiguous: every access instruction is 256 coalesced bytes)
  const int64_t plane = p.E / 2;
  float* agg = c.agg + (int64_t)b * c.C * 4 * plane + lp;
  if (chunk != c.C - 1) {
    // 1. summary of this chunk (from h0 for chunk 0, from 0 otherwise)
    float P0 = 1.f, P1 = 1.f, H0 = h0v, H1 = h1v;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (i < n) {
        const bool r = POS && ps[i] == 0;
        const float a0 = r ? 0.f : bflo(as[i]), a1 = r ? 0.f : bfhi(as[i]);
        H0 = add_rn(mul_rn(a0, H0), bflo(xs[i]));
        H1 = add_rn(mul_rn(a1, H1), bfhi(xs[i]));
        P0 = mul_rn(P0, a0);
        P1 = mul_rn(P1, a1);
      }
    }
    if (chunk == 0) P0 = P1 = 0.f;
    // 2. publish
    float* q = agg + (int64_t)chunk * 4 * plane;
    agg_put(q, P0);
    agg_put(q + plane, H0);
    agg_put(q + 2 * plane, P1);
    agg_put(q + 3 * plane, H1);
  }
  // 3. carry-in from the summaries of chunks 0 .. chunk-1, in order, 8 in
  // flight; a value still NaN (not yet written) is polled again
  for (int j0 = 0; j0 < chunk; j0 += 8) {
    float v[8][4];
    int spins = 0;
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float* q = agg + (int64_t)min(j0 + k, chunk - 1) * 4 * plane;
#pragma unroll
        for (int u = 0; u < 4; ++u) v[k][u] = agg_get(q + u * plane);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) ready = ready && !__builtin_isnan(v[k][u]);
      if (__all(ready) || ++spins > (1 << 20)) break;
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (j0 + k < chunk) {
        h0v = add_rn(mul_rn(v[k][0], h0v), v[k][1]);
        h1v = add_rn(mul_rn(v[k][2], h1v), v[k][3]);
      }
    }
  }
  // 4. exact rescan from the carry-in, writing y
  u16* op = p.out + (row0 + t0) * p.ldo + e;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (i < n) {
      const bool r = POS && ps[i] == 0;
      const float a0 = r ? 0.f : bflo(as[i]), a1 = r ? 0.f : bfhi(as[i]);
      h0v = add_rn(mul_rn(a0, h0v), bflo(xs[i]));
      h1v = add_rn(mul_rn(a1, h1v), bfhi(xs[i]));
      float y0 = rbf(h0v), y1 = rbf(h1v);
      if constexpr (GATE) {
        y0 = bmul(y0, bflo(gs[i]));
        y1 = bmul(y1, bfhi(gs[i]));
      }
      *reinterpret_cast<uint32_t*>(op + (int64_t)i * p.ldo) =
          (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
    }
  }
  if (chunk == c.C - 1 && p.h_last) {
    p.h_last[(int64_t)b * p.E + e] = h0v;
    p.h_last[(int64_t)b * p.E + e + 1] = h1v;
  }
}

// Chunk plan: 0 = the one-lane-per-sequence kernel (enough lanes to fill the
// chip, or too short a sequence to cut), else the chunk length S: the
// shortest of 8 / 16 / 32 / 64 steps that cuts L into at most 32 chunks
// (64 for L up to 4096).
int chunk_plan(int64_t B, int64_t L, int64_t E, int* chunks) {
  const int64_t lanes = B * E / 2;
  if (E % 128 || lanes >= 32768 || L < 16 || L > 4096) return 0;
  int S = 8;
  while (S < 64 && (L + S - 1) / S > 32) S *= 2;
  *chunks = (int)((L + S - 1) / S);
  return S;
}

int64_t chunk_ws_bytes(int64_t B, int64_t E, int64_t C) {
  return B * (E / 2) * C * 16 + B * (E / 128) * 4 + 256;
}

template <int S>
void launch_scan_chunked(const ScanArgs& p, const ChunkArgs& c, hipStream_t st) {
  const dim3 grid((unsigned)((int64_t)p.B * (p.E / 128) * c.C)), block(64);
  const bool g = p.gate != nullptr, q = p.pos != nullptr;
  if (g && q) hipLaunchKernelGGL((rnn_scan_chunk_kernel<S, true, true>), grid, block, 0, st, p, c);
  else if (g) hipLaunchKernelGGL((rnn_scan_chunk_kernel<S, true, false>), grid, block, 0, st, p, c);
  else if (q) hipLaunchKernelGGL((rnn_scan_chunk_kernel<S, false, true>), grid, block, 0, st, p, c);
  else hipLaunchKernelGGL((rnn_scan_chunk_kernel<S, false, false>), grid, block, 0, st, p, c);
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
    if (temporal_width == 4 && L >= 4)
      hipLaunchKernelGGL((conv1d_prefill_ts_kernel<4, 4>),
                         dim3(grid_for(B * ((L + 3) / 4) * E / 8)),
                         dim3(256), 0, st, static_cast<const u16*>(x), ldx,
                         static_cast<const u16*>(w), static_cast<const u16*>(b),
                         segment_pos, static_cast<u16*>(out), ldo,
                         static_cast<u16*>(cache_out), (int)B, (int)L, (int)E,
                         compat);
    else if (temporal_width == 4)
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

int64_t cadence_rnn_scan_workspace_bytes(int64_t B, int64_t L, int64_t E) {
  int C = 0;
  if (!chunk_plan(B, L, E, &C)) return 0;
  return chunk_ws_bytes(B, E, C);
}

int cadence_rnn_scan(const void* x, int64_t ldx, const void* a, int64_t lda,
                     const int32_t* segment_pos, const float* h0,
                     const void* gate, int64_t ldg, void* out, int64_t ldo,
                     float* h_last, int64_t B, int64_t L, int64_t E,
                     void* workspace, int64_t ws_bytes, void* stream) {
  if (E % 2 || ldx % 2 || lda % 2 || ldo % 2 || (gate && ldg % 2))
    return (int)hipErrorInvalidValue;
  if (L <= 0 || B <= 0) return 0;
  ScanArgs p{static_cast<const u16*>(x), ldx, static_cast<const u16*>(a), lda,
             segment_pos, h0, static_cast<const u16*>(gate), ldg,
             static_cast<u16*>(out), ldo, h_last, (int)B, (int)L, (int)E};
  hipStream_t st = static_cast<hipStream_t>(stream);
  int C = 0;
  const int S = chunk_plan(B, L, E, &C);
  if (S && workspace && ws_bytes >= chunk_ws_bytes(B, E, C) &&
      (uintptr_t)workspace % 16 == 0) {
    // small batch: chunked scan (one wave per sequence x 128 channels x
    // chunk); summaries start as NaN, chunk counters as -1 (one memset)
    char* w = static_cast<char*>(workspace);
    const int64_t agg_bytes = B * (E / 2) * C * 16;
    ChunkArgs c{reinterpret_cast<float*>(w),
                reinterpret_cast<int32_t*>(w + agg_bytes), C};
    hipError_t e = hipMemsetAsync(w, 0xff, agg_bytes + B * (E / 128) * 4, st);
    if (e != hipSuccess) return (int)e;
    if (S == 8) launch_scan_chunked<8>(p, c, st);
    else if (S == 16) launch_scan_chunked<16>(p, c, st);
    else if (S == 32) launch_scan_chunked<32>(p, c, st);
    else launch_scan_chunked<64>(p, c, st);
    return (int)hipGetLastError();
  }
  // Otherwise two channels per lane, an 8-step register ring (two chunks in
  // flight), one-wave workgroups.  Graph-replayed at B = 32, E = 2560 with
  // the y gate (tools/scan_ab.py, profiles/r04zj_scan_ab.log): L = 319
  // 40.4 -> 36.2 us against the 16-step ring (5.8 TB/s), L = 2048 289.9 ->
  // 282.1 us; one channel per lane and a 4-step ring are slower, 24 / 32-step
  // rings were slower in round 3 (profiles/r03ai_*).  Bitwise identical.
  launch_scan<2, 8>(p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
