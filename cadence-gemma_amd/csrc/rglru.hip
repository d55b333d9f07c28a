// Recurrent-block kernels: Conv1D (temporal width 4) and the RG-LRU linear
// recurrence.
//
// Scan design (HBM-bound, SURVEY §8d: 8 B per (b,t,e) element here: x and a
// in, gate in, out):  one lane owns two channels of one sequence and walks
// the sequence in order, so h_t = a_t*h_{t-1} + x_t is evaluated with the
// reference's exact fp32 op order (separate mul, add; layers.py:195-197).
// Memory parallelism comes from a register ring: the next CH time steps of
// x / a / gate are in flight while the current CH steps are combined, so each
// wave keeps 3*CH loads (256 B each) outstanding.  The per-step dependent
// chain (two VALU ops) is far shorter than the HBM time per step.
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

// Single-token decode: full = [state (TW-1 rows), x]; no document mask
// (layers.py:478-483).  cache_out may alias cache_in (each thread reads its
// 8 channels of every state row before writing them).
__global__ __launch_bounds__(256) void conv1d_decode_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ bias, const u16* cache_in, u16* out, int64_t ldo,
    u16* cache_out, int B, int E, int TW) {
  const int ch8 = E / 8;
  const int64_t total = (int64_t)B * ch8;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int c = idx % ch8, b = idx / ch8;
    const int e0 = c * 8;
    uint4 rows[8];  // TW <= 8
    for (int r = 0; r < TW - 1; ++r)
      rows[r] = ld16(cache_in + ((int64_t)b * (TW - 1) + r) * E + e0);
    rows[TW - 1] = ld16(x + (int64_t)b * ldx + e0);
    float acc[8];
    for (int s = 0; s < TW; ++s) {
      float xv[8], wv[8];
      unpack8(rows[TW - 1 - s], xv);
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
    st16(out + (int64_t)b * ldo + e0, pack8(acc));
    for (int r = 0; r < TW - 1; ++r)
      st16(cache_out + ((int64_t)b * (TW - 1) + r) * E + e0, rows[r + 1]);
  }
}

// ------------------------------------------------------------------- scan

constexpr int CH = 16;  // time steps per register stage

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

__device__ __forceinline__ void scan_load(const ScanArgs& p, int b, int e,
                                          int t0, uint32_t (&xs)[CH],
                                          uint32_t (&as)[CH],
                                          uint32_t (&gs)[CH], int32_t (&ps)[CH]) {
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int t = t0 + i;
    if (t < p.L) {
      const int64_t row = (int64_t)b * p.L + t;
      xs[i] = *reinterpret_cast<const uint32_t*>(p.x + row * p.ldx + e);
      as[i] = *reinterpret_cast<const uint32_t*>(p.a + row * p.lda + e);
      gs[i] = p.gate ? *reinterpret_cast<const uint32_t*>(p.gate + row * p.ldg + e)
                     : 0u;
      ps[i] = p.pos ? p.pos[row] : 1;
    }
  }
}

__device__ __forceinline__ void scan_step(const ScanArgs& p, int b, int e,
                                          int t0, float& h0v, float& h1v,
                                          const uint32_t (&xs)[CH],
                                          const uint32_t (&as)[CH],
                                          const uint32_t (&gs)[CH],
                                          const int32_t (&ps)[CH]) {
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int t = t0 + i;
    if (t < p.L) {
      const bool reset = ps[i] == 0;
      const float x0 = __uint_as_float(xs[i] << 16);
      const float x1 = __uint_as_float(xs[i] & 0xffff0000u);
      const float a0 = reset ? 0.0f : __uint_as_float(as[i] << 16);
      const float a1 = reset ? 0.0f : __uint_as_float(as[i] & 0xffff0000u);
      h0v = add_rn(mul_rn(a0, h0v), x0);
      h1v = add_rn(mul_rn(a1, h1v), x1);
      float y0 = rbf(h0v), y1 = rbf(h1v);
      if (p.gate) {
        y0 = bmul(y0, __uint_as_float(gs[i] << 16));
        y1 = bmul(y1, __uint_as_float(gs[i] & 0xffff0000u));
      }
      const int64_t row = (int64_t)b * p.L + t;
      *reinterpret_cast<uint32_t*>(p.out + row * p.ldo + e) =
          (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
    }
  }
}

__global__ __launch_bounds__(256) void rnn_scan_kernel(ScanArgs p) {
  const int pairs = p.E / 2;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)p.B * pairs) return;
  const int b = gid / pairs;
  const int e = (gid % pairs) * 2;
  float h0v = p.h0 ? p.h0[(int64_t)b * p.E + e] : 0.0f;
  float h1v = p.h0 ? p.h0[(int64_t)b * p.E + e + 1] : 0.0f;
  uint32_t xa[CH], aa[CH], ga[CH], xb[CH], ab[CH], gb[CH];
  int32_t pa[CH], pb[CH];
  scan_load(p, b, e, 0, xa, aa, ga, pa);
  for (int t0 = 0; t0 < p.L; t0 += 2 * CH) {
    if (t0 + CH < p.L) scan_load(p, b, e, t0 + CH, xb, ab, gb, pb);
    scan_step(p, b, e, t0, h0v, h1v, xa, aa, ga, pa);
    if (t0 + CH >= p.L) break;
    if (t0 + 2 * CH < p.L) scan_load(p, b, e, t0 + 2 * CH, xa, aa, ga, pa);
    scan_step(p, b, e, t0 + CH, h0v, h1v, xb, ab, gb, pb);
  }
  if (p.h_last) {
    p.h_last[(int64_t)b * p.E + e] = h0v;
    p.h_last[(int64_t)b * p.E + e + 1] = h1v;
  }
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
    hipLaunchKernelGGL(conv1d_decode_kernel, dim3(grid_for(B * E / 8)), dim3(256),
                       0, st, static_cast<const u16*>(x), ldx,
                       static_cast<const u16*>(w), static_cast<const u16*>(b),
                       static_cast<const u16*>(cache_in), static_cast<u16*>(out),
                       ldo, static_cast<u16*>(cache_out), (int)B, (int)E,
                       (int)temporal_width);
  } else {
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
  const int64_t threads = B * E / 2;
  hipLaunchKernelGGL(rnn_scan_kernel, dim3((unsigned)((threads + 255) / 256)),
                     dim3(256), 0, static_cast<hipStream_t>(stream), p);
  return (int)hipGetLastError();
}

}  // extern "C"
