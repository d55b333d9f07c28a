// Shared device helpers for the CadenceGemma gfx950 kernels.
//
// Storage is bf16 (raw 16-bit in HBM), arithmetic is fp32 with explicit
// bf16 rounding points where the reference rounds.
// No FMA contraction is allowed where the reference performs separate eager
// ops (see `mul_rn` / `add_rn`).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16;

#define CADENCE_DEV __device__ __forceinline__

namespace {
// 1 KiB of zeros (never written): a kernel reads a fragment that must be
// zero from here (lane-linear 16-B loads) instead of loading under a branch
// or masking a loaded value -- either makes the waitcnt pass serialise a
// full memory round trip.
__device__ __attribute__((aligned(16))) uint4 kZeroPage[64] = {};
}  // namespace

CADENCE_DEV float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
CADENCE_DEV float bf2f(bf16 v) { return (float)v; }
// Round-to-nearest-even fp32 -> bf16 (v_cvt_pk_bf16_f32 on gfx950; keeps NaN).
CADENCE_DEV u16 f2bf(float f) {
  bf16 h = (bf16)f;
  return __builtin_bit_cast(u16, h);
}
// Round an fp32 value through bf16 and back (one reference rounding point).
CADENCE_DEV float rbf(float f) { return bf2f(f2bf(f)); }

// Separate IEEE multiply / add (the reference's eager ops never fuse).
CADENCE_DEV float mul_rn(float a, float b) { return __fmul_rn(a, b); }
CADENCE_DEV float add_rn(float a, float b) { return __fadd_rn(a, b); }
CADENCE_DEV float sub_rn(float a, float b) { return __fsub_rn(a, b); }

// bf16 elementwise ops as torch computes them for bf16 tensors: promote to
// fp32, compute, round once.
CADENCE_DEV float bmul(float a, float b) { return rbf(mul_rn(a, b)); }
CADENCE_DEV float badd(float a, float b) { return rbf(add_rn(a, b)); }
CADENCE_DEV float bsub(float a, float b) { return rbf(sub_rn(a, b)); }

// Pairs: both values rounded by ONE v_cvt_pk_bf16_f32 (the same rounding as
// two rbf calls), unpacked by a shift and a mask.
CADENCE_DEV uint32_t pk2bf(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
CADENCE_DEV f32x2 rbf2(f32x2 v) {
  const uint32_t w = pk2bf(v);
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
CADENCE_DEV f32x2 bmul2(f32x2 a, f32x2 b) {
  return rbf2(f32x2{mul_rn(a.x, b.x), mul_rn(a.y, b.y)});
}
CADENCE_DEV f32x2 badd2(f32x2 a, f32x2 b) {
  return rbf2(f32x2{add_rn(a.x, b.x), add_rn(a.y, b.y)});
}

CADENCE_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// Hardware transcendentals (v_exp_f32 / v_rcp_f32 / v_sqrt_f32, ~1-2 ulp in
// fp32) for element chains whose results are rounded to bf16 right after:
// a flip of the bf16 rounding needs the fp32 error to straddle a bf16
// midpoint (~1e-5 per op).  Used where an accurate libm chain made the
// kernel VALU-bound (RG-LRU gate chain).
CADENCE_DEV float hw_exp(float x) {
  return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
}
CADENCE_DEV float hw_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + hw_exp(-x));
}
CADENCE_DEV float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
CADENCE_DEV float softplusf_(float x) {
  // torch softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}
// Exact (erf) GELU, 0.5 x (1 + erf(x / sqrt 2)) (timm / projector
// nn.GELU()), branch-free: 1 + erf(u) = erfc(-u) for u < 0 and 2 - erfc(u)
// for u >= 0, erfc by the Chebyshev fit of Numerical Recipes' erfcc
// (fractional error < 1.2e-7 on all of z >= 0, so the negative tail keeps
// its relative accuracy) with the hardware exp / reciprocal; rounded to bf16
// right after by every caller.  libm erff branches on |u| (both paths run
// when a wave diverges, ~50 VALU per element) and made the fc1 GEMM
// epilogue cost twice its MFMA time at K = 1024.
CADENCE_DEV float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float q = t * hw_exp(p - z * z);       // erfc(z)
  return 0.5f * x * (x >= 0.0f ? 2.0f - q : q);
}
// tanh-approximated GELU, 0.5 x (1 + tanh(z)) with z = sqrt(2/pi) (x +
// 0.044715 x^3) (modules.py:293-295), evaluated as the identical x *
// sigmoid(2z) with the hardware exp / reciprocal: ~3 fp32 ulp, rounded to
// bf16 right after by every caller (a flip needs the error to straddle a
// bf16 midpoint).  The libm tanhf chain was ~45 VALU per element and made
// the gated-GELU GEMM epilogue a third of that kernel's time; this form is
// also free of the 1 + tanh(z) cancellation for z << 0.
CADENCE_DEV float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
  const float k1 = 0.044715f;
  const float z = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.0f + hw_exp(-2.0f * z));
}

// gelu_erf / gelu_tanh of two values: the same IEEE operations in the same
// order (bit-identical per element), with the multiplies, adds and fmas on
// packed fp32 (v_pk_mul / v_pk_add / v_pk_fma_f32, two values per
// instruction); only the transcendentals run per element.
CADENCE_DEV f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
CADENCE_DEV f32x2 splat2(float v) { return f32x2{v, v}; }
CADENCE_DEV f32x2 gelu_erf2(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * splat2(0.70710678118654752440f);
  const f32x2 d = splat2(1.0f) + splat2(0.5f) * z;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = splat2(0.17087277f);
  p = fma2(p, t, splat2(-0.82215223f));
  p = fma2(p, t, splat2(1.48851587f));
  p = fma2(p, t, splat2(-1.13520398f));
  p = fma2(p, t, splat2(0.27886807f));
  p = fma2(p, t, splat2(-0.18628806f));
  p = fma2(p, t, splat2(0.09678418f));
  p = fma2(p, t, splat2(0.37409196f));
  p = fma2(p, t, splat2(1.00002368f));
  p = fma2(p, t, splat2(-1.26551223f));
  const f32x2 ea = (p - z * z) * splat2(1.4426950408889634f);
  const f32x2 q = t * f32x2{__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  const f32x2 two_q = splat2(2.0f) - q;
  const f32x2 s = f32x2{x.x >= 0.0f ? two_q.x : q.x, x.y >= 0.0f ? two_q.y : q.y};
  return splat2(0.5f) * x * s;
}
CADENCE_DEV f32x2 gelu_tanh2(f32x2 x) {
  const f32x2 z = splat2(0.7978845608028654f) * (x + splat2(0.044715f) * x * x * x);
  const f32x2 ea = (splat2(-2.0f) * z) * splat2(1.4426950408889634f);
  const f32x2 d = splat2(1.0f) + f32x2{__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// 16-byte vector of 8 bf16 (raw) for global/LDS traffic.
struct alignas(16) u16x8 {
  u16 v[8];
};

CADENCE_DEV uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
// Non-temporal 16-B load for bytes read once (decode weights): `nt` policy.
CADENCE_DEV uint4 ld16_nt(const void* p) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
CADENCE_DEV void st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

CADENCE_DEV void unpack8(uint4 v, float (&f)[8]) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
CADENCE_DEV uint4 pack8(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

CADENCE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
CADENCE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Decode activation layout ("packed rows"; leading dimension 0 at the C ABI,
// M <= 32 rows): the A-operand fragment order of mfma_f32_16x16x32_bf16, so
// a decode GEMV's activation load is one contiguous 1 KiB per wave
// instruction (row-major fragment loads touch 16 rows x 16 B per
// instruction and halve the weight stream's rate).  mt = ceil(M / 16).
//   Xp[((k / 32) * mt + m / 16) * 512 + (m % 16 + 16 * ((k % 32) / 8)) * 8 + k % 8]
// Eight consecutive k of one row (k % 8 == 0) are one 16-B chunk.
CADENCE_DEV int64_t xpk(int m, int k, int mt) {
  return ((((int64_t)(k >> 5) * mt + (m >> 4)) * 64 + (m & 15) + ((k >> 3) & 3) * 16)
          << 3) + (k & 7);
}
// Offset of row m, column k in either layout (ld == 0: packed).
// RoPE sin / cos of rotation pair fi at position pos (half = rope dims):
// modules.py:73-81: fp32 inverse frequency (10000 ** (2i / rope_dim))^-1,
// fp32 angle pos * inv, sin / cos rounded to the activation dtype.
CADENCE_DEV void rope_sincos(int pos, int fi, int half, float& sn, float& cs) {
  const float expo = (float)(2 * fi) / (float)half;
  const float timescale = (float)pow(10000.0, (double)expo);
  const float inv = 1.0f / timescale;
  const float ang = (float)pos * inv;
  sn = rbf((float)sin((double)ang));
  cs = rbf((float)cos((double)ang));
}

CADENCE_DEV int64_t xoff(int m, int k, int64_t ld, int mt) {
  return ld ? (int64_t)m * ld + k : xpk(m, k, mt);
}

#define CADENCE_CHECK_LAUNCH() return (int)hipGetLastError()
