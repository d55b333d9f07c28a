// Decode-GEMV lab (not part of the product library): a pure-read bandwidth
// probe and a split-K weight-streaming GEMV with an in-kernel, fixed-order
// last-arriver combine, swept over (waves per block, k-steps per wave, K
// splits) by tools/gemv_lab.py.  Weights are fragment-packed
// ([N/16][K/32][64 lanes][8], include/cadence_kernels.h), M <= 32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../cadence-gemma_amd/csrc/common.hpp"

namespace {

__global__ __launch_bounds__(512) void read_kernel(const uint4* __restrict__ p,
                                                   int64_t n16, int per,
                                                   float* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * per + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < per; ++i) {
    const int64_t idx = base + (int64_t)i * blockDim.x;
    if (idx < n16) {
      const uint4 v = p[idx];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = 1.0f;
}

// grid (N/16/NTW, S); NW waves; wave w owns k-steps kb + w + NW*u, u < KSW,
// for NTW adjacent 16-column tiles (the A fragments are reused NTW times).
// NOA: ablation, no activation loads (A fragment = constant).
template <int NW, int KSW, int NTW, int AMODE, bool NT = false>
__global__ __launch_bounds__(NW * 64) void gemv_kernel(
    const u16* __restrict__ A, int64_t lda, const u16* __restrict__ Wp, int M,
    int N, int K, float* __restrict__ parts, int* __restrict__ cnt,
    const u16* __restrict__ bias, u16* __restrict__ out, int64_t ldo) {
  constexpr int OUTS = 32 * 16 * NTW;
  constexpr int KRMAX = NW * KSW * 32;      // k elements per block
  __shared__ float red[NW][OUTS];
  __shared__ int ticket;
  constexpr bool kLds = AMODE == 3 && KRMAX * 64 <= 98304;
  __shared__ __attribute__((aligned(16))) u16 as[kLds ? 32 * KRMAX : 8];
  const int grp = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kst = K >> 5;
  const int per = (kst + S - 1) / S;
  const int kb = split * per, ke = min(kst, kb + per);
  const uint4 zero = make_uint4(0, 0, 0, 0);
  uint4 wb[KSW][NTW], xa[KSW][2];
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kb + wave + NW * u;
#pragma unroll
    for (int t = 0; t < NTW; ++t)
      wb[u][t] = k < ke ? (NT ? ld16_nt(Wp + (((int64_t)(grp * NTW + t) * kst + k) * 64 + lane) * 8)
                              : ld16(Wp + (((int64_t)(grp * NTW + t) * kst + k) * 64 + lane) * 8))
                        : zero;
  }
  if constexpr (kLds) {
    // rows of A[kb*32 .. ke*32) -> LDS [32][KRMAX], 16-B chunk c of row r at
    // slot c ^ (r & 15) inside its 256-B group; one DMA instruction = 1 KiB.
    typedef const void __attribute__((address_space(1)))* gptr_t;
    typedef void __attribute__((address_space(3)))* lptr_t;
    const int cpr = KRMAX / 8;                 // chunks per row
    const int total = 32 * cpr;                // chunks
    for (int base = wave * 64; base < total; base += NW * 64) {
      const int idx = base + lane;
      const int r = idx / cpr, slot = idx % cpr;
      const int c = (slot & ~15) | ((slot & 15) ^ (r & 15));
      const int m = min(r, M - 1);
      const int kk = min(kb * 32 + c * 8, K - 8);
      __builtin_amdgcn_global_load_lds((gptr_t)(A + (int64_t)m * lda + kk),
                                       (lptr_t)(as + base * 8), 16, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kb + wave + NW * u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = i * 16 + (lane & 15);
      if constexpr (AMODE == 1)
        xa[u][i] = make_uint4(0x3f803f80u, 0, 0, (uint32_t)k);
      else if constexpr (AMODE == 2)
        xa[u][i] = k < ke ? ld16(A + (((int64_t)k * 2 + i) * 64 + lane) * 8) : zero;
      else if constexpr (AMODE == 0)
        xa[u][i] = (k < ke && m < M) ? ld16(A + (int64_t)m * lda + k * 32 + 8 * (lane >> 4))
                                     : zero;
    }
  }
  if constexpr (kLds) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KSW; ++u) {
      const int kl = wave + NW * u;            // local k-step
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = i * 16 + (lane & 15);
        const int c = kl * 4 + (lane >> 4);
        const int slot = (c & ~15) | ((c & 15) ^ (r & 15));
        xa[u][i] = kb + kl < ke ? *reinterpret_cast<const uint4*>(as + (r * (KRMAX / 8) + slot) * 8)
                                : zero;
      }
    }
  }
  f32x4 acc[2][NTW];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[i][t] = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < KSW; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < NTW; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[u][i]), __builtin_bit_cast(bf16x8, wb[u][t]),
            acc[i][t], 0, 0, 0);
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
  // red layout: [m][t][16]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][((i * 16 + rsub + r) * NTW + t) * 16 + csub] = acc[i][t][r];
  __syncthreads();
  for (int o = threadIdx.x; o < OUTS; o += NW * 64) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][o];
    red[0][o] = v;
  }
  if (S > 1) {
    __syncthreads();
    float* dst = parts + ((int64_t)grp * S + split) * OUTS;
    for (int o = threadIdx.x * 4; o < OUTS; o += NW * 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&red[0][o]);
      asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(dst + o), "v"(v) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      ticket = __hip_atomic_fetch_add(&cnt[grp], 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (ticket != S - 1) return;
    const float* src = parts + (int64_t)grp * S * OUTS;
    for (int o = threadIdx.x; o < OUTS; o += NW * 64) {
      float v = 0.0f;
      for (int s = 0; s < S; ++s)
        v += __hip_atomic_load(src + s * OUTS + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      red[0][o] = v;
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(&cnt[grp], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < OUTS; o += NW * 64) {
    const int m = o / (16 * NTW), tc = o % (16 * NTW);
    if (m >= M) continue;
    const int n = grp * NTW * 16 + tc;
    float v = red[0][o];
    if (bias) v += bf2f(bias[n]);
    out[(int64_t)m * ldo + n] = f2bf(v);
  }
}

}  // namespace

extern "C" {

int lab_read(const void* p, int64_t bytes, float* out, int blocks, void* stream) {
  const int64_t n16 = bytes / 16;
  const int per = (int)((n16 + (int64_t)blocks * 512 - 1) / ((int64_t)blocks * 512));
  hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream,
                     (const uint4*)p, n16, per, out);
  return (int)hipGetLastError();
}

int lab_gemv(const void* A, int64_t lda, const void* Wp, int M, int N, int K,
             int nw, int ksw, int ntw, int amode, int splits, float* parts, int* cnt,
             const void* bias, void* out, int64_t ldo, void* stream) {
  const dim3 grid(N / 16 / ntw, splits);
  hipStream_t st = (hipStream_t)stream;
#define L1(NW_, KSW_, NTW_, AM_)                                                   \
  if (nw == NW_ && ksw == KSW_ && ntw == NTW_ && (amode & 15) == AM_) {            \
    if (amode & 16)                                                                \
      hipLaunchKernelGGL((gemv_kernel<NW_, KSW_, NTW_, AM_, true>), grid,          \
                         dim3(NW_ * 64), 0, st, (const u16*)A, lda, (const u16*)Wp, \
                         M, N, K, parts, cnt, (const u16*)bias, (u16*)out, ldo);   \
    else                                                                           \
      hipLaunchKernelGGL((gemv_kernel<NW_, KSW_, NTW_, AM_, false>), grid,         \
                         dim3(NW_ * 64), 0, st, (const u16*)A, lda, (const u16*)Wp, \
                         M, N, K, parts, cnt, (const u16*)bias, (u16*)out, ldo);   \
    return (int)hipGetLastError();                                                 \
  }
#define L(NW_, KSW_, NTW_) L1(NW_, KSW_, NTW_, 0) L1(NW_, KSW_, NTW_, 2)
  L(8, 10, 1) L(8, 4, 2) L(8, 5, 2) L(4, 5, 2) L(4, 5, 4) L(8, 5, 4) L(16, 2, 2) L(4, 10, 2) L(8, 10, 2)
  L(4, 10, 1) L(8, 5, 1) L(4, 20, 1) L(8, 2, 1) L(8, 4, 1) L(16, 5, 1) L(16, 1, 1)
#undef L1
#undef L
  return 1;
}

}  // extern "C"
