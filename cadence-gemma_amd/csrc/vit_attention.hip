// ViT (bidirectional) attention for short image sequences on gfx950.
//
// One workgroup per (image, head).  The whole K (row-major, XOR-swizzled
// 16-B chunks) and V^T of the sequence are staged in LDS once; each wave then
// takes 16-query tiles.  "Swapped" QK^T: S^T = K . Q^T on
// mfma_f32_16x16x32_bf16, so a lane owns ONE query (lane & 15) and four keys
// per 16-key tile.  The softmax reductions are in-lane plus two
// xor-shuffles, and the S^T accumulator of a 32-key chunk is directly the B
// operand of O^T = V^T . P^T under the key-slot permutation
//   slot 8g + j  <->  key 4g + j (j < 4),  16 + 4g + (j - 4) (j >= 4)
// which the V^T fragment reads (two 8-B runs of 4 keys) match.  Online
// softmax over 32-key chunks, exp2 with log2(e) folded into the scale; O^T
// leaves as 8-B runs of 4 head dims of one query.
//
// Replaces timm `Attention.forward` (F.scaled_dot_product_attention,
// bidirectional, scale hd^-1/2) called from recurrentgemma/vit/dino_siglip.py
// :85-86,149-151 (timm not vendored).
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

template <int CPR>
CADENCE_DEV int kswz(int ch, int row) {
  return (CPR % 8 == 0) ? (ch ^ (row & 7)) : (ch ^ (row & 3));
}

// HDK: head dim padded to a multiple of 32 (QK^T k-steps); HDV: padded to 16
// (O^T row tiles); NPMAX: LDS capacity in keys (multiple of 32); NW waves.
template <int HDK, int HDV, int NPMAX, int NW>
__global__ __launch_bounds__(NW * 64) void vit_attn_kernel(
    const u16* __restrict__ qkv, u16* __restrict__ out, int N, int H, int hd,
    float scale_log2) {
  constexpr int CPR = HDK / 8;        // 16-B chunks per K row
  constexpr int KS = HDK / 32;
  constexpr int NDT = HDV / 16;
  constexpr int VCH = HDV / 8;
  constexpr int VTS = NPMAX + 8;      // V^T row stride (elements): 16-B pad
  constexpr int KIMG = NPMAX * CPR;   // uint4 of the K image
  // one LDS array (K image, then V^T)
  __shared__ __attribute__((aligned(16))) uint4 smem[KIMG + (HDV * VTS) / 8];
  uint4* kimg = smem;
  u16* vt = reinterpret_cast<u16*>(smem + KIMG);

  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = H * hd;
  const int64_t rs = 3 * (int64_t)D;  // qkv row stride: [q | k | v] per token
  const u16* qb = qkv + (int64_t)b * N * rs + (int64_t)h * hd;
  const u16* kb = qb + D;
  const u16* vb = qb + 2 * D;
  const int np = (N + 31) & ~31;
  const uint4 zero = make_uint4(0, 0, 0, 0);

  // K -> LDS, zero-filled past N and past hd
  for (int c = tid; c < np * CPR; c += NW * 64) {
    const int key = c / CPR, ch = c % CPR;
    uint4 v = zero;
    if (key < N && ch * 8 < hd) v = ld16(kb + key * rs + ch * 8);
    kimg[key * CPR + kswz<CPR>(ch, key)] = v;
  }
  // V^T -> LDS: one item = 4 keys x 8 dims, written as 8 runs of 4 keys
  for (int it = tid; it < (np / 4) * VCH; it += NW * 64) {
    const int kq = it / VCH, dc = it % VCH;
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kq * 4 + j;
      v[j] = (key < N && dc * 8 < hd) ? ld16(vb + key * rs + dc * 8) : zero;
    }
    const uint32_t w[4][4] = {{v[0].x, v[0].y, v[0].z, v[0].w},
                              {v[1].x, v[1].y, v[1].z, v[1].w},
                              {v[2].x, v[2].y, v[2].z, v[2].w},
                              {v[3].x, v[3].y, v[3].z, v[3].w}};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int sh = (i & 1) * 16;
      const uint32_t e0 = (w[0][i >> 1] >> sh) & 0xffffu, e1 = (w[1][i >> 1] >> sh) & 0xffffu;
      const uint32_t e2 = (w[2][i >> 1] >> sh) & 0xffffu, e3 = (w[3][i >> 1] >> sh) & 0xffffu;
      *reinterpret_cast<uint2*>(&vt[(dc * 8 + i) * VTS + kq * 4]) =
          make_uint2(e0 | (e1 << 16), e2 | (e3 << 16));
    }
  }
  __syncthreads();

  const int g = lane >> 4, c16 = lane & 15;
  const int nqt = (N + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int q = qt * 16 + c16;
    bf16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = ks * 32 + 8 * g;
      qf[ks] = __builtin_bit_cast(bf16x8, (q < N && d < hd) ? ld16(qb + q * rs + d) : zero);
    }
    f32x4 o[NDT];
#pragma unroll
    for (int j = 0; j < NDT; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.0f;
    for (int c0 = 0; c0 < np; c0 += 32) {
      f32x4 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int kr = c0 + 16 * t + c16;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kf = __builtin_bit_cast(bf16x8, kimg[kr * CPR + kswz<CPR>(ks * 4 + g, kr)]);
          s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[t], 0, 0, 0);
        }
      }
      float p[8];
      float cm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = c0 + 16 * t + 4 * g + r;
          const float v = key < N ? s[t][r] * scale_log2 : -INFINITY;
          p[t * 4 + r] = v;
          cm = fmaxf(cm, v);
        }
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      const float mn = fmaxf(m, cm);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);   // m = -inf: 0
      float ps = 0.0f;
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float e0 = __builtin_amdgcn_exp2f(p[j] - mn);
        const float e1 = __builtin_amdgcn_exp2f(p[j + 1] - mn);
        ps += e0 + e1;
        pk[j >> 1] = (uint32_t)f2bf(e0) | ((uint32_t)f2bf(e1) << 16);
      }
      l = l * alpha + ps;
      m = mn;
      const bf16x8 pf = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
        const u16* vr = vt + (dt * 16 + c16) * VTS + c0 + 4 * g;
        const uint2 lo = *reinterpret_cast<const uint2*>(vr);
        const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
        const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    if (q < N) {
      u16* orow = out + ((int64_t)b * N + q) * D + (int64_t)h * hd;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < hd) {
          const uint32_t lo = (uint32_t)f2bf(o[dt][0] * inv) | ((uint32_t)f2bf(o[dt][1] * inv) << 16);
          const uint32_t hi = (uint32_t)f2bf(o[dt][2] * inv) | ((uint32_t)f2bf(o[dt][3] * inv) << 16);
          *reinterpret_cast<uint2*>(orow + d0) = make_uint2(lo, hi);
        }
      }
    }
  }
}

}  // namespace

// LDS-resident form for the sequence lengths it covers (224-px towers:
// DINO N = 261, SigLIP N = 256); returns -1 when the caller should use the
// streaming flash kernel instead (longer sequences).
__attribute__((visibility("hidden"))) int vit_attention_lds_launch(const void* qkv, void* out, int64_t B, int64_t N,
                              int64_t H, int64_t hd, void* stream) {
  const float sl2 = 1.4426950408889634f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)H, (unsigned)B);
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
  if (hd == 64 && N <= 288) {
    hipLaunchKernelGGL((vit_attn_kernel<64, 64, 288, 4>), grid, dim3(256), 0, st, in, o,
                       (int)N, (int)H, (int)hd, sl2);
  } else if (hd == 72 && N <= 256) {
    hipLaunchKernelGGL((vit_attn_kernel<96, 80, 256, 8>), grid, dim3(512), 0, st, in, o,
                       (int)N, (int)H, (int)hd, sl2);
  } else if (hd == 72 && N <= 288) {
    hipLaunchKernelGGL((vit_attn_kernel<96, 80, 288, 8>), grid, dim3(512), 0, st, in, o,
                       (int)N, (int)H, (int)hd, sl2);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}
