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
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// max of scores that are finite or -inf.  Compiler-visible (not inline
// asm): the hazard recognizer must see these reads of fresh MFMA results
// (an MFMA's D read by an asm VALU within ~12 wait states reads stale
// accumulators -- observed as run-to-run differences in the output).
CADENCE_DEV float max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
CADENCE_DEV float max2(float a, float b) { return __builtin_fmaxf(a, b); }
// max over lanes l, l ^ 16, l ^ 32, l ^ 48 (the four 16-lane rows) with the
// gfx950 row swaps instead of two LDS-routed ds_bpermute
CADENCE_DEV float max_rows(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float m = max2(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const uint32_t w = __float_as_uint(m);
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return max2(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// two fp32 -> packed bf16 pair in one v_cvt_pk_bf16_f32 (RNE)
CADENCE_DEV uint32_t pk2bf(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// V^T columns are stored in the P^T slot order of each 32-key group (slot
// 8g + j <-> key 4g + j for j < 4, 16 + 4g + j - 4 for j >= 4), so a lane's 8
// keys of a PV k-step are one 16-B run.  vslot(k) for a key k = 4q.
CADENCE_DEV int vslot(int k) {
  const int k0 = k & 31;
  return (k & ~31) + (k0 < 16 ? 8 * (k0 >> 2) : 8 * ((k0 - 16) >> 2) + 4);
}

// K image: KW stored 16-B chunks per key row, XOR-swizzled so that the
// 16-lane ds_read_b128 groups of a k-step are conflict-free (checked
// exhaustively for both row strides): 8 chunks (128-B rows): ch ^ (row & 7);
// 10 chunks (160-B rows): chunks 0-7 ^ ((row >> 2) & 7), the pair 8-9 ^ (row & 1).
template <int KW>
CADENCE_DEV int kswz(int ch, int row) {
  if constexpr (KW == 8) return ch ^ (row & 7);
  return ch < 8 ? (ch ^ ((row >> 2) & 7)) : (8 + ((ch - 8) ^ (row & 1)));
}

// HDK: head dim padded to a multiple of 32 (QK^T k-steps); HDV: padded to 16
// (O^T row tiles); NPMAX: LDS capacity in keys (multiple of 32); NW waves;
// QT query tiles per wave pass.  Only what the head dim needs is stored:
// KW = ceil(hd / 8) chunks of each K row (a k-step chunk past KW re-reads
// chunk KW - 2 or KW - 1 of the same row: finite, and its Q fragment is
// zero) and VR = hd rows of V^T (O^T rows >= hd read row VR - 1 and are
// discarded) -- for hd 72 that is 79 KB, two workgroups per CU.
template <int HDK, int HDV, int NPMAX, int NW, int QT, int KW = HDK / 8, int VR = HDV>
__global__ __launch_bounds__(NW * 64, 4) void vit_attn_kernel(
    const u16* __restrict__ qkv, u16* __restrict__ out, int N, int H, int hd,
    float scale_log2) {
  constexpr int CPR = KW;             // stored 16-B chunks per K row
  constexpr int KS = HDK / 32;
  constexpr int NDT = HDV / 16;
  constexpr int VCH = VR / 8;         // stored V^T row groups of 8 dims
  constexpr int VTS = NPMAX + 16;     // V^T row stride: 32-B pad (b128 reads conflict-free)
  constexpr int KIMG = NPMAX * CPR;   // uint4 of the K image
  static_assert(KW % 2 == 0 && KW >= 8 && KW * 8 <= HDK && VR % 8 == 0, "layout");
  // one LDS array (K image, then V^T)
  __shared__ __attribute__((aligned(16))) uint4 smem[KIMG + (VR * VTS) / 8];
  uint4* kimg = smem;
  u16* vt = reinterpret_cast<u16*>(smem + KIMG);

  // XCD-aware (image, head) order: workgroups are dispatched round-robin
  // over the 8 XCDs, so remap the dispatch index (bijectively) to give each
  // XCD a contiguous range of images -- all heads of an image then share
  // one L2 for the image's q|k|v rows (SigLIP's 144-B head slices straddle
  // 128-B lines shared by neighbouring heads).
  int h, b;
  {
    const int nh = gridDim.x, total = nh * gridDim.y;
    const int lin = blockIdx.x + blockIdx.y * nh;
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int p = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    h = p % nh;
    b = p / nh;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = H * hd;
  const int64_t rs = 3 * (int64_t)D;  // qkv row stride: [q | k | v] per token
  const u16* qb = qkv + (int64_t)b * N * rs + (int64_t)h * hd;
  const u16* kb = qb + D;
  const u16* vb = qb + 2 * D;
  const int np = (N + 31) & ~31;
  const uint4 zero = make_uint4(0, 0, 0, 0);

  const int g = lane >> 4, c16 = lane & 15;
  const int nqt = (N + 15) >> 4;
  // QT query tiles per pass share every K / V^T fragment read and give the
  // wave QT independent S -> softmax -> PV chains to interleave.
  // Q fragments: unconditional loads from clamped addresses (a branch around
  // a load costs a full vmcnt(0) round trip), the next pass's prefetched
  // while this one computes.
  auto load_q = [&](int qt0, uint4 (&dst)[QT][KS]) {
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const int qq = min((qt0 + u) * 16 + c16, N - 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        dst[u][ks] = ld16(qb + qq * rs + min(ks * 32 + 8 * g, hd - 8));
    }
  };
  // K -> LDS (zero-filled past N and past hd) and V^T -> LDS (one item = 4
  // keys x 8 dims, written as 8 runs of 4 keys).  Every staging load of the
  // thread is issued before the first LDS write (branch-free: absent chunks
  // read the zero page), and the first Q fragments with them: one memory
  // round trip for the whole staging instead of one per loop iteration.
  constexpr int NT = NW * 64;
  constexpr int KIT = (NPMAX * CPR + NT - 1) / NT;
  constexpr int VIT = ((NPMAX / 4) * VCH + NT - 1) / NT;
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  uint4 kv[KIT], vv[VIT][4];
#pragma unroll
  for (int i = 0; i < KIT; ++i) {
    const int c = tid + i * NT;
    const int key = c / CPR, ch = c % CPR;
    const bool ok = c < np * CPR && key < N && ch * 8 < hd;
    kv[i] = ld16(ok ? kb + key * rs + ch * 8 : zpage);
  }
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int it = tid + i * NT;
    const int kq = it / VCH, dc = it % VCH;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kq * 4 + j;
      const bool ok = it < (np / 4) * VCH && key < N && dc * 8 < hd;
      vv[i][j] = ld16(ok ? vb + key * rs + dc * 8 : zpage);
    }
  }
  uint4 qn[QT][KS];
  load_q(wave * QT, qn);
#pragma unroll
  for (int i = 0; i < KIT; ++i) {
    const int c = tid + i * NT;
    if (c < np * CPR) {
      const int key = c / CPR, ch = c % CPR;
      kimg[key * CPR + kswz<CPR>(ch, key)] = kv[i];
    }
  }
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int it = tid + i * NT;
    if (it < (np / 4) * VCH) {
      const int kq = it / VCH, dc = it % VCH;
      const uint32_t w[4][4] = {{vv[i][0].x, vv[i][0].y, vv[i][0].z, vv[i][0].w},
                                {vv[i][1].x, vv[i][1].y, vv[i][1].z, vv[i][1].w},
                                {vv[i][2].x, vv[i][2].y, vv[i][2].z, vv[i][2].w},
                                {vv[i][3].x, vv[i][3].y, vv[i][3].z, vv[i][3].w}};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int sh = (e & 1) * 16;
        const uint32_t e0 = (w[0][e >> 1] >> sh) & 0xffffu, e1 = (w[1][e >> 1] >> sh) & 0xffffu;
        const uint32_t e2 = (w[2][e >> 1] >> sh) & 0xffffu, e3 = (w[3][e >> 1] >> sh) & 0xffffu;
        *reinterpret_cast<uint2*>(&vt[(dc * 8 + e) * VTS + vslot(kq * 4)]) =
            make_uint2(e0 | (e1 << 16), e2 | (e3 << 16));
      }
    }
  }
  __syncthreads();

  for (int qt0 = wave * QT; qt0 < nqt; qt0 += NW * QT) {
    int q[QT];
    bf16x8 qf[QT][KS];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      q[u] = (qt0 + u) * 16 + c16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bool ok = q[u] < N && ks * 32 + 8 * g < hd;
        qf[u][ks] = __builtin_bit_cast(bf16x8, ok ? qn[u][ks] : zero);
      }
    }
    load_q(min(qt0 + NW * QT, nqt - 1), qn);
    f32x4 o[QT][NDT];
    float m[QT], l[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      m[u] = -INFINITY;
      l[u] = 0.0f;
#pragma unroll
      for (int j = 0; j < NDT; ++j) o[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // 64-key chunks (the last one may be a 32-key tail), masking only where
    // a chunk runs past N, the scale folded into one FMA before exp2, and the
    // running max updated only when it grows by more than 2^8 (deferred
    // rescale: P <= 256 is exact enough in bf16, l and O stay fp32).
    constexpr float kThr = 8.0f;
    // one 64-key chunk; MASK / TWO (32-key tail) only on the last chunk, so
    // the full chunks carry no masking code
    auto chunk = [&](int c0, auto mask_tag, auto two_tag) {
      constexpr bool mask = decltype(mask_tag)::value;
      constexpr bool two = decltype(two_tag)::value;
      f32x4 s[QT][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int u = 0; u < QT; ++u) s[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t >= 2 && two) continue;
        const int kr = c0 + 16 * t + c16;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int lc = ks * 4 + g;
          const int ch = lc < CPR ? lc : lc - 2;   // past the stored chunks
          const bf16x8 kf = __builtin_bit_cast(bf16x8, kimg[kr * CPR + kswz<CPR>(ch, kr)]);
#pragma unroll
          for (int u = 0; u < QT; ++u)
            s[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[u][ks], s[u][t], 0, 0, 0);
        }
      }
      bf16x8 pf[QT][2];
#pragma unroll
      for (int u = 0; u < QT; ++u) {
        if (mask) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (c0 + 16 * t + 4 * g + r >= N) s[u][t][r] = -INFINITY;
        }
        float smax = max3(s[u][0][0], s[u][0][1], s[u][0][2]);
        smax = max3(smax, s[u][0][3], s[u][1][0]);
        smax = max3(smax, s[u][1][1], s[u][1][2]);
        if (two) {
          smax = max2(smax, s[u][1][3]);
        } else {
          smax = max3(smax, s[u][1][3], s[u][2][0]);
          smax = max3(smax, s[u][2][1], s[u][2][2]);
          smax = max3(smax, s[u][2][3], s[u][3][0]);
          smax = max3(smax, s[u][3][1], s[u][3][2]);
          smax = max2(smax, s[u][3][3]);
        }
        smax = max_rows(smax);
        const float mt = smax * scale_log2;
        const bool need = mt > m[u] + kThr;
        if (__any(need)) {
          const float mn = need ? mt : m[u];
          const float alpha = __builtin_amdgcn_exp2f(m[u] - mn);   // m = -inf: 0
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[u][dt][r] *= alpha;
          l[u] *= alpha;
          m[u] = mn;
        }
        const float nm = -m[u];
        float ps0 = 0.0f, ps1 = 0.0f;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          uint32_t pk[4] = {0u, 0u, 0u, 0u};
          if (!(kk == 1 && two)) {
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const int t = 2 * kk + (j >> 2), r = j & 3;
              const float e0 = __builtin_amdgcn_exp2f(fmaf(s[u][t][r], scale_log2, nm));
              const float e1 = __builtin_amdgcn_exp2f(fmaf(s[u][t][r + 1], scale_log2, nm));
              ps0 += e0;
              ps1 += e1;
              pk[j >> 1] = pk2bf(f32x2{e0, e1});   // one cvt for the pair
            }
          }
          pf[u][kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
        }
        l[u] += ps0 + ps1;
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (kk == 1 && two) continue;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int vrow = min(dt * 16 + c16, VR - 1);   // rows >= VR: discarded dims
          const bf16x8 vf = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(vt + vrow * VTS + c0 + 32 * kk + 8 * g));
#pragma unroll
          for (int u = 0; u < QT; ++u)
            o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[u][kk], o[u][dt], 0, 0, 0);
        }
      }
    };
    using F = std::false_type;
    using T = std::true_type;
    int c0 = 0;
    for (; c0 + 64 <= N; c0 += 64) chunk(c0, F{}, F{});
    if (c0 < N) {
      if (c0 + 32 >= np) chunk(c0, T{}, T{});
      else chunk(c0, T{}, F{});
    }

#pragma unroll
    for (int u = 0; u < QT; ++u) {
      float lt = l[u];
      lt += __shfl_xor(lt, 16, 64);
      lt += __shfl_xor(lt, 32, 64);
      const float inv = 1.0f / lt;
      if (q[u] < N) {
        u16* orow = out + ((int64_t)b * N + q[u]) * D + (int64_t)h * hd;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int d0 = dt * 16 + 4 * g;
          if (d0 < hd) {
            const uint32_t lo = (uint32_t)f2bf(o[u][dt][0] * inv) |
                                ((uint32_t)f2bf(o[u][dt][1] * inv) << 16);
            const uint32_t hi = (uint32_t)f2bf(o[u][dt][2] * inv) |
                                ((uint32_t)f2bf(o[u][dt][3] * inv) << 16);
            *reinterpret_cast<uint2*>(orow + d0) = make_uint2(lo, hi);
          }
        }
      }
    }
  }
}

}  // namespace

// LDS-resident form for the sequence lengths it covers (224-px towers:
// DINO N = 261, SigLIP N = 256); returns -1 when the caller should use the
// streaming flash kernel instead (longer sequences).
__attribute__((visibility("hidden"))) int vit_attention_lds_launch(
    const void* qkv, void* out, int64_t B, int64_t N, int64_t H, int64_t hd,
    void* stream) {
  const float sl2 = 1.4426950408889634f / sqrtf((float)hd);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)H, (unsigned)B);
  const u16* in = static_cast<const u16*>(qkv);
  u16* o = static_cast<u16*>(out);
#define VA(HDK_, HDV_, NP_, NW_, QT_, KW_, VR_)                                       \
  hipLaunchKernelGGL((vit_attn_kernel<HDK_, HDV_, NP_, NW_, QT_, KW_, VR_>), grid,       \
                     dim3(NW_ * 64), 0, st, in, o, (int)N, (int)H, (int)hd, sl2)
  // 8 waves x 1 query tile (DINO's 17 tiles on 9 waves measured 10 % slower:
  // 18 waves per CU do not split evenly over the 4 SIMDs)
  if (hd == 64 && N <= 288) {
    VA(64, 64, 288, 8, 1, 8, 64);
  } else if (hd == 72 && N <= 256) {
    VA(96, 80, 256, 8, 1, 10, 72);
  } else if (hd == 72 && N <= 288) {
    VA(96, 80, 288, 8, 1, 10, 72);
  } else {
    return -1;
  }
#undef VA
  return (int)hipGetLastError();
}
