// Vision-tower glue kernels: patch extraction with the per-encoder Normalize
// folded in (dino_siglip.py:88-124 transforms, timm PatchEmbed), prefix
// tokens, and the bf16 feature concat that feeds the projector
// (dino_siglip.py:153-154, projector/mlp.py:30).
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

__global__ __launch_bounds__(256) void im2col_kernel(
    const float* __restrict__ pix, u16* __restrict__ out, int64_t ldp, int B,
    int S, int P, float m0, float m1, float m2, float s0, float s1, float s2) {
  const int g = S / P;
  const int kreal = 3 * P * P;
  const int64_t rows = (int64_t)B * g * g;
  const int64_t total = rows * ldp;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int k = idx % ldp;
    const int64_t m = idx / ldp;
    float v = 0.0f;
    if (k < kreal) {
      const int b = m / (g * g), pp = m % (g * g);
      const int py = pp / g, px = pp % g;
      const int c = k / (P * P), r = k % (P * P);
      const int ky = r / P, kx = r % P;
      const float x = pix[(((int64_t)b * 3 + c) * S + py * P + ky) * S + px * P + kx];
      const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
      const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
      v = (x - mean) / sd;
    }
    out[m * ldp + k] = f2bf(v);
  }
}

__global__ __launch_bounds__(256) void prefix_kernel(const u16* __restrict__ tok,
                                                     float* __restrict__ resid,
                                                     int B, int ntok, int prefix,
                                                     int D) {
  const int64_t total = (int64_t)B * prefix * D;
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int d = idx % D;
    const int64_t bp = idx / D;
    const int p = bp % prefix, b = bp / prefix;
    resid[((int64_t)b * ntok + p) * D + d] = bf2f(tok[(int64_t)p * D + d]);
  }
}

__global__ __launch_bounds__(256) void features_kernel(
    const float* __restrict__ resid, u16* __restrict__ out, int64_t ldo,
    int64_t col_off, int B, int ntok, int prefix, int D) {
  const int P = ntok - prefix;
  const int64_t total = (int64_t)B * P * (D / 4);
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int d = (idx % (D / 4)) * 4;
    const int64_t bp = idx / (D / 4);
    const int p = bp % P, b = bp / P;
    const float4 v =
        *reinterpret_cast<const float4*>(resid + ((int64_t)b * ntok + prefix + p) * D + d);
    const uint32_t lo = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    const uint32_t hi = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(out + ((int64_t)b * P + p) * ldo + col_off + d) =
        make_uint2(lo, hi);
  }
}

int grid_cap(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

}  // namespace

extern "C" {

int cadence_im2col_normalize(const float* pixels, void* patches, int64_t ldp,
                             int64_t B, int64_t S, int64_t patch,
                             const float* mean3, const float* std3,
                             void* stream) {
  if (ldp < 3 * patch * patch || ldp % 8) return (int)hipErrorInvalidValue;
  const int64_t g = S / patch;
  if (B <= 0 || g <= 0) return 0;
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_cap(B * g * g * ldp)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), pixels,
                     static_cast<u16*>(patches), ldp, (int)B, (int)S, (int)patch,
                     mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  return (int)hipGetLastError();
}

int cadence_vit_prefix(const void* tokens, float* resid, int64_t B,
                       int64_t ntok, int64_t prefix, int64_t D, void* stream) {
  if (prefix <= 0 || B <= 0) return 0;
  hipLaunchKernelGGL(prefix_kernel, dim3(grid_cap(B * prefix * D)), dim3(256), 0,
                     static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(tokens), resid, (int)B, (int)ntok,
                     (int)prefix, (int)D);
  return (int)hipGetLastError();
}

int cadence_vit_features(const float* resid, void* out, int64_t ldo,
                         int64_t col_off, int64_t B, int64_t ntok,
                         int64_t prefix, int64_t D, void* stream) {
  if (D % 4 || col_off % 4 || ldo % 4) return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  hipLaunchKernelGGL(features_kernel,
                     dim3(grid_cap(B * (ntok - prefix) * (D / 4))), dim3(256), 0,
                     static_cast<hipStream_t>(stream), resid,
                     static_cast<u16*>(out), ldo, col_off, (int)B, (int)ntok,
                     (int)prefix, (int)D);
  return (int)hipGetLastError();
}

}  // extern "C"
