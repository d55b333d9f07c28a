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

// ---------------------------------------------------------------------------
// Image preprocessing: Resize((S, S), BICUBIC) of torchvision on a PIL image
// (dino_siglip.py:12-16, 88-124, 148-151) is Pillow's ImagingResample
// (libImaging/Resample.c; Pillow is a third-party dependency, restated here):
//   * per output index i: center = (i + 0.5) * scale, scale = in / S,
//     filterscale = max(scale, 1), support = 2 * filterscale,
//     taps [xmin, xmin + n) with xmin = (int)(center - support + 0.5) >= 0,
//     xmax = min((int)(center + support + 0.5), in); weights
//     w = cubic((x + xmin - center + 0.5) / filterscale), a = -0.5,
//     normalised by their double sum, then fixed point:
//     k = (int)(w * 2^22 +- 0.5) (PRECISION_BITS = 32 - 8 - 2)
//   * horizontal pass first into a uint8 image [H, S, 3], then the vertical
//     pass; each output = clamp((2^21 + sum u8 * k) >> 22, 0, 255)
//   * ToTensor: u8 / 255 in fp32; CenterCrop(S) after a square resize is a
//     no-op.
// The coefficient tables are built on the device in IEEE double (no FMA
// contraction: -ffp-contract=off), exactly as Pillow builds them on the host.
// Ragged batch: meta[b] = {byte offset of image b in `images` (packed HWC
// RGB), H, W, byte offset of its [H, S, 3] row-pass image in tmp}.

__device__ __forceinline__ double pil_bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// One thread per (image, axis, output index).  Table of image b, axis ax:
// bounds at coef + ((b * 2 + ax) * S) * (2 + KS), row i = {xmin, n, k[KS]}.
__global__ __launch_bounds__(256) void resize_coeff_kernel(
    const int64_t* __restrict__ meta, int32_t* __restrict__ coef, int S,
    int KS) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int ax = blockIdx.y, b = blockIdx.z;
  if (i >= S) return;
  const int in_size = (int)meta[b * 4 + 1 + (ax == 0 ? 1 : 0)];  // ax 0: W, 1: H
  int32_t* row = coef + ((int64_t)(b * 2 + ax) * S + i) * (2 + KS);
  const double scale = (double)(float)in_size / S;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double center = (i + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += pil_bicubic((x + xmin - center + 0.5) * ss);
  row[0] = xmin;
  row[1] = xmax < KS ? xmax : KS;   // host sizes KS >= every n
  for (int x = 0; x < KS; ++x) {
    double w = 0.0;
    if (x < xmax) {
      w = pil_bicubic((x + xmin - center + 0.5) * ss);
      if (ww != 0.0) w /= ww;
    }
    const double f = w * (double)(1 << 22);
    row[2 + x] = w < 0 ? (int32_t)(-0.5 + f) : (int32_t)(0.5 + f);
  }
}

__device__ __forceinline__ uint8_t pil_clip8(int32_t ss) {
  const int32_t v = ss >> 22;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

constexpr int kResizeRows = 8;          // input rows per row-pass block
constexpr int kResizeLds = 16384;       // staged pixel bytes per block
constexpr int kResizeCoefLds = 16384;   // coefficient table bytes (if it fits)

// Loads bytes [start, start + len) of `src` (valid up to `nbytes`; `src`
// 16-byte aligned) into LDS as aligned 16-byte quads, all of a thread's
// loads issued before its LDS stores: lds byte j + head holds
// src[start + j]; returns head (< 16).  LDS needs head + len + 15 bytes.
__device__ __forceinline__ int stage_bytes(const uint8_t* __restrict__ src,
                                          int64_t nbytes, int64_t start,
                                          int len, uint4* lds) {
  const int64_t base = start & ~(int64_t)15;
  const int head = (int)(start - base);
  const int nq = (head + len + 15) >> 4;
  int64_t full = (nbytes - base) >> 4;            // quads wholly inside src
  const int nfull = full < nq ? (int)full : nq;
  const uint4* q = reinterpret_cast<const uint4*>(src + base);
  constexpr int kU = 4;      // loads in flight per thread before the stores
  const int bd = blockDim.x;
  int i = threadIdx.x;
  for (; i + (kU - 1) * bd < nfull; i += kU * bd) {
    uint4 v[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) v[j] = q[i + j * bd];
#pragma unroll
    for (int j = 0; j < kU; ++j) lds[i + j * bd] = v[j];
  }
  for (; i < nfull; i += bd) lds[i] = q[i];
  // at most one quad runs past the end of src: byte loads
  for (int i = nfull + (int)threadIdx.x; i < nq; i += blockDim.x) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; ++k) {
      const int64_t a = base + 16 * (int64_t)i + k;
      if (a < nbytes) w[k >> 2] |= (uint32_t)src[a] << (8 * (k & 3));
    }
    lds[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  return head;
}

// Row pass: block (8 input rows, image b).  The rows (contiguous in the
// packed HWC image) and the image's horizontal coefficient table are staged
// in LDS; a thread produces all 3 channels of one output column of a row,
// so each fixed-point coefficient is read once for 3 multiply-adds.
template <bool kCoefInLds>
__global__ __launch_bounds__(256) void resize_rows_kernel(
    const uint8_t* __restrict__ images, int64_t nbytes,
    const int64_t* __restrict__ meta, const int32_t* __restrict__ coef,
    uint8_t* __restrict__ tmp, int S, int KS) {
  __shared__ uint4 spix[kResizeLds / 16];
  __shared__ uint4 scoef[kCoefInLds ? kResizeCoefLds / 16 : 1];
  const int b = blockIdx.y;
  const int H = (int)meta[b * 4 + 1], W = (int)meta[b * 4 + 2];
  const int y0 = blockIdx.x * kResizeRows;
  if (y0 >= H) return;
  const int rb = W * 3, ld = 2 + KS;
  const int64_t tab_off = (int64_t)(b * 2 + 0) * S * ld;
  const int32_t* ct = coef + tab_off;
  if (kCoefInLds) {    // host: S * ld * 4 <= kResizeCoefLds - 32
    const int64_t coef_bytes = (int64_t)gridDim.y * 2 * S * ld * 4;
    const int h = stage_bytes(reinterpret_cast<const uint8_t*>(coef), coef_bytes,
                              tab_off * 4, S * ld * 4, scoef);
    ct = reinterpret_cast<const int32_t*>(reinterpret_cast<const uint8_t*>(scoef) + h);
  }
  const int nrows = min(kResizeRows, H - y0);
  uint8_t* dst = tmp + meta[b * 4 + 3];
  // rows wider than the LDS buffer (W > 5450) are read from global directly
  const bool staged = rb <= kResizeLds - 32;
  const int fit = staged ? (kResizeLds - 32) / rb : nrows;
  // one output pixel (3 channels) of row-pass row r; PX is the LDS image
  // (taps in fours: tables are zero-padded to KS % 4 == 0 and the staged
  // region has slack, so extra taps add 0 * in-bounds bytes) or, for rows
  // too wide to stage, the global image (exact tap count)
  auto pixel = [&](const uint8_t* px, const int32_t* row, int n, bool four,
                   uint8_t* d) {
    int32_t a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
    if (four) {
      for (int x = 0; x < n; x += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t k = row[2 + x + u];
          a0 += __mul24((int32_t)px[3 * (x + u) + 0], k);   // |k| < 2^23
          a1 += __mul24((int32_t)px[3 * (x + u) + 1], k);
          a2 += __mul24((int32_t)px[3 * (x + u) + 2], k);
        }
      }
    } else {
      for (int x = 0; x < n; ++x) {
        const int32_t k = row[2 + x];
        a0 += __mul24((int32_t)px[3 * x + 0], k);
        a1 += __mul24((int32_t)px[3 * x + 1], k);
        a2 += __mul24((int32_t)px[3 * x + 2], k);
      }
    }
    d[0] = pil_clip8(a0);
    d[1] = pil_clip8(a1);
    d[2] = pil_clip8(a2);
  };
  for (int r0 = 0; r0 < nrows; r0 += fit) {
    const int nr = min(fit, nrows - r0);
    const int64_t src0 = meta[b * 4 + 0] + (int64_t)(y0 + r0) * rb;
    if (staged) {
      const int head = stage_bytes(images, nbytes, src0, nr * rb, spix);
      __syncthreads();
      const uint8_t* pix = reinterpret_cast<const uint8_t*>(spix) + head;
      for (int o = threadIdx.x; o < nr * S; o += 256) {
        const int r = o / S, xx = o - r * S;
        const int32_t* row = ct + xx * ld;
        pixel(pix + r * rb + row[0] * 3, row, row[1], true,
              dst + ((int64_t)(y0 + r0 + r) * S + xx) * 3);
      }
      __syncthreads();
    } else {
      for (int o = threadIdx.x; o < nr * S; o += 256) {
        const int r = o / S, xx = o - r * S;
        const int32_t* row = ct + xx * ld;
        pixel(images + src0 + (int64_t)r * rb + row[0] * 3, row, row[1], false,
              dst + ((int64_t)(y0 + r0 + r) * S + xx) * 3);
      }
    }
  }
}

// Column pass + ToTensor: block (output row yy, image b); the coefficient
// row is block-uniform (scalar loads); a thread produces the 3 channels of
// one output pixel from the L2-resident row-pass image (each coefficient
// read once for 3 multiply-adds) and writes the 3 fp32 planes, coalesced
// over xx.
__global__ __launch_bounds__(256) void resize_cols_kernel(
    const uint8_t* __restrict__ tmp, const int64_t* __restrict__ meta,
    const int32_t* __restrict__ coef, float* __restrict__ out, int S, int KS) {
  const int yy = blockIdx.x, b = blockIdx.y;
  const int ld = 2 + KS, rb = S * 3;
  const int32_t* row = coef + ((int64_t)(b * 2 + 1) * S + yy) * ld;
  const int ymin = row[0], n = row[1];
  const uint8_t* src = tmp + meta[b * 4 + 3] + (int64_t)ymin * rb;
  float* plane = out + (int64_t)b * 3 * S * S + (int64_t)yy * S;
  for (int xx = threadIdx.x; xx < S; xx += 256) {
    const uint8_t* px = src + xx * 3;
    int32_t a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
    for (int y = 0; y < n; ++y) {
      const int32_t k = row[2 + y];
      const uint8_t* p = px + (int64_t)y * rb;
      a0 += __mul24((int32_t)p[0], k);
      a1 += __mul24((int32_t)p[1], k);
      a2 += __mul24((int32_t)p[2], k);
    }
    plane[xx] = (float)pil_clip8(a0) / 255.0f;
    plane[(int64_t)S * S + xx] = (float)pil_clip8(a1) / 255.0f;
    plane[(int64_t)2 * S * S + xx] = (float)pil_clip8(a2) / 255.0f;
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

int cadence_resize_bicubic(const void* images, int64_t images_bytes,
                           const int64_t* meta, int64_t B, int64_t S,
                           int64_t KS, int64_t max_h, int64_t max_w, void* coef,
                           void* tmp, int64_t tmp_bytes, float* out,
                           void* stream) {
  if (B <= 0) return 0;
  if (S <= 0 || KS < 5 || KS % 4 || max_h <= 0 || max_w <= 0 || tmp_bytes <= 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int32_t* tab = static_cast<int32_t*>(coef);
  const uint8_t* img = static_cast<const uint8_t*>(images);
  uint8_t* t = static_cast<uint8_t*>(tmp);
  hipLaunchKernelGGL(resize_coeff_kernel, dim3((S + 255) / 256, 2, B), dim3(256),
                     0, s, meta, tab, (int)S, (int)KS);
  const dim3 rgrid((max_h + kResizeRows - 1) / kResizeRows, B);
  if (S * (2 + KS) * 4 <= kResizeCoefLds - 32)
    hipLaunchKernelGGL(resize_rows_kernel<true>, rgrid, dim3(256), 0, s, img,
                       images_bytes, meta, tab, t, (int)S, (int)KS);
  else
    hipLaunchKernelGGL(resize_rows_kernel<false>, rgrid, dim3(256), 0, s, img,
                       images_bytes, meta, tab, t, (int)S, (int)KS);
  hipLaunchKernelGGL(resize_cols_kernel, dim3(S, B), dim3(256), 0, s, t, meta,
                     tab, out, (int)S, (int)KS);
  return (int)hipGetLastError();
}

}  // extern "C"
