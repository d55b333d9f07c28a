// Row-wise kernels: Griffin RMSNorm, ViT LayerNorm, token embedding, and the
// small int bookkeeping kernels (image-splice positions, segment ids).
// One wave per row, 16-byte vector accesses (G13), fp32 reductions.
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

// layers.py:73-78 on bf16 tensors: square (rounded), mean (fp32 sum,
// rounded), + eps (rounded), rsqrt (rounded), x * r (rounded),
// scale + 1 (rounded), product (rounded).
// Rows up to 64 * 8 * RC wide stay in registers between the two passes:
// x and scale are loaded once, up front (one memory round trip per row).
template <int RC>
__global__ __launch_bounds__(256) void rmsnorm_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ scale,
    u16* __restrict__ out, int64_t ldo, int64_t rows, int width, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const u16* xr = x + row * ldx;
  uint4 xv[RC], sv[RC];
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = min(lane * 8 + i * 512, width - 8);
    xv[i] = ld16(xr + c);
    sv[i] = ld16(scale + c);
  }
  float ss = 0.0f;
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    if (lane * 8 + i * 512 < width) {
      float v[8];
      unpack8(xv[i], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += rbf(v[j] * v[j]);
    }
  }
  ss = wave_sum(ss);
  const float var = rbf(ss / (float)width);
  const float r = rbf(1.0f / sqrtf(rbf(var + eps)));
  const int mt = (int)((rows + 15) >> 4);   // ldo == 0: packed rows
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = lane * 8 + i * 512;
    if (c < width) {
      float v[8], sc[8];
      unpack8(xv[i], v);
      unpack8(sv[i], sc);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bmul(bmul(v[j], r), badd(sc[j], 1.0f));
      st16(out + xoff((int)row, c, ldo, mt), pack8(v));
    }
  }
}

// Wider rows: two passes over global memory.
__global__ __launch_bounds__(256) void rmsnorm_wide_kernel(
    const u16* __restrict__ x, int64_t ldx, const u16* __restrict__ scale,
    u16* __restrict__ out, int64_t ldo, int64_t rows, int width, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const u16* xr = x + row * ldx;
  float ss = 0.0f;
  for (int c = lane * 8; c < width; c += 512) {
    float v[8];
    unpack8(ld16(xr + c), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += rbf(v[i] * v[i]);
  }
  ss = wave_sum(ss);
  const float var = rbf(ss / (float)width);
  const float r = rbf(1.0f / sqrtf(rbf(var + eps)));
  const int mt = (int)((rows + 15) >> 4);   // ldo == 0: packed rows
  for (int c = lane * 8; c < width; c += 512) {
    float v[8], s[8];
    unpack8(ld16(xr + c), v);
    unpack8(ld16(scale + c), s);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bmul(bmul(v[i], r), badd(s[i], 1.0f));
    st16(out + xoff((int)row, c, ldo, mt), pack8(v));
  }
}

// timm LayerNorm (eps 1e-6) over the fp32 residual stream, bf16 out.
// Rows up to 256 * RC wide (ViT widths 1024, 1152): the row is loaded once
// into registers, with w / b, all before the first reduction (one memory
// round trip instead of three); the sums keep layernorm_kernel's order, so
// the results are identical.
template <int RC>
__global__ __launch_bounds__(256) void layernorm_reg_kernel(
    const float* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ b, u16* __restrict__ out, int64_t ldo,
    int64_t rows, int width, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float4 v[RC];
  uint2 wq[RC], bq[RC];
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = min(lane * 4 + i * 256, width - 4);
    v[i] = *reinterpret_cast<const float4*>(xr + c);
    wq[i] = *reinterpret_cast<const uint2*>(w + c);
    bq[i] = *reinterpret_cast<const uint2*>(b + c);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < RC; ++i)
    if (lane * 4 + i * 256 < width) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)width;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < RC; ++i)
    if (lane * 4 + i * 256 < width) {
      const float d0 = v[i].x - mean, d1 = v[i].y - mean, d2 = v[i].z - mean,
                  d3 = v[i].w - mean;
      q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)width + eps);
  u16* orow = out + row * ldo;
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = lane * 4 + i * 256;
    if (c >= width) continue;
    const float vv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    const uint32_t wv[2] = {wq[i].x, wq[i].y}, bv[2] = {bq[i].x, bq[i].y};
    uint32_t o[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float w0 = __uint_as_float(wv[j] << 16), w1 = __uint_as_float(wv[j] & 0xffff0000u);
      const float b0 = __uint_as_float(bv[j] << 16), b1 = __uint_as_float(bv[j] & 0xffff0000u);
      const float y0 = (vv[2 * j] - mean) * rstd * w0 + b0;
      const float y1 = (vv[2 * j + 1] - mean) * rstd * w1 + b1;
      o[j] = (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
    }
    *reinterpret_cast<uint2*>(orow + c) = make_uint2(o[0], o[1]);
  }
}

__global__ __launch_bounds__(256) void layernorm_kernel(
    const float* __restrict__ x, int64_t ldx, const u16* __restrict__ w,
    const u16* __restrict__ b, u16* __restrict__ out, int64_t ldo,
    int64_t rows, int width, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float s = 0.0f;
  for (int c = lane * 4; c < width; c += 256) {
    const float4 v = *reinterpret_cast<const float4*>(xr + c);
    s += (v.x + v.y) + (v.z + v.w);
  }
  const float mean = wave_sum(s) / (float)width;
  float q = 0.0f;
  for (int c = lane * 4; c < width; c += 256) {
    const float4 v = *reinterpret_cast<const float4*>(xr + c);
    const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)width + eps);
  u16* orow = out + row * ldo;
  for (int c = lane * 4; c < width; c += 256) {
    const float4 v = *reinterpret_cast<const float4*>(xr + c);
    const float vv[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float y0 = (vv[2 * i] - mean) * rstd * bf2f(w[c + 2 * i]) + bf2f(b[c + 2 * i]);
      const float y1 = (vv[2 * i + 1] - mean) * rstd * bf2f(w[c + 2 * i + 1]) +
                       bf2f(b[c + 2 * i + 1]);
      o[i] = (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
    }
    *reinterpret_cast<uint2*>(orow + c) = make_uint2(o[0], o[1]);
  }
}

__global__ __launch_bounds__(256) void embed_kernel(
    const int32_t* __restrict__ tok, const u16* __restrict__ E,
    u16* __restrict__ out, int64_t ldo, int64_t M, int D, int64_t V,
    float scale, int64_t div, int64_t mul, int64_t off, u16* __restrict__ packed,
    int mt) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  // an id outside [0, V) reads row 0 instead of faulting (the reference's
  // nn.Embedding raises; a device kernel cannot)
  const int64_t t = tok[m];
  const u16* src = E + (t >= 0 && t < V ? t : 0) * D;
  u16* dst = out + ((m / div) * mul + (m % div) + off) * ldo;
  for (int c = lane * 8; c < D; c += 512) {
    uint4 v = ld16(src + c);
    if (scale != 1.0f) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = bmul(f[i], scale);
      v = pack8(f);
    }
    st16(dst + c, v);
    // (decode, identity row map) the same 8 columns in the packed layout
    if (packed) st16(packed + xoff((int)m, c, 0, mt), v);
  }
}

__global__ void splice_positions_kernel(const int32_t* __restrict__ text,
                                        int32_t* __restrict__ out, int B, int T,
                                        int n_vis) {
  const int L = n_vis + T;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < (int64_t)B * L;
       i += (int64_t)gridDim.x * 256) {
    const int b = i / L, t = i % L;
    out[i] = t < n_vis ? t : text[(int64_t)b * T + t - n_vis];
  }
}

// seg_id = cumsum(pos == 0) (modules.py:145); seg_start = first index of
// the row's segment (0 before the first reset).  One workgroup per sequence:
// each thread counts the resets of a contiguous slice, a block-wide
// Hillis-Steele scan gives every slice its running count and last reset
// index, then each thread writes its slice.
__global__ __launch_bounds__(256) void segment_info_kernel(
    const int32_t* __restrict__ pos, int32_t* __restrict__ seg,
    int32_t* __restrict__ start, int B, int L) {
  __shared__ int sc[256], sl[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int per = (L + 255) / 256;
  const int t0 = min(L, tid * per), t1 = min(L, t0 + per);
  const int32_t* p = pos + (int64_t)b * L;
  int cnt = 0, last = -1;
  for (int t = t0; t < t1; ++t)
    if (p[t] == 0) {
      ++cnt;
      last = t;
    }
  sc[tid] = cnt;
  sl[tid] = last;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const int c = tid >= d ? sc[tid - d] : 0;
    const int l = tid >= d ? sl[tid - d] : -1;
    __syncthreads();
    sc[tid] += c;
    sl[tid] = max(sl[tid], l);
    __syncthreads();
  }
  int s = tid ? sc[tid - 1] : 0;
  int st = tid ? max(sl[tid - 1], 0) : 0;
  for (int t = t0; t < t1; ++t) {
    if (p[t] == 0) {
      ++s;
      st = t;
    }
    seg[(int64_t)b * L + t] = s;
    start[(int64_t)b * L + t] = st;
  }
}

// Greedy-decode bookkeeping on device (no host sync per step):
// out[b, *step] = next[b] (pad once row b is done); pos[b] += 1; cur[b] = the
// token written; done[b] latches when row b emits EOS in a column >= eos_from
// (1 = the reference's loop: the token sampled from the prompt is never
// tested, recurrentgemma/torch/sampler.py:177-187,291-300), done[B] = all rows
// done (read by the host a few steps late, so it never stalls the GPU);
// ++*step.
__global__ void decode_advance_kernel(const int32_t* __restrict__ next,
                                      int32_t* __restrict__ out, int64_t ldo,
                                      int32_t* __restrict__ step,
                                      int32_t* __restrict__ pos,
                                      int32_t* __restrict__ cur,
                                      int32_t* __restrict__ done, int eos_id,
                                      int pad_id, int eos_from, int B) {
  const int b = threadIdx.x;
  const int s = *step;
  int fin = 1;
  if (b < B) {
    int32_t t = next[b];
    if (done) {
      const int d = done[b];
      if (d) t = pad_id;
      fin = d | (t == eos_id && s >= eos_from);
      done[b] = fin;
    }
    out[(int64_t)b * ldo + s] = t;
    pos[b] += 1;
    if (cur) cur[b] = t;
  }
  const int all = __syncthreads_and(fin);
  if (threadIdx.x == 0) {
    *step = s + 1;
    if (done) done[B] = all;
  }
}

// Batched row-strided device copies (the decode graph's cache hand-over):
// blockIdx.y = descriptor, blocks grid-stride over its 16-B (or 4-B) units.
constexpr int kCopyBatch = 32;
struct CopyBatch {
  CadenceCopyDesc d[kCopyBatch];
};
__global__ __launch_bounds__(256) void copy_batched_kernel(CopyBatch cb) {
  const CadenceCopyDesc d = cb.d[blockIdx.y];
  const bool wide = d.row_bytes % 16 == 0 && d.src_stride % 16 == 0 &&
                    d.dst_stride % 16 == 0 && (uintptr_t)d.src % 16 == 0 &&
                    (uintptr_t)d.dst % 16 == 0;
  const int64_t unit = wide ? 16 : 4;
  const int64_t per_row = d.row_bytes / unit, total = d.rows * per_row;
  const char* src = static_cast<const char*>(d.src);
  char* dst = static_cast<char*>(d.dst);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = (i % per_row) * unit;
    if (wide)
      *reinterpret_cast<uint4*>(dst + r * d.dst_stride + c) =
          *reinterpret_cast<const uint4*>(src + r * d.src_stride + c);
    else
      *reinterpret_cast<uint32_t*>(dst + r * d.dst_stride + c) =
          *reinterpret_cast<const uint32_t*>(src + r * d.src_stride + c);
  }
}

}  // namespace

extern "C" {

int cadence_decode_advance(const int32_t* next_token, int32_t* tokens_out,
                           int64_t ld_out, int32_t* step, int32_t* positions,
                           int32_t* cur_out, int32_t* done, int32_t eos_id,
                           int32_t pad_id, int32_t eos_from, int64_t B,
                           void* stream) {
  if (B <= 0) return 0;
  if (B > 1024) return (int)hipErrorInvalidValue;
  const unsigned threads = (unsigned)((B + 63) / 64 * 64);
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(threads), 0,
                     static_cast<hipStream_t>(stream), next_token, tokens_out,
                     ld_out, step, positions, cur_out, done, eos_id, pad_id,
                     (int)eos_from, (int)B);
  return (int)hipGetLastError();
}


int cadence_rmsnorm(const void* x, int64_t ldx, const void* scale, void* out,
                    int64_t ldo, int64_t rows, int64_t width, float eps,
                    void* stream) {
  if (width % 8 || ldx % 8 || ldo % 8) return (int)hipErrorInvalidValue;
  if (ldo == 0 && (rows > 32 || width % 32)) return (int)hipErrorInvalidValue;
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const u16* xp = static_cast<const u16*>(x);
  const u16* sp = static_cast<const u16*>(scale);
  u16* op = static_cast<u16*>(out);
  if (width <= 1024)
    hipLaunchKernelGGL(rmsnorm_kernel<2>, grid, block, 0, st, xp, ldx, sp, op, ldo,
                       rows, (int)width, eps);
  else if (width <= 4096)
    hipLaunchKernelGGL(rmsnorm_kernel<8>, grid, block, 0, st, xp, ldx, sp, op, ldo,
                       rows, (int)width, eps);
  else
    hipLaunchKernelGGL(rmsnorm_wide_kernel, grid, block, 0, st, xp, ldx, sp, op, ldo,
                       rows, (int)width, eps);
  return (int)hipGetLastError();
}

int cadence_layernorm(const float* x, int64_t ldx, const void* weight,
                      const void* bias, void* out, int64_t ldo, int64_t rows,
                      int64_t width, float eps, void* stream) {
  if (width % 4 || ldx % 4 || ldo % 4) return (int)hipErrorInvalidValue;
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const u16* wp = static_cast<const u16*>(weight);
  const u16* bp = static_cast<const u16*>(bias);
  u16* op = static_cast<u16*>(out);
  if (width <= 1280)
    hipLaunchKernelGGL(layernorm_reg_kernel<5>, grid, block, 0, st, x, ldx, wp, bp, op,
                       ldo, rows, (int)width, eps);
  else
    hipLaunchKernelGGL(layernorm_kernel, grid, block, 0, st, x, ldx, wp, bp, op, ldo,
                       rows, (int)width, eps);
  return (int)hipGetLastError();
}

int cadence_embed(const int32_t* tokens, const void* E, void* out,
                  int64_t ldo, int64_t M, int64_t D, int64_t V, float scale,
                  int64_t row_div, int64_t row_mul, int64_t row_off,
                  void* stream) {
  if (D % 8 || ldo % 8 || row_div <= 0) return (int)hipErrorInvalidValue;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(embed_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), tokens,
                     static_cast<const u16*>(E), static_cast<u16*>(out), ldo, M,
                     (int)D, V, scale, row_div, row_mul, row_off, nullptr, 0);
  return (int)hipGetLastError();
}

int cadence_embed_packed(const int32_t* tokens, const void* E, void* out,
                         int64_t ldo, void* packed, int64_t M, int64_t D,
                         int64_t V, float scale, void* stream) {
  if (D % 32 || ldo % 8 || M > 32 || !packed) return (int)hipErrorInvalidValue;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(embed_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), tokens,
                     static_cast<const u16*>(E), static_cast<u16*>(out), ldo, M,
                     (int)D, V, scale, M, (int64_t)0, (int64_t)0,
                     static_cast<u16*>(packed), (int)((M + 15) / 16));
  return (int)hipGetLastError();
}

int cadence_copy_batched(const CadenceCopyDesc* desc, int64_t n, void* stream) {
  if (n < 0 || (n > 0 && !desc)) return (int)hipErrorInvalidValue;
  for (int64_t i = 0; i < n; ++i) {
    const CadenceCopyDesc& d = desc[i];
    if (d.rows < 0 || d.row_bytes < 0 || d.row_bytes % 4 || d.src_stride % 4 ||
        d.dst_stride % 4 || (uintptr_t)d.src % 4 || (uintptr_t)d.dst % 4 ||
        (d.rows > 1 && (d.src_stride < d.row_bytes || d.dst_stride < d.row_bytes)) ||
        (d.rows * d.row_bytes > 0 && (!d.src || !d.dst)))
      return (int)hipErrorInvalidValue;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  bool launched = false;
  for (int64_t i0 = 0; i0 < n; i0 += kCopyBatch) {
    CopyBatch cb{};
    const int m = (int)(n - i0 < kCopyBatch ? n - i0 : kCopyBatch);
    int64_t most = 0;
    for (int j = 0; j < m; ++j) {
      cb.d[j] = desc[i0 + j];
      const int64_t units = cb.d[j].rows * (cb.d[j].row_bytes / 4);
      most = units > most ? units : most;
    }
    if (most == 0) continue;
    // ~4 (wide) units per thread for the largest region, at most 1024 blocks
    int64_t g = (most / 4 + 1023) / 1024;
    g = g < 1 ? 1 : g > 1024 ? 1024 : g;
    hipLaunchKernelGGL(copy_batched_kernel, dim3((unsigned)g, (unsigned)m), dim3(256), 0,
                       st, cb);
    launched = true;
  }
  return launched ? (int)hipGetLastError() : 0;
}

int cadence_splice_positions(const int32_t* text_pos, int32_t* out,
                             int64_t B, int64_t T, int64_t n_vis,
                             void* stream) {
  const int64_t n = B * (n_vis + T);
  if (n <= 0) return 0;
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(splice_positions_kernel, dim3((unsigned)g), dim3(256), 0,
                     static_cast<hipStream_t>(stream), text_pos, out, (int)B,
                     (int)T, (int)n_vis);
  return (int)hipGetLastError();
}

int cadence_segment_info(const int32_t* segment_pos, int32_t* seg_id,
                         int32_t* seg_start, int64_t B, int64_t L,
                         void* stream) {
  if (B <= 0 || L <= 0) return 0;
  hipLaunchKernelGGL(segment_info_kernel, dim3((unsigned)B),
                     dim3(256), 0, static_cast<hipStream_t>(stream), segment_pos,
                     seg_id, seg_start, (int)B, (int)L);
  return (int)hipGetLastError();
}

}  // extern "C"
