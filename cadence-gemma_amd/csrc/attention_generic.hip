// Local attention for the shapes the tuned kernels do not cover: any head
// dim (multiple of 4, up to 1024 -- the reference's own test grids use 16
// and 1024, recurrentgemma/torch/modules_test.py:77-116), and a multi-token
// step against an existing cache (modules.py:206-225: n_fill == window, the
// prompt-in-chunks path).  Plain per-(query row, head) workgroups: scores in
// LDS, one softmax, then the value sum -- correctness over speed; the
// 2B / 9B shapes (hd 256) never come here.
//
// Rounding follows the reference op by op: logits = bf16(bf16(q . k) *
// hd^-1/2) (the bf16 einsum, then the Python-float scale), masked to
// MIN_LOGIT, softmax in fp32, probs rounded to bf16, encoded = bf16(sum p v).
#include "common.hpp"
#include "../../include/cadence_kernels.h"

namespace {

constexpr int kGenMaxKeys = 4096 + 2048;   // scores held in LDS per workgroup
constexpr float kMinLogit = -2.3819763e38f;  // modules.py:29

// mode 0 (prefill, no cache): keys = the T prompt rows; key k visible to
//   query t iff seg_start[t] <= k <= t and t <= k + W  (modules.py:130-152).
// mode 1 (cached step): keys = [W ring slots | T new rows]; positions from
//   num_tokens as _compute_cache_mask (modules.py:155-185): query t at
//   nt + t, slot j at j + kblk W (or the previous block's), new key i at
//   nt + i; visible iff kpos >= 0, kpos <= qpos <= kpos + W.
__global__ __launch_bounds__(256) void generic_attn_kernel(
    const u16* __restrict__ q, const u16* __restrict__ kn,
    const u16* __restrict__ vn, const u16* __restrict__ ck,
    const u16* __restrict__ cv, const int32_t* __restrict__ num_tokens,
    const int32_t* __restrict__ seg_start, u16* __restrict__ out, int T,
    int H, int hd, int W, float scale, int mode) {
  __shared__ float qs[1024];
  __shared__ float sc[kGenMaxKeys];
  __shared__ float red[8];
  const int row = blockIdx.x;          // b * T + t
  const int h = blockIdx.y;
  const int b = row / T, t = row % T;
  const int tid = threadIdx.x;
  const u16* qrow = q + (int64_t)row * H * hd + (int64_t)h * hd;
  for (int d = tid; d < hd; d += 256) qs[d] = bf2f(qrow[d]);
  __syncthreads();
  const int nt = mode ? num_tokens[b] : 0;
  const int nring = mode ? W : 0;
  const int nkeys = nring + T;
  const int qpos = mode ? nt + t : t;
  const int kblk = mode ? nt / W : 0;
  const int lo = mode ? 0 : seg_start[row];
  auto key_row = [&](int j, const u16* cache, const u16* fresh) -> const u16* {
    return j < nring ? cache + ((int64_t)b * W + j) * hd
                     : fresh + ((int64_t)b * T + (j - nring)) * hd;
  };
  float mx = -INFINITY;
  for (int j = tid; j < nkeys; j += 256) {
    bool ok;
    if (mode) {
      int kpos;
      if (j < nring) {
        const int now = j + kblk * W;
        kpos = now < nt ? now : j + (kblk - 1) * W;
      } else {
        kpos = nt + (j - nring);
      }
      ok = kpos >= 0 && qpos >= kpos && qpos <= kpos + W;
    } else {
      ok = j >= lo && j <= t && t <= j + W;
    }
    float v = kMinLogit;
    if (ok) {
      const u16* kr = key_row(j, ck, kn);
      float acc = 0.0f;
      for (int d = 0; d < hd; ++d) acc = fmaf(qs[d], bf2f(kr[d]), acc);
      v = bmul(rbf(acc), scale);
    }
    sc[j] = v;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.0f;
  for (int j = tid; j < nkeys; j += 256) {
    const float e = expf(sc[j] - mx);
    sc[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  sum = (red[0] + red[1]) + (red[2] + red[3]);
  const float inv = 1.0f / sum;
  for (int j = tid; j < nkeys; j += 256) sc[j] = rbf(sc[j] * inv);   // probs, bf16
  __syncthreads();
  u16* orow = out + (int64_t)row * H * hd + (int64_t)h * hd;
  for (int d = tid; d < hd; d += 256) {
    float acc = 0.0f;
    for (int j = 0; j < nkeys; ++j) {
      const float p = sc[j];
      if (p != 0.0f) acc = fmaf(p, bf2f(key_row(j, cv, vn)[d]), acc);
    }
    orow[d] = f2bf(acc);
  }
}

// RoPE on the first half of each head for any hd % 4 == 0 (modules.py:53-87),
// one thread per rotation pair; v copied.
__global__ __launch_bounds__(256) void rope_qkv_generic_kernel(
    const u16* __restrict__ qkv, int64_t ld, const int32_t* __restrict__ pos,
    u16* __restrict__ qo, u16* __restrict__ ko, u16* __restrict__ vo, int64_t M,
    int H, int hd) {
  const int half = hd / 2, quarter = hd / 4;
  const int64_t total = M * (H + 1) * (int64_t)half;   // pairs + pass-through
  for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int i = idx % half;
    const int64_t mh = idx / half;
    const int hh = mh % (H + 1);
    const int64_t m = mh / (H + 1);
    const u16* src = qkv + m * ld + hh * hd;
    u16* dst = hh < H ? qo + m * (int64_t)H * hd + hh * hd : ko + m * hd;
    if (i < quarter) {
      float sn, cs;
      rope_sincos(pos[m], i, half, sn, cs);
      const float x1 = bf2f(src[i]), x2 = bf2f(src[quarter + i]);
      dst[i] = f2bf(bsub(bmul(x1, cs), bmul(x2, sn)));
      dst[quarter + i] = f2bf(badd(bmul(x2, cs), bmul(x1, sn)));
    } else {
      const int d = half + 2 * (i - quarter);     // two pass-through dims
      dst[d] = src[d];
      dst[d + 1] = src[d + 1];
    }
    if (hh == H) {
      const u16* vs = qkv + m * ld + (H + 1) * hd;
      vo[m * hd + 2 * i] = vs[2 * i];
      vo[m * hd + 2 * i + 1] = vs[2 * i + 1];
    }
  }
}

// Single-token ring update (modules.py:206-215): slot num_tokens % W of
// each sequence <- the new key / value; num_tokens += 1.
__global__ __launch_bounds__(256) void kv_ring_update_kernel(
    const u16* __restrict__ kn, const u16* __restrict__ vn, u16* __restrict__ ck,
    u16* __restrict__ cv, int32_t* __restrict__ num_tokens, int hd, int W) {
  const int b = blockIdx.x;
  const int nt = num_tokens[b];
  const int slot = ((nt % W) + W) % W;
  for (int d = threadIdx.x; d < hd; d += 256) {
    ck[((int64_t)b * W + slot) * hd + d] = kn[(int64_t)b * hd + d];
    cv[((int64_t)b * W + slot) * hd + d] = vn[(int64_t)b * hd + d];
  }
  __syncthreads();
  if (threadIdx.x == 0) num_tokens[b] = nt + 1;
}

int gen_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

__attribute__((visibility("hidden"))) int generic_attention_launch(
    const void* q, const void* k, const void* v, const void* cache_k,
    const void* cache_v, const int32_t* num_tokens, const int32_t* seg_start,
    void* out, int64_t B, int64_t T, int64_t H, int64_t hd, int64_t window,
    void* stream) {
  const int mode = cache_k ? 1 : 0;
  if (hd % 4 || hd > 1024 || (mode ? window : 0) + T > kGenMaxKeys)
    return (int)hipErrorInvalidValue;
  if (B <= 0 || T <= 0) return 0;
  // the reference multiplies the bf16 logits by the Python float hd^-1/2
  const float scale = 1.0f / sqrtf((float)hd);
  hipLaunchKernelGGL(generic_attn_kernel, dim3((unsigned)(B * T), (unsigned)H),
                     dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(q), static_cast<const u16*>(k),
                     static_cast<const u16*>(v), static_cast<const u16*>(cache_k),
                     static_cast<const u16*>(cache_v), num_tokens, seg_start,
                     static_cast<u16*>(out), (int)T, (int)H, (int)hd, (int)window,
                     scale, mode);
  return (int)hipGetLastError();
}

__attribute__((visibility("hidden"))) int rope_qkv_generic_launch(
    const void* qkv, int64_t ld, const int32_t* positions, void* q_out,
    void* k_out, void* v_out, int64_t M, int64_t H, int64_t hd, void* stream) {
  if (hd % 4 || M <= 0) return hd % 4 ? (int)hipErrorInvalidValue : 0;
  hipLaunchKernelGGL(rope_qkv_generic_kernel, dim3(gen_grid(M * (H + 1) * (hd / 2))),
                     dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(qkv), ld, positions,
                     static_cast<u16*>(q_out), static_cast<u16*>(k_out),
                     static_cast<u16*>(v_out), M, (int)H, (int)hd);
  return (int)hipGetLastError();
}

extern "C" {

int cadence_local_attention_cached(const void* q, const void* k_new,
                                   const void* v_new, const void* cache_k,
                                   const void* cache_v,
                                   const int32_t* num_tokens, void* out,
                                   int64_t B, int64_t T, int64_t H, int64_t hd,
                                   int64_t window, void* stream) {
  if (!cache_k || !cache_v || !num_tokens) return (int)hipErrorInvalidValue;
  return generic_attention_launch(q, k_new, v_new, cache_k, cache_v, num_tokens,
                                  nullptr, out, B, T, H, hd, window, stream);
}

int cadence_kv_ring_update(const void* k_new, const void* v_new, void* cache_k,
                           void* cache_v, int32_t* num_tokens, int64_t B,
                           int64_t hd, int64_t window, void* stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(kv_ring_update_kernel, dim3((unsigned)B), dim3(256), 0,
                     static_cast<hipStream_t>(stream),
                     static_cast<const u16*>(k_new), static_cast<const u16*>(v_new),
                     static_cast<u16*>(cache_k), static_cast<u16*>(cache_v),
                     num_tokens, (int)hd, (int)window);
  return (int)hipGetLastError();
}

}  // extern "C"
