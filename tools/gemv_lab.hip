// Decode GEMV lab: cold-weight timing of the stream engine's variants on the
// decode shapes (M = 32 packed rows, fragment-packed weights), each variant
// captured as a hipGraph of back-to-back launches cycling over enough weight
// copies that nothing is served from the 256 MB Infinity Cache.  Also a pure
// streaming-read kernel over the same bytes (the bandwidth this size can
// reach).  Not part of the library; built by tools/gemv_lab.sh.
#include "../cadence-gemma_amd/csrc/gemm.hip"

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)

namespace {

__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ p, int64_t n16,
                                                   uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint4 v = ld16_nt(reinterpret_cast<const u16*>(p + i));
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// Lab copy of the stream engine's core: MODE 0 = weights + packed-row
// activations (as shipped), 1 = weights only (activation fragments are a
// constant), 2 = weights only and no MFMA (XOR of the loads).
template <int KSW, int NREP, int MODE>
__global__ __launch_bounds__(512) void lab_gemv(const u16* __restrict__ A,
                                                const u16* __restrict__ W, int N, int K,
                                                int klen, float* __restrict__ out) {
  constexpr int MR = 2;
  __shared__ float red[8][32 * 16 * NREP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kbeg = blockIdx.y * klen, kend = min(K, kbeg + klen);
  const uint4 zero = make_uint4(0, 0, 0, 0);
  uint4 wb[KSW][NREP], xa[KSW][MR];
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kbeg + (wave + 8 * u) * 32;
    const bool ok = k < kend;
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      const int col = (blockIdx.x * NREP + j) * 16;
      wb[u][j] = ok ? ld16_nt(W + (((int64_t)(col >> 4) * (K >> 5) + (k >> 5)) * 64 + lane) * 8)
                    : zero;
    }
#pragma unroll
    for (int i = 0; i < MR; ++i)
      xa[u][i] = (MODE == 0 && ok) ? ld16(A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3))
                                   : make_uint4(0x3c003c00u, 0x3c003c00u, lane, i);
  }
  if constexpr (MODE == 2) {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < KSW; ++u)
#pragma unroll
      for (int j = 0; j < NREP; ++j) acc ^= wb[u][j].x ^ wb[u][j].y ^ wb[u][j].z ^ wb[u][j].w;
    if (acc == 0x12345678u) out[0] = 1.0f;
    return;
  }
  f32x4 acc[MR][NREP];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KSW; ++u)
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, xa[u][i]), __builtin_bit_cast(bf16x8, wb[u][j]),
            acc[i][j], 0, 0, 0);
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][((i * 16 + rsub + r) * NREP + j) * 16 + csub] = acc[i][j][r];
  __syncthreads();
  for (int o = threadIdx.x; o < 32 * 16 * NREP; o += 512) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w][o];
    out[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 32 * 16 * NREP + o] = v;
  }
}

// Pipelined core: each wave walks its KSW k-steps in chunks of CH k-steps and
// keeps INF chunks of weight + activation fragments in flight; chunk c +
// INF's loads are issued right after chunk c's MFMAs (the registers they
// overwrite are free then), so one workgroup streams its whole slice with a
// bounded register budget -- NREP = 4 column tiles (240 workgroups on the
// gated shape: one round) instead of 2 (480: two rounds).
template <int KSW, int NREP, int CH, int INF>
__global__ __launch_bounds__(512) void lab_pipe_gemv(const u16* __restrict__ A,
                                                     const u16* __restrict__ W, int N, int K,
                                                     float* __restrict__ out) {
  constexpr int MR = 2, NC = KSW / CH;
  static_assert(KSW % CH == 0 && INF <= NC, "chunking");
  __shared__ float red[8][32 * 16 * NREP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  uint4 wb[INF][CH][NREP], xa[INF][CH][MR];
  f32x4 acc[MR][NREP];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int c, int slot) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = (wave + 8 * (c * CH + u)) * 32;
      const bool ok = k < K;
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const int col = (blockIdx.x * NREP + j) * 16;
        wb[slot][u][j] = ld16_nt(ok ? W + (((int64_t)(col >> 4) * (K >> 5) + (k >> 5)) * 64 + lane) * 8
                                    : zpage);
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
        xa[slot][u][i] = ld16(ok ? A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3) : zpage);
    }
  };
#pragma unroll
  for (int c = 0; c < INF; ++c) issue(c, c);
  // pin the issue order: the scheduler otherwise sinks loads to their first
  // use (to save registers) and the wave has a third of the bytes in flight
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int slot = c % INF;
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NREP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, xa[slot][u][i]), __builtin_bit_cast(bf16x8, wb[slot][u][j]),
              acc[i][j], 0, 0, 0);
    if (c + INF < NC) issue(c + INF, slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  const int rsub = (lane >> 4) * 4, csub = lane & 15;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave][((i * 16 + rsub + r) * NREP + j) * 16 + csub] = acc[i][j][r];
  __syncthreads();
  for (int o = threadIdx.x; o < 32 * 16 * NREP; o += 512) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w][o];
    out[(int64_t)blockIdx.x * 32 * 16 * NREP + o] = v;
  }
}

struct Lab {
  hipStream_t st;
  std::vector<u16*> w;
  u16* x;
  float* parts;
  u16* out;
  u16* bias;
  int copies;
  int64_t wbytes;
};

template <class F>
double time_graph(Lab& L, int reps, F&& launch_one) {
  hipGraph_t g;
  hipGraphExec_t ge;
  for (int i = 0; i < 3; ++i) launch_one(i % L.copies);
  CK(hipStreamSynchronize(L.st));
  CK(hipStreamBeginCapture(L.st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < reps; ++i) launch_one(i % L.copies);
  CK(hipStreamEndCapture(L.st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, L.st));
  CK(hipStreamSynchronize(L.st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double best = 1e30;
  for (int t = 0; t < 5; ++t) {
    CK(hipEventRecord(a, L.st));
    CK(hipGraphLaunch(ge, L.st));
    CK(hipEventRecord(b, L.st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, (double)ms * 1e3 / reps);
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return best;
}

void report(const char* name, double us, int64_t bytes) {
  printf("%-58s %8.2f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  fflush(stdout);
}

template <int MS, int KSW, int NTW, class Epi>
void run_stream(Lab& L, const char* name, int N, int K, int splits, const Epi& epi,
                bool with_reduce) {
  const int nblk = Epi::kPaired ? N / 32 : N / 16 / NTW;
  const int ks = K / 32;
  const int klen = ((ks + splits - 1) / splits) * 32;
  const int need_steps = (klen / 32 + 7) / 8;
  if (need_steps > KSW) { printf("%-58s skipped (KSW too small)\n", name); return; }
  dim3 grid(nblk, splits, 1);
  float* parts = splits > 1 ? L.parts : nullptr;
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((gemm_stream_kernel<MS, KSW, NTW, Epi>), grid, dim3(512), 0, L.st,
                       L.x, (int64_t)0, L.w[c], (int64_t)0, 32, N, K, klen, (int64_t)0,
                       (int64_t)0, parts, epi, 1, nullptr, 0.0f);
    if (with_reduce && splits > 1) {
      int rb = (32 * N + 255) / 256;
      hipLaunchKernelGGL((splitk_reduce_kernel<Epi>), dim3(rb, 1), dim3(256), 0, L.st,
                         parts, splits, 1, 32, N, epi);
    }
  });
  report(name, us, (int64_t)N * K * 2);
}

template <int KSW, int NREP, int MODE>
void run_lab(Lab& L, const char* name, int N, int K, int splits) {
  const int ks = K / 32;
  const int klen = ((ks + splits - 1) / splits) * 32;
  if ((klen / 32 + 7) / 8 > KSW) { printf("%-58s skipped\n", name); return; }
  dim3 grid(N / 16 / NREP, splits);
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((lab_gemv<KSW, NREP, MODE>), grid, dim3(512), 0, L.st, L.x, L.w[c],
                       N, K, klen, L.parts);
  });
  report(name, us, (int64_t)N * K * 2);
}

template <int KSW, int NREP, int CH, int INF>
void run_pipe(Lab& L, const char* name, int N, int K) {
  dim3 grid(N / 16 / NREP);
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((lab_pipe_gemv<KSW, NREP, CH, INF>), grid, dim3(512), 0, L.st, L.x,
                       L.w[c], N, K, L.parts);
  });
  report(name, us, (int64_t)N * K * 2);
}

void run_read(Lab& L, const char* name, int64_t bytes, int blocks) {
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(256), 0, L.st,
                       reinterpret_cast<const uint4*>(L.w[c]), bytes / 16,
                       reinterpret_cast<uint32_t*>(L.out));
  });
  report(name, us, bytes);
}

}  // namespace

int main() {
  Lab L;
  CK(hipStreamCreate(&L.st));
  L.wbytes = (int64_t)15360 * 2560 * 2;     // largest shape: gated up-projection
  L.copies = 8;                              // 8 x 78.6 MB > 256 MB MALL
  for (int i = 0; i < L.copies; ++i) {
    u16* p;
    CK(hipMalloc(&p, L.wbytes));
    CK(hipMemset(p, 0x3c, L.wbytes));
    L.w.push_back(p);
  }
  CK(hipMalloc(&L.x, 32 * 7680 * 2));
  CK(hipMemset(L.x, 0x3c, 32 * 7680 * 2));
  CK(hipMalloc(&L.parts, (int64_t)8 * 32 * 15360 * 4));
  CK(hipMalloc(&L.out, (int64_t)32 * 15360 * 2 * 2));
  CK(hipMalloc(&L.bias, 15360 * 2));
  CK(hipMemset(L.bias, 0, 15360 * 2));

  printf("== pure streaming read (nt 16-B loads)\n");
  for (int blocks : {1024, 2048}) {
    char nm[96];
    snprintf(nm, sizeof nm, "read 79 MB, %d blocks x 256", blocks);
    run_read(L, nm, 15360LL * 2560 * 2, blocks);
  }
  EpiGatedGelu gg{L.out, 0, L.bias, L.bias, 2};
  printf("== gated up-projection N=15360 (2F) K=2560\n");
  run_stream<32, 10, 1>(L, "stream<32,10,1,Gated> s1 (shipped)", 15360, 2560, 1, gg, false);
  run_lab<10, 2, 0>(L, "lab<10,2> act+w s1 (all loads up front)", 15360, 2560, 1);
  run_pipe<10, 2, 2, 3>(L, "pipe<10,2> chunk 2 x 3 in flight (480 wg)", 15360, 2560);
  run_pipe<10, 4, 2, 3>(L, "pipe<10,4> chunk 2 x 3 in flight (240 wg)", 15360, 2560);
  run_pipe<10, 4, 2, 4>(L, "pipe<10,4> chunk 2 x 4 in flight (240 wg)", 15360, 2560);
  run_pipe<10, 4, 1, 6>(L, "pipe<10,4> chunk 1 x 6 in flight (240 wg)", 15360, 2560);
  run_pipe<10, 4, 5, 2>(L, "pipe<10,4> chunk 5 x 2 in flight (240 wg)", 15360, 2560);
  run_pipe<10, 6, 2, 3>(L, "pipe<10,6> chunk 2 x 3 in flight (160 wg)", 15360, 2560);
  printf("== down-projection shape N=2560 K=2560 split slice (one K split of 7680)\n");
  run_lab<10, 2, 0>(L, "lab<10,2> act+w s1 (80 wg)", 2560, 2560, 1);
  run_pipe<10, 2, 2, 3>(L, "pipe<10,2> chunk 2 x 3 (80 wg)", 2560, 2560);
  printf("done\n");
  return 0;
}
