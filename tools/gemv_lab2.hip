// Decode residual-projection lab: cold-weight timing of the two residual
// GEMV shapes of a decode token step (out projection N = 2560, K = 2560;
// MLP down projection N = 2560, K = 7680; M = 32 packed rows, fragment-packed
// weights), shipped split-K stream kernel (in-kernel last-arriver combine)
// against unsplit pipelined variants that write the EpiResidRows epilogue
// directly, and a pure streaming read of the same bytes.  Each variant is a
// hipGraph of back-to-back launches cycling over weight copies larger than
// the Infinity Cache.  Not part of the library; built by tools/gemv_lab2.sh.
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

// Unsplit residual GEMV: NW waves per workgroup walk the whole K of NREP
// 16-column tiles round-robin in 32-deep k-steps, in chunks of CH k-steps
// with INF chunks of weight + activation fragments in flight; fixed-order LDS
// reduction; EpiResidRows epilogue (bias / residual prefetched at start).
template <int NW, int KSW, int NREP, int CH, int INF>
__global__ __launch_bounds__(NW * 64) void resid_pipe(const u16* __restrict__ A,
                                                      const u16* __restrict__ W, int M, int K,
                                                      EpiResidRows epi) {
  constexpr int MR = 2, NC = KSW / CH;
  static_assert(KSW % CH == 0 && INF <= NC, "chunking");
  __shared__ float red[NW][32 * 16 * NREP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  const int ks32 = K >> 5;
  // epilogue operands: thread t owns (row t / 16, column t % 16) of each tile
  constexpr int EPT = (32 * 16 * NREP + NW * 64 - 1) / (NW * 64);
  EpiResidRows::Pref pf[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = min((int)threadIdx.x + e * NW * 64, 32 * 16 * NREP - 1);
    const int m = min(o / (16 * NREP), M - 1), j = (o / 16) % NREP, c = o % 16;
    pf[e] = epi.prefetch(m, (blockIdx.x * NREP + j) * 16 + c);
  }
  uint4 wb[INF][CH][NREP], xa[INF][CH][MR];
  auto issue = [&](int c, int slot) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = (wave + NW * (c * CH + u)) * 32;
      const bool ok = k < K;
#pragma unroll
      for (int j = 0; j < NREP; ++j)
        wb[slot][u][j] = ld16_nt(ok ? W + (((int64_t)(blockIdx.x * NREP + j) * ks32 + (k >> 5)) * 64 + lane) * 8
                                    : zpage);
#pragma unroll
      for (int i = 0; i < MR; ++i)
        xa[slot][u][i] = ld16(ok ? A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3) : zpage);
    }
  };
  f32x4 acc[MR][NREP];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < INF; ++c) issue(c, c);
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
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = threadIdx.x + e * NW * 64;
    if (o >= 32 * 16 * NREP) break;
    const int m = o / (16 * NREP), j = (o / 16) % NREP, c = o % 16;
    if (m >= M) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][o];
    epi.apply_pf(m, (blockIdx.x * NREP + j) * 16 + c, v, 0, pf[e]);
  }
}


// Split-K residual GEMV with many small workgroups: NW waves per workgroup,
// NREP 16-column tiles, K split over gridDim.y; every load issued before the
// first MFMA (as the shipped engine); in-kernel last-arriver combine in split
// order (sc1 slabs, one relaxed agent atomic per workgroup, sc1 loads).
template <int NW, int KSW, int NREP, int OCC>
__global__ __launch_bounds__(NW * 64, OCC) void resid_split(
    const u16* __restrict__ A, const u16* __restrict__ W, int M, int K, int klen,
    float* __restrict__ parts, int32_t* __restrict__ counters, EpiResidRows epi) {
  constexpr int MR = 2, NT = NW * 64, NE = 32 * 16 * NREP;
  constexpr int EPT = (NE + NT - 1) / NT;
  constexpr int SMAX = 8;
  __shared__ float red[NW][NE];
  __shared__ int ticket;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u16* zpage = reinterpret_cast<const u16*>(kZeroPage + lane);
  const int ks32 = K >> 5, N = gridDim.x * 16 * NREP;
  EpiResidRows::Pref pf[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = min((int)threadIdx.x + e * NT, NE - 1);
    const int m = min(o / (16 * NREP), M - 1), j = (o / 16) % NREP, c = o % 16;
    pf[e] = epi.prefetch(m, (blockIdx.x * NREP + j) * 16 + c);
  }
  const int kbeg = blockIdx.y * klen, kend = min(K, kbeg + klen);
  uint4 wb[KSW][NREP], xa[KSW][MR];
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kbeg + (wave + NW * u) * 32;
    const bool ok = k < kend;
#pragma unroll
    for (int i = 0; i < MR; ++i)
      xa[u][i] = ld16(ok ? A + ((((int64_t)(k >> 5) * MR + i) * 64 + lane) << 3) : zpage);
  }
#pragma unroll
  for (int u = 0; u < KSW; ++u) {
    const int k = kbeg + (wave + NW * u) * 32;
    const bool ok = k < kend;
#pragma unroll
    for (int j = 0; j < NREP; ++j)
      wb[u][j] = ld16_nt(ok ? W + (((int64_t)(blockIdx.x * NREP + j) * ks32 + (k >> 5)) * 64 + lane) * 8
                            : zpage);
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
  float v[EPT];
  const int64_t sstride = (int64_t)M * N;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = min((int)threadIdx.x + e * NT, NE - 1);
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w][o];
    v[e] = t;
    const int m = min(o / (16 * NREP), M - 1), j = (o / 16) % NREP, c = o % 16;
    if ((int)threadIdx.x + e * NT < NE)
      __hip_atomic_store(parts + blockIdx.y * sstride + (int64_t)m * N + (blockIdx.x * NREP + j) * 16 + c,
                         t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    ticket = __hip_atomic_fetch_add(counters + blockIdx.x, 1, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int S = gridDim.y;
  if (ticket != S - 1) return;
  float p[EPT][SMAX];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = min((int)threadIdx.x + e * NT, NE - 1);
    const int m = min(o / (16 * NREP), M - 1), j = (o / 16) % NREP, c = o % 16;
#pragma unroll
    for (int sp = 0; sp < SMAX; ++sp)
      p[e][sp] = __hip_atomic_load(parts + min(sp, S - 1) * sstride + (int64_t)m * N +
                                   (blockIdx.x * NREP + j) * 16 + c,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = threadIdx.x + e * NT;
    if (o >= NE) break;
    const int m = o / (16 * NREP), j = (o / 16) % NREP, c = o % 16;
    if (m >= M) continue;
    float t = 0.f;
#pragma unroll
    for (int sp = 0; sp < SMAX; ++sp)
      if (sp < S) t += sp == (int)blockIdx.y ? v[e] : p[e][sp];
    epi.apply_pf(m, (blockIdx.x * NREP + j) * 16 + c, t, 0, pf[e]);
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(counters + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Lab {
  hipStream_t st;
  std::vector<u16*> w;
  u16* x;
  float* parts;
  int32_t* counters;
  u16* out;
  u16* rows;
  u16* bias;
  u16* resid;
  int copies;
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

EpiResidRows make_epi(Lab& L, int N) {
  EpiResidRows e{};
  e.out = L.out;
  e.ldo = N;
  e.bias = L.bias;
  e.resid = L.resid;
  e.ldr = N;
  e.act = 0;
  e.map = RowMap{1 << 30, 0, 0};
  e.rows = L.rows;
  e.mt = 2;
  return e;
}

// the shipped launch (launch_stream_t's choice: MS 32, NTW 2, in-kernel combine)
template <int KSW>
void run_shipped(Lab& L, const char* name, int N, int K, int splits) {
  const int ks = K / 32;
  const int klen = ((ks + splits - 1) / splits) * 32;
  if ((klen / 32 + 7) / 8 > KSW) { printf("%-58s skipped\n", name); return; }
  EpiResidRows e = make_epi(L, N);
  dim3 grid(N / 32, splits, 1);
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((gemm_stream_kernel<32, KSW, 2, EpiResidRows>), grid, dim3(512), 0, L.st,
                       L.x, (int64_t)0, L.w[c], (int64_t)0, 32, N, K, klen, (int64_t)0,
                       (int64_t)0, L.parts, e, 1, L.counters, 0.0f);
  });
  report(name, us, (int64_t)N * K * 2);
}

template <int NW, int KSW, int NREP, int CH, int INF>
void run_pipe(Lab& L, const char* name, int N, int K) {
  if ((K / 32 + NW - 1) / NW > KSW) { printf("%-58s skipped\n", name); return; }
  EpiResidRows e = make_epi(L, N);
  dim3 grid(N / 16 / NREP);
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((resid_pipe<NW, KSW, NREP, CH, INF>), grid, dim3(NW * 64), 0, L.st, L.x,
                       L.w[c], 32, K, e);
  });
  report(name, us, (int64_t)N * K * 2);
}


template <int NW, int KSW, int NREP, int OCC>
void run_split(Lab& L, int N, int K, int splits) {
  const int ks = K / 32;
  const int klen = ((ks + splits - 1) / splits) * 32;
  char name[96];
  const int nblk = N / 16 / NREP;
  snprintf(name, sizeof name, "split nw%d nrep%d ksw%d occ%d S%d (%d wg)", NW, NREP, KSW, OCC,
           splits, nblk * splits);
  if ((klen / 32 + NW - 1) / NW > KSW) { printf("%-58s skipped\n", name); return; }
  EpiResidRows e = make_epi(L, N);
  dim3 grid(nblk, splits);
  const double us = time_graph(L, 60, [&](int c) {
    hipLaunchKernelGGL((resid_split<NW, KSW, NREP, OCC>), grid, dim3(NW * 64), 0, L.st, L.x,
                       L.w[c], 32, K, klen, L.parts, L.counters, e);
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
  const int64_t wbytes = (int64_t)2560 * 7680 * 2;   // down projection, 39.3 MB
  L.copies = 10;                                      // 393 MB > 256 MB MALL
  for (int i = 0; i < L.copies; ++i) {
    u16* p;
    CK(hipMalloc(&p, wbytes));
    CK(hipMemset(p, 0x3c, wbytes));
    L.w.push_back(p);
  }
  CK(hipMalloc(&L.x, 32 * 7680 * 2));
  CK(hipMemset(L.x, 0x3c, 32 * 7680 * 2));
  CK(hipMalloc(&L.parts, (int64_t)8 * 32 * 2560 * 4));
  CK(hipMalloc(&L.counters, 4096 * 4));
  CK(hipMemset(L.counters, 0, 4096 * 4));
  CK(hipMalloc(&L.out, (int64_t)32 * 2560 * 2));
  CK(hipMalloc(&L.rows, (int64_t)32 * 2560 * 2));
  CK(hipMalloc(&L.bias, 2560 * 2));
  CK(hipMemset(L.bias, 0, 2560 * 2));
  CK(hipMalloc(&L.resid, (int64_t)32 * 2560 * 2));
  CK(hipMemset(L.resid, 0, (int64_t)32 * 2560 * 2));

  printf("== pure streaming read (nt 16-B loads)\n");
  for (int blocks : {512, 1024}) {
    char nm[96];
    snprintf(nm, sizeof nm, "read 13.1 MB, %d blocks x 256", blocks);
    run_read(L, nm, 2560LL * 2560 * 2, blocks);
    snprintf(nm, sizeof nm, "read 39.3 MB, %d blocks x 256", blocks);
    run_read(L, nm, 2560LL * 7680 * 2, blocks);
  }
  printf("== down projection N=2560 K=7680 (39.3 MB): wider column tiles\n");
  run_shipped<10>(L, "shipped stream<32,10,2> S3 combine (240 wg)", 2560, 7680, 3);
  run_split<8, 5, 4, 1>(L, 2560, 7680, 6);
  run_split<8, 4, 4, 1>(L, 2560, 7680, 8);
  run_split<8, 8, 4, 1>(L, 2560, 7680, 4);
  run_split<8, 10, 3, 1>(L, 2560, 7680, 3);
  run_shipped<10>(L, "shipped stream<32,10,2> S3 combine (240 wg)", 2560, 7680, 3);
  printf("== out projection N=2560 K=2560 (13.1 MB)\n");
  run_shipped<5>(L, "shipped stream<32,5,2> S2 combine (160 wg)", 2560, 2560, 2);
  run_split<8, 2, 4, 1>(L, 2560, 2560, 5);
  run_split<8, 3, 2, 1>(L, 2560, 2560, 4);
  run_pipe<16, 5, 1, 1, 5>(L, "pipe nw16 nrep1 ch1x5 unsplit (160 wg)", 2560, 2560);
  run_shipped<5>(L, "shipped stream<32,5,2> S2 combine (160 wg)", 2560, 2560, 2);
  // round 5: more waves in flight (two or four workgroups per CU), after the
  // pure reads above reached their rate only at 2048 x 4 waves
  printf("== occupancy sweep: down projection\n");
  run_shipped<10>(L, "shipped stream<32,10,2> S3 combine (240 wg)", 2560, 7680, 3);
  run_split<8, 5, 2, 2>(L, 2560, 7680, 6);
  run_split<8, 4, 2, 2>(L, 2560, 7680, 8);
  run_split<16, 5, 2, 1>(L, 2560, 7680, 3);
  run_split<16, 3, 2, 1>(L, 2560, 7680, 5);
  run_split<8, 4, 1, 2>(L, 2560, 7680, 8);
  printf("== occupancy sweep: out projection\n");
  run_pipe<16, 5, 1, 1, 5>(L, "pipe nw16 nrep1 ch1x5 unsplit (160 wg)", 2560, 2560);
  run_split<8, 5, 2, 2>(L, 2560, 2560, 2);
  run_split<8, 3, 1, 2>(L, 2560, 2560, 4);
  run_split<4, 5, 1, 4>(L, 2560, 2560, 4);
  run_split<8, 2, 1, 2>(L, 2560, 2560, 5);
  printf("done\n");
  return 0;
}
