// Cross-launch weight prefetch lab (decode token step): does a streaming
// kernel that also touches the first bytes of the NEXT launch's weights
// (plain loads, so they allocate in L2 / the Infinity Cache) shorten the pair?
// A decode step is ~130 back-to-back GEMV launches whose weights do not
// depend on the previous launch's output, and each pays a ramp of ~2 us
// (profiles/r03u_decode_resid_lab_wide.log: 13.1 MB reads at 3.7 TB/s).
// Pure streaming reads stand in for the GEMVs (the bound on any gain): a
// hipGraph of alternating 13.1 MB (out projection) and 39.3 MB (down
// projection) reads cycling over 8 pairs of copies (419 MB > the 256 MB
// Infinity Cache), each launch prefetching `pf` bytes of the next one's
// buffer -- at its start (head) or after its own loop (tail).  Not part of
// the library; built by tools/mall_prefetch_lab.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: no prefetch; 1: prefetch issued at kernel start, consumed at the
// end; 2: prefetch after the own loop.  At most 4 prefetch loads per thread
// (pf16 <= 4 * grid threads).
template <int MODE>
__global__ __launch_bounds__(256) void read_pf(const u32x4* __restrict__ p, int64_t n16,
                                               const u32x4* __restrict__ nxt, int64_t pf16,
                                               uint32_t* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  u32x4 pf[4] = {};
  if constexpr (MODE == 1) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * stride < pf16) pf[u] = nxt[t + u * stride];
  }
  for (int64_t i = t; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if constexpr (MODE == 2) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * stride < pf16) pf[u] = nxt[t + u * stride];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) acc ^= pf[u].x ^ pf[u].w;
  if (acc == 0x12345678u) sink[0] = acc;
}

struct Lab {
  hipStream_t st;
  std::vector<u32x4*> a, b;   // 13.1 MB and 39.3 MB copies
  uint32_t* sink;
  int copies = 8;
};

constexpr int64_t kABytes = 2560LL * 2560 * 2;
constexpr int64_t kBBytes = 2560LL * 7680 * 2;

template <int MODE>
double time_pairs(Lab& L, int blocks, int64_t pf_bytes) {
  const int64_t pf16 = std::min<int64_t>(pf_bytes / 16, 4LL * blocks * 256);
  auto launch_pair = [&](int c) {
    const int cn = (c + 1) % L.copies;
    // the prefetch never reads past the next buffer
    hipLaunchKernelGGL(read_pf<MODE>, dim3(blocks), dim3(256), 0, L.st, L.a[c], kABytes / 16,
                       L.b[c], std::min(pf16, kBBytes / 16), L.sink);
    hipLaunchKernelGGL(read_pf<MODE>, dim3(blocks), dim3(256), 0, L.st, L.b[c], kBBytes / 16,
                       L.a[cn], std::min(pf16, kABytes / 16), L.sink);
  };
  const int pairs = 40;
  for (int i = 0; i < 3; ++i) launch_pair(i % L.copies);
  CK(hipStreamSynchronize(L.st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(L.st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < pairs; ++i) launch_pair(i % L.copies);
  CK(hipStreamEndCapture(L.st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, L.st));
  CK(hipStreamSynchronize(L.st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double best = 1e30;
  for (int t = 0; t < 7; ++t) {
    CK(hipEventRecord(e0, L.st));
    CK(hipGraphLaunch(ge, L.st));
    CK(hipEventRecord(e1, L.st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, (double)ms * 1e3 / pairs);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return best;
}

void report(const char* mode, int blocks, int64_t pf, double us) {
  printf("%-5s blocks %5d  prefetch %5.1f MB   pair %7.2f us  (%5.2f TB/s over 52.4 MB)\n", mode,
         blocks, pf / 1048576.0, us, (kABytes + kBBytes) / (us * 1e-6) / 1e12);
  fflush(stdout);
}

}  // namespace

int main() {
  Lab L;
  CK(hipStreamCreate(&L.st));
  for (int i = 0; i < L.copies; ++i) {
    u32x4* p;
    CK(hipMalloc(&p, kABytes));
    CK(hipMemset(p, 0x3c, kABytes));
    L.a.push_back(p);
    CK(hipMalloc(&p, kBBytes));
    CK(hipMemset(p, 0x3c, kBBytes));
    L.b.push_back(p);
  }
  CK(hipMalloc(&L.sink, 64));
  for (int blocks : {1024, 2048}) {
    for (int rep = 0; rep < 2; ++rep) {
      report("none", blocks, 0, time_pairs<0>(L, blocks, 0));
      for (int64_t mb : {2, 4, 8, 16}) {
        const int64_t pf = mb << 20;
        if (pf / 16 > 4LL * blocks * 256) continue;
        report("head", blocks, pf, time_pairs<1>(L, blocks, pf));
        report("tail", blocks, pf, time_pairs<2>(L, blocks, pf));
      }
    }
  }
  printf("done\n");
  return 0;
}
