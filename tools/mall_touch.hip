// Lab only (tools/mall_graph_probe.py): read a byte range with ordinary
// (cache-allocating) vector loads, so it lands in the Infinity Cache ahead of
// a decode GEMV that streams it with non-temporal loads.  Built by
// tools/mall_graph_probe.py into tools/_build/libmall_touch.so; not part of
// the library.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void touch_kernel(const uint4* __restrict__ p, int64_t n16,
                                                    uint32_t* __restrict__ sink) {
  const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t b = (int64_t)blockIdx.x * per;
  const int64_t e = b + per < n16 ? b + per : n16;
  uint32_t x = 0;
  for (int64_t i = b + threadIdx.x; i < e; i += 4 * 256) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + u * 256;
      v[u] = j < e ? p[j] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (x == 0x9e3779b9u) sink[blockIdx.x & 255] = x;   // keeps the loads alive
}

extern "C" int mall_touch(const void* p, int64_t bytes, int nwg, void* sink, void* stream) {
  if (bytes <= 0) return 0;
  hipLaunchKernelGGL(touch_kernel, dim3((unsigned)nwg), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint4*>(p),
                     bytes / 16, static_cast<uint32_t*>(sink));
  return (int)hipGetLastError();
}
