// Calibrates what one sparse narrow read costs at the memory side on gfx950:
// does an isolated 12-byte load fill a whole 128-B L2 line (one EA request)
// or a 64-B half?  Run under rocprofv3 --pmc TCC_EA0_RDREQ_sum ... and compare
// requests per line for: (a) one 12-B load per line, (b) loads at both
// halves (offsets 0 and 64) of the same line, (c) 12-B loads at offset 60
// (straddling the 64-B halves).   hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t line_of(uint64_t i, uint64_t nlines) {
  return (i * 0x9E3779B97F4A7C15ull >> 17) % nlines;  // scattered, distinct-ish lines
}

template <int MODE>
__global__ void sparse(const uint8_t* __restrict__ buf, uint64_t nlines, uint64_t n,
                       uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* l = buf + line_of(i, nlines) * 128;
  uint32_t acc;
  if (MODE == 0) {
    const uint3 v = *reinterpret_cast<const uint3*>(l + 16);
    acc = v.x ^ v.y ^ v.z;
  } else if (MODE == 1) {
    const uint3 v = *reinterpret_cast<const uint3*>(l + 16);
    const uint3 w = *reinterpret_cast<const uint3*>(l + 80);
    acc = v.x ^ v.y ^ w.z ^ w.x;
  } else {
    const uint3 v = *reinterpret_cast<const uint3*>(l + 60);
    acc = v.x ^ v.y ^ v.z;
  }
  if (acc == 0x12345678u) *sink = acc;
}

int main() {
  const uint64_t bytes = 4ull << 30, nlines = bytes / 128, n = 16ull << 20;
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = (int)((n + 255) / 256);
  float ms;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(sparse<0>, blocks, 256, 0, 0, buf, nlines, n, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode0 one 12B load/line      %llu loads  %.3f ms  %.2f Gloads/s\n",
           (unsigned long long)n, ms, n / ms / 1e6);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(sparse<1>, blocks, 256, 0, 0, buf, nlines, n, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode1 loads at both halves   %llu lines  %.3f ms  %.2f Glines/s\n",
           (unsigned long long)n, ms, n / ms / 1e6);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(sparse<2>, blocks, 256, 0, 0, buf, nlines, n, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode2 12B load across halves %llu loads  %.3f ms  %.2f Gloads/s\n",
           (unsigned long long)n, ms, n / ms / 1e6);
  }
  return 0;
}
