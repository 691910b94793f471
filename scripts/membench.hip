// Calibration microbenchmarks for the extraction kernel's memory patterns on
// MI355X: streaming 16-byte stores (the nucleotide/peptide output pattern),
// streaming reads, and 8-byte gathers at tile-local random windows.
//   hipcc -O3 --offload-arch=gfx950 scripts/membench.hip -o /tmp/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void store16(uint4* __restrict__ out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void read16(const uint4* __restrict__ in, size_t n16, uint32_t* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) *sink = acc;
}

// Each lane reads an 8-byte window at a pseudo-random word of a large table
// (the genome code plane), then stores 16 bytes contiguously (the output).
__global__ void gather_store(const uint32_t* __restrict__ table, size_t words,
                             uint4* __restrict__ out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    // windows are contiguous within groups of 64 lanes (one interval), random across groups
    const size_t grp = i >> 6;
    const size_t base = (grp * 0x9E3779B97F4A7C15ull) % (words - 128);
    const uint2 w = *reinterpret_cast<const uint2*>(table + base + (i & 63));
    out[i] = make_uint4(w.x, w.y, w.x ^ w.y, (uint32_t)i);
  }
}

int main() {
  const size_t out_bytes = 800ull << 20, tab_bytes = 256ull << 20;
  uint4* out;
  uint32_t *tab, *sink;
  CK(hipMalloc(&out, out_bytes));
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(tab, 1, tab_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t n16 = out_bytes / 16;
  for (int blocks_per_cu : {4, 8, 16}) {
    const int grid = ncu * blocks_per_cu;
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(store16, grid, 256, 0, 0, out, n16);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("store16     grid=%6d  %.3f ms  %.0f GB/s\n", grid, ms / 10, out_bytes / (ms / 10) / 1e6);
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(read16, grid, 256, 0, 0, out, n16, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("read16      grid=%6d  %.3f ms  %.0f GB/s\n", grid, ms / 10, out_bytes / (ms / 10) / 1e6);
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL(gather_store, grid, 256, 0, 0, tab, tab_bytes / 4, out, n16);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("gather+st   grid=%6d  %.3f ms  %.0f GB/s (stored bytes)\n", grid, ms / 10,
           out_bytes / (ms / 10) / 1e6);
  }
  return 0;
}
